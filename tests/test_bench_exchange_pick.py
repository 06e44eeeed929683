"""bench.py's choice between the two one-shot exchange forms at N > 1 (pick_fused_exchange),
on CPU with a gloo world of 2 and a stand-in engine (no GPU): both forms must reproduce the
checked tokens on every rank, then the faster by the slowest rank is kept; a rank whose
fused tokens differ, or whose timing raises, makes EVERY rank keep the exchange launches
(mode 1) -- never a split decision, never a collective left waiting."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FakeEngine:
    def __init__(self, rank, fused_ok=True, slow_mode=2, raise_in_timing=False):
        self.rank, self.fused_ok, self.slow_mode, self.raise_in_timing = rank, fused_ok, slow_mode, raise_in_timing
        self.mode, self.modes_set = 1, []

        class C:
            max_seq = 64
        self.cfg = C()

    def set_exchange(self, m):
        self.mode = m
        self.modes_set.append(m)

    def generate(self, prompt, n):
        t = np.arange(n, dtype=np.int32)
        return t + 1 if (self.mode == 2 and not self.fused_ok) else t

    def set_prompt(self, p):
        pass

    def decode(self, n):
        import time
        if self.raise_in_timing and self.mode == 2:
            raise RuntimeError("device error flag 8")
        time.sleep(0.02 if self.mode == self.slow_mode else 0.001)

    def sync(self):
        pass


def _worker(rank, world, port, case, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, REPO)
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        kw = {"ok": {}, "slow_fused": {"slow_mode": 2}, "slow_launches": {"slow_mode": 1},
              "bad_tokens": {"fused_ok": rank != 1}, "raises": {"raise_in_timing": rank == 0}}[case]
        eng = FakeEngine(rank, **kw)
        out = bench.pick_fused_exchange(eng, dist, np.zeros(4, np.int32), world, np.arange(8, dtype=np.int32))
        q.put((rank, out, eng.mode))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,want_mode", [("slow_fused", 1), ("slow_launches", 2), ("bad_tokens", 1),
                                            ("raises", 1)])
def test_pick_is_consistent_across_ranks(case, want_mode):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    modes = {r: m for r, _, m in res}
    assert modes[0] == modes[1] == want_mode, res
    for _, out, _ in res:
        if want_mode == 2:
            assert out["mode"] == "fused" and len(out["us_per_forward_oneshot_vs_fused"]) == 2
        elif case in ("bad_tokens", "raises"):
            assert out["fused_rejected"]
        else:
            assert out["mode"] == "oneshot"
