#!/usr/bin/env python3
"""One rank of a tensor-parallel engine group that exchanges through the one-shot
peer path (llmi_engine_xchg_*) instead of RCCL: run as a separate process per rank
by tests/test_gpu_xchg.py. The 64-byte inbox handles are exchanged through files in
a rendezvous directory (any side channel works; bench.py uses torch.distributed).

    python xchg_worker.py <rank> <world> <device> <rendezvous_dir> <fixture.npz> <preset> <n_new>
Writes <rendezvous_dir>/out_<rank>.npz: tokens, logits (this rank's vocab shard)."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "llm-inference_amd"))

from llmi import _lib  # noqa: E402
from llmi.engine import Engine, preset  # noqa: E402


def wait_for(paths, timeout=60.0):
    t0 = time.time()
    while not all(os.path.exists(p) for p in paths):
        if time.time() - t0 > timeout:
            raise TimeoutError(f"rendezvous: missing {[p for p in paths if not os.path.exists(p)]}")
        time.sleep(0.02)


def main():
    rank, world, device, rdv, fixture, pname, n_new = sys.argv[1:8]
    rank, world, device, n_new = int(rank), int(world), int(device), int(n_new)
    f = np.load(fixture, allow_pickle=False)
    cfg = preset(pname, tp_rank=rank, tp_world=world)
    if os.environ.get("XCHG_LAYERS"):  # timing runs: a thin model of the preset's width
        cfg.layers, cfg.max_seq = int(os.environ["XCHG_LAYERS"]), 64
    cfg.kv_dtype = _lib.F32
    with Engine(cfg, device=device) as e:  # no RCCL id: the one-shot exchange only
        e.load_synthetic(int(f["seed"]))
        h = e.xchg_handle()
        tmp = os.path.join(rdv, f".h{rank}")
        with open(tmp, "wb") as fh:
            fh.write(h)
        os.replace(tmp, os.path.join(rdv, f"h{rank}"))
        paths = [os.path.join(rdv, f"h{q}") for q in range(world)]
        wait_for(paths)
        e.xchg_open([open(p, "rb").read() for p in paths])
        mode = int(os.environ.get("XCHG_MODE", "1"))  # 1: exchange launches, 2: fused into the producers
        e.set_exchange(mode)
        toks = {}
        for g in (True, False):
            toks[g] = e.generate(f["prompt"], n_new, use_graph=g)
        logits = e.logits()
        timing = {}
        if os.environ.get("XCHG_TIME"):  # a collective: every rank times the same calls
            e.set_exchange(1)
            timing = {k: e.time_kernel(k, 256)[0] for k in ("xchg", "xchg_graph")}
            n_loop = min(cfg.max_seq - 1, 48)
            for m in (1, 2, 1, 2):  # graph-replayed decode per exchange form, alternating
                e.set_exchange(m)
                e.generate(f["prompt"], 4)  # capture + warm
                e.set_prompt(f["prompt"])
                e.sync()
                t0 = time.perf_counter()
                e.decode(n_loop)
                e.sync()
                us = (time.perf_counter() - t0) / n_loop * 1e6
                timing[f"loop_mode{m}"] = min(us, timing.get(f"loop_mode{m}", us))
        np.savez(os.path.join(rdv, f"out_{rank}.npz"), tokens=toks[True], tokens_eager=toks[False], logits=logits,
                 **{f"us_{k}": np.float64(v) for k, v in timing.items()})
        # stay alive until every rank is done (no inbox freed while a peer may still write it)
        open(os.path.join(rdv, f"done{rank}"), "w").close()
        wait_for([os.path.join(rdv, f"done{q}") for q in range(world)])
    print(f"rank {rank}: ok", flush=True)


if __name__ == "__main__":
    main()
