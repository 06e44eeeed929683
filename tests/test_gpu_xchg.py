"""The one-shot peer exchange of tensor-parallel decode (config 4; csrc/xchg.hip):
each exchange is one kernel per rank that writes the rank's int64 residual partial into
every peer's inbox, raises per-slice flags, waits for every rank and sums the slots in
rank order -- the RCCL all-reduce of modeling_llama.py's pretraining_tp sums
(:251-266, :443-446) without a collective library.

On one GPU it is checked two ways:
  * inside the in-process group (llmi_group_set_exchange 1): the same kernels, every
    rank's push then every rank's reduce, must give BITWISE the reduction-kernel path's
    tokens, logits and hidden states (int64 sums are exact) and the reference fixtures;
  * across real processes: two engines in two processes on the same device, inboxes
    shared through hipIpcGetMemHandle / hipIpcOpenMemHandle, flags polled across
    processes while both run -- tokens equal the fixture and logits equal the group's."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from llmi import _lib  # noqa: E402
from llmi.engine import TPGroup, preset  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden")


def load(name):
    return np.load(os.path.join(G, name), allow_pickle=False)


def group_run(name, cfg, world, mode, use_graph):
    f = load(name)
    with TPGroup(cfg, world) as g:
        g.set_exchange(mode)
        g.load_synthetic(int(f["seed"]))
        toks = g.generate(f["prompt"], len(f["tokens"]), use_graph=use_graph)
        per_rank = [g.tokens(r) for r in range(world)]
        return f, toks, per_rank, g.logits(), [g.hidden(r) for r in range(world)]


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("name,pname,kw,world,use_graph", [
    ("tiny.npz", "tiny", {}, 2, True),
    ("tiny.npz", "tiny", {}, 4, False),
    ("f4_tp8.npz", "llama2-7b", {"layers": 2, "max_seq": 64}, 8, True),
])
def test_group_oneshot_equals_reduce_kernel_bitwise(name, pname, kw, world, use_graph, mode):
    """mode 1: exchange launches; mode 2: the push fused into the o_proj / down / lm_head
    launches (their tails), then the reduce kernels."""
    cfg = preset(pname, **kw)
    cfg.kv_dtype = _lib.F32
    f, t0, r0, l0, h0 = group_run(name, cfg, world, 0, use_graph)
    _, t1, r1, l1, h1 = group_run(name, cfg, world, mode, use_graph)
    np.testing.assert_array_equal(t1, f["tokens"])
    np.testing.assert_array_equal(t1, t0)
    for a, b in zip(r1, r0):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(l1, l0)
    for a, b in zip(h1, h0):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("mode", [1, 2])
def test_oneshot_two_processes_one_gpu_ipc(tmp_path, mode):
    """Two rank processes on device 0 (RCCL refuses that; the one-shot exchange does not
    care where the peer's inbox lives): IPC handles through files, cross-process flags.
    mode 2: each process's o_proj / down / lm_head launches push, wait for the other
    process and reduce from inside the launch."""
    f = load("tiny.npz")
    n_new = len(f["tokens"])
    worker = os.path.join(HERE, "helpers", "xchg_worker.py")
    env = dict(os.environ, XCHG_MODE=str(mode))
    procs = [subprocess.Popen([sys.executable, worker, str(r), "2", "0", str(tmp_path), os.path.join(G, "tiny.npz"),
                               "tiny", str(n_new)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                              env=env)
             for r in range(2)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o
    res = [np.load(os.path.join(tmp_path, f"out_{r}.npz")) for r in range(2)]
    for r in res:
        np.testing.assert_array_equal(r["tokens"], f["tokens"])
        np.testing.assert_array_equal(r["tokens_eager"], f["tokens"])
    cfg = preset("tiny")
    cfg.kv_dtype = _lib.F32
    _, _, _, lg, _ = group_run("tiny.npz", cfg, 2, 0, True)
    np.testing.assert_array_equal(np.concatenate([r["logits"] for r in res]), lg)


@pytest.mark.parametrize("world", [2, 8])
def test_loopback_rank_exchange_modes_agree_bitwise(world):
    """llmi_engine_xchg_loopback (the one-GPU pricing of a single TP rank): every peer inbox is
    the rank's own, the push writes its partial into its own slot and zeros into the others,
    so the one-shot exchange (mode 1) and the producer-fused tail (mode 2) must reduce to the
    rank's own partial -- tokens, logits and hidden state bitwise those of running with no
    exchange at all (mode 0), graph replay and eager alike."""
    from llmi.engine import Engine
    cfg = preset("llama2-7b", layers=2, max_seq=160, tp_rank=0, tp_world=world)
    out = {}
    with Engine(cfg) as e:
        e.load_synthetic(3)
        e.xchg_loopback()
        prompt = np.array([1, 5, 9, 13, 17, 21, 25, 29], np.int32)
        for mode in (0, 1, 2):
            e.set_exchange(mode)
            for graph in (True, False):
                toks = e.generate(prompt, 70, use_graph=graph)  # crosses a split-count boundary
                out[(mode, graph)] = (toks.copy(), e.logits().copy(), e.hidden().copy())
    ref = out[(0, True)]
    for k, v in out.items():
        np.testing.assert_array_equal(v[0], ref[0], err_msg=str(k))
        np.testing.assert_array_equal(v[1], ref[1], err_msg=str(k))
        np.testing.assert_array_equal(v[2], ref[2], err_msg=str(k))
