"""Ring layer (ring.hip, LLMI_FUSED=4) and merged attention + row-GEMV o_proj
(LLMI_FUSED=5) on the MI355X. Ring: attention with the in-kernel
merge, then o_proj + gate_up + down as one persistent launch fed by an LDS-DMA
weight ring. Bars: the reference fixtures (tokens exact, logits within the
north-star 1e-3; fp32-KV parity runs within 2e-6 like the five-launch path), and
the five-launch engine on the full 7B model (tokens exact)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from llmi import _lib  # noqa: E402
from llmi.engine import Engine, preset, synth_prompt  # noqa: E402

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def run(cfg, seed, prompt, n_new, mode, use_graph=True):
    old = os.environ.get("LLMI_FUSED")
    os.environ["LLMI_FUSED"] = mode
    try:
        with Engine(cfg) as e:
            e.load_synthetic(seed)
            toks = e.generate(prompt, n_new, use_graph=use_graph)
            return toks, e.logits(), e.hidden()
    finally:
        if old is None:
            os.environ.pop("LLMI_FUSED", None)
        else:
            os.environ["LLMI_FUSED"] = old


@pytest.mark.parametrize("mode", ["4", "5"])
@pytest.mark.parametrize("name,cfgname,over,kv", [
    ("tiny.npz", "tiny", {}, _lib.F32),
    ("f3_decode.npz", "llama2-7b", dict(layers=2, max_seq=64), _lib.F32),
    ("f3_decode.npz", "llama2-7b", dict(layers=2, max_seq=64), _lib.F16),
])
def test_ring_matches_reference(name, cfgname, over, kv, mode):
    f = np.load(os.path.join(G, name))
    cfg = preset(cfgname, **over)
    cfg.kv_dtype = kv
    n = len(f["tokens"])
    t, lg, _ = run(cfg, int(f["seed"]), f["prompt"], n, mode)
    np.testing.assert_array_equal(t, f["tokens"])
    r = rel(lg, f["last_logits"])
    print(f"{name} ring logits rel-L2 vs reference: {r:.3e}")
    assert r < (2e-6 if kv == _lib.F32 else 1e-3)


@pytest.mark.parametrize("mode", ["4", "5"])
def test_ring_eager_equals_graph_bitwise(mode):
    cfg = preset("llama2-7b", layers=2, max_seq=128)
    prompt = synth_prompt(0, 8, cfg.vocab)
    tg, lg, hg = run(cfg, 0, prompt, 40, mode)
    te, le, he = run(cfg, 0, prompt, 40, mode, use_graph=False)
    np.testing.assert_array_equal(tg, te)
    np.testing.assert_array_equal(lg, le)
    np.testing.assert_array_equal(hg, he)


@pytest.mark.parametrize("mode", ["4", "5"])
def test_ring_full_7b_matches_five_launches(mode):
    cfg = preset("llama2-7b", max_seq=512)
    prompt = synth_prompt(0, 8, cfg.vocab)
    tr, lr, _ = run(cfg, 0, prompt, 300, mode)
    tu, lu, _ = run(cfg, 0, prompt, 300, "0")
    np.testing.assert_array_equal(tr, tu)
    r = rel(lr, lu)
    print(f"ring vs five launches, 7B 300 tokens: logits rel-L2 {r:.3e}")
    assert r < 1e-4


def test_ring_timing_reported():
    cfg = preset("llama2-7b", layers=8, max_seq=2048)
    os.environ["LLMI_FUSED"] = "4"
    try:
        with Engine(cfg) as e:
            e.load_synthetic(0)
            e.generate(synth_prompt(0, 8, cfg.vocab), 1000)
            us, b = e.time_kernel("ring", 50)
            am, _ = e.time_kernel("attn_merge", 50)
    finally:
        os.environ.pop("LLMI_FUSED", None)
    print(f"ring layer {us:.1f} us ({b / us / 1e3:.0f} GB/s), attention+merge {am:.1f} us")
    assert us > 0
