"""Dataflow layer kernel (layer.hip, LLMI_FUSED=1) and the co-scheduled
attention + o_proj launch (attn.hip, LLMI_FUSED=3) on the MI355X: in-launch
counter hand-offs must produce exactly what the standalone launches produce -- same device bodies, same arithmetic, and the o_proj's
int64 fixed-point atomics are order-independent -- so the bar is bitwise
equality of tokens and logits, plus the reference fixtures as usual."""
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


def run(cfg, seed, prompt, n_new, fused, use_graph=True):
    old = os.environ.get("LLMI_FUSED")
    os.environ["LLMI_FUSED"] = fused if isinstance(fused, str) else ("1" if fused else "0")
    os.environ["LLMI_DOWN_KSPLIT"] = "4"  # both paths run the same down slicing (bitwise comparison)
    try:
        with Engine(cfg) as e:
            e.load_synthetic(seed)
            toks = e.generate(prompt, n_new, use_graph=use_graph)
            return toks, e.logits(), e.hidden()
    finally:
        os.environ.pop("LLMI_DOWN_KSPLIT", None)
        if old is None:
            os.environ.pop("LLMI_FUSED", None)
        else:
            os.environ["LLMI_FUSED"] = old


@pytest.mark.parametrize("mode", ["1", "3"])
@pytest.mark.parametrize("name,cfgname,over,wdt,kv", [
    ("tiny.npz", "tiny", {}, _lib.F16, _lib.F32),
    ("f3_decode.npz", "llama2-7b", dict(layers=2, max_seq=64), _lib.F16, _lib.F32),
    ("f3_decode.npz", "llama2-7b", dict(layers=2, max_seq=64), _lib.F16, _lib.F16),
    ("f5_int8.npz", "llama2-13b", dict(layers=1, max_seq=32), _lib.I8, _lib.F32),
])
def test_fused_equals_unfused_bitwise(name, cfgname, over, wdt, kv, mode):
    f = np.load(os.path.join(G, name))
    cfg = preset(cfgname, **over)
    cfg.weight_dtype, cfg.kv_dtype = wdt, kv
    n = len(f["tokens"])
    tf, lf, hf = run(cfg, int(f["seed"]), f["prompt"], n, mode)
    tu, lu, hu = run(cfg, int(f["seed"]), f["prompt"], n, False)
    np.testing.assert_array_equal(tf, tu)
    np.testing.assert_array_equal(lf, lu)
    np.testing.assert_array_equal(hf, hu)
    np.testing.assert_array_equal(tf, f["tokens"])
    if kv == _lib.F32:
        r = rel(lf, f["last_logits"])
        print(f"{name} fused logits rel-L2 vs reference: {r:.3e}")
        assert r < 1e-3


@pytest.mark.parametrize("mode", ["1", "3"])
def test_fused_full_7b_long_context_bitwise(mode):
    """Bench model past many split-KV chunks: 300 forwards, graph replay and eager."""
    cfg = preset("llama2-7b", max_seq=512)
    prompt = synth_prompt(0, 8, cfg.vocab)
    tf, lf, _ = run(cfg, 0, prompt, 300, mode)
    tu, lu, _ = run(cfg, 0, prompt, 300, False)
    te, le, _ = run(cfg, 0, prompt, 40, mode, use_graph=False)
    np.testing.assert_array_equal(tf, tu)
    np.testing.assert_array_equal(lf, lu)
    np.testing.assert_array_equal(te, tu[:40])


def test_fused_layer_timing_reported():
    cfg = preset("llama2-7b", layers=2, max_seq=2048)
    os.environ["LLMI_FUSED"] = "1"
    try:
        with Engine(cfg) as e:
            e.load_synthetic(0)
            e.generate(synth_prompt(0, 8, cfg.vocab), 1000)
            us, b = e.time_kernel("layer", 50)
            parts = {k: e.time_kernel(k, 50)[0] for k in ("qkv", "attn", "o", "gate_up", "down")}
    finally:
        os.environ.pop("LLMI_FUSED", None)
    print(f"fused layer {us:.1f} us ({b / us / 1e3:.0f} GB/s) vs five kernels back to back "
          f"{sum(parts.values()):.1f} us {parts}")
    assert us > 0
