"""The fused q/k/v GEMV + split-KV attention launch (csrc/qkv_attn.hip, engine option "qkv_attn")
against the two separate launches it replaces (masked_self_attention.cpp:54-92's qkv linear +
RoPE + decoder MHA): the GEMV and attention bodies are the same code, only the q/k/v hand-off
differs (tagged 8-byte granules polled inside the launch instead of a kernel boundary), so
tokens, logits and the final hidden state must be bitwise equal -- in graph replay and eager
launches, across split-count boundaries, for every weight / cache dtype the engine runs -- and
the reference fixtures must still hold with the fused launch."""
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


CASES = {
    "7b_f16_f16kv": ("llama2-7b", _lib.F16, _lib.F16),
    "7b_f16_f32kv": ("llama2-7b", _lib.F16, _lib.F32),
    "13b_i8_f16kv": ("llama2-13b", _lib.I8, _lib.F16),
    "tiny_f32_f32kv": ("tiny", _lib.F32, _lib.F32),
    "tiny_gqa_f16kv": ("tiny", _lib.F16, _lib.F16),  # kv_heads = heads / 2: natural row order
}


@pytest.mark.parametrize("case", list(CASES))
def test_fused_equals_two_launches(case):
    pname, wdt, kv = CASES[case]
    cfg = preset(pname, layers=2, max_seq=200)
    cfg.weight_dtype, cfg.kv_dtype = wdt, kv
    if "gqa" in case:
        cfg.kv_heads = cfg.heads // 2
    prompt = synth_prompt(3, 8, cfg.vocab)
    out = {}
    variants = {0: (0, 0), 1: (1, 0), 2: (1, 1)}  # separate launches / fused q/k/v + attention / + o_proj
    with Engine(cfg) as e:
        e.load_synthetic(7)
        for v, (qa, qo) in variants.items():
            e.set_option("qkv_attn", qa)
            e.set_option("qa_o", qo)
            for g in (True, False):
                n = 150 if g else 70  # graph: ctx 158, three split counts
                toks = e.generate(prompt, n, use_graph=g)
                out[(v, g)] = (toks.copy(), e.logits().copy(), e.hidden().copy())
    for v in (1, 2):
        for g in (True, False):
            for i in range(3):
                np.testing.assert_array_equal(out[(v, g)][i], out[(0, g)][i])
    print(f"{case}: fused q/k/v + attention (+ o_proj) bitwise equal to the separate launches (graph and eager)")


def test_fused_reference_fixtures():
    """F3 (7B width, 2 layers, fp32 KV) and F7 (ctx 2048 through the decode graph, fp16 KV
    against the oracle's cache rounding) with the fused launch."""
    f = np.load(os.path.join(G, "f3_decode.npz"), allow_pickle=False)
    cfg = preset("llama2-7b", layers=2, max_seq=64)
    cfg.kv_dtype = _lib.F32
    with Engine(cfg) as e:
        e.set_option("qkv_attn", 1)
        e.set_option("qa_o", 1)
        e.load_synthetic(int(f["seed"]))
        toks = e.generate(f["prompt"], len(f["tokens"]))
        np.testing.assert_array_equal(toks, f["tokens"])
        r = rel(e.logits(), f["last_logits"])
    print(f"f3 fused: logits rel-L2 vs reference {r:.3e}")
    assert r < 1e-3
    f = np.load(os.path.join(G, "f7_longctx.npz"), allow_pickle=False)
    cfg = preset("llama2-7b", layers=2, max_seq=2048)
    cfg.kv_dtype = _lib.F16
    with Engine(cfg) as e:
        e.set_option("qkv_attn", 1)
        e.set_option("qa_o", 1)
        e.load_synthetic(int(f["seed"]))
        toks = e.generate(f["prompt"], len(f["tokens"]))
        np.testing.assert_array_equal(toks, f["f16kv_tokens"])
        r = rel(e.logits(), f["f16kv_last_logits"])
    print(f"f7 ctx 2048 fused (fp16 KV): logits rel-L2 vs oracle {r:.3e}")
    assert r < 1e-3


def test_fused_one_layer_across_prompts():
    """One layer and one-token prompts: the granule buffer then holds the tag of the same layer
    index from the previous forward, so tags must come from a per-forward epoch that set_prompt
    does not reset (a reset epoch would let the attention read the previous prompt's q/k/v)."""
    cfg = preset("tiny", layers=1, max_seq=64)
    cfg.kv_dtype = _lib.F32
    res = {}
    with Engine(cfg) as e:
        e.load_synthetic(5)
        for v in (0, 1):
            e.set_option("qkv_attn", v)
            e.set_option("qa_o", v)
            res[v] = []
            for p in ([3], [11], [3], [29, 4]):
                t = e.generate(np.array(p, np.int32), 1)
                res[v].append((t.copy(), e.logits().copy()))
    for a, b in zip(res[0], res[1]):
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])


@pytest.mark.parametrize("use_graph", [True, False])
def test_fused_position_mismatch_is_reported(use_graph):
    """The fused launch keeps the attention's host/device split-count check (error bit 4)."""
    cfg = preset("tiny", max_seq=256)
    cfg.kv_dtype = _lib.F32
    prompt = synth_prompt(1, 8, cfg.vocab)
    with Engine(cfg) as e:
        e.set_option("qkv_attn", 1)
        e.set_option("qa_o", 1)
        e.load_synthetic(2)
        e.set_prompt(prompt)
        e.decode(len(prompt), use_graph=use_graph)
        e.tokens()
        e.debug_set_next_pos(100)
        e.decode(1, use_graph=use_graph)
        with pytest.raises(_lib.LlmiError, match="device error flag 4"):
            e.tokens()
