"""llmi_engine_load_bin / llmi_group_load_bin: the reference's raw fp32 .bin files
(written by llmi/convert.py from the oracle's weights) loaded into the engine must give
exactly the synthetic-weight engine's tokens and logits (the PRNG weights are fp16 values,
so fp32 -> fp16 on load is exact), and the golden fixture's tokens. Bars: tokens bit-exact,
logits bit-exact against the synthetic load (same device arithmetic)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import llama_ref as R  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def tiny(tmp_path_factory):
    import llmi
    from llmi import convert as CV
    f = np.load(os.path.join(REPO, "tests", "golden", "tiny.npz"), allow_pickle=False)
    seed = int(f["seed"])
    cfg = R.LlamaConfig(hidden=512, heads=4, kv_heads=4, inter=1024, layers=2, max_seq=64)
    w = R.make_model_weights(cfg, seed)
    t = {"model.embed_tokens.weight": w.embed, "lm_head.weight": w.lm_head, "model.norm.weight": w.final_norm}
    for l, L in enumerate(w.layers):
        p = f"model.layers.{l}."
        t.update({p + "input_layernorm.weight": L.attn_norm, p + "post_attention_layernorm.weight": L.ffn_norm,
                  p + "self_attn.qkv.weight": L.qkv, p + "self_attn.o_proj.weight": L.o,
                  p + "mlp.gate_up_proj.weight": L.gate_up, p + "mlp.down_proj.weight": L.down})
    prefix = str(tmp_path_factory.mktemp("bin")) + "/"
    CV.write_bin(prefix, t)
    llmi.lib()
    return f, seed, prefix


def _run(make, load, prompt, n):
    with make() as e:
        load(e)
        toks = e.generate(prompt, n)
        return toks, e.logits()


@pytest.mark.parametrize("kv", ["f32", "f16"])
def test_engine_load_bin_matches_synthetic(tiny, kv):
    import llmi
    from llmi.engine import Engine, preset
    f, seed, prefix = tiny
    cfg = preset("tiny")
    cfg.kv_dtype = llmi.F32 if kv == "f32" else llmi.F16
    a_t, a_l = _run(lambda: Engine(cfg), lambda e: e.load_bin(prefix), f["prompt"], 8)
    b_t, b_l = _run(lambda: Engine(cfg), lambda e: e.load_synthetic(seed), f["prompt"], 8)
    np.testing.assert_array_equal(a_t, b_t)
    np.testing.assert_array_equal(a_l, b_l)
    if kv == "f32":
        np.testing.assert_array_equal(a_t, f["tokens"][:8])


def test_group_load_bin_tp2(tiny):
    from llmi.engine import TPGroup, preset
    import llmi
    f, seed, prefix = tiny
    cfg = preset("tiny")
    cfg.kv_dtype = llmi.F32
    a_t, a_l = _run(lambda: TPGroup(cfg, 2), lambda g: g.load_bin(prefix), f["prompt"], 8)
    b_t, b_l = _run(lambda: TPGroup(cfg, 2), lambda g: g.load_synthetic(seed), f["prompt"], 8)
    np.testing.assert_array_equal(a_t, b_t)
    np.testing.assert_array_equal(a_l, b_l)


def test_load_errors(tiny, tmp_path):
    import llmi
    from llmi._lib import LlmiError
    from llmi.engine import Engine, preset
    _, _, prefix = tiny
    cfg = preset("tiny")
    with Engine(cfg) as e:
        with pytest.raises(LlmiError, match="cannot open"):
            e.load_bin(str(tmp_path) + "/missing/")
        with pytest.raises(LlmiError, match="expected"):
            e.load_tensor("model.norm.weight", np.ones(7, np.float32))
        with pytest.raises(LlmiError, match="unknown tensor"):
            e.load_tensor("model.layers.0.self_attn.q_proj.weight", np.ones(7, np.float32))
        with pytest.raises(LlmiError, match="layer out of range"):
            e.load_tensor("model.layers.9.input_layernorm.weight", np.ones(512, np.float32))
    with Engine(preset("tiny", weight_dtype=llmi.I8)) as e:
        with pytest.raises(LlmiError, match="int8"):
            e.load_bin(prefix)
