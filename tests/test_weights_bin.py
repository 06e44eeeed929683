"""The reference's fp32 .bin weight format (llmi/convert.py) on CPU: the HF -> fused-name
converter, file round trips (raw .bin and safetensors), and the loader's C-ABI argument
checks. The device upload is covered by tests/test_gpu_weights_bin.py."""
import numpy as np

from oracle import llama_ref as R
from llmi import convert as CV

CFG = R.LlamaConfig(hidden=128, heads=2, kv_heads=1, inter=256, layers=2, vocab=300, max_seq=16)


def _hf_state(cfg, seed=3):
    w = R.make_model_weights(cfg, seed)
    st = {"model.embed_tokens.weight": w.embed, "lm_head.weight": w.lm_head, "model.norm.weight": w.final_norm}
    for l, L in enumerate(w.layers):
        p = f"model.layers.{l}."
        q, k, v = np.split(L.qkv, [cfg.q_rows, cfg.q_rows + cfg.kv_rows])
        g, u = np.split(L.gate_up, 2)
        st.update({p + "self_attn.q_proj.weight": q, p + "self_attn.k_proj.weight": k,
                   p + "self_attn.v_proj.weight": v, p + "self_attn.o_proj.weight": L.o,
                   p + "mlp.gate_proj.weight": g, p + "mlp.up_proj.weight": u, p + "mlp.down_proj.weight": L.down,
                   p + "input_layernorm.weight": L.attn_norm, p + "post_attention_layernorm.weight": L.ffn_norm})
    return w, st


def test_convert_hf_fuses_in_reference_order():
    w, st = _hf_state(CFG)
    out = CV.convert_hf(st, CFG.layers)
    assert sorted(out) == sorted(CV.tensor_names(CFG.layers))
    for l, L in enumerate(w.layers):
        p = f"model.layers.{l}."
        np.testing.assert_array_equal(out[p + "self_attn.qkv.weight"], L.qkv.astype(np.float32))
        np.testing.assert_array_equal(out[p + "mlp.gate_up_proj.weight"], L.gate_up.astype(np.float32))
        assert out[p + "self_attn.qkv.weight"].shape == (CFG.q_rows + 2 * CFG.kv_rows, CFG.hidden)
    tied = {k: v for k, v in st.items() if k != "lm_head.weight"}
    np.testing.assert_array_equal(CV.convert_hf(tied, CFG.layers)["lm_head.weight"], w.embed.astype(np.float32))


def test_bin_and_safetensors_round_trip(tmp_path):
    from safetensors.numpy import save_file
    _, st = _hf_state(CFG)
    ref = CV.convert_hf(st, CFG.layers)
    CV.write_bin(str(tmp_path / "a") + "/", ref)
    for n, t in ref.items():
        np.testing.assert_array_equal(CV.read_bin(str(tmp_path / "a") + "/", n), t.reshape(-1))
    save_file({k: np.ascontiguousarray(v) for k, v in st.items()}, str(tmp_path / "m.safetensors"))
    CV.convert_safetensors([str(tmp_path / "m.safetensors")], CFG.layers, str(tmp_path / "b") + "/")
    for n, t in ref.items():
        np.testing.assert_array_equal(CV.read_bin(str(tmp_path / "b") + "/", n), t.reshape(-1))


def test_loader_c_abi_argument_checks():
    from llmi import _lib
    L = _lib.lib()
    assert L.llmi_engine_load_bin(None, b"/nonexistent/") == -1
    assert L.llmi_engine_load_tensor(None, b"model.norm.weight", None, 0) == -1
    assert L.llmi_group_load_bin(None, b"/nonexistent/") == -1
