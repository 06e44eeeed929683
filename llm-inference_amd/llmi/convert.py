"""The reference's on-disk weight format and a Hugging Face checkpoint converter.

Format (what LlamaWeight<T>::loadWeights reads, llama_weights.cc:41-53,
layer_weights.cc:48-66, loadWeightFromBin weight_utils.cu:90-187): one raw
little-endian fp32 file per tensor, named `<prefix><name>.bin`, with the attention
projections fused as `self_attn.qkv.weight` = [q; k; v] rows and the MLP as
`mlp.gate_up_proj.weight` = [gate; up] rows. The reference ships no converter
(SURVEY.md §8f rank 2); `convert_hf` below builds those files from an HF Llama
state dict (`q_proj/k_proj/v_proj/o_proj/gate_proj/up_proj/down_proj`, norms,
`embed_tokens`, `lm_head`), e.g. one loaded with `safetensors.numpy.load_file`.
Host-side file I/O only; the engine (llmi_engine_load_bin) does the device upload.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, Mapping

import numpy as np

LAYER_LEAVES = ("input_layernorm.weight", "post_attention_layernorm.weight", "self_attn.qkv.weight",
                "self_attn.o_proj.weight", "mlp.gate_up_proj.weight", "mlp.down_proj.weight")
GLOBAL_NAMES = ("model.norm.weight", "lm_head.weight", "model.embed_tokens.weight")


def tensor_names(layers: int) -> Iterable[str]:
    yield from GLOBAL_NAMES
    for l in range(layers):
        for leaf in LAYER_LEAVES:
            yield f"model.layers.{l}.{leaf}"


def write_bin(prefix: str, tensors: Mapping[str, np.ndarray]) -> None:
    """Write each tensor as `<prefix><name>.bin` (raw fp32). A directory prefix needs its
    trailing separator, as the reference's weight_path does (user_entry.cpp:8)."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    for name, t in tensors.items():
        np.ascontiguousarray(t, dtype=np.float32).tofile(prefix + name + ".bin")


def read_bin(prefix: str, name: str) -> np.ndarray:
    return np.fromfile(prefix + name + ".bin", dtype=np.float32)


def convert_hf(state: Mapping[str, np.ndarray], layers: int) -> Dict[str, np.ndarray]:
    """HF Llama names -> the reference's fused names (fp32). lm_head falls back to the
    embedding when the checkpoint ties them."""
    f = lambda k: np.asarray(state[k], dtype=np.float32)  # noqa: E731
    out = {
        "model.embed_tokens.weight": f("model.embed_tokens.weight"),
        "lm_head.weight": f("lm_head.weight") if "lm_head.weight" in state else f("model.embed_tokens.weight"),
        "model.norm.weight": f("model.norm.weight"),
    }
    for l in range(layers):
        p = f"model.layers.{l}."
        out[p + "input_layernorm.weight"] = f(p + "input_layernorm.weight")
        out[p + "post_attention_layernorm.weight"] = f(p + "post_attention_layernorm.weight")
        out[p + "self_attn.qkv.weight"] = np.concatenate(
            [f(p + "self_attn.q_proj.weight"), f(p + "self_attn.k_proj.weight"), f(p + "self_attn.v_proj.weight")])
        out[p + "self_attn.o_proj.weight"] = f(p + "self_attn.o_proj.weight")
        out[p + "mlp.gate_up_proj.weight"] = np.concatenate(
            [f(p + "mlp.gate_proj.weight"), f(p + "mlp.up_proj.weight")])
        out[p + "mlp.down_proj.weight"] = f(p + "mlp.down_proj.weight")
    return out


def convert_safetensors(files: Iterable[str], layers: int, prefix: str) -> None:
    """Convert HF `*.safetensors` shards (loaded without pickle) and write the .bin set."""
    from safetensors.numpy import load_file
    state: Dict[str, np.ndarray] = {}
    for fn in files:
        state.update(load_file(fn))
    write_bin(prefix, convert_hf(state, layers))
