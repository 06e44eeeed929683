"""ctypes binding of libllmi.so (include/llmi.h).

The shared library is the product: this module only declares signatures and
turns negative return codes into exceptions. There is no fallback -- if the
library is missing the import fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(_HERE)
REPO = os.path.dirname(PKG)
LIB_PATH = os.environ.get("LLMI_LIB_PATH") or os.path.join(PKG, "lib", "libllmi.so")
HEADER = os.path.join(REPO, "include", "llmi.h")

F32, F16, I8, I32, I64 = 0, 1, 2, 3, 4
SYN_LINEAR, SYN_EMBED, SYN_GAMMA, SYN_INT8, SYN_INT8_SCALE = 0, 1, 2, 3, 4


class LlmiError(RuntimeError):
    pass


class Config(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("hidden", "heads", "kv_heads", "head_dim", "inter", "layers",
                                        "vocab", "max_seq")] + \
               [("rms_eps", C.c_float), ("rope_base", C.c_float)] + \
               [(n, C.c_int) for n in ("weight_dtype", "kv_dtype", "tp_rank", "tp_world")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


_P, _I, _U64, _U32, _F, _SZ = C.c_void_p, C.c_int, C.c_uint64, C.c_uint32, C.c_float, C.c_size_t
_SIGS = {
    "llmi_last_error": (C.c_char_p, []),
    "llmi_version": (C.c_char_p, []),
    "llmi_embedding": (_I, [_P, _I, _P, _I, _I, _I, _P, _P]),
    "llmi_rmsnorm": (_I, [_P, _P, _P, _P, _I, _I, _I, _F, _P]),
    "llmi_add_residual_rmsnorm": (_I, [_P, _P, _P, _I, _P, _I, _I, _I, _F, _P]),
    "llmi_add_residual": (_I, [_P, _P, _I, _I, _P]),
    "llmi_silu_mul": (_I, [_P, _P, _I, _I, _P]),
    "llmi_convert": (_I, [_P, _I, _P, _I, _SZ, _P]),
    "llmi_linear": (_I, [_P, _P, _I, _P, _P, _I, _I, _I, _P]),
    "llmi_linear_trans": (_I, [_P, _P, _I, _P, _P, _I, _I, _I, _I, _I, _P]),
    "llmi_linear_fused": (_I, [_P, _P, _I, _P, _P, _I, _I, _P, _I, _F, _I, _P, _P]),
    "llmi_rope_decode": (_I, [_P, _I, _I, _I, _I, _F, _P]),
    "llmi_attn_workspace_bytes": (_SZ, [_I, _I, _I]),
    "llmi_attn_decode": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _F, _P, _P, _P]),
    "llmi_argmax": (_I, [_P, _I, _P, _P]),
    "llmi_topk": (_I, [_P, _I, _I, _I, _I, _P, _P, _P]),
    "llmi_sampling": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _I, _I, _I, _P]),
    "llmi_repeat_kv": (_I, [_P, _P, _I, _I, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "llmi_padding_offset": (_I, [_P, _P, _P, _I, _I, _P]),
    "llmi_rope_qkv_prefill": (_I, [_P, _P, _P, _P, _I, _P, _P, _I, _I, _I, _I, _I, _I, _F, _P]),
    "llmi_kv_append": (_I, [_P, _P, _I, _I, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "llmi_causal_mask": (_I, [_P, _I, _P, _P, _I, _I, _I, _P]),
    "llmi_masked_softmax": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _F, _P]),
    "llmi_context_attention": (_I, [_P, _P, _P, _I, _I, _P, _P, _I, _I, _I, _I, _I, _I, _F, _P, _P]),
    "llmi_context_attention_qkv": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _F, _P, _P, _I, _I, _I, _F, _P,
                                        _P, _P]),
    "llmi_context_attention_proj": (_I, [_P, _P, _I, _I, _P, _P, _P, _I, _I, _I, _I, _I, _I, _F, _P, _P, _I, _I, _I,
                                         _F, _P, _P, _P]),
    "llmi_ffn": (_I, [_P, _P, _P, _I, _P, _I, _I, _I, _P]),
    "llmi_linear_residual": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _I, _F, _P]),
    "llmi_ffn_residual": (_I, [_P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _I, _F, _P]),
    "llmi_stream_errors": (_I, [_P, _P]),
    "llmi_debug_stream_k": (_I, [_I, _I]),
    "llmi_debug_prefill_stamps": (_I, [_P]),
    "llmi_hbm_read_bench": (_I, [_SZ, _I, _P, _P, _P]),
    "llmi_batched_matmul": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "llmi_transpose_remove_pad": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "llmi_synth_fill": (_I, [_P, _I, _I, _U64, _U32, _I, _I, _I, _I, _I, _P]),
    "llmi_synth_fill_host": (_I, [_P, _I, _I, _U64, _U32, _I, _I, _I, _I, _I]),
    "llmi_synth_prompt": (_I, [_U64, _I, _I, _P]),
    "llmi_device_alloc": (_I, [C.POINTER(_P), _SZ]),
    "llmi_device_memset": (_I, [_P, _I, _SZ]),
    "llmi_device_memset_async": (_I, [_P, _I, _SZ, _P]),
    "llmi_device_free": (_I, [_P]),
    "llmi_memcpy": (_I, [_P, _P, _SZ, _I]),
    "llmi_device_sync": (_I, []),
    "llmi_config_preset": (_I, [C.c_char_p, C.POINTER(Config)]),
    "llmi_tp_unique_id": (_I, [_P]),
    "llmi_tp_comm_create": (_I, [_P, _I, _I, _I, C.POINTER(_P)]),
    "llmi_tp_allreduce": (_I, [_P, _P, _SZ, _I, _P]),
    "llmi_tp_comm_destroy": (_I, [_P]),
    "llmi_engine_create": (_I, [C.POINTER(Config), _I, _P, C.POINTER(_P)]),
    "llmi_engine_destroy": (_I, [_P]),
    "llmi_engine_load_synthetic": (_I, [_P, _U64]),
    "llmi_engine_load_bin": (_I, [_P, C.c_char_p]),
    "llmi_engine_set_sampling": (_I, [_P, _I, _U64]),
    "llmi_engine_load_tensor": (_I, [_P, C.c_char_p, _P, _SZ]),
    "llmi_engine_set_prompt": (_I, [_P, _P, _I]),
    "llmi_engine_decode": (_I, [_P, _I, _I]),
    "llmi_engine_prefill": (_I, [_P, _I, _I]),
    "llmi_engine_sync": (_I, [_P]),
    "llmi_engine_tokens": (_I, [_P, _P, _I, C.POINTER(_I)]),
    "llmi_engine_logits": (_I, [_P, _P, _I]),
    "llmi_engine_hidden": (_I, [_P, _P, _I]),
    "llmi_engine_kv_slot": (_I, [_P, _I, _I, _I, _P]),
    "llmi_engine_bytes": (_I, [_P, C.POINTER(_U64), C.POINTER(_U64)]),
    "llmi_engine_stream": (_P, [_P]),
    "llmi_engine_time_kernel": (_I, [_P, _I, _I, C.POINTER(_F), C.POINTER(_U64)]),
    "llmi_engine_debug_stamps": (_I, [_P, _P]),
    "llmi_engine_debug_timeline": (_I, [_P, _P, _SZ, _I]),
    "llmi_curand_uniform": (_I, [_U64, _U32, C.POINTER(_F)]),
    "llmi_engine_debug_set_next_pos": (_I, [_P, _I]),
    "llmi_engine_xchg_handle": (_I, [_P, _P]),
    "llmi_engine_xchg_open": (_I, [_P, _P]),
    "llmi_engine_xchg_loopback": (_I, [_P]),
    "llmi_engine_set_option": (_I, [_P, C.c_char_p, _I]),
    "llmi_engine_set_exchange": (_I, [_P, _I]),
    "llmi_engine_set_decode_mode": (_I, [_P, _I]),
    "llmi_group_set_exchange": (_I, [_P, _I]),
    "llmi_group_create": (_I, [C.POINTER(Config), _I, _I, C.POINTER(_P)]),
    "llmi_group_destroy": (_I, [_P]),
    "llmi_group_load_synthetic": (_I, [_P, _U64]),
    "llmi_group_load_bin": (_I, [_P, C.c_char_p]),
    "llmi_group_set_prompt": (_I, [_P, _P, _I]),
    "llmi_group_decode": (_I, [_P, _I, _I]),
    "llmi_group_tokens": (_I, [_P, _I, _P, _I, C.POINTER(_I)]),
    "llmi_group_logits": (_I, [_P, _P, _I]),
    "llmi_group_hidden": (_I, [_P, _I, _P, _I]),
}

_lib = None


def lib() -> C.CDLL:
    """Load libllmi.so once. Raises if it has not been built -- no fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libllmi.so not found at {LIB_PATH}; build it with "
                              f"`python llm-inference_amd/build.py` (HIP extension is required)")
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().llmi_last_error().decode(errors="replace")
        raise LlmiError(f"{what} failed ({rc}): {msg}")


def call(name: str, *args):
    rc = getattr(lib(), name)(*args)
    check(rc, name)
    return rc


def header_functions() -> list:
    """Names of the functions include/llmi.h declares (for the export check)."""
    import re
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(llmi_[a-z0-9_]+)\s*\(", src)))
