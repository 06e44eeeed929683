"""Python handle on the native decode engine (llmi_engine_* in include/llmi.h).

Mirrors the reference's model-level API (src/models/basemodel.h:14-42,
src/utils/model_utils.h:63-70): build a Llama with dummy (here: synthetic
PRNG) weights, feed a prompt, greedy-decode. All compute runs in
libllmi.so on the GPU; this class only moves ids/logits across the boundary.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _lib
from ._lib import F16, F32, I8, Config, call


def preset(name: str, **overrides) -> Config:
    cfg = Config()
    call("llmi_config_preset", name.encode(), C.byref(cfg))
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return cfg


def tp_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    call("llmi_tp_unique_id", buf)
    return buf.raw


def synth_prompt(seed: int, n: int, vocab: int) -> np.ndarray:
    out = np.zeros(n, np.int32)
    call("llmi_synth_prompt", seed, n, vocab, out.ctypes.data)
    return out


class Engine:
    def __init__(self, cfg: Config, device: int = 0, tp_id: Optional[bytes] = None):
        self.cfg = cfg
        h = C.c_void_p()
        idbuf = C.create_string_buffer(tp_id, 128) if tp_id else None
        call("llmi_engine_create", C.byref(cfg), device, idbuf, C.byref(h))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().llmi_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ------------------------------------------------------------------ api
    def load_synthetic(self, seed: int):
        call("llmi_engine_load_synthetic", self._h, seed)

    def set_sampling(self, k: int, seed: int = 0):
        """Top-k stochastic sampling in the decode step (k = 0: greedy, the default)."""
        call("llmi_engine_set_sampling", self._h, int(k), int(seed))

    def load_bin(self, weight_path: str):
        """Llama<T>::loadWeights(weight_path): weight_path + "<name>.bin" raw fp32 files
        (llmi/convert.py writes them); the path is used as a prefix, like the reference's."""
        call("llmi_engine_load_bin", self._h, weight_path.encode())

    def load_tensor(self, name: str, values: np.ndarray):
        v = np.ascontiguousarray(values, dtype=np.float32)
        call("llmi_engine_load_tensor", self._h, name.encode(), v.ctypes.data, v.size)

    def set_prompt(self, ids):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        call("llmi_engine_set_prompt", self._h, ids.ctypes.data, len(ids))

    def decode(self, n_steps: int, use_graph: bool = True):
        call("llmi_engine_decode", self._h, n_steps, 1 if use_graph else 0)

    def prefill(self, n_tokens: int, exact=True):
        """exact: True / 1 fp32-faithful (two fp16 planes), 2 fp16 hi + e4m3 lo planes on
        the fp8 MFMA (~1e-4), False / 0 fp16 activations (llmi_engine_prefill)."""
        mode = int(exact)
        if mode not in (0, 1, 2):
            raise ValueError("prefill: exact must be False/0, True/1 or 2")
        call("llmi_engine_prefill", self._h, n_tokens, mode)

    def sync(self):
        call("llmi_engine_sync", self._h)

    def tokens(self, n: Optional[int] = None) -> np.ndarray:
        n = self.cfg.max_seq + 1 if n is None else n
        out = np.zeros(n, np.int32)
        valid = C.c_int()
        call("llmi_engine_tokens", self._h, out.ctypes.data, n, C.byref(valid))
        return out[:min(n, valid.value)]

    def logits(self) -> np.ndarray:
        n = self.cfg.vocab // self.cfg.tp_world
        out = np.zeros(n, np.float32)
        call("llmi_engine_logits", self._h, out.ctypes.data, n)
        return out

    def hidden(self) -> np.ndarray:
        out = np.zeros(self.cfg.hidden, np.float32)
        call("llmi_engine_hidden", self._h, out.ctypes.data, self.cfg.hidden)
        return out

    def kv_slot(self, layer: int, pos: int, which_v: bool = False) -> np.ndarray:
        kvl = self.cfg.kv_heads // self.cfg.tp_world
        out = np.zeros((kvl, self.cfg.head_dim), np.float32)
        call("llmi_engine_kv_slot", self._h, layer, pos, 1 if which_v else 0, out.ctypes.data)
        return out

    def bytes_per_token(self):
        w, kv = C.c_uint64(), C.c_uint64()
        call("llmi_engine_bytes", self._h, C.byref(w), C.byref(kv))
        return w.value, kv.value

    def debug_set_next_pos(self, next_pos: int):
        """Test hook: move the device decode state's next position only (not the host's)."""
        call("llmi_engine_debug_set_next_pos", self._h, int(next_pos))

    def stream(self) -> int:
        return _lib.lib().llmi_engine_stream(self._h) or 0

    # allreduce / allreduce_graph: one residual all-reduce of the TP exchange (needs a tp_id),
    # launched eagerly / replayed from a captured graph of `iters` calls
    KERNELS = {"qkv": 0, "attn": 1, "o": 2, "gate_up": 3, "down": 4, "lm_head": 5, "allreduce": 6,
               "allreduce_graph": 7, "xchg": 8, "xchg_graph": 9, "ring": 10, "qkv_attn": 11}

    # one-shot peer exchange (tensor parallel without RCCL in the token graph)
    def xchg_handle(self) -> bytes:
        buf = C.create_string_buffer(64)
        call("llmi_engine_xchg_handle", self._h, buf)
        return buf.raw

    def xchg_open(self, handles):
        """handles: every rank's 64-byte inbox handle, in rank order."""
        blob = b"".join(bytes(h) for h in handles)
        assert len(blob) == 64 * self.cfg.tp_world
        buf = C.create_string_buffer(blob, len(blob))
        call("llmi_engine_xchg_open", self._h, buf)

    def set_option(self, name: str, value: int):
        """llmi_engine_set_option: tuning switches for same-process A/B ("kpar": 0 / 1)."""
        call("llmi_engine_set_option", self._h, name.encode(), int(value))

    def xchg_loopback(self):
        """Price ONE tensor-parallel rank on one GPU (llmi_engine_xchg_loopback): every peer
        inbox is this rank's own; the timing and launch structure are a rank's, the tokens
        are not the TP model's. Then set_exchange(0 | 1 | 2)."""
        call("llmi_engine_xchg_loopback", self._h)

    def set_exchange(self, mode: int):
        """0: RCCL all-reduces (needs a tp_id at create); 1: the one-shot peer exchange;
        2: the same exchange fused into the producing launches (o_proj / down / lm_head)."""
        call("llmi_engine_set_exchange", self._h, int(mode))

    def set_decode_mode(self, mode: int):
        """0: five launches per layer; 1: the persistent ring layer (ring.hip: attention +
        one launch per layer). Raises LlmiError where mode 1 is unsupported."""
        call("llmi_engine_set_decode_mode", self._h, int(mode))

    def time_kernel(self, which: str, iters: int = 50):
        us, b = C.c_float(), C.c_uint64()
        call("llmi_engine_time_kernel", self._h, self.KERNELS[which], iters, C.byref(us), C.byref(b))
        return us.value, b.value

    def generate(self, prompt, n_new: int, use_graph: bool = True, prefill: bool = False,
                 exact: bool = True) -> np.ndarray:
        """Greedy: feed the prompt, produce n_new tokens (Llama<T>::Response).
        prefill=True runs the prompt as one batched pass (firstTokenGen)."""
        prompt = np.asarray(prompt, np.int32)
        self.set_prompt(prompt)
        if prefill:
            self.prefill(len(prompt), exact)
            self.decode(n_new - 1, use_graph)
        else:
            self.decode(len(prompt) + n_new - 1, use_graph)
        toks = self.tokens(len(prompt) + n_new)
        return toks[len(prompt):]


class TPGroup:
    """In-process tensor-parallel group (llmi_group_* in include/llmi.h): `world`
    rank engines on one device, stepped together, reductions by a kernel in
    place of RCCL. The single-GPU parity harness for the sharded decode path."""

    def __init__(self, cfg: Config, world: int, device: int = 0):
        self.cfg, self.world = cfg, world
        h = C.c_void_p()
        call("llmi_group_create", C.byref(cfg), world, device, C.byref(h))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().llmi_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def load_synthetic(self, seed: int):
        call("llmi_group_load_synthetic", self._h, seed)

    def load_bin(self, weight_path: str):
        call("llmi_group_load_bin", self._h, weight_path.encode())

    def tokens(self, rank: int = 0, n: Optional[int] = None) -> np.ndarray:
        n = self.cfg.max_seq + 1 if n is None else n
        out = np.zeros(n, np.int32)
        valid = C.c_int()
        call("llmi_group_tokens", self._h, rank, out.ctypes.data, n, C.byref(valid))
        return out[:min(n, valid.value)]

    def logits(self) -> np.ndarray:
        out = np.zeros(self.cfg.vocab, np.float32)
        call("llmi_group_logits", self._h, out.ctypes.data, self.cfg.vocab)
        return out

    def hidden(self, rank: int = 0) -> np.ndarray:
        out = np.zeros(self.cfg.hidden, np.float32)
        call("llmi_group_hidden", self._h, rank, out.ctypes.data, self.cfg.hidden)
        return out

    def set_exchange(self, mode: int):
        """0: in-place reduction kernel; 1: the one-shot peer exchange kernels; 2: the push
        fused into every rank's producing launches, then the reduce kernels."""
        call("llmi_group_set_exchange", self._h, int(mode))

    def generate(self, prompt, n_new: int, use_graph: bool = True) -> np.ndarray:
        prompt = np.ascontiguousarray(prompt, np.int32)
        call("llmi_group_set_prompt", self._h, prompt.ctypes.data, len(prompt))
        call("llmi_group_decode", self._h, len(prompt) + n_new - 1, 1 if use_graph else 0)
        return self.tokens(0, len(prompt) + n_new)[len(prompt):]
