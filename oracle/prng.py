"""Portable counter-based PRNG for synthetic Llama weights ("llmi-prng-v1").

TEST INFRASTRUCTURE. Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import anything under oracle/. The product path
(llm-inference_amd/csrc/prng.hip) regenerates the same bits on the GPU; this
numpy copy is the checker.

There is no checkpoint in this environment (no hub access,
user_entry.cpp:8 points at a path that does not exist), so every weight of
every test and bench model is a pure function of (seed, tensor id, global
element index). The reference's own dummy loader
(src/weights/llama/layer_weights.cc:69-146, llama_weights.cc:56-88) fills
weights with rand()%100/100000 on the host; we replace that with a
splitmix64 stream whose values are exactly representable so the fp16 bits
are identical on host and device:

  key      = mix64(seed * GOLD + tensor_id)
  r(i)     = mix64(key + (i + 1) * GOLD)          i = global element index
  i24(i)   = (r >> 40) - 2^23                      in [-2^23, 2^23)
  linear   = fp16_rne(i24 * 2^-28)                 |w| < 2^-5
  embed    = fp16_rne(i24 * 2^-23)                 |w| < 1
  gamma    = fp16_rne(1 + i24 * 2^-26)             in [0.875, 1.125)
  int8 q   = (r >> 56) - 128                       in [-128, 127]
  int8 s   = fp16_rne((1 + i24 * 2^-24) * 2^-12)   per output row

The products are exact (power-of-two scaling of a 24-bit integer); the
sums `1 + t` are rounded once by IEEE fp32 addition, identically on host and
device; the last step is fp32->fp16 round-to-nearest-even on both sides.
"""
from __future__ import annotations

import numpy as np

GOLD = np.uint64(0x9E3779B97F4A7C15)
_C1 = np.uint64(0xBF58476D1CE4E5B9)
_C2 = np.uint64(0x94D049BB133111EB)

# tensor-kind ids (low 8 bits); layer tensors use (layer + 1) << 8 | kind
KIND_Q, KIND_K, KIND_V, KIND_O = 0, 1, 2, 3
KIND_GATE, KIND_UP, KIND_DOWN = 4, 5, 6
KIND_ATTN_NORM, KIND_FFN_NORM = 7, 8
KIND_Q_SCALE = 16  # + kind: per-row int8 scales of tensor `kind`
GLOBAL_EMBED, GLOBAL_LM_HEAD, GLOBAL_FINAL_NORM = 1, 2, 3


def layer_tid(layer: int, kind: int) -> int:
    return ((layer + 1) << 8) | kind


def mix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _C1
        z = (z ^ (z >> np.uint64(27))) * _C2
    return z ^ (z >> np.uint64(31))


def tensor_key(seed: int, tid: int) -> np.uint64:
    with np.errstate(over="ignore"):
        z = np.array([np.uint64(seed) * GOLD + np.uint64(tid)], dtype=np.uint64)
    return mix64(z)[0]


def raw_bits(seed: int, tid: int, idx: np.ndarray) -> np.ndarray:
    """64-bit stream value for global element indices `idx` (uint64 array)."""
    key = tensor_key(seed, tid)
    with np.errstate(over="ignore"):
        z = key + (idx.astype(np.uint64) + np.uint64(1)) * GOLD
    return mix64(z)


def _index_grid(rows: int, cols: int, row0: int, col0: int, ld: int) -> np.ndarray:
    r = np.arange(row0, row0 + rows, dtype=np.uint64)[:, None]
    c = np.arange(col0, col0 + cols, dtype=np.uint64)[None, :]
    return r * np.uint64(ld) + c


def _i24(bits: np.ndarray) -> np.ndarray:
    return (bits >> np.uint64(40)).astype(np.int64) - (1 << 23)


def _chunked(fn, rows, cols, row0, col0, ld, out_dtype, chunk_rows=None):
    """Row blocks of ~256K elements (cache-sized temporaries) on a thread pool: numpy's
    integer ufuncs release the GIL, and every element is a pure function of its index."""
    import concurrent.futures as cf
    import os
    out = np.empty((rows, cols), dtype=out_dtype)
    step = chunk_rows or max(1, (1 << 18) // max(cols, 1))

    def block(r):
        n = min(step, rows - r)
        out[r:r + n] = fn(_index_grid(n, cols, row0 + r, col0, ld))

    starts = range(0, rows, step)
    if rows * cols < (1 << 20):
        for r in starts:
            block(r)
    else:
        with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
            list(ex.map(block, starts))
    return out


def linear_fp16(seed, tid, rows, cols, row0=0, col0=0, ld=None) -> np.ndarray:
    """[rows, cols] slice of a linear weight whose full row length is `ld`."""
    ld = cols if ld is None else ld
    f = lambda idx: (_i24(raw_bits(seed, tid, idx)).astype(np.float32)
                     * np.float32(2.0 ** -28)).astype(np.float16)
    return _chunked(f, rows, cols, row0, col0, ld, np.float16)


def embed_fp16(seed, tid, rows, cols, row0=0, col0=0, ld=None) -> np.ndarray:
    ld = cols if ld is None else ld
    f = lambda idx: (_i24(raw_bits(seed, tid, idx)).astype(np.float32)
                     * np.float32(2.0 ** -23)).astype(np.float16)
    return _chunked(f, rows, cols, row0, col0, ld, np.float16)


def gamma_fp16(seed, tid, n) -> np.ndarray:
    idx = np.arange(n, dtype=np.uint64)
    t = _i24(raw_bits(seed, tid, idx)).astype(np.float32) * np.float32(2.0 ** -26)
    return (np.float32(1.0) + t).astype(np.float16)


def int8_weight(seed, tid, rows, cols, row0=0, col0=0, ld=None) -> np.ndarray:
    ld = cols if ld is None else ld
    f = lambda idx: ((raw_bits(seed, tid, idx) >> np.uint64(56)).astype(np.int16) - 128).astype(np.int8)
    return _chunked(f, rows, cols, row0, col0, ld, np.int8)


def int8_row_scale(seed, tid, rows, row0=0) -> np.ndarray:
    idx = np.arange(row0, row0 + rows, dtype=np.uint64)
    t = _i24(raw_bits(seed, tid | KIND_Q_SCALE, idx)).astype(np.float32) * np.float32(2.0 ** -24)
    return ((np.float32(1.0) + t) * np.float32(2.0 ** -12)).astype(np.float16)


def prompt_ids(seed: int, n: int, vocab: int) -> np.ndarray:
    """Synthetic prompt token ids ('prompt = 8 PRNG token ids')."""
    bits = raw_bits(seed, 0xFFFF, np.arange(n, dtype=np.uint64))
    return (bits % np.uint64(vocab)).astype(np.int32)
