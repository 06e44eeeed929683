"""CPU restatement (numpy) of the reference's sampling operators and GQA repeat_kv.

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker for llmi_topk,
llmi_sampling and llmi_repeat_kv (include/llmi.h); never by the product path.

* topk      -- launchTopKforBeamSearch (src/kernels/topK.cu:24-191, topK.h:6-56).
* sampling  -- launchSampling / SamplingKernel (src/kernels/sampling.cu:28-115).
* repeat_kv -- launchRepeatKVCache / repeat_value_cache (src/kernels/repeat_kv.cu:7-91).

Pinning: the reference's unit tests for these kernels print their outputs instead of
checking them (tests/unittests/test_topk.cu, test_sampling.cu, test_repeat_kv.cu), so
there are no golden vectors; tests/test_sampling_oracle.py works the reference tests'
own inputs (probs = arange, topk values K-1-(i%K), caches = arange) by hand. The
sampling draw is the reference's own, curand_uniform(curand_init(step, row, 0))
(sampling.cu:66-69), restated in oracle/xorwow.py from cuRAND's published XORWOW (a
CUDA toolkit header absent here): parity unpinned against cuRAND itself (no CUDA in
this image), bit-exact between the device kernel and this restatement.
"""
from __future__ import annotations

import numpy as np

from . import xorwow


def topk(logits: np.ndarray, k: int):
    """logits [rows, vocab] -> (ids int32 [rows, k], vals [rows, k]) in descending order.
    The reference's insertHeap sort (topK.h:22-44); ties -> lower index (the reference's
    tie order follows its CUB reduction tree). vocab < k pads id -1 / value 1e-20
    (topK.h:15-20)."""
    x = np.asarray(logits)
    rows, vocab = x.shape
    ids = np.full((rows, k), -1, dtype=np.int32)
    vals = np.full((rows, k), 1e-20, dtype=x.dtype)
    for r in range(rows):
        order = np.lexsort((np.arange(vocab), -x[r].astype(np.float64)))[:k]
        ids[r, :len(order)] = order
        vals[r, :len(order)] = x[r, order]
    return ids, vals


def uniform(step: int, row: int) -> np.float32:
    """curand_uniform(curand_init(step, row, 0)) (sampling.cu:66-69), in (0, 1]."""
    return xorwow.curand_uniform(int(step) & 0xFFFFFFFFFFFFFFFF, int(row))


def sampling(topk_ids, topk_vals, seqlen, is_finished, step: int, end_id: int, vocab: int):
    """SamplingKernel (sampling.cu:28-84) per row. Returns (output_id, vals_after,
    seqlen_after, finished_after); output_id is -1 where the row was already finished
    (the kernel leaves output_id untouched there)."""
    ids = np.asarray(topk_ids, dtype=np.int32)
    vals = np.array(topk_vals, copy=True)
    dt = vals.dtype
    rows, K = ids.shape
    out = np.full(rows, -1, dtype=np.int32)
    seq = np.array(seqlen, dtype=np.int32, copy=True)
    fin = np.array(is_finished, dtype=np.uint8, copy=True)
    for b in range(rows):
        if fin[b]:
            continue
        mx = np.float32(vals[b, 0])
        s = np.float32(0.0)
        for i in range(K):
            vals[b, i] = dt.type(np.exp(np.float32(vals[b, i]) - mx, dtype=np.float32))
            s = np.float32(s + np.float32(vals[b, i]))
        thr = np.float32(uniform(step, b) * s)
        o = int(ids[b, 0])
        for i in range(K):
            thr = np.float32(thr - np.float32(vals[b, i]))
            if thr <= 0:
                o = int(ids[b, i]) % vocab
                break
        out[b] = o
        seq[b] += 1
        fin[b] = 1 if o == end_id else 0
    return out, vals, seq, fin


def sampling_margin(topk_vals_after, step: int, row: int) -> float:
    """Smallest |running threshold| over the row's subtraction chain, relative to the sum:
    rows where it is ~1 ulp can flip between two correct expf implementations."""
    v = np.asarray(topk_vals_after[row], dtype=np.float32)
    s = np.float32(v.sum(dtype=np.float32))
    thr = np.float32(uniform(step, row) * s)
    m = abs(float(thr))
    for x in v:
        thr = np.float32(thr - x)
        m = min(m, abs(float(thr)))
    return m / max(float(s), 1e-30)


def repeat_kv(k_cache, v_cache, layer: int, context_length, heads: int, max_k_len: int, k_dst=None, v_dst=None):
    """caches [layers, batch, kv_heads, max_seq, d] -> [batch, heads, max_k_len, d]; query
    head h reads kv head h // (heads // kv_heads); positions >= context_length[b] keep the
    destination's previous contents (repeat_kv.cu:33-48)."""
    _, batch, kv_heads, _, d = k_cache.shape
    rep = heads // kv_heads
    kd = np.zeros((batch, heads, max_k_len, d), k_cache.dtype) if k_dst is None else np.array(k_dst, copy=True)
    vd = np.zeros((batch, heads, max_k_len, d), v_cache.dtype) if v_dst is None else np.array(v_dst, copy=True)
    for b in range(batch):
        n = min(int(context_length[b]), max_k_len)
        for h in range(heads):
            kd[b, h, :n] = k_cache[layer, b, h // rep, :n]
            vd[b, h, :n] = v_cache[layer, b, h // rep, :n]
    return kd, vd
