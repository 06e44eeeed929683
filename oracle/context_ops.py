"""CPU restatement (numpy) of the reference's context-phase (prefill) operators.

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker for the llmi_* context
operators (include/llmi.h); never by the product path.

Each function follows the reference launcher it names (file:line under
/root/reference/src/kernels). Pinning: their composition for one sequence must
reproduce `llama_ref.attention_prefill` with `llama_ref.apply_rope`, which are pinned
against the reference model's golden vectors (tests/test_oracle_golden.py); the
ragged-batch layouts (padding offsets, history lengths) are the reference kernels'
index arithmetic restated, checked by the hand-worked cases in
tests/test_context_oracle.py (parity for batch > 1 is otherwise unpinned: the
reference ships no fixtures for it).
"""
from __future__ import annotations

import math

import numpy as np


def padding_offset(input_lengths, max_q_len: int) -> np.ndarray:
    """CalPaddingoffset (cal_paddingoffset.cu:51-72): token i of the packed batch sits at
    padded position i + padding_offset[i]."""
    out, cum = [], 0
    for n in input_lengths:
        out += [cum] * int(n)
        cum += max_q_len - int(n)
    return np.asarray(out, np.int32)


def rope_angles(pos: int, d: int, base: float):
    """Angle arithmetic of llmi_rope_decode: inv_freq = 1 / fp32(base^(2i/d)) (the power
    correctly rounded, as torch's fp32 pow), angle = fp32(pos * inv_freq), cos/sin of the
    fp32 angle rounded to fp32 (modeling_llama.py:123-146)."""
    i = np.arange(d // 2, dtype=np.float64)
    p = np.power(np.float64(base), 2.0 * i / d).astype(np.float32)
    inv = (np.float32(1.0) / p).astype(np.float32)
    ang = (np.float32(pos) * inv).astype(np.float32)
    return np.cos(ang.astype(np.float64)).astype(np.float32), np.sin(ang.astype(np.float64)).astype(np.float32)


def rope_qkv_prefill(qkv: np.ndarray, pad_off: np.ndarray, history: np.ndarray, batch: int, seq_len: int,
                     heads: int, kv_heads: int, d: int, base: float = 10000.0):
    """add_fusedQKV_bias_transpose_kernel (qkv_bias_and_RoPE.cu:49-144) without bias:
    qkv [num_tokens, (heads + 2 kv) * d] -> q [batch, heads, seq_len, d], k, v
    [batch, kv, seq_len, d]; q, k rotated (pairs (i, i + d/2), :39-46, :131-143) at
    position history[b] + s. v is copied (the reference leaves v_buf unwritten: the
    copy is commented out at :94-119) and the position uses the sequence index s (the
    reference's `history + token_id` at :125 is the packed index, equal at batch 1)."""
    n = qkv.shape[0]
    q = np.zeros((batch, heads, seq_len, d), np.float32)
    k = np.zeros((batch, kv_heads, seq_len, d), np.float32)
    v = np.zeros((batch, kv_heads, seq_len, d), np.float32)
    x = qkv.astype(np.float32).reshape(n, heads + 2 * kv_heads, d)
    h2 = d // 2
    for t in range(n):
        p = t + int(pad_off[t])
        b, s = p // seq_len, p % seq_len
        c, sn = rope_angles(int(history[b]) + s, d, base)
        for dst, src in ((q[b, :, s], x[t, :heads]), (k[b, :, s], x[t, heads:heads + kv_heads])):
            x0, x1 = src[:, :h2], src[:, h2:]
            dst[:, :h2] = x0 * c - x1 * sn
            dst[:, h2:] = x1 * c + x0 * sn
        v[b, :, s] = x[t, heads + kv_heads:]
    return q, k, v


def kv_append(k_src, v_src, layer: int, cur_q, history, k_cache, v_cache):
    """append_key_cache / append_value_cache (concat_past_kv.cu:16-91, launcher :102-143):
    src [batch, kv, max_q, d] -> cache [layers, batch, kv, max_seq, d] at slot
    history[b] + t for t < cur_q[b]; caches updated in place."""
    for b in range(k_src.shape[0]):
        h0, n = int(history[b]), int(cur_q[b])
        k_cache[layer, b, :, h0:h0 + n] = k_src[b, :, :n]
        v_cache[layer, b, :, h0:h0 + n] = v_src[b, :, :n]
    return k_cache, v_cache


def causal_mask(q_lens, k_lens, max_q: int, max_k: int) -> np.ndarray:
    """BuildCausalMasksConsideringContextPastKV (build_causal_mask.cu:4-45), the :29 test
    without its `k >= klen - qlen` term: that term hides the history positions from the
    chunk's queries, which modeling_llama.py's cached forward (its 4-D causal mask over
    past + current keys, :1043-1046) does not -- pinned by tests/golden/f8_*.npz. With no
    history (klen == qlen) the reference's test and this one agree."""
    q = np.arange(max_q)[:, None]
    k = np.arange(max_k)[None, :]
    out = []
    for ql, kl in zip(q_lens, k_lens):
        ql, kl = int(ql), int(kl)
        out.append((q < ql) & (k < kl) & (k <= q + (kl - ql)))
    return np.asarray(out, np.float32)


def masked_softmax(qk: np.ndarray, mask: np.ndarray, scale: float) -> np.ndarray:
    """ScaleMaskAndSoftmax_float (attn_softmax_kernel.cu:79-174): x = scale * qk +
    (1 - mask) * -10000 (:130), p = exp(x - max) / (sum + 1e-6) (:151, :158, :171)."""
    x = np.float32(scale) * qk.astype(np.float32) + (np.float32(1) - mask.astype(np.float32))[:, None] * np.float32(
        -10000.0)
    e = np.exp(x - x.max(axis=-1, keepdims=True))
    return (e * (np.float32(1) / (e.sum(axis=-1, keepdims=True, dtype=np.float32) + np.float32(1e-6)))).astype(
        np.float32)


def transpose_remove_pad(src: np.ndarray, pad_off: np.ndarray, num_tokens: int) -> np.ndarray:
    """fused_transpose_reshape_remv_pad (fused_transpose_and_remv_pad.cu:17-47)."""
    b_, heads, seq_len, d = src.shape
    out = np.zeros((num_tokens, heads * d), src.dtype)
    for i in range(num_tokens):
        p = i + int(pad_off[i])
        out[i] = src[p // seq_len, :, p % seq_len].reshape(-1)
    return out


def context_attention(qkv, input_lengths, history, heads, kv_heads, d, k_cache, v_cache, layer=0,
                      base: float = 10000.0):
    """The reference's unfused context attention (context_attention.cpp:108-161) composed
    from the operators above, QK^T and PV as the strided-batch GEMMs of
    launchLinearStridedBatchGemm (linear.cu:126-229): k_len = history + q_len, keys read
    back from the cache. Returns [num_tokens, heads * d]."""
    batch = len(input_lengths)
    max_q = int(max(input_lengths))
    po = padding_offset(input_lengths, max_q)
    q, k, v = rope_qkv_prefill(qkv, po, history, batch, max_q, heads, kv_heads, d, base)
    kv_append(k, v, layer, input_lengths, history, k_cache, v_cache)
    k_lens = [int(h) + int(n) for h, n in zip(history, input_lengths)]
    max_k = max(k_lens)
    group = heads // kv_heads
    kc = np.repeat(k_cache[layer, :, :, :max_k].astype(np.float32), group, axis=1)
    vc = np.repeat(v_cache[layer, :, :, :max_k].astype(np.float32), group, axis=1)
    qk = np.einsum("bhqd,bhkd->bhqk", q, kc)
    mask = causal_mask(input_lengths, k_lens, max_q, max_k)
    p = masked_softmax(qk, mask, 1.0 / math.sqrt(d))
    o = np.einsum("bhqk,bhkd->bhqd", p, vc).astype(np.float32)
    return transpose_remove_pad(o, po, int(sum(input_lengths)))
