"""Operator API on torch device tensors -> libllmi.so kernels.

One function per reference launcher on the decode path (src/kernels/*.h),
same names and argument meaning, fp32 activations. torch is only the
device-memory / stream plumbing here: every op launches the HIP kernel
through the C ABI on torch's current stream and raises on a non-zero status.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib
from ._lib import F16, F32, I8, I32, I64, call

_DT = {torch.float32: F32, torch.float16: F16, torch.int8: I8, torch.int32: I32, torch.int64: I64}


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    return None if t is None else t.data_ptr()


def _dt(t):
    return _DT[t.dtype]


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("llmi ops need device tensors")


def launchInputEmbedding(input_ids: torch.Tensor, embed_table: torch.Tensor) -> torch.Tensor:
    _dev(input_ids, embed_table)
    ids = input_ids.to(torch.int32).contiguous().view(-1)
    out = torch.empty(ids.numel(), embed_table.shape[1], device=ids.device, dtype=torch.float32)
    call("llmi_embedding", ids.data_ptr(), ids.numel(), embed_table.data_ptr(), _dt(embed_table),
         embed_table.shape[0], embed_table.shape[1], out.data_ptr(), _stream())
    return out


def launchRMSNorm(decoder_out: torch.Tensor, gamma: torch.Tensor, eps: float,
                  decoder_residual: torch.Tensor = None) -> torch.Tensor:
    """In place on decoder_out (the reference's convention); optionally saves pre-norm x."""
    _dev(decoder_out, gamma)
    n, h = decoder_out.shape
    call("llmi_rmsnorm", decoder_out.data_ptr(), decoder_out.data_ptr(), _p(decoder_residual),
         gamma.data_ptr(), _dt(gamma), n, h, float(eps), _stream())
    return decoder_out


def launchFusedAddBiasResidualRMSNorm(residual, decoder_out, gamma, eps, bias=None):
    _dev(residual, decoder_out, gamma)
    n, h = decoder_out.shape
    call("llmi_add_residual_rmsnorm", residual.data_ptr(), decoder_out.data_ptr(), _p(bias),
         _dt(bias) if bias is not None else F32, gamma.data_ptr(), _dt(gamma), n, h, float(eps), _stream())
    return residual, decoder_out


def launchAddResidual(residual, decoder_out):
    _dev(residual, decoder_out)
    n, h = decoder_out.shape
    call("llmi_add_residual", residual.data_ptr(), decoder_out.data_ptr(), n, h, _stream())
    return decoder_out


def launchAct(gate_up: torch.Tensor) -> torch.Tensor:
    """gate_up [n, 2, inter] -> silu(gate) * up [n, inter]."""
    _dev(gate_up)
    n, _, inter = gate_up.shape
    out = torch.empty(n, inter, device=gate_up.device, dtype=torch.float32)
    call("llmi_silu_mul", gate_up.data_ptr(), out.data_ptr(), n, inter, _stream())
    return out


def launchLinearGemm(x: torch.Tensor, w: torch.Tensor, scales: torch.Tensor = None, trans_a: bool = False,
                     trans_b: bool = True) -> torch.Tensor:
    """y = op_a(x) @ op_b(w) (llmi_linear_trans; linear.cu:38-99). This Python mirror keeps
    torch's nn.Linear layout as its default (trans_b = True: w [n, k], y = x @ w^T); the C++
    mirror (include/llmi/kernels.h) keeps the reference's defaults (trans_a = trans_b = false).
    trans_b False: w [k, n], y = x @ w; trans_a True: x [k, m], y = x^T @ op_b(w).
    w f32/f16, or i8 (+ per-row f16 scales) with trans_b only."""
    _dev(x, w)
    m, k = (x.shape[1], x.shape[0]) if trans_a else x.shape
    n = w.shape[0] if trans_b else w.shape[1]
    if (w.shape[1] if trans_b else w.shape[0]) != k:
        raise ValueError(f"launchLinearGemm: x gives k = {k}, w has shape {tuple(w.shape)} (trans_b={trans_b})")
    y = torch.empty(m, n, device=x.device, dtype=torch.float32)
    call("llmi_linear_trans", x.contiguous().data_ptr(), w.contiguous().data_ptr(), _dt(w), _p(scales), y.data_ptr(),
         m, n, k, int(trans_a), int(trans_b), _stream())
    return y


def launchRoPE(qkv: torch.Tensor, pos: int, heads: int, kv_heads: int, head_dim: int = 128,
               base: float = 10000.0) -> torch.Tensor:
    _dev(qkv)
    call("llmi_rope_decode", qkv.data_ptr(), int(pos), heads, kv_heads, head_dim, float(base), _stream())
    return qkv


def attn_workspace(heads: int, max_seq: int, head_dim: int = 128, device="cuda") -> torch.Tensor:
    n = _lib.lib().llmi_attn_workspace_bytes(heads, head_dim, max_seq)
    return torch.zeros(n, dtype=torch.uint8, device=device)


def launchDecoderMaskedMHA(qkv, k_cache, v_cache, layer: int, pos: int, heads: int, kv_heads: int,
                           workspace, rope: bool = False, base: float = 10000.0, head_dim: int = 128):
    """k_cache/v_cache [layers, kv_heads, max_seq, d] f16/f32; returns out [heads * d] fp32."""
    _dev(qkv, k_cache, v_cache, workspace)
    max_seq = k_cache.shape[2]
    out = torch.empty(heads * head_dim, device=qkv.device, dtype=torch.float32)
    call("llmi_attn_decode", qkv.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), _dt(k_cache), layer,
         max_seq, int(pos), heads, kv_heads, head_dim, 1 if rope else 0, float(base), out.data_ptr(),
         workspace.data_ptr(), _stream())
    return out


def argmax(logits: torch.Tensor) -> torch.Tensor:
    _dev(logits)
    out = torch.empty(1, device=logits.device, dtype=torch.int32)
    call("llmi_argmax", logits.data_ptr(), logits.numel(), out.data_ptr(), _stream())
    return out


def launchTopKforBeamSearch(probs: torch.Tensor, k: int = 5):
    """probs [rows, vocab] f32/f16 -> (final_topk_ids int32 [rows, k], final_topk_vals [rows, k]),
    descending (topK.cu:24-191; the reference fixes K = 5, topK.cu:154). One launch: the
    reference's round-1 / round-2 scratch buffers are not needed."""
    _dev(probs)
    x = probs.contiguous().view(-1, probs.shape[-1])
    ids = torch.empty(x.shape[0], k, device=x.device, dtype=torch.int32)
    vals = torch.empty(x.shape[0], k, device=x.device, dtype=x.dtype)
    call("llmi_topk", x.data_ptr(), _dt(x), x.shape[0], x.shape[1], int(k), ids.data_ptr(), vals.data_ptr(),
         _stream())
    return ids, vals


def launchSampling(topk_id, topk_val, seqlen, is_finished, output_id, step: int, end_id: int, vocab_size: int):
    """In place, like the reference (sampling.cu:87-115, params step/end_id/vocab_size from
    its IntDict): topk_val <- exp(v - v[0]); output_id, seqlen, is_finished (uint8/bool)
    updated for unfinished rows."""
    _dev(topk_id, topk_val, seqlen, is_finished, output_id)
    for t, dt in ((topk_id, torch.int32), (seqlen, torch.int32), (output_id, torch.int32)):
        if t.dtype != dt or not t.is_contiguous():
            raise ValueError("launchSampling: ids, seqlen and output_id must be contiguous int32")
    if is_finished.dtype not in (torch.bool, torch.uint8) or not topk_val.is_contiguous():
        raise ValueError("launchSampling: is_finished must be bool/uint8, topk_val contiguous")
    rows, k = topk_id.shape
    call("llmi_sampling", topk_id.data_ptr(), topk_val.data_ptr(), _dt(topk_val), rows, k, output_id.data_ptr(),
         seqlen.data_ptr(), is_finished.data_ptr(), int(step), int(end_id), int(vocab_size), _stream())
    return output_id


def launchRepeatKVCache(k_cache_src, v_cache_src, context_length, layer: int, k_cache_dst, v_cache_dst):
    """caches [layers, batch, kv_heads, max_seq, d] -> dst [batch, heads, max_k_len, d]
    (repeat_kv.cu:52-91); positions >= context_length[b] are left as they were."""
    _dev(k_cache_src, v_cache_src, context_length, k_cache_dst, v_cache_dst)
    _, b, kv, max_seq, d = k_cache_src.shape
    heads, max_k = k_cache_dst.shape[1], k_cache_dst.shape[2]
    ctx = _i32(context_length)
    call("llmi_repeat_kv", k_cache_src.data_ptr(), v_cache_src.data_ptr(), _dt(k_cache_src), int(layer),
         ctx.data_ptr(), b, kv, max_seq, heads, max_k, d, k_cache_dst.data_ptr(), v_cache_dst.data_ptr(), _stream())
    return k_cache_dst, v_cache_dst


def synth_fill(out: torch.Tensor, kind: int, seed: int, tid: int, rows: int, cols: int,
               row0: int = 0, col0: int = 0, ld: int = 0) -> torch.Tensor:
    _dev(out)
    call("llmi_synth_fill", out.data_ptr(), _dt(out), kind, seed, tid, rows, cols, row0, col0, ld, _stream())
    return out


# ---------------------------------------------- context-phase (prefill) operators
def _i32(t):
    return t.to(torch.int32).contiguous()


def launchCalPaddingoffset(input_lengths, max_q_len: int):
    """-> (padding_offset [num_tokens], cum_seqlens [batch + 1]) (cal_paddingoffset.cu:51-86)."""
    _dev(input_lengths)
    lens = _i32(input_lengths)
    n = int(lens.sum().item())
    po = torch.empty(max(n, 1), device=lens.device, dtype=torch.int32)
    cum = torch.empty(lens.numel() + 1, device=lens.device, dtype=torch.int32)
    call("llmi_padding_offset", po.data_ptr(), cum.data_ptr(), lens.data_ptr(), lens.numel(), int(max_q_len),
         _stream())
    return po[:n], cum


def launchAddFusedQKVBiasTransposeAndRoPE(qkv, padding_offset, history_length, batch: int, seq_len: int,
                                          heads: int, kv_heads: int, head_dim: int = 128, base: float = 10000.0):
    """qkv [num_tokens, (heads + 2 kv) * d] -> q [batch, heads, seq_len, d], k, v [batch, kv, seq_len, d]
    (qkv_bias_and_RoPE.cu:49-144; no bias for Llama). Padded slots of q/k/v are zero."""
    _dev(qkv, padding_offset, history_length)
    n = qkv.shape[0]
    po, hist = _i32(padding_offset), _i32(history_length)
    q = torch.zeros(batch, heads, seq_len, head_dim, device=qkv.device, dtype=qkv.dtype)
    k = torch.zeros(batch, kv_heads, seq_len, head_dim, device=qkv.device, dtype=qkv.dtype)
    v = torch.zeros_like(k)
    call("llmi_rope_qkv_prefill", qkv.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), _dt(qkv), po.data_ptr(),
         hist.data_ptr(), n, batch, seq_len, heads, kv_heads, head_dim, float(base), _stream())
    return q, k, v


def launchConcatKVCache(k_src, v_src, layer: int, cur_query_length, history_length, k_dst, v_dst):
    """k_src/v_src [batch, kv, max_q_len, d]; k_dst/v_dst [layers, batch, kv, max_seq, d] (concat_past_kv.cu)."""
    _dev(k_src, v_src, cur_query_length, history_length, k_dst, v_dst)
    b, kv, max_q, d = k_src.shape
    cq, hist = _i32(cur_query_length), _i32(history_length)
    call("llmi_kv_append", k_src.data_ptr(), v_src.data_ptr(), _dt(k_src), int(layer), cq.data_ptr(),
         hist.data_ptr(), b, kv, max_q, d, k_dst.shape[3], k_dst.data_ptr(), v_dst.data_ptr(), _stream())
    return k_dst, v_dst


def launchBuildCausalMasks(q_lens, k_lens, max_q_len: int, max_k_len: int, dtype=torch.float32):
    _dev(q_lens, k_lens)
    ql, kl = _i32(q_lens), _i32(k_lens)
    mask = torch.empty(ql.numel(), max_q_len, max_k_len, device=ql.device, dtype=dtype)
    call("llmi_causal_mask", mask.data_ptr(), _dt(mask), ql.data_ptr(), kl.data_ptr(), ql.numel(), max_q_len,
         max_k_len, _stream())
    return mask


def launchScaleMaskAndSoftmax(qk, mask, scale: float, out=None):
    """qk [batch, heads, q_len, k_len], mask [batch, q_len, k_len] -> attention scores."""
    _dev(qk, mask)
    b, h, ql, kl = qk.shape
    out = torch.empty_like(qk) if out is None else out
    call("llmi_masked_softmax", qk.data_ptr(), mask.data_ptr(), out.data_ptr(), _dt(qk), b, h, ql, kl, float(scale),
         _stream())
    return out


def launchTransposeOutRemovePadding(src, padding_offset, num_tokens: int):
    """src [batch, heads, seq_len, d] -> [num_tokens, heads * d]."""
    _dev(src, padding_offset)
    b, h, s, d = src.shape
    po = _i32(padding_offset)
    out = torch.empty(num_tokens, h * d, device=src.device, dtype=src.dtype)
    call("llmi_transpose_remove_pad", src.data_ptr(), po.data_ptr(), out.data_ptr(), _dt(src), num_tokens, b, s, h,
         d, _stream())
    return out


def context_attention_qkv(qkv, padding_offset, history_length, input_length, batch: int, max_q_len: int,
                          heads: int, kv_heads: int, k_cache, v_cache, layer: int = 0, base: float = 10000.0,
                          scale: float = None):
    """LLaMAContextAttentionLayer's middle fused (llmi_context_attention_qkv): qkv rows
    [num_tokens, (heads + 2 kv) * 128] fp32 -> RoPE, k / v into the caches [layers, batch, kv,
    max_seq, 128] (fp32 or fp16) after each sequence's history, ragged causal attention ->
    [num_tokens, heads * 128] fp32."""
    _dev(qkv, padding_offset, history_length, input_length, k_cache, v_cache)
    n, d = qkv.shape[0], 128
    po, hist, ql = _i32(padding_offset), _i32(history_length), _i32(input_length)
    qs = torch.empty(batch, heads, max_q_len, d, device=qkv.device, dtype=torch.float32)
    out = torch.empty(n, heads * d, device=qkv.device, dtype=torch.float32)
    sc = 1.0 / math.sqrt(d) if scale is None else scale
    call("llmi_context_attention_qkv", qkv.contiguous().data_ptr(), po.data_ptr(), hist.data_ptr(), ql.data_ptr(), n,
         batch, max_q_len, heads, kv_heads, d, float(base), k_cache.data_ptr(), v_cache.data_ptr(), _dt(k_cache),
         int(layer), k_cache.shape[3], float(sc), qs.data_ptr(), out.data_ptr(), _stream())
    return out


def context_attention_proj(x, w_qkv, padding_offset, history_length, input_length, batch: int, max_q_len: int,
                           heads: int, kv_heads: int, k_cache, v_cache, layer: int = 0, base: float = 10000.0,
                           scale: float = None):
    """context_attention_qkv with the q/k/v projection in front (llmi_context_attention_proj):
    x [num_tokens, hidden] fp32, w_qkv [(heads + 2 kv) * 128, hidden] fp16. Raises LlmiError
    (unsupported) where the fused form does not apply."""
    _dev(x, w_qkv, padding_offset, history_length, input_length, k_cache, v_cache)
    n, hidden, d = x.shape[0], x.shape[1], 128
    po, hist, ql = _i32(padding_offset), _i32(history_length), _i32(input_length)
    qs = torch.empty(batch, heads, max_q_len, d, device=x.device, dtype=torch.float32)
    out = torch.empty(n, heads * d, device=x.device, dtype=torch.float32)
    sc = 1.0 / math.sqrt(d) if scale is None else scale
    call("llmi_context_attention_proj", x.contiguous().data_ptr(), w_qkv.data_ptr(), _dt(w_qkv), hidden,
         po.data_ptr(), hist.data_ptr(), ql.data_ptr(), n, batch, max_q_len, heads, kv_heads, d, float(base),
         k_cache.data_ptr(), v_cache.data_ptr(), _dt(k_cache), int(layer), k_cache.shape[3], float(sc), qs.data_ptr(),
         out.data_ptr(), _stream())
    return out


def check_stream(what: str) -> None:
    """Raise LlmiError when a launch on the current stream recorded a device error bit
    (llmi_stream_errors; 16 = a stream-K partial never arrived, the output is incomplete) --
    the reference's DeviceSyncAndCheckCudaError (macro.h:98-109). Synchronises the stream
    only when a launch on it could have recorded one."""
    f = stream_errors()
    if f:
        why = " (a stream-K partial never arrived within 2 s: the output is incomplete)" if f & 16 else ""
        raise _lib.LlmiError(f"{what}: device error bits {f:#x}{why}")


def ffn(x, w_gate_up, w_down, check: bool = True):
    """LLaMAFFNLayer for context rows in one call (llmi_ffn): x [m, hidden] fp32, w_gate_up
    [2 inter, hidden] and w_down [hidden, inter] fp16 -> [m, hidden] fp32. Raises
    LlmiError (unsupported) where the fused form does not apply, and (check) when the
    stream-K hand-off failed (check_stream; False leaves that to the caller, e.g. once per
    forward of many layers)."""
    _dev(x, w_gate_up, w_down)
    m, hidden = x.shape
    inter = w_down.shape[1]
    y = torch.empty(m, hidden, device=x.device, dtype=torch.float32)
    call("llmi_ffn", x.contiguous().data_ptr(), w_gate_up.data_ptr(), w_down.data_ptr(), _dt(w_gate_up), y.data_ptr(),
         m, hidden, inter, _stream())
    if check:
        check_stream("llmi_ffn")
    return y


def linear_residual(x, w, residual, gamma=None, eps: float = 1e-5, out: bool = True, check: bool = True):
    """llmi_linear_residual: residual += x . w^T (in place), then returns RMSNorm(residual) *
    gamma (gamma None: a copy of the residual; out False: None). x [m, k] fp32, w [n, k] fp16,
    residual [m, n] fp32, gamma [n] fp16 / fp32. check: as ffn."""
    _dev(x, w, residual)
    m, k = x.shape
    n = w.shape[0]
    y = torch.empty(m, n, device=x.device, dtype=torch.float32) if out else None
    call("llmi_linear_residual", x.contiguous().data_ptr(), w.data_ptr(), _dt(w), m, n, k, residual.data_ptr(),
         y.data_ptr() if out else None, gamma.data_ptr() if gamma is not None else None,
         _dt(gamma) if gamma is not None else 0, float(eps), _stream())
    if check:
        check_stream("llmi_linear_residual")
    return y


def ffn_residual(x, w_gate_up, w_down, residual, gamma=None, eps: float = 1e-5, out: bool = True,
                 check: bool = True):
    """llmi_ffn_residual: residual += FFN(x) (in place), then the output as linear_residual."""
    _dev(x, w_gate_up, w_down, residual)
    m, hidden = x.shape
    inter = w_down.shape[1]
    y = torch.empty(m, hidden, device=x.device, dtype=torch.float32) if out else None
    call("llmi_ffn_residual", x.contiguous().data_ptr(), w_gate_up.data_ptr(), w_down.data_ptr(), _dt(w_gate_up), m,
         hidden, inter, residual.data_ptr(), y.data_ptr() if out else None,
         gamma.data_ptr() if gamma is not None else None, _dt(gamma) if gamma is not None else 0, float(eps),
         _stream())
    if check:
        check_stream("llmi_ffn_residual")
    return y


def debug_stream_k(mode: int, launches: int = 1) -> None:
    """llmi_debug_stream_k (test hook): the next `launches` stream-K launches never publish a
    later piece (mode 1) or publish it 2.5 s late (mode 2); mode 0 clears."""
    call("llmi_debug_stream_k", int(mode), int(launches))


def stream_errors() -> int:
    """llmi_stream_errors: read and clear the device error bits recorded on the current stream
    by the layer-API GEMM calls (16: a stream-K partial never arrived; synchronises)."""
    flags = ctypes.c_int(0)
    call("llmi_stream_errors", _stream(), ctypes.addressof(flags))
    return flags.value


def launchLinearStridedBatchGemm(input1, input2, trans_a: bool = False, trans_b: bool = False):
    """input1 [bs, heads, m|k, k|m], input2 [bs, heads, k|n, n|k] -> [bs, heads, m, n] =
    op(input1) @ op(input2) (linear.cu:126-229; QK^T with trans_b, PV without)."""
    _dev(input1, input2)
    b, h = input1.shape[0], input1.shape[1]
    m, k = (input1.shape[3], input1.shape[2]) if trans_a else (input1.shape[2], input1.shape[3])
    k2, n = (input2.shape[3], input2.shape[2]) if trans_b else (input2.shape[2], input2.shape[3])
    if k != k2 or input2.shape[0] * input2.shape[1] != b * h:
        raise ValueError("launchLinearStridedBatchGemm: inner dims / batch counts differ")
    a, bb = input1.contiguous(), input2.contiguous()
    out = torch.empty(b, h, m, n, device=input1.device, dtype=input1.dtype)
    call("llmi_batched_matmul", a.data_ptr(), bb.data_ptr(), out.data_ptr(), _dt(a), b * h, m, n, k,
         1 if trans_a else 0, 1 if trans_b else 0, _stream())
    return out


# ------------------------------------------------------ tensor-parallel all-reduce
def tp_unique_id() -> bytes:
    import ctypes as C
    buf = C.create_string_buffer(128)
    call("llmi_tp_unique_id", C.cast(buf, C.c_void_p))
    return buf.raw


class TPComm:
    """One rank's RCCL communicator (llmi_tp_comm_*): all_reduce sums a device tensor in
    place across the ranks -- the TP reduction of row-parallel partials."""

    def __init__(self, unique_id: bytes, world: int, rank: int, device: int = 0):
        import ctypes as C
        self._h = C.c_void_p()
        idb = C.create_string_buffer(unique_id, 128)
        call("llmi_tp_comm_create", C.cast(idb, C.c_void_p), world, rank, device, C.byref(self._h))

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        _dev(t)
        if not t.is_contiguous():
            raise ValueError("all_reduce needs a contiguous tensor")
        call("llmi_tp_allreduce", self._h, t.data_ptr(), t.numel(), _dt(t), _stream())
        return t

    def close(self):
        if self._h:
            call("llmi_tp_comm_destroy", self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
