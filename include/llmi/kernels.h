// The reference's operator API (src/kernels/*.h launchers), same names and
// argument meaning, implemented over the llmi C ABI (include/llmi.h) -- so code
// written against Mr-wang27/llm-inference's launchers compiles against this
// header and runs the MI355X kernels. Activations are TensorWrapper<float> (the
// reference's working instantiation, user_entry.cpp:21 / llama.h:207) or
// TensorWrapper<half_t> (its fp16 instantiation: staged through the fp32 operators by
// llmi_convert, results rounded back to fp16); weights may be float, half_t or int8_t
// (+ per-row scales).
//
// Differences, all deliberate and documented per launcher:
//  * every launcher takes an optional trailing stream (hipStream_t as void*);
//    the reference stored a stream and never used it (model_utils.h:36);
//  * errors throw std::runtime_error("[oneLLM][ERROR] ...") immediately (the
//    reference surfaced them at DeviceSyncAndCheckCudaError, macro.h:98-109);
//  * launchRMSNorm's decoder_residual really receives the pre-norm x (its kernel
//    aliased it).
#pragma once
#include "tensor.h"
#include "weights.h"

namespace llmi_detail {
inline void* attn_workspace(int heads, int head_dim, int max_seq) {
    thread_local void* ws = nullptr;
    thread_local size_t cap = 0;
    const size_t need = llmi_attn_workspace_bytes(heads, head_dim, max_seq);
    if (need > cap) {
        if (ws) LLMI_CALL(llmi_device_free(ws));
        LLMI_CALL(llmi_device_alloc(&ws, need));
        cap = need;
    }
    return ws;
}
inline int tokens_of(const Tensor* t) { return t->shape.size() >= 2 ? t->size() / t->shape.back() : 1; }

// Device-side failures of launches with no error word of their own (the stream-K hand-off
// in llmi_linear / llmi_ffn / the *_residual calls: bit 16 = a partial never arrived, the
// output is incomplete) surface here as the reference's exception. The reference found its
// errors at DeviceSyncAndCheckCudaError (macro.h:98-109) after each launch; the layer
// classes call this once per forward. Synchronises the stream only when a launch on it
// could have recorded a bit (llmi_stream_errors returns at once otherwise).
inline void checkStreamErrors(void* stream, const char* who) {
    int flags = 0;
    LLMI_CALL(llmi_stream_errors(stream, &flags));
    if (flags) {
        std::ostringstream os;
        os << "[oneLLM][ERROR] " << who << ": device error bits 0x" << std::hex << flags << std::dec
           << ((flags & 16) ? " (a stream-K partial never arrived within 2 s -- another stream or process held "
                              "CUs the launch needed -- so this forward's output is incomplete)"
                            : "");
        throw std::runtime_error(os.str());
    }
}

// fp32 view of an activation tensor: TensorWrapper<float> as is; TensorWrapper<half_t>
// converted into a device scratch buffer (load = copy the values in) and written back
// rounded to fp16 by back(). The scratch is per (host thread, stream, slot): launchers
// on different streams never share one, and a buffer that must grow is freed only
// after the device has drained (earlier launches may still read it). The buffers live
// for the thread (the reference's launchers allocate nothing; this is their staging).
inline float* f32_scratch(int slot, size_t n, void* stream) {
    struct Slots {
        void* buf[4] = {nullptr, nullptr, nullptr, nullptr};
        size_t cap[4] = {0, 0, 0, 0};
    };
    thread_local std::unordered_map<void*, Slots> per_stream;
    Slots& s = per_stream[stream];
    if (n * sizeof(float) > s.cap[slot]) {
        if (s.buf[slot]) {
            LLMI_CALL(llmi_device_sync());
            LLMI_CALL(llmi_device_free(s.buf[slot]));
        }
        LLMI_CALL(llmi_device_alloc(&s.buf[slot], n * sizeof(float)));
        s.cap[slot] = n * sizeof(float);
    }
    return static_cast<float*>(s.buf[slot]);
}
template <typename AT> struct Act;
template <> struct Act<float> {
    float* p;
    Act(TensorWrapper<float>* t, int, void*, bool) : p(t ? t->data : nullptr) {}
    void back(void*) {}
};
template <> struct Act<half_t> {
    TensorWrapper<half_t>* t;
    float* p = nullptr;
    Act(TensorWrapper<half_t>* t_, int slot, void* stream, bool load) : t(t_) {
        if (!t) return;
        p = f32_scratch(slot, t->size(), stream);
        if (load) LLMI_CALL(llmi_convert(t->data, LLMI_F16, p, LLMI_F32, t->size(), stream));
    }
    void back(void* stream) {
        if (t) LLMI_CALL(llmi_convert(p, LLMI_F32, t->data, LLMI_F16, t->size(), stream));
    }
};
}  // namespace llmi_detail

// input_embedding.h:6-9 -- out[t, :] = table[ids[t], :]
template <typename AT, typename T>
void launchInputEmbedding(TensorWrapper<int>* input_ids, TensorWrapper<AT>* output, EmbeddingWeight<T>* embed_table,
                          void* stream = nullptr) {
    LLM_CHECK_WITH_INFO(embed_table->shape.size() == 2, "embedding table must be [vocab, hidden]");
    llmi_detail::Act<AT> out(output, 0, stream, false);
    LLMI_CALL(llmi_embedding(input_ids->data, input_ids->size(), embed_table->data,
                             llmiWeightDtype(getWeightType<T>()), embed_table->shape[0], embed_table->shape[1],
                             out.p, stream));
    out.back(stream);
}

// rmsnorm_kernel.h:11-17 -- in place on decoder_out; decoder_residual <- pre-norm x
template <typename AT, typename T>
void launchRMSNorm(TensorWrapper<AT>* decoder_out, TensorWrapper<AT>* decoder_residual,
                   LayerNormWeight<T>& attn_norm_weight, float eps, bool is_last = false, void* stream = nullptr) {
    (void)is_last;
    const int hidden = decoder_out->shape.back();
    llmi_detail::Act<AT> out(decoder_out, 0, stream, true), res(decoder_residual, 1, stream, false);
    LLMI_CALL(llmi_rmsnorm(out.p, out.p, res.p, attn_norm_weight.gamma, llmiWeightDtype(getWeightType<T>()),
                           llmi_detail::tokens_of(decoder_out), hidden, eps, stream));
    out.back(stream);
    res.back(stream);
}

// fused_addresidual_norm.h:9-15 -- residual += decoder_out (+bias); decoder_out = rmsnorm(residual) * scale
template <typename AT, typename T>
void launchFusedAddBiasResidualRMSNorm(TensorWrapper<AT>* residual, TensorWrapper<AT>* decoder_out,
                                       BaseWeight<T>& norm, T* scale, float eps, void* stream = nullptr) {
    const int hidden = decoder_out->shape.back();
    const int dt = llmiWeightDtype(getWeightType<T>());
    llmi_detail::Act<AT> res(residual, 0, stream, true), out(decoder_out, 1, stream, true);
    LLMI_CALL(llmi_add_residual_rmsnorm(res.p, out.p, norm.bias, dt, scale, dt, llmi_detail::tokens_of(decoder_out),
                                        hidden, eps, stream));
    res.back(stream);
    out.back(stream);
}

// add_residual.h:8-13 -- decoder_out += residual
template <typename AT>
void launchAddResidual(TensorWrapper<AT>* residual, TensorWrapper<AT>* decoder_out, bool is_print = false,
                       void* stream = nullptr) {
    (void)is_print;
    llmi_detail::Act<AT> res(residual, 0, stream, true), out(decoder_out, 1, stream, true);
    LLMI_CALL(llmi_add_residual(res.p, out.p, llmi_detail::tokens_of(decoder_out), decoder_out->shape.back(), stream));
    out.back(stream);
}

// act_kernel.h:8-9 -- input [n, 2, inter] (gate, up) -> out [n, inter] = silu(gate) * up
template <typename AT>
void launchAct(TensorWrapper<AT>* input, TensorWrapper<AT>* out, void* stream = nullptr) {
    LLM_CHECK_WITH_INFO(input->shape.size() == 3 && input->shape[1] == 2, "launchAct input must be [n, 2, inter]");
    llmi_detail::Act<AT> in(input, 0, stream, true), o(out, 1, stream, false);
    LLMI_CALL(llmi_silu_mul(in.p, o.p, input->shape[0], input->shape[2], stream));
    o.back(stream);
}

// cublasWrapper stand-in: the reference's launchLinearGemm takes one (linear.h:16-22);
// here it only carries the stream.
struct cublasWrapper {
    void* stream = nullptr;
};

// linear.h:16-22, linear.cu:38-99 -- output = op_a(input) . op_b(weight), row-major, with the
// reference's defaults (trans_a = trans_b = false):
//   trans_b = false: weight [k, n] (in, out) and op_b(W) = W      (linear.cu:60-66)
//   trans_b = true:  weight [n, k] (out, in) and op_b(W) = W^T    (linear.cu:71-76; every
//                    layer of the reference passes this, masked_self_attention.cpp:62)
//   trans_a = false: input [m, k] (its trailing dims flattened: [tokens, heads, head])
//   trans_a = true:  input [k, m] and op_a(x) = x^T               (linear.cu:78-84)
// m = output->shape[0], as the reference's Cn (linear.cu:50). Every form runs llmi_linear's
// arithmetic (the non-default ones transpose their operands first, llmi_linear_trans).
template <typename AT, typename T>
void launchLinearGemm(TensorWrapper<AT>* input, BaseWeight<T>& weight, TensorWrapper<AT>* output,
                      cublasWrapper* cublas_wrapper = nullptr, bool trans_a = false, bool trans_b = false) {
    LLM_CHECK_WITH_INFO(weight.shape.size() == 2, "launchLinearGemm: weight must be 2-D");
    LLM_CHECK_WITH_INFO(input->shape.size() >= 2 && output->shape.size() >= 2,
                        "launchLinearGemm: input and output must be at least 2-D");
    const int k = trans_b ? weight.shape[1] : weight.shape[0], n = trans_b ? weight.shape[0] : weight.shape[1];
    const int in_rows = input->shape[0], in_cols = input->size() / input->shape[0];
    const int m = trans_a ? in_cols : in_rows;
    LLM_CHECK_WITH_INFO((trans_a ? in_rows : in_cols) == k, "2nd dim of input MUST = 1st dim of weight");
    LLM_CHECK_WITH_INFO(output->shape[0] == m && output->size() == m * n, "launchLinearGemm: output must be [m, n]");
    void* stream = cublas_wrapper ? cublas_wrapper->stream : nullptr;
    llmi_detail::Act<AT> in(input, 0, stream, true), out(output, 1, stream, false);
    LLMI_CALL(llmi_linear_trans(in.p, weight.data, llmiWeightDtype(getWeightType<T>()), weight.scale, out.p, m, n, k,
                                trans_a ? 1 : 0, trans_b ? 1 : 0, stream));
    out.back(stream);
}

// qkv_bias_and_RoPE.h:40-42 -- one decode token, in place on q and k of the fused
// qkv row [1, qkv_head_num, head_size] at position step - 1 (step: host tensor).
// The reference assumed MHA (head_num = qkv_head_num / 3, :416); kv_head_num may be given.
template <typename AT>
void launchRoPE(TensorWrapper<AT>* qkv_buf, TensorWrapper<int>* step, LLaMAAttentionStaticParams& params,
                int kv_head_num = -1, void* stream = nullptr) {
    const int qkv_heads = qkv_buf->shape[qkv_buf->shape.size() - 2];
    const int head_size = qkv_buf->shape.back();
    const int kv = kv_head_num > 0 ? kv_head_num : qkv_heads / 3;
    llmi_detail::Act<AT> q(qkv_buf, 0, stream, true);
    LLMI_CALL(llmi_rope_decode(q.p, step->getVal() - 1, qkv_heads - 2 * kv, kv, head_size, params.rotary_embedding_base,
                               stream));
    q.back(stream);
}

// fused_decoder_self_attention.h:10-19 -- write k, v of the (already rotated) fused qkv
// into cache slot step - 1 of layer layer_id, then masked MHA over positions
// 0..step-1. caches [layers, batch(=1), kv_heads, max_seq, head] f32 or f16 bits.
template <typename AT, typename T, typename CT>
void launchDecoderMaskedMHA(TensorWrapper<AT>* qkv_buf, BaseWeight<T>& qkv, TensorWrapper<int>* layer_id,
                            TensorWrapper<CT>* k_cache, TensorWrapper<CT>* v_cache, TensorWrapper<bool>* finished,
                            TensorWrapper<int>* step, TensorWrapper<AT>* mha_output,
                            LLaMAAttentionStaticParams& static_params, void* stream = nullptr) {
    (void)qkv;
    (void)finished;
    LLM_CHECK_WITH_INFO(k_cache->shape.size() == 5, "kv cache must be [layers, batch, kv_heads, max_seq, head]");
    LLM_CHECK_WITH_INFO(k_cache->shape[1] == 1, "batch size 1 only");
    const int kv = k_cache->shape[2], max_seq = k_cache->shape[3], head = k_cache->shape[4];
    const int qkv_heads = qkv_buf->shape[qkv_buf->shape.size() - 2];
    const int heads = qkv_heads - 2 * kv;
    const int cdt = llmiDtype(getTensorType<CT>());
    void* ws = llmi_detail::attn_workspace(heads, head, max_seq);
    llmi_detail::Act<AT> q(qkv_buf, 0, stream, true), out(mha_output, 1, stream, false);
    LLMI_CALL(llmi_attn_decode(q.p, k_cache->data, v_cache->data, cdt, layer_id->getVal(), max_seq, step->getVal() - 1,
                               heads, kv, head, /*rope=*/0, static_params.rotary_embedding_base, out.p, ws, stream));
    out.back(stream);
}

// topK.h:51-56 + sampling.h:12-18 as Llama<T> wires them: beam width 1 and
// K = 1 (llama.cpp:59, sampling.cu:99), i.e. greedy argmax of probs [1, vocab];
// final_topk_id receives the token id (device int).
template <typename AT>
void launchTopKforBeamSearch(TensorWrapper<AT>* probs, TensorWrapper<int>* final_topk_id, void* stream = nullptr) {
    llmi_detail::Act<AT> p(probs, 0, stream, true);
    LLMI_CALL(llmi_argmax(p.p, probs->shape.back(), final_topk_id->data, stream));
}

// topK.h:51-56 -- the reference's full signature. topk_ids / topK_values are the
// reference's round-1 scratch [bs, beam, BlockPerBeam, K]; the build selects in one
// launch and leaves them untouched. K = final_topk_ids->shape.back() (the reference
// fixes 5). Values descending, ties -> lower index (include/llmi.h: llmi_topk).
template <typename T>
void launchTopKforBeamSearch(TensorWrapper<T>* probs, TensorWrapper<int>* topk_ids, TensorWrapper<T>* topK_values,
                             TensorWrapper<int>* final_topk_ids, TensorWrapper<T>* final_topk_values,
                             void* stream = nullptr) {
    (void)topk_ids;
    (void)topK_values;
    const int vocab = probs->shape.back(), rows = probs->size() / vocab;
    const int k = final_topk_ids->shape.back();
    LLM_CHECK_WITH_INFO(final_topk_values->size() == rows * k && final_topk_ids->size() == rows * k,
                        "topk: final buffers must be [bs * beam, K]");
    LLMI_CALL(llmi_topk(probs->data, llmiDtype(getTensorType<T>()), rows, vocab, k, final_topk_ids->data,
                        final_topk_values->data, stream));
}

// sampling.h:12-18 -- params "step" (the draw's seed), "end_id", "vocab_size"
// (sampling.cu:92-95); topk_val is overwritten with exp(v - v[0]) as in the reference.
template <typename T>
void launchSampling(TensorWrapper<int>* topk_id, TensorWrapper<T>* topk_val, TensorWrapper<int>* seqlen,
                    TensorWrapper<bool>* is_finished, TensorWrapper<int>* output_id, IntDict& params,
                    void* stream = nullptr) {
    LLM_CHECK_WITH_INFO(topk_id->shape.size() == 2, "sampling: topk_id must be [bs, K]");
    LLMI_CALL(llmi_sampling(topk_id->data, topk_val->data, llmiDtype(getTensorType<T>()), topk_id->shape[0],
                            topk_id->shape[1], output_id->data, seqlen->data,
                            reinterpret_cast<uint8_t*>(is_finished->data), params.at("step"), params.at("end_id"),
                            params.at("vocab_size"), stream));
}

// ---- context-phase launchers (prefill; the engine fuses them, see llmi_engine_prefill).
// T = float or half_t storage; padding_offset, history_length, input_length, q_lens,
// k_lens, cur_query_length are device int tensors; layer_id is a host tensor.

// qkv_bias_and_RoPE.h:26-36 -- QKV [num_tokens, heads + 2 kv_heads, head] ->
// q [batch, heads, seq, head], k, v [batch, kv_heads, seq, head], RoPE at history + s.
// Llama has no qkv bias (qkv.bias is ignored); v is written (the reference leaves it
// unset) and positions are per sequence (include/llmi.h: llmi_rope_qkv_prefill).
template <typename T, typename WT>
void launchAddFusedQKVBiasTransposeAndRoPE(TensorWrapper<T>* q_buf, TensorWrapper<T>* k_buf, TensorWrapper<T>* v_buf,
                                           TensorWrapper<T>* QKV, BaseWeight<WT>& qkv,
                                           TensorWrapper<int>* padding_offset, TensorWrapper<int>* history_length,
                                           TensorWrapper<int>* input_length, LLaMAAttentionStaticParams& params,
                                           void* stream = nullptr) {
    (void)qkv;
    (void)input_length;
    LLM_CHECK_WITH_INFO(q_buf->shape.size() == 4 && k_buf->shape.size() == 4, "q/k/v bufs must be [bs, heads, seq, head]");
    const int batch = q_buf->shape[0], heads = q_buf->shape[1], seq = q_buf->shape[2], head = q_buf->shape[3];
    const int kv = k_buf->shape[1];
    const int tokens = QKV->size() / ((heads + 2 * kv) * head);
    LLMI_CALL(llmi_rope_qkv_prefill(QKV->data, q_buf->data, k_buf->data, v_buf->data, llmiDtype(getTensorType<T>()),
                                    padding_offset->data, history_length->data, tokens, batch, seq, heads, kv, head,
                                    params.rotary_embedding_base, stream));
}

// concat_past_kv.h:11-18 -- k/v [bs, kv_heads, max_q_len, head] -> caches
// [layers, bs, kv_heads, max_seq, head] at slots history_length[b] + t, t < cur_query_length[b].
template <typename T>
void launchConcatKVCache(TensorWrapper<T>* k_src, TensorWrapper<T>* v_src, TensorWrapper<int>* layer_id,
                         TensorWrapper<int>* cur_query_length, TensorWrapper<int>* history_length,
                         TensorWrapper<T>* k_dst, TensorWrapper<T>* v_dst, void* stream = nullptr) {
    LLM_CHECK_WITH_INFO(k_src->shape.size() == 4 && k_dst->shape.size() == 5, "concat kv: bad shapes");
    LLMI_CALL(llmi_kv_append(k_src->data, v_src->data, llmiDtype(getTensorType<T>()), layer_id->getVal(),
                             cur_query_length->data, history_length->data, k_src->shape[0], k_src->shape[1],
                             k_src->shape[2], k_src->shape[3], k_dst->shape[3], k_dst->data, v_dst->data, stream));
}

// build_causal_mask.h:8-11 -- mask [bs, max_q_len, max_k_len]
template <typename T>
void launchBuildCausalMasks(TensorWrapper<T>* mask, TensorWrapper<int>* q_lens, TensorWrapper<int>* k_lens,
                            void* stream = nullptr) {
    LLM_CHECK_WITH_INFO(mask->shape.size() == 3, "mask must be [bs, max_q_len, max_k_len]");
    LLMI_CALL(llmi_causal_mask(mask->data, llmiDtype(getTensorType<T>()), q_lens->data, k_lens->data, mask->shape[0],
                               mask->shape[1], mask->shape[2], stream));
}

// attn_softmax_kernel.h:8-12 -- qk, attn_score [bs, heads, q_len, k_len], mask [bs, q_len, k_len]
template <typename T>
void launchScaleMaskAndSoftmax(TensorWrapper<T>* qk, TensorWrapper<T>* mask, TensorWrapper<T>* attn_score, float scale,
                               void* stream = nullptr) {
    LLM_CHECK_WITH_INFO(qk->shape.size() == 4 && mask->shape.size() == 3, "softmax: bad shapes");
    LLMI_CALL(llmi_masked_softmax(qk->data, mask->data, attn_score->data, llmiDtype(getTensorType<T>()), qk->shape[0],
                                  qk->shape[1], qk->shape[2], qk->shape[3], scale, stream));
}

// fused_transpose_and_remv_pad.h:7-9 -- [bs, heads, seq, head] -> [num_tokens, heads, head]
template <typename T>
void launchTransposeOutRemovePadding(TensorWrapper<T>* qkv_buf_w_pad, TensorWrapper<int>* padding_offset,
                                     TensorWrapper<T>* qkv_buf_wo_pad_1, void* stream = nullptr) {
    const int batch = qkv_buf_w_pad->shape[0], heads = qkv_buf_w_pad->shape[1];
    const int seq = qkv_buf_w_pad->shape[2], head = qkv_buf_w_pad->shape[3];
    LLMI_CALL(llmi_transpose_remove_pad(qkv_buf_w_pad->data, padding_offset->data, qkv_buf_wo_pad_1->data,
                                        llmiDtype(getTensorType<T>()), qkv_buf_wo_pad_1->shape[0], batch, seq, heads,
                                        head, stream));
}

// linear.h:29-36 -- output[b, h] = op(input1[b, h]) . op(input2[b, h]) (QK^T: input1 = q,
// input2 = k, trans_b = true; PV: input1 = scores, input2 = v). The intended semantics of
// linear.cu:126-229 (its strideC = Cm * Cm is only right for square outputs); heads of
// input2 must equal input1's (expand GQA k/v first, as the reference's repeat_kv).
template <typename T>
void launchLinearStridedBatchGemm(TensorWrapper<T>* input1, TensorWrapper<T>* input2, TensorWrapper<T>* output,
                                  cublasWrapper* cublas_wrapper = nullptr, bool trans_a = false, bool trans_b = false) {
    LLM_CHECK_WITH_INFO(input1->shape.size() == 4 && input2->shape.size() == 4 && output->shape.size() == 4,
                        "strided batch gemm: tensors must be [bs, heads, rows, cols]");
    const int batch = input1->shape[0] * input1->shape[1];
    const int m = trans_a ? input1->shape[3] : input1->shape[2], k = trans_a ? input1->shape[2] : input1->shape[3];
    const int k2 = trans_b ? input2->shape[3] : input2->shape[2], n = trans_b ? input2->shape[2] : input2->shape[3];
    LLM_CHECK_WITH_INFO(k == k2, "2nd dim of input MUST = 1st dim of weight");
    LLM_CHECK_WITH_INFO(input2->shape[0] * input2->shape[1] == batch, "strided batch gemm: batch counts differ");
    LLM_CHECK_WITH_INFO(output->shape[2] == m && output->shape[3] == n, "strided batch gemm: bad output shape");
    LLMI_CALL(llmi_batched_matmul(input1->data, input2->data, output->data, llmiDtype(getTensorType<T>()), batch, m, n,
                                  k, trans_a ? 1 : 0, trans_b ? 1 : 0, cublas_wrapper ? cublas_wrapper->stream : nullptr));
}

// repeat_kv.h -- caches [layers, bs, kv_heads, max_seq, head] -> k/v_cache_dst
// [bs, heads, max_k_len, head]; positions < context_length[b] (device int) are written.
template <typename T>
void launchRepeatKVCache(TensorWrapper<T>* k_cache_src, TensorWrapper<T>* v_cache_src,
                         TensorWrapper<int>* context_length, TensorWrapper<int>* layer_id,
                         TensorWrapper<T>* k_cache_dst, TensorWrapper<T>* v_cache_dst, void* stream = nullptr) {
    LLM_CHECK_WITH_INFO(k_cache_src->shape.size() == 5 && k_cache_dst->shape.size() == 4, "repeat kv: bad shapes");
    LLMI_CALL(llmi_repeat_kv(k_cache_src->data, v_cache_src->data, llmiDtype(getTensorType<T>()), layer_id->getVal(),
                             context_length->data, context_length->shape[0], k_cache_src->shape[2],
                             k_cache_src->shape[3], k_cache_dst->shape[1], k_cache_dst->shape[2],
                             k_cache_dst->shape[3], k_cache_dst->data, v_cache_dst->data, stream));
}

// cal_paddingoffset.h -- padding_offset [batch, max_q_len] (its first num_tokens entries
// are written), cum_seqlens [batch + 1], input_lengths [batch] (all device int)
inline void launchCalPaddingoffset(TensorWrapper<int>* padding_offset, TensorWrapper<int>* cum_seqlens,
                                   TensorWrapper<int>* input_lengths, void* stream = nullptr) {
    const int batch = padding_offset->shape[0], max_q_len = padding_offset->shape[1];
    LLM_CHECK_WITH_INFO(batch == input_lengths->shape[0], "input lengths numbers should equal to padding offset bs dim");
    LLM_CHECK_WITH_INFO(batch == cum_seqlens->shape[0] - 1,
                        "cum seqlen numbers should equal to padding offset bs dim + 1!");
    LLMI_CALL(llmi_padding_offset(padding_offset->data, cum_seqlens->data, input_lengths->data, batch, max_q_len,
                                  stream));
}
