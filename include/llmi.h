/*
 * llmi.h -- C ABI of the MI355X-native Llama-2 decode engine (libllmi.so).
 *
 * This is the drop-in boundary for the reference's decode hot path
 * (Mr-wang27/llm-inference, the src/kernels launcher headers + the Llama<T> decode
 * loop). Every entry point is plain C: device pointers, sizes, dtype enums,
 * an opaque hipStream_t. No torch or C++ types cross it. Each function cites
 * the reference interface it replaces (paths relative to the reference root).
 *
 * Conventions
 *  - return 0 (LLMI_OK) on success, negative on error; never throws.
 *    LLMI_EINVAL = bad argument, LLMI_EUNSUPPORTED = valid but not built,
 *    LLMI_EHIP - hipError_t = HIP runtime error. llmi_last_error() returns a
 *    thread-local message "[llmi][ERROR] ..." (the reference's LLM_CHECK text
 *    convention, src/utils/macro.h:113-133).
 *  - Row-major tensors. Linear weights are [out_features, in_features]
 *    (PyTorch nn.Linear layout; every layer of the reference calls cuBLAS with
 *    trans_b on exactly this layout, src/kernels/linear.cu:38-99); the
 *    launcher's other forms (weight [in, out], a transposed input) are
 *    llmi_linear_trans.
 *  - Activations are fp32 unless a dtype argument says otherwise; weights
 *    may be fp32, fp16 or int8 (+ per-row fp16 scales, W8A16).
 *  - Nothing here blocks the host or allocates, except engine create/destroy and
 *    the engine's host<->device copy helpers; all launches are stream-ordered
 *    and graph-capturable.
 */
#ifndef LLMI_H_
#define LLMI_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* llmi_stream_t; /* hipStream_t; NULL = legacy default stream */

enum llmi_dtype { LLMI_F32 = 0, LLMI_F16 = 1, LLMI_I8 = 2, LLMI_I32 = 3, LLMI_I64 = 4 };

#define LLMI_OK 0
#define LLMI_EINVAL (-1)
#define LLMI_EUNSUPPORTED (-2)
#define LLMI_ENOMEM (-3)
#define LLMI_EHIP (-1000)

const char* llmi_last_error(void);
const char* llmi_version(void);

/* ======================================================================
 * Operator API: one entry per reference launcher on the decode path.
 * ==================================================================== */

/* launchInputEmbedding (src/kernels/input_embedding.h:6-9):
 * out[t, :] = table[ids[t], :] for t < n_tokens; out fp32 [n_tokens, hidden].
 * Bit-exact copy (fp16 -> fp32 widening is exact). ids out of range -> error flag. */
int llmi_embedding(const int32_t* ids, int n_tokens, const void* table, int table_dtype,
                   int vocab, int hidden, float* out, llmi_stream_t stream);

/* launchRMSNorm (src/kernels/rmsnorm_kernel.h:11-17):
 * out = gamma * (x * rsqrt(mean(x^2) + eps)) per row (modeling_llama.py:112-117).
 * residual_out (nullable) receives the pre-norm x (the reference's intent;
 * its kernel aliases it). x may alias out. */
int llmi_rmsnorm(const float* x, float* out, float* residual_out, const void* gamma, int gamma_dtype,
                 int n_tokens, int hidden, float eps, llmi_stream_t stream);

/* launchFusedAddBiasResidualRMSNorm (src/kernels/fused_addresidual_norm.h:9-15):
 * residual = residual + decoder_out (+ bias); decoder_out = rmsnorm(residual) * gamma.
 * bias is nullable (Llama-2 has none). */
int llmi_add_residual_rmsnorm(float* residual, float* decoder_out, const void* bias, int bias_dtype,
                              const void* gamma, int gamma_dtype, int n_tokens, int hidden, float eps,
                              llmi_stream_t stream);

/* launchAddResidual (src/kernels/add_residual.h:8-13): decoder_out += residual. */
int llmi_add_residual(const float* residual, float* decoder_out, int n_tokens, int hidden,
                      llmi_stream_t stream);

/* Elementwise f16 <-> f32 (round to nearest even): no reference counterpart; the
 * C++ mirror (include/llmi/kernels.h) stages TensorWrapper<half> activations of the
 * reference's fp16 instantiation through the fp32 operators with it. */
int llmi_convert(const void* src, int src_dtype, void* dst, int dst_dtype, size_t n, llmi_stream_t stream);

/* launchAct (src/kernels/act_kernel.h:8-9): in [n, 2, inter] (gate then up),
 * out[n, i] = silu(gate) * up. */
int llmi_silu_mul(const float* gate_up, float* out, int n_tokens, int inter, llmi_stream_t stream);

/* launchLinearGemm (src/kernels/linear.h:16-22) with trans_b = true:
 * y[m, n] = sum_k x[m, k] * W[n, k] (* scales[n] for int8). fp32 accumulate.
 * decode (m <= 8): HBM-streaming GEMV; m > 8: batched (prefill) path. */
int llmi_linear(const float* x, const void* w, int w_dtype, const void* w_scales, float* y, int m,
                int n, int k, llmi_stream_t stream);

/* launchLinearGemm (src/kernels/linear.h:16-22, linear.cu:38-99) with both of its flags,
 * row-major: y[m, n] = op_a(x) . op_b(W), where
 *   op_a(x) = x [m, k]            (trans_a = 0)  or  x^T with x stored [k, m]  (trans_a = 1),
 *   op_b(W) = W stored [k, n]     (trans_b = 0, the reference's default: weight [in, out])
 *          or W^T with W [n, k]   (trans_b = 1: nn.Linear's [out, in], llmi_linear).
 * trans_b = 1, trans_a = 0 is llmi_linear itself; the other forms transpose the operand(s)
 * into a per-(device, stream) scratch (grown outside stream capture: run the shape once
 * before capturing) and then run llmi_linear, so every form has llmi_linear's arithmetic.
 * f16 / f32 weights; int8 weights only with trans_b = 1 (their scales are per output row).
 * Cost: trans_b = 0 transposes the WHOLE weight on every call (one extra n*k read and write,
 * so a weight-bound call moves ~3x the bytes of trans_b = 1); store weights [out, in] and pass
 * trans_b = 1 on a hot path, as every reference layer does. The scratch is kept per (device,
 * stream) for the process's lifetime, sized by the largest call. */
int llmi_linear_trans(const float* x, const void* w, int w_dtype, const void* w_scales, float* y, int m, int n, int k,
                      int trans_a, int trans_b, llmi_stream_t stream);

/* LLaMAFFNLayer::forward (ffn.cpp:52-93) for context rows as one call: y [m, hidden] =
 * W_down (silu(W_gate x) * (W_up x)), x [m, hidden] fp32, w_gate_up [2 inter, hidden] (gate
 * rows then up rows, the reference's fused gate_up_proj) and w_down [hidden, inter] fp16.
 * On the matrix cores with fp32-faithful split activations (llmi_linear's arithmetic); the
 * SiLU*up product goes from the gate_up epilogue straight into the down GEMM's input, never
 * to memory in fp32. LLMI_EUNSUPPORTED (nothing launched) for other dtypes / shapes: the
 * caller then runs llmi_linear + llmi_silu_mul + llmi_linear. */
int llmi_ffn(const float* x, const void* w_gate_up, const void* w_down, int w_dtype, float* y, int m, int hidden,
             int inter, llmi_stream_t stream);

/* The context decoder's projection + residual pair in one call (LlamaContextDecoder,
 * context_decoder.cpp:104-139): launchLinearGemm(o_proj) followed by
 * launchFusedAddBiasResidualRMSNorm (no bias), or the FFN followed by launchAddResidual and
 * the next layer's launchRMSNorm. With p = x . W^T (llmi_linear's arithmetic, K slices summed
 * in slice order): residual[m, n] += p, then out[m, n] = RMSNorm(residual) * gamma (gamma
 * null: out = residual; out null: the residual update alone). out may alias x (it is written
 * after x is read), not residual. fp16 weights, m >= 16, GEMM-tileable n / k, n <= 8192;
 * other cases return LLMI_EUNSUPPORTED with nothing launched (the caller runs the separate
 * launches). */
int llmi_linear_residual(const float* x, const void* w, int w_dtype, int m, int n, int k, float* residual, float* out,
                         const void* gamma, int gamma_dtype, float eps, llmi_stream_t stream);
/* llmi_ffn with the same residual epilogue: residual[m, hidden] += FFN(x), then out as above. */
int llmi_ffn_residual(const float* x, const void* w_gate_up, const void* w_down, int w_dtype, int m, int hidden,
                      int inter, float* residual, float* out, const void* gamma, int gamma_dtype, float eps,
                      llmi_stream_t stream);

/* Sticky device error bits recorded by launches on `stream` (current device) that have no
 * error word of their own -- llmi_linear / llmi_ffn / the *_residual calls: 16 = a stream-K
 * partial never arrived within 2 s (its workgroup could not run alongside the others), so
 * that output is incomplete. Synchronises the stream, stores the bits in *flags and clears
 * them. No counterpart in the reference (its cuBLAS calls have no cross-workgroup wait).
 * Concurrency: the stream-K control words (epoch, arrival count) live in a per-(device,
 * stream) workspace; launches on one workspace must not overlap, i.e. do not replay a graph
 * captured on stream S on another stream while eager stream-K launches run on S (the epoch
 * count would race silently). Launches on different streams use different workspaces. */
int llmi_stream_errors(llmi_stream_t stream, int* flags);

/* Test hook for the stream-K hand-off (no reference counterpart): the next `launches`
 * stream-K launches (any stream, this process) run with fault `mode` -- 1: no later piece
 * ever publishes its flag (every owner waiting on one times out after 2 s and sets bit 16),
 * 2: every later piece publishes 2.5 s late, after its owner gave up (a launch that follows
 * must still be correct: flags carry a per-launch epoch). 0 / launches 0 clears it. */
int llmi_debug_stream_k(int mode, int launches);

/* Diagnostics (no reference counterpart): while `stamps` (device memory, 8 u64 per
 * workgroup) is non-null, every launch of the transposed prefill attention kernel writes its
 * per-workgroup timeline there (WgStamp: start, copies of the first block landed, loop end,
 * end, __smid(), then query block | head << 16, key blocks). Null turns it off. */
int llmi_debug_prefill_stamps(void* stamps);

/* One decode row through the HBM-streaming GEMV with its fused prologue/epilogue -- what
 * LlamaSelfDecoder::forward strings together for a token (self_decoder.cpp:59-81 fused):
 *   gamma != NULL: x is RMS-normalised and scaled by gamma (dtype gamma_dtype) first;
 *   epilogue 0: y[n] = W x;  1: y[n] = W x + resid[n] (resid may not alias y);
 *   2: W is [gate; up] (n = 2 inter rows), y[inter] = silu(W_gate x) * (W_up x).
 * fp32 x / y / resid, W f16, f32 or i8 (+ scales). */
int llmi_linear_fused(const float* x, const void* w, int w_dtype, const void* w_scales, float* y, int n, int k,
                      const void* gamma, int gamma_dtype, float eps, int epilogue, const float* resid,
                      llmi_stream_t stream);

/* launchRoPE (src/kernels/qkv_bias_and_RoPE.h:40-42) for one decode token:
 * rotates q (heads) and k (kv_heads) of the fused qkv row [ (h + 2kv) * d ]
 * in place at position `pos` (= step - 1), pairs (i, i + d/2),
 * theta_i = base^(-2i/d) (modeling_llama.py:123-156, 204-236). */
int llmi_rope_decode(float* qkv, int pos, int heads, int kv_heads, int head_dim, float base,
                     llmi_stream_t stream);

/* launchDecoderMaskedMHA (src/kernels/fused_decoder_self_attention.h:10-19):
 * writes k, v of the fused qkv row into the cache slot `pos` of `layer`
 * (cache [layers, kv_heads, max_seq, head_dim], dtype f16 or f32), then
 * out[h] = softmax(q_h . K^T / sqrt(d)) V over positions 0..pos (fp32
 * softmax, split-KV over workgroups, log-sum-exp merge in a second launch).
 * rope != 0 additionally applies RoPE to q/k first (the engine's fused form).
 * workspace: >= llmi_attn_workspace_bytes(...) bytes of device memory (split
 * partials; no initialisation needed). */
size_t llmi_attn_workspace_bytes(int heads, int head_dim, int max_seq);
int llmi_attn_decode(const float* qkv, void* k_cache, void* v_cache, int cache_dtype, int layer,
                     int max_seq, int pos, int heads, int kv_heads, int head_dim, int rope,
                     float rope_base, float* out, void* workspace, llmi_stream_t stream);

/* launchTopKforBeamSearch + launchSampling (src/kernels/topK.h:51-56,
 * sampling.h:12-18) as wired by Llama<T> (K = beamwidth = 1, llama.cpp:59):
 * greedy argmax over logits[n]; ties -> lowest index. out_id: device int32. */
int llmi_argmax(const float* logits, int n, int32_t* out_id, llmi_stream_t stream);

/* launchTopKforBeamSearch (src/kernels/topK.h:51-56, topK.cu:24-191): per row of
 * logits [rows, vocab] (f32/f16), the k largest values in descending order -> topk_ids
 * [rows, k] (device int32) and topk_vals [rows, k] (same dtype). Ties -> lower index
 * (the reference's tie order follows its CUB reduction tree). k in [1, 16]; the
 * reference fixes K = 5 (topK.cu:154). vocab < k pads with id -1, value 1e-20 (topK.h:15-20). */
int llmi_topk(const void* logits, int dtype, int rows, int vocab, int k, int32_t* topk_ids, void* topk_vals,
              llmi_stream_t stream);

/* launchSampling (src/kernels/sampling.h:12-18, sampling.cu:28-115): for each row not yet
 * finished, topk_vals <- exp(v - v[0]) in place, threshold u * sum, output_id = the first id
 * whose running subtraction reaches <= 0 (% vocab), seqlen += 1, is_finished = (id == end_id).
 * u in (0, 1] is the reference's draw, curand_uniform of curand_init(step, row, 0): cuRAND's
 * XORWOW restated (rows < 65536). is_finished: device uint8 (C++ bool). */
int llmi_sampling(const int32_t* topk_ids, void* topk_vals, int dtype, int rows, int k, int32_t* output_id,
                  int32_t* seqlen, uint8_t* is_finished, int step, int end_id, int vocab, llmi_stream_t stream);

/* The draw llmi_sampling makes, computed on the host (no device work): the first
 * curand_uniform of curand_init(seed, subsequence, 0) -- cuRAND's XORWOW as restated in
 * csrc/xorwow.h (subsequence < 65536). For checking the restatement against a CPU oracle. */
int llmi_curand_uniform(uint64_t seed, uint32_t subsequence, float* out);

/* launchRepeatKVCache (src/kernels/repeat_kv.h, repeat_kv.cu:7-91): caches [layers, batch,
 * kv_heads, max_seq, d] -> k_dst/v_dst [batch, heads, max_k_len, d], query head h reading kv
 * head h / (heads / kv_heads), positions < context_length[b] only. */
int llmi_repeat_kv(const void* k_cache, const void* v_cache, int dtype, int layer, const int32_t* context_length,
                   int batch, int kv_heads, int max_seq, int heads, int max_k_len, int head_dim, void* k_dst,
                   void* v_dst, llmi_stream_t stream);

/* ---- context-phase (prefill) operators of the reference's unfused attention layer
 * (LLaMAContextAttentionLayer::forward, context_attention.cpp:108-161). The engine's
 * llmi_engine_prefill fuses them; these are the per-launcher equivalents. dtype is
 * LLMI_F32 or LLMI_F16 for every tensor of a call (fp32 arithmetic); integer arrays
 * are device int32. Layouts are the reference's. */

/* launchCalPaddingoffset (src/kernels/cal_paddingoffset.h, .cu:51-86): input_lengths
 * [batch] -> padding_offset [sum of lengths] (token i sits at padded position
 * i + padding_offset[i] of [batch, max_q_len]) and cum_seqlens [batch + 1]. Lengths must
 * be <= max_q_len (the reference does not check; not checked on the device either). */
int llmi_padding_offset(int32_t* padding_offset, int32_t* cum_seqlens, const int32_t* input_lengths, int batch,
                        int max_q_len, llmi_stream_t stream);

/* launchAddFusedQKVBiasTransposeAndRoPE (src/kernels/qkv_bias_and_RoPE.h:26-36,
 * .cu:49-144), Llama (no bias): qkv [num_tokens, (heads + 2 kv_heads) * d] ->
 * q [batch, heads, seq_len, d], k, v [batch, kv_heads, seq_len, d]; token i goes to
 * padded position i + padding_offset[i]; q and k are rotated at position
 * history_length[b] + s (s = the token's index in its sequence), pairs (i, i + d/2),
 * with llmi_rope_decode's angle arithmetic. Two deliberate differences from the
 * reference kernel (bugs there): v is written (the reference leaves v_buf unset) and
 * the position is per sequence (the reference adds the packed token index, which is
 * the same thing at batch 1). */
int llmi_rope_qkv_prefill(const void* qkv, void* q, void* k, void* v, int dtype, const int32_t* padding_offset,
                          const int32_t* history_length, int num_tokens, int batch, int seq_len, int heads,
                          int kv_heads, int head_dim, float rope_base, llmi_stream_t stream);

/* launchConcatKVCache (src/kernels/concat_past_kv.h:11-18, .cu:16-143): k_src, v_src
 * [batch, kv_heads, max_q_len, d] -> caches [layers, batch, kv_heads, max_seq, d] at
 * slots history_length[b] + t for t < cur_query_length[b] of layer `layer`. */
int llmi_kv_append(const void* k_src, const void* v_src, int dtype, int layer, const int32_t* cur_query_length,
                   const int32_t* history_length, int batch, int kv_heads, int max_q_len, int head_dim, int max_seq,
                   void* k_cache, void* v_cache, llmi_stream_t stream);

/* launchBuildCausalMasks (src/kernels/build_causal_mask.h:8-11, .cu:4-45): mask
 * [batch, max_q_len, max_k_len] = 1 where q < q_lens[b], k < k_lens[b] and
 * k <= q + k_lens[b] - q_lens[b], else 0. (The reference's :29 also requires
 * k >= k_lens[b] - q_lens[b], which hides every history key from the chunk's queries;
 * identical without history. DESIGN.md §4.) */
int llmi_causal_mask(void* mask, int dtype, const int32_t* q_lens, const int32_t* k_lens, int batch,
                     int max_q_len, int max_k_len, llmi_stream_t stream);

/* The attention core of LLaMAContextAttentionLayer::forward after the cache append
 * (context_attention.cpp:125-161: launchRepeatKVCache -> QK^T launchLinearStridedBatchGemm
 * -> launchScaleMaskAndSoftmax with llmi_causal_mask's mask -> PV GEMM ->
 * launchTransposeOutRemovePadding) as ONE fused launch: q [batch, heads, max_q_len, d]
 * (rotated, fp32), caches [layers, batch, kv_heads, max_seq, d] (dtype LLMI_F32 or
 * LLMI_F16) of layer `layer` already holding each sequence's history and this chunk;
 * sequence b's query s (< input_length[b]) attends to slots k <= history_length[b] + s;
 * softmax(scale * qk) normalised by 1 / (sum + 1e-6) as the reference; out [num_tokens,
 * heads, d] fp32 with the sequences packed in batch order (launchCalPaddingoffset's
 * packing). head_dim 128. */
int llmi_context_attention(const float* q, const void* k_cache, const void* v_cache, int cache_dtype, int layer,
                           const int32_t* history_length, const int32_t* input_length, int batch, int heads,
                           int kv_heads, int max_q_len, int max_seq, int head_dim, float scale, float* out,
                           llmi_stream_t stream);

/* The same core with the two launchers in front of it fused in (launchAddFusedQKVBiasTransposeAndRoPE
 * + launchConcatKVCache, context_attention.cpp:108-124): qkv [num_tokens, (heads + 2 kv_heads) d]
 * fp32 rows (padding_offset as llmi_padding_offset makes it) are rotated at position
 * history_length[b] + s (llmi_rope_qkv_prefill's arithmetic), q goes to q_scratch [batch,
 * heads, max_q_len, d] and k / v straight into the cache slots llmi_kv_append would write
 * (rounded to the cache dtype), then llmi_context_attention runs. */
int llmi_context_attention_qkv(const float* qkv, const int32_t* padding_offset, const int32_t* history_length,
                               const int32_t* input_length, int num_tokens, int batch, int max_q_len, int heads,
                               int kv_heads, int head_dim, float rope_base, void* k_cache, void* v_cache,
                               int cache_dtype, int layer, int max_seq, float scale, float* q_scratch, float* out,
                               llmi_stream_t stream);
/* llmi_context_attention_qkv preceded by its q/k/v projection (context_attention.cpp:99's
 * launchLinearGemm): qkv = x [num_tokens, hidden] . w_qkv^T ((heads + 2 kv_heads) * head_dim
 * rows, fp16) with llmi_linear's arithmetic, its K slices summed in slice order by the RoPE
 * kernel as it reads them (the same values, no [num_tokens, qkv] pass). LLMI_EUNSUPPORTED
 * (nothing launched) for other weight dtypes / shapes: the caller runs llmi_linear first. */
int llmi_context_attention_proj(const float* x, const void* w_qkv, int w_dtype, int hidden,
                                const int32_t* padding_offset, const int32_t* history_length,
                                const int32_t* input_length, int num_tokens, int batch, int max_q_len, int heads,
                                int kv_heads, int head_dim, float rope_base, void* k_cache, void* v_cache,
                                int cache_dtype, int layer, int max_seq, float scale, float* q_scratch, float* out,
                                llmi_stream_t stream);

/* launchScaleMaskAndSoftmax (src/kernels/attn_softmax_kernel.h:8-12, .cu:79-174):
 * score[b, h, q, :] = softmax(scale * qk[b, h, q, :] + (1 - mask[b, q, :]) * -10000)
 * normalised by 1 / (sum + 1e-6) as the reference; qk, score [batch, heads, q_len,
 * k_len], mask [batch, q_len, k_len]. score may alias qk. */
int llmi_masked_softmax(const void* qk, const void* mask, void* score, int dtype, int batch, int heads, int q_len,
                        int k_len, float scale, llmi_stream_t stream);

/* launchLinearStridedBatchGemm (src/kernels/linear.h:29-36, .cu:126-229): for each of
 * `batch` matrices (contiguous, row-major) c[z] = op(a[z]) . op(b[z]); op(a) [m, k] is a
 * [m, k] or, with trans_a, a [k, m]; op(b) [k, n] is b [k, n] or, with trans_b, b [n, k];
 * c [m, n]; fp32 accumulate. QK^T: a = q, b = k, trans_b = 1; PV: a = scores, b = v. */
int llmi_batched_matmul(const void* a, const void* b, void* c, int dtype, int batch, int m, int n, int k, int trans_a,
                        int trans_b, llmi_stream_t stream);

/* launchTransposeOutRemovePadding (src/kernels/fused_transpose_and_remv_pad.h:7-9,
 * .cu:17-75): src [batch, heads, seq_len, d] -> dst [num_tokens, heads * d], token i
 * read from padded position i + padding_offset[i]. */
int llmi_transpose_remove_pad(const void* src, const int32_t* padding_offset, void* dst, int dtype, int num_tokens,
                              int batch, int seq_len, int heads, int head_dim, llmi_stream_t stream);

/* Synthetic-weight generator (replaces LlamaLayerWeight::loadWeights() dummy
 * path, src/weights/llama/layer_weights.cc:69-146). Fills the [rows, cols]
 * slice (row0, col0) of a logical [*, ld] tensor `tid` with llmi-prng-v1
 * values (spec: oracle/prng.py). kind: 0 linear, 1 embedding, 2 norm gamma
 * (rows = 1), 3 int8 weight, 4 int8 per-row scale (cols = 1).
 * out_dtype: F16 or F32 (values identical), I8 for kind 3, F16 for kind 4. */
enum llmi_synth_kind { LLMI_SYN_LINEAR = 0, LLMI_SYN_EMBED = 1, LLMI_SYN_GAMMA = 2,
                       LLMI_SYN_INT8 = 3, LLMI_SYN_INT8_SCALE = 4 };
int llmi_synth_fill(void* out, int out_dtype, int kind, uint64_t seed, uint32_t tid, int rows,
                    int cols, int row0, int col0, int ld, llmi_stream_t stream);
/* Host (CPU) twin of llmi_synth_fill, for checking the generator without a GPU. */
int llmi_synth_fill_host(void* out, int out_dtype, int kind, uint64_t seed, uint32_t tid, int rows,
                         int cols, int row0, int col0, int ld);
/* Device memory for host-side callers that include no HIP headers (the C++
 * mirror in include/llmi/): hipMalloc / hipFree / hipMemcpy / hipDeviceSynchronize.
 * kind: 0 host->device, 1 device->host, 2 device->device. */
int llmi_device_alloc(void** ptr, size_t bytes);
int llmi_device_free(void* ptr);
int llmi_device_memset(void* ptr, int value, size_t bytes);
/* stream-ordered form (hipMemsetAsync): the layer classes' scratch on their stream */
int llmi_device_memset_async(void* ptr, int value, size_t bytes, llmi_stream_t stream);
int llmi_memcpy(void* dst, const void* src, size_t bytes, int kind);
int llmi_device_sync(void);

/* Measured HBM read peak (the roofline's second denominator, SURVEY.md §8d timing rules):
 * one-shot launches that each read `bytes` (rounded down to whole 32-KB pieces per
 * workgroup) with non-temporal 16-B loads, 8 in flight per lane, cycling through the regions
 * of a 2 GiB buffer so every launch streams from HBM (not the 256 MiB Infinity Cache), timed
 * with HIP events over `iters` launches for grids of 512 / 1024 / 2048 / 4096 workgroups; the
 * best grid's average microseconds per launch, its GB/s and the bytes one launch read. */
int llmi_hbm_read_bench(size_t bytes, int iters, float* us, float* gbps, size_t* bytes_read);

/* Synthetic prompt ids (bench config: 8 PRNG ids). Host only. */
int llmi_synth_prompt(uint64_t seed, int n, int vocab, int32_t* out);

/* ======================================================================
 * Engine API: the Llama<T> decode loop (src/models/llama/llama.cpp:318-349
 * continueTokenGen, :362-457 Response) with the per-layer sequence of
 * LlamaSelfDecoder::forward (src/layers/decoder/self_decoder.cpp:23-89).
 * One engine per GPU (per TP rank). The whole token step -- embedding,
 * L x {rmsnorm+QKV, rope+kv-write+attention, O+residual, rmsnorm+gate_up+silu,
 * down+residual}, final norm + lm_head + argmax -- is one hipGraph replay;
 * positions and token ids live in device memory, so no host sync per token.
 * ==================================================================== */
typedef struct llmi_config {
    int hidden, heads, kv_heads, head_dim, inter, layers, vocab, max_seq;
    float rms_eps, rope_base;
    int weight_dtype; /* LLMI_F16 (default), LLMI_F32 (reference Llama<float>), LLMI_I8 (W8A16) */
    int kv_dtype;     /* LLMI_F16 (throughput) or LLMI_F32 (parity) */
    int tp_rank, tp_world;
} llmi_config;

typedef struct llmi_engine llmi_engine;

/* Fill `cfg` with a preset: "llama2-7b", "llama2-13b", "tiny". */
int llmi_config_preset(const char* name, llmi_config* cfg);

/* RCCL unique id (128 bytes) for tensor parallel: rank 0 creates it, the
 * launcher broadcasts it (any side channel), every rank passes it to create. */
int llmi_tp_unique_id(void* out128);

/* Tensor-parallel all-reduce for operator-level callers (the sum of the
 * row-parallel partials after o_proj and down, modeling_llama.py pretraining_tp
 * semantics; the reference has none). One communicator per rank over RCCL (xGMI):
 * llmi_tp_comm_create on `device` with the broadcast id; llmi_tp_allreduce sums `count`
 * elements of buf in place across the ranks on `stream` (dtype LLMI_F32, LLMI_F16,
 * LLMI_I32 or LLMI_I64 -- the engine reduces its int64 fixed-point residual, exact and
 * order-independent). The engine owns its own communicator (llmi_engine_create). */
typedef struct llmi_tp_comm llmi_tp_comm;
int llmi_tp_comm_create(const void* tp_id, int world, int rank, int device, llmi_tp_comm** out);
int llmi_tp_allreduce(llmi_tp_comm* comm, void* buf, size_t count, int dtype, llmi_stream_t stream);
int llmi_tp_comm_destroy(llmi_tp_comm* comm);

/* device: HIP device ordinal. tp_id: 128-byte RCCL id (llmi_tp_unique_id, broadcast
 * to every rank): the engine creates an RCCL communicator and the token graph all-reduces
 * over it (with tp_world == 1 too: identities). With tp_world > 1 and tp_id NULL there is
 * no RCCL communicator: the ranks must open the one-shot peer exchange (below) before
 * they decode. */
int llmi_engine_create(const llmi_config* cfg, int device, const void* tp_id, llmi_engine** out);
int llmi_engine_destroy(llmi_engine* e);
/* Llama<T>::loadWeightsFromDummy (src/models/llama/llama.h) with llmi-prng-v1 weights. */
int llmi_engine_load_synthetic(llmi_engine* e, uint64_t seed);
/* LlamaWeight<T>::loadWeights(weight_path) (llama_weights.cc:41-53, layer_weights.cc:48-66,
 * loadWeightFromBin weight_utils.cu:90-187): reads weight_path + "<name>.bin", raw fp32, for
 * model.embed_tokens.weight, lm_head.weight, model.norm.weight and per layer l
 * model.layers.<l>.{input_layernorm, post_attention_layernorm, self_attn.qkv, self_attn.o_proj,
 * mlp.gate_up_proj, mlp.down_proj}.weight (unsharded shapes; this rank's slice is taken).
 * fp32 -> fp16 is round-to-nearest-even. int8 engines are refused (no reference format). */
int llmi_engine_load_bin(llmi_engine* e, const char* weight_path);
/* One tensor of the same set from a host fp32 buffer (name without ".bin"; count checked). */
int llmi_engine_load_tensor(llmi_engine* e, const char* name, const float* host, size_t count);
/* Llama<T>::Sampling (llama.cpp:245-262: launchTopKforBeamSearch + launchSampling) inside the
 * decode step: k in [1, 16] samples each generated token from the top k logits with
 * sampling.cu's rule, u = curand_uniform(curand_init(step, 0, 0)) (cuRAND XORWOW restated)
 * at step = seed + (tokens so far, the sampled token's position) (seed 0: the reference's step,
 * llama.cpp:405-423);
 * k = 0 restores greedy argmax (the default). Needs tp_world == 1. Applies to tokens chosen
 * by decode steps (a batched prefill's first token stays greedy). */
int llmi_engine_set_sampling(llmi_engine* e, int k, uint64_t seed);
/* Reset the sequence and stage a prompt (device copy). */
int llmi_engine_set_prompt(llmi_engine* e, const int32_t* ids, int n);
/* Run n forward steps (one token each). use_graph: replay the captured hipGraph. */
int llmi_engine_decode(llmi_engine* e, int n_steps, int use_graph);
/* Prefill (Llama<T>::firstTokenGen, llama.cpp:273-316; LlamaContextDecoder::forward,
 * context_decoder.cpp:47-143): the next n_tokens prompt rows in one batched pass
 * (chunks of 512) -- MFMA GEMMs, causal prefill attention, KV slots written --
 * then the last row's lm_head + argmax. Afterwards the engine is exactly where
 * n_tokens decode steps would have left it, so llmi_engine_decode continues.
 * exact = 1: fp32-faithful GEMMs (activations split into two fp16 halves);
 * exact = 2: the fp16 hi half exact, the remainder as e4m3 against e4m3 weight
 *   copies on the block-scaled fp8 MFMA (~1e-4 relative; the copies are made on the
 *   first such call and kept at the fp16 row stride, i.e. as many bytes as the fp16
 *   GEMM weights; an fp32 KV cache or shapes without K % 128 == 0 fall back to
 *   exact = 1);
 * exact = 0: activations rounded to fp16 (faster, ~1e-3 relative at 32 layers).
 * Rows must lie inside the prompt; tp_world must be 1. fp32 weights run the
 * decode kernels row by row. */
int llmi_engine_prefill(llmi_engine* e, int n_tokens, int exact);
/* Block until the engine stream is idle. */
int llmi_engine_sync(llmi_engine* e);
/* Tokens[0 .. n) of the sequence so far: prompt ids followed by generated ids
 * (position p's token; the token after the last forward is included). */
int llmi_engine_tokens(llmi_engine* e, int32_t* out, int n, int* n_valid);
/* fp32 logits of the last forward (this rank's vocab shard under TP). */
int llmi_engine_logits(llmi_engine* e, float* out, int n);
/* fp32 residual stream (hidden) after the last forward. */
int llmi_engine_hidden(llmi_engine* e, float* out, int n);
/* Read one cache slot (layer, pos) of K or V as fp32 [kv_heads_local, head_dim]. */
int llmi_engine_kv_slot(llmi_engine* e, int layer, int pos, int which_v, float* out);
/* Bytes of weights (and KV per position) one forward streams on this rank. */
int llmi_engine_bytes(llmi_engine* e, uint64_t* weight_bytes, uint64_t* kv_bytes_per_pos);
/* hipStream_t the engine launches on. */
llmi_stream_t llmi_engine_stream(llmi_engine* e);
/* Time `iters` eager launches of one kernel (HIP events on the engine stream);
 * launch i runs layer i % layers, so its weights stream from HBM as in decode.
 * which: 0 qkv, 1 attn, 2 o, 3 gate_up, 4 down, 5 lm_head; 6 / 7 one TP residual
 * all-reduce (RCCL int64, hidden elements; engines created with a tp_id) launched
 * eagerly / replayed from one captured graph of `iters` calls -- a collective: every
 * rank must make the same call.
 * avg_us receives the mean duration; bytes the algorithmic bytes per launch. */
int llmi_engine_time_kernel(llmi_engine* e, int which, int iters, float* avg_us, uint64_t* bytes);
/* which 8 / 9: the same residual exchange over the one-shot peer path (below), eager /
 * graph-replayed -- also a collective. which 10: the persistent ring layer (decode mode 1,
 * below): o_proj + gate_up + down + the next layer's q/k/v in one launch. */

/* Decode structure of a token (no reference counterpart: the reference launches ~326
 * kernels per token). mode 0: 5 L + 2 launches (q/k/v, attention, o_proj, gate_up, down
 * per layer). mode 1: the persistent ring layer -- per layer the attention launch plus
 * ONE launch for o_proj, RMSNorm + gate_up + SiLU*up, down (K split by CU) and the next
 * layer's RMSNorm + q/k/v, one workgroup per CU whose loader waves stream the weights
 * through an LDS ring ahead of the in-launch hand-offs (2 L + 3 launches). Mode 1 needs
 * fp16 weights, hidden 4096, head_dim 128, heads dividing the CU count and tp_world 1
 * (else LLMI_EUNSUPPORTED); it keeps a transposed copy of every W_down (rebuilt after a
 * weight load). The two modes differ only in the down projection's fp32 summation order.
 * Graphs are re-captured. */
int llmi_engine_set_decode_mode(llmi_engine* e, int mode);

/* ---- One-shot peer exchange for tensor parallel decode (config 4; replaces the RCCL
 * all-reduces of the token graph: the sum of the row-parallel partials of
 * modeling_llama.py's pretraining_tp, :251-266 / :443-446, and the argmax-key max).
 * Every rank owns an inbox in its HBM; each exchange is ONE kernel that writes this rank's
 * int64 partial into every peer's inbox over xGMI, raises per-slice flags, waits for every
 * rank's flags and sums the slots in rank order (exact: bitwise the RCCL result).
 *   1. llmi_engine_xchg_handle: allocate the inbox, return its 64-byte IPC handle;
 *   2. the launcher all-gathers the handles (any side channel; rank order);
 *   3. llmi_engine_xchg_open(e, handles[world * 64]): map every peer's inbox;
 *   4. llmi_engine_set_exchange(e, 1) (0 = RCCL again; graphs are re-captured).
 *      Mode 2 runs the same protocol from INSIDE the producing launches: the o_proj, down
 *      and lm_head kernels end with an arrival ticket; their last workgroups push the
 *      finished vector to every inbox, wait for the peers and reduce in rank order (no
 *      exchange launch, 2 L + 1 fewer launches and kernel boundaries per token); results
 *      are bitwise those of modes 0 and 1.
 * A peer that never arrives (2 s) sets error bit 8: llmi_engine_tokens fails, no hang. */
int llmi_engine_xchg_handle(llmi_engine* e, void* out64);
int llmi_engine_xchg_open(llmi_engine* e, const void* handles);

/* One-GPU pricing of ONE tensor-parallel rank (no reference counterpart): a tp_world > 1
 * engine without peers runs its shard's whole token loop with every peer inbox replaced by
 * its own -- the push writes this rank's slice into its own slot and zeros into the W - 1
 * others (the same bytes a real push writes), raises all W flags, and the reduce sums to
 * this rank's own partial. Tokens are NOT the TP model's (the other ranks' partials are
 * zero); the launch / exchange structure and its timing are. set_exchange 0 then runs no
 * exchange at all (the compute-only floor), 1 the one-shot exchange launches, 2 the
 * exchange fused into the producers. */
int llmi_engine_xchg_loopback(llmi_engine* e);

/* Engine tuning switches for same-process A/B (no reference counterpart); the captured
 * token graphs are rebuilt on the next decode. "kpar": 1 (default) lets a TP rank's q/k/v and
 * gate_up GEMVs split K over 2 or 4 waves of a workgroup when one row group per wave would
 * leave CUs idle or doubled (tp_world > 1 only), 0 keeps one wave per row group.
 * "qkv_attn": 1 (default) runs a layer's q/k/v GEMV and split-KV attention as one launch (q/k/v
 * handed over as tagged 8-byte granules; bitwise the two launches), 0 as two. "qa_o": 1 adds the
 * o_proj to that launch (fp16 MHA, single rank; default 0, measured slower). "qa_grid" (workgroups
 * of the fused launch's GEMV part, 0 = every resident slot), "qa_order" (1 head-major rows and
 * attention blocks, default), "qa_poll" (1 poll every granule from the start): A/B only. */
int llmi_engine_set_option(llmi_engine* e, const char* name, int value);
int llmi_engine_set_exchange(llmi_engine* e, int mode);
/* Diagnostics: kernels launched by llmi_engine_time_kernel (and graphs built
 * afterwards) write a per-workgroup timeline into dev_buf (8 x uint64 per
 * workgroup at 8 * linear block id: start, two kernel-defined marks, end, CU id;
 * 100 MHz clock). NULL switches it off. */
int llmi_engine_debug_stamps(llmi_engine* e, void* dev_buf);
/* Graph-replay timeline: like llmi_engine_debug_stamps, but every stamped launch of a
 * recorded token step (qkv, attention, o_proj, gate_up, down per layer, then lm_head)
 * writes its own region of slot_wgs workgroups x 64 B, in launch order, so one replay of
 * a captured token graph leaves the whole step's per-workgroup timeline. Captured graphs
 * are dropped (re-captured with the stamp pointers on the next graph decode); launches
 * past bytes / (slot_wgs * 64) regions are not stamped. slot_wgs must cover the largest
 * decode grid (the error names the bound). dev_buf NULL switches it off. */
int llmi_engine_debug_timeline(llmi_engine* e, void* dev_buf, size_t bytes, int slot_wgs);
/* Test hook: overwrite the device decode state's next position only (the host's copy is
 * left alone), to check that a host/device position mismatch is reported (error bit 4). */
int llmi_engine_debug_set_next_pos(llmi_engine* e, int next_pos);

/* ---- In-process tensor-parallel group (no reference counterpart: the
 * reference has no TP). W rank engines with tp_rank 0..W-1 on ONE device and
 * one stream, stepped phase by phase with an in-place reduction kernel where
 * the RCCL path all-reduces. RCCL refuses two ranks on one device, so this is
 * the single-GPU parity harness for the sharded path (per-rank weight shards,
 * rank-0 residual, vocab-parallel argmax keys). cfg->tp_rank/tp_world are
 * ignored; the group sets them. Same status codes as the engine. */
typedef struct llmi_group llmi_group;
int llmi_group_create(const llmi_config* cfg, int world, int device, llmi_group** out);
int llmi_group_destroy(llmi_group* g);
int llmi_group_load_synthetic(llmi_group* g, uint64_t seed);
int llmi_group_load_bin(llmi_group* g, const char* weight_path);
int llmi_group_set_prompt(llmi_group* g, const int32_t* ids, int n);
int llmi_group_decode(llmi_group* g, int n_steps, int use_graph);
/* tokens as seen by one rank (every rank must agree) */
int llmi_group_tokens(llmi_group* g, int rank, int32_t* out, int n, int* n_valid);
/* last logits over the full vocab: the ranks' slices concatenated */
int llmi_group_logits(llmi_group* g, float* out, int n);
int llmi_group_hidden(llmi_group* g, int rank, float* out, int n);
/* mode 0: the in-place reduction kernel; 1: the one-shot peer exchange's kernels (every
 * rank's push, then every rank's wait + rank-order reduce; the ranks' inboxes are the
 * group's own device buffers) -- the single-GPU parity check of that protocol; 2: the
 * push fused into every rank's o_proj / down / lm_head launch (their tails), then every
 * rank's reduce kernel (one stream: an in-launch wait for a later rank cannot finish). */
int llmi_group_set_exchange(llmi_group* g, int mode);

#ifdef __cplusplus
}
#endif
#endif /* LLMI_H_ */
