// extern "C" operator API (include/llmi.h): thin argument checks over the
// kernels in gemv.hip / attn.hip / ops.hip. Never throws; errors are return
// codes plus a thread-local message.
#include <map>
#include <mutex>
#include <string>

#include "kernels.h"
#include "prng.h"

namespace llmi {
namespace {
thread_local std::string g_last_error;
}
void set_last_error(const std::string& msg) { g_last_error = msg; }
}  // namespace llmi

using namespace llmi;

#define STREAM(s) reinterpret_cast<hipStream_t>(s)

extern "C" {

const char* llmi_last_error(void) { return llmi::g_last_error.c_str(); }
const char* llmi_version(void) { return "llmi 0.1 (gfx950)"; }

int llmi_embedding(const int32_t* ids, int n_tokens, const void* table, int table_dtype, int vocab, int hidden,
                   float* out, llmi_stream_t stream) {
    return embedding_launch(ids, n_tokens, table, table_dtype, vocab, hidden, out, STREAM(stream));
}

int llmi_rmsnorm(const float* x, float* out, float* residual_out, const void* gamma, int gamma_dtype, int n_tokens,
                 int hidden, float eps, llmi_stream_t stream) {
    return rmsnorm_launch(x, out, residual_out, gamma, gamma_dtype, n_tokens, hidden, eps, STREAM(stream));
}

int llmi_add_residual_rmsnorm(float* residual, float* decoder_out, const void* bias, int bias_dtype,
                              const void* gamma, int gamma_dtype, int n_tokens, int hidden, float eps,
                              llmi_stream_t stream) {
    return add_resid_rmsnorm_launch(residual, decoder_out, bias, bias_dtype, gamma, gamma_dtype, n_tokens, hidden,
                                    eps, STREAM(stream));
}

int llmi_add_residual(const float* residual, float* decoder_out, int n_tokens, int hidden, llmi_stream_t stream) {
    return add_resid_launch(residual, decoder_out, n_tokens, hidden, STREAM(stream));
}

int llmi_convert(const void* src, int src_dtype, void* dst, int dst_dtype, size_t n, llmi_stream_t stream) {
    return convert_launch(src, src_dtype, dst, dst_dtype, n, STREAM(stream));
}

int llmi_silu_mul(const float* gate_up, float* out, int n_tokens, int inter, llmi_stream_t stream) {
    return silu_mul_launch(gate_up, out, n_tokens, inter, STREAM(stream));
}

int llmi_ffn(const float* x, const void* w_gate_up, const void* w_down, int w_dtype, float* y, int m, int hidden,
             int inter, llmi_stream_t stream) {
    LLMI_REQUIRE(x && w_gate_up && w_down && y && m >= 1 && hidden >= 1 && inter >= 1, "ffn: bad arguments");
    if (w_dtype != LLMI_F16 || !ffn_mfma_supported(m, hidden, inter) || (reinterpret_cast<uintptr_t>(x) & 15) ||
        (reinterpret_cast<uintptr_t>(y) & 15) || (reinterpret_cast<uintptr_t>(w_gate_up) & 15) ||
        (reinterpret_cast<uintptr_t>(w_down) & 15)) {
        set_last_error("[llmi][ERROR] ffn: the fused context FFN needs fp16 weights, M >= 16, 16-B aligned buffers "
                       "and GEMM-tileable hidden / inter (use llmi_linear + llmi_silu_mul)");
        return LLMI_EUNSUPPORTED;
    }
    return ffn_mfma_launch(x, w_gate_up, w_down, y, m, hidden, inter, STREAM(stream));
}

namespace {
bool resid_args_ok(const float* x, const void* w, int w_dtype, float* residual, float* out, const void* gamma,
                   int gamma_dtype, int n) {
    auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    return w_dtype == LLMI_F16 && a16(x) && a16(w) && a16(residual) && a16(out) && n % 4 == 0 && n <= 8192 &&
           (!gamma || gamma_dtype == LLMI_F16 || gamma_dtype == LLMI_F32);
}
}  // namespace

int llmi_linear_residual(const float* x, const void* w, int w_dtype, int m, int n, int k, float* residual, float* out,
                         const void* gamma, int gamma_dtype, float eps, llmi_stream_t stream) {
    LLMI_REQUIRE(x && w && residual && m >= 1 && n >= 1 && k >= 1, "linear_residual: bad arguments");
    LLMI_REQUIRE(out != residual, "linear_residual: out must not alias the residual");
    if (!resid_args_ok(x, w, w_dtype, residual, out, gamma, gamma_dtype, n) || !linear_mfma_supported(m, n, k)) {
        set_last_error("[llmi][ERROR] linear_residual: needs fp16 weights, M >= 16, GEMM-tileable n / k, n <= 8192 "
                       "and 16-B aligned buffers (use llmi_linear + llmi_add_residual_rmsnorm)");
        return LLMI_EUNSUPPORTED;
    }
    ResidEpi re;
    re.resid = residual; re.out = out; re.gamma = gamma; re.g_dtype = gamma ? gamma_dtype : LLMI_F32; re.eps = eps;
    return linear_mfma_launch(x, w, nullptr, m, n, k, STREAM(stream), &re);
}

int llmi_ffn_residual(const float* x, const void* w_gate_up, const void* w_down, int w_dtype, int m, int hidden,
                      int inter, float* residual, float* out, const void* gamma, int gamma_dtype, float eps,
                      llmi_stream_t stream) {
    LLMI_REQUIRE(x && w_gate_up && w_down && residual && m >= 1 && hidden >= 1 && inter >= 1,
                 "ffn_residual: bad arguments");
    LLMI_REQUIRE(out != residual, "ffn_residual: out must not alias the residual");
    if (!resid_args_ok(x, w_gate_up, w_dtype, residual, out, gamma, gamma_dtype, hidden) ||
        (reinterpret_cast<uintptr_t>(w_down) & 15) || !ffn_mfma_supported(m, hidden, inter)) {
        set_last_error("[llmi][ERROR] ffn_residual: needs fp16 weights, M >= 16, GEMM-tileable hidden / inter, "
                       "hidden <= 8192 and 16-B aligned buffers (use llmi_ffn + llmi_add_residual)");
        return LLMI_EUNSUPPORTED;
    }
    ResidEpi re;
    re.resid = residual; re.out = out; re.gamma = gamma; re.g_dtype = gamma ? gamma_dtype : LLMI_F32; re.eps = eps;
    return ffn_mfma_launch(x, w_gate_up, w_down, nullptr, m, hidden, inter, STREAM(stream), &re);
}

int llmi_stream_errors(llmi_stream_t stream, int* flags) { return stream_errors(STREAM(stream), flags); }

int llmi_debug_stream_k(int mode, int launches) {
    LLMI_REQUIRE(mode >= 0 && mode <= 2 && launches >= 0, "debug_stream_k: mode 0..2, launches >= 0");
    gemm3_sk_debug(mode, launches);
    return LLMI_OK;
}

int llmi_debug_prefill_stamps(void* stamps) {
    prefill_stamps_debug(static_cast<unsigned long long*>(stamps));
    return LLMI_OK;
}

int llmi_linear(const float* x, const void* w, int w_dtype, const void* w_scales, float* y, int m, int n, int k,
                llmi_stream_t stream) {
    LLMI_REQUIRE(m >= 1 && n >= 1 && k >= 1, "linear: m, n, k must be >= 1");
    GemvArgs a;
    a.w = w;
    a.w_dtype = w_dtype;
    a.scales = reinterpret_cast<const __half*>(w_scales);
    a.n_rows = n;
    a.k = k;
    a.epi = EPI_STORE;
    if (w_dtype == LLMI_F16 && linear_mfma_supported(m, n, k) && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
        (reinterpret_cast<uintptr_t>(y) & 15) == 0 && (reinterpret_cast<uintptr_t>(w) & 15) == 0)
        return linear_mfma_launch(x, w, y, m, n, k, STREAM(stream));  // context rows: the prefill's GEMMs
    if (m > 8 && gemm_supported(w_dtype, n, k, EPI_STORE) && (k % 4) == 0 &&
        (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(w) & 15) == 0) {
        GemmArgs g;  // prefill: MFMA GEMM, fp32-faithful (split activations)
        g.a = x; g.lda = k;
        g.w = w; g.w_dtype = w_dtype; g.scales = a.scales;
        g.m = m; g.n = n; g.k = k; g.split = 2;
        g.epi = EPI_STORE; g.y = y; g.ldy = n;
        return gemm_launch(g, STREAM(stream));
    }
    for (int i = 0; i < m; ++i) {  // decode rows (and shapes the GEMM tiles do not cover): GEMV
        a.x = x + (size_t)i * k;
        a.y = y + (size_t)i * n;
        LLMI_TRY(gemv_launch(a, STREAM(stream)));
    }
    return LLMI_OK;
}

}  // extern "C"

namespace {
// llmi_linear_trans's operand scratch per (device, stream): [0] the transposed weight,
// [1] the transposed input. Grown only outside stream capture, freed after a sync (earlier
// launches on the stream may still read it).
std::mutex g_tr_mu;
std::map<std::pair<int, hipStream_t>, std::pair<void*, size_t>> g_tr[2];
int trans_scratch(int slot, hipStream_t s, size_t bytes, void** out) {
    int dev = 0;
    LLMI_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lock(g_tr_mu);
    auto& e = g_tr[slot][{dev, s}];
    if (bytes > e.second) {
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        LLMI_HIP(hipStreamIsCapturing(s, &cap));
        LLMI_REQUIRE(cap == hipStreamCaptureStatusNone,
                     "linear_trans: the transpose scratch must grow, which cannot happen while the stream is "
                     "capturing (run the same shape once before capture)");
        if (e.first) {
            LLMI_HIP(hipStreamSynchronize(s));
            LLMI_HIP(hipFree(e.first));
            e = {nullptr, 0};
        }
        LLMI_HIP(hipMalloc(&e.first, bytes));
        e.second = bytes;
    }
    *out = e.first;
    return LLMI_OK;
}
}  // namespace

extern "C" {

int llmi_linear_trans(const float* x, const void* w, int w_dtype, const void* w_scales, float* y, int m, int n, int k,
                      int trans_a, int trans_b, llmi_stream_t stream) {
    LLMI_REQUIRE(x && w && y && m >= 1 && n >= 1 && k >= 1, "linear_trans: null pointer or empty shape");
    if (trans_b && !trans_a) return llmi_linear(x, w, w_dtype, w_scales, y, m, n, k, stream);
    LLMI_REQUIRE(w_dtype == LLMI_F16 || w_dtype == LLMI_F32 || trans_b,
                 "linear_trans: int8 weights are [out, in] with per-row scales (trans_b = 1 only)");
    hipStream_t s = STREAM(stream);
    const void* wt = w;
    if (!trans_b) {  // W [k, n] -> [n, k]
        void* buf = nullptr;
        const int eb = w_dtype == LLMI_F16 ? 2 : 4;
        LLMI_TRY(trans_scratch(0, s, (size_t)n * k * eb, &buf));
        LLMI_TRY(transpose_launch(w, buf, k, n, eb, s));
        wt = buf;
    }
    const float* xt = x;
    if (trans_a) {  // x [k, m] -> [m, k]
        void* buf = nullptr;
        LLMI_TRY(trans_scratch(1, s, (size_t)m * k * sizeof(float), &buf));
        LLMI_TRY(transpose_launch(x, buf, k, m, 4, s));
        xt = static_cast<const float*>(buf);
    }
    return llmi_linear(xt, wt, w_dtype, w_scales, y, m, n, k, stream);
}

int llmi_linear_fused(const float* x, const void* w, int w_dtype, const void* w_scales, float* y, int n, int k,
                      const void* gamma, int gamma_dtype, float eps, int epilogue, const float* resid,
                      llmi_stream_t stream) {
    LLMI_REQUIRE(x && w && y && n >= 1 && k >= 1, "linear_fused: null pointer or empty shape");
    LLMI_REQUIRE(epilogue >= 0 && epilogue <= 2, "linear_fused: epilogue must be 0 (store), 1 (add) or 2 (silu_mul)");
    LLMI_REQUIRE(epilogue != 1 || (resid && resid != y), "linear_fused: the add epilogue needs resid != y");
    LLMI_REQUIRE(epilogue != 2 || n % 2 == 0, "linear_fused: silu_mul needs 2 * inter rows");
    GemvArgs a;
    a.w = w;
    a.w_dtype = w_dtype;
    a.scales = reinterpret_cast<const __half*>(w_scales);
    a.n_rows = n;
    a.k = k;
    a.x = x;
    a.gamma = gamma;
    a.g_dtype = gamma_dtype;
    a.eps = eps;
    a.y = y;
    if (epilogue == 0) {
        a.epi = EPI_STORE;
    } else if (epilogue == 1) {
        a.epi = EPI_ADD;
        a.resid = resid;
    } else {
        a.epi = EPI_SILU_MUL;
        a.pair_off = n / 2;
    }
    return gemv_launch(a, STREAM(stream));
}

int llmi_rope_decode(float* qkv, int pos, int heads, int kv_heads, int head_dim, float base, llmi_stream_t stream) {
    return rope_decode_launch(qkv, pos, heads, kv_heads, head_dim, base, STREAM(stream));
}

size_t llmi_attn_workspace_bytes(int heads, int head_dim, int max_seq) {
    return attn_workspace_bytes(heads, head_dim, max_seq);
}

int llmi_attn_decode(const float* qkv, void* k_cache, void* v_cache, int cache_dtype, int layer, int max_seq, int pos,
                     int heads, int kv_heads, int head_dim, int rope, float rope_base, float* out, void* workspace,
                     llmi_stream_t stream) {
    LLMI_REQUIRE(layer >= 0, "attn: layer must be >= 0");
    AttnArgs a;
    const size_t off = (size_t)layer * kv_heads * max_seq * head_dim * dtype_size(cache_dtype);
    a.qkv = qkv;
    a.k_cache = (char*)k_cache + off;
    a.v_cache = (char*)v_cache + off;
    a.cache_dtype = cache_dtype;
    a.max_seq = max_seq;
    a.pos_host = pos;
    a.heads = heads;
    a.kv_heads = kv_heads;
    a.head_dim = head_dim;
    a.rope = rope;
    a.rope_base = rope_base;
    a.out = out;
    a.workspace = workspace;
    return attn_decode_launch(a, STREAM(stream));
}

int llmi_topk(const void* logits, int dtype, int rows, int vocab, int k, int32_t* topk_ids, void* topk_vals,
              llmi_stream_t stream) {
    return topk_launch(logits, dtype, rows, vocab, k, topk_ids, topk_vals, STREAM(stream));
}

int llmi_sampling(const int32_t* topk_ids, void* topk_vals, int dtype, int rows, int k, int32_t* output_id,
                  int32_t* seqlen, uint8_t* is_finished, int step, int end_id, int vocab, llmi_stream_t stream) {
    return sampling_launch(topk_ids, topk_vals, dtype, rows, k, output_id, seqlen, is_finished, step, end_id, vocab,
                           STREAM(stream));
}

int llmi_repeat_kv(const void* k_cache, const void* v_cache, int dtype, int layer, const int32_t* context_length,
                   int batch, int kv_heads, int max_seq, int heads, int max_k_len, int head_dim, void* k_dst,
                   void* v_dst, llmi_stream_t stream) {
    return repeat_kv_launch(k_cache, v_cache, dtype, layer, context_length, batch, kv_heads, max_seq, heads,
                            max_k_len, head_dim, k_dst, v_dst, STREAM(stream));
}

int llmi_padding_offset(int32_t* padding_offset, int32_t* cum_seqlens, const int32_t* input_lengths, int batch,
                        int max_q_len, llmi_stream_t stream) {
    return padding_offset_launch(padding_offset, cum_seqlens, input_lengths, batch, max_q_len, STREAM(stream));
}

int llmi_rope_qkv_prefill(const void* qkv, void* q, void* k, void* v, int dtype, const int32_t* padding_offset,
                          const int32_t* history_length, int num_tokens, int batch, int seq_len, int heads,
                          int kv_heads, int head_dim, float rope_base, llmi_stream_t stream) {
    return rope_qkv_prefill_launch(qkv, q, k, v, dtype, padding_offset, history_length, num_tokens, batch, seq_len,
                                   heads, kv_heads, head_dim, rope_base, STREAM(stream));
}

int llmi_kv_append(const void* k_src, const void* v_src, int dtype, int layer, const int32_t* cur_query_length,
                   const int32_t* history_length, int batch, int kv_heads, int max_q_len, int head_dim, int max_seq,
                   void* k_cache, void* v_cache, llmi_stream_t stream) {
    return kv_append_launch(k_src, v_src, dtype, layer, cur_query_length, history_length, batch, kv_heads, max_q_len,
                            head_dim, max_seq, k_cache, v_cache, STREAM(stream));
}

int llmi_context_attention(const float* q, const void* k_cache, const void* v_cache, int cache_dtype, int layer,
                           const int32_t* history_length, const int32_t* input_length, int batch, int heads,
                           int kv_heads, int max_q_len, int max_seq, int head_dim, float scale, float* out,
                           llmi_stream_t stream) {
    return context_attention_launch(q, k_cache, v_cache, cache_dtype, layer, history_length, input_length, batch,
                                    heads, kv_heads, max_q_len, max_seq, head_dim, scale, out, STREAM(stream));
}

int llmi_context_attention_qkv(const float* qkv, const int32_t* padding_offset, const int32_t* history_length,
                               const int32_t* input_length, int num_tokens, int batch, int max_q_len, int heads,
                               int kv_heads, int head_dim, float rope_base, void* k_cache, void* v_cache,
                               int cache_dtype, int layer, int max_seq, float scale, float* q_scratch, float* out,
                               llmi_stream_t stream) {
    return context_attention_qkv_launch(qkv, padding_offset, history_length, input_length, num_tokens, batch,
                                        max_q_len, heads, kv_heads, head_dim, rope_base, k_cache, v_cache, cache_dtype,
                                        layer, max_seq, scale, q_scratch, out, STREAM(stream));
}

int llmi_context_attention_proj(const float* x, const void* w_qkv, int w_dtype, int hidden,
                                const int32_t* padding_offset, const int32_t* history_length,
                                const int32_t* input_length, int num_tokens, int batch, int max_q_len, int heads,
                                int kv_heads, int head_dim, float rope_base, void* k_cache, void* v_cache,
                                int cache_dtype, int layer, int max_seq, float scale, float* q_scratch, float* out,
                                llmi_stream_t stream) {
    LLMI_REQUIRE(x && w_qkv && num_tokens >= 1 && hidden >= 1 && heads >= 1 && kv_heads >= 1 && head_dim >= 1,
                 "context_attention_proj: bad arguments");
    const int n = (heads + 2 * kv_heads) * head_dim;
    if (w_dtype != LLMI_F16 || !linear_mfma_supported(num_tokens, n, hidden) ||
        ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(w_qkv)) & 15)) {
        set_last_error("[llmi][ERROR] context_attention_proj: needs fp16 weights, >= 16 rows, GEMM-tileable "
                       "shapes and 16-B aligned x / w (use llmi_linear + llmi_context_attention_qkv)");
        return LLMI_EUNSUPPORTED;
    }
    const float* slab = nullptr;
    int ks = 0;
    LLMI_TRY(linear_mfma_launch(x, w_qkv, nullptr, num_tokens, n, hidden, STREAM(stream), nullptr, &slab, &ks));
    return context_attention_qkv_launch(slab, padding_offset, history_length, input_length, num_tokens, batch,
                                        max_q_len, heads, kv_heads, head_dim, rope_base, k_cache, v_cache, cache_dtype,
                                        layer, max_seq, scale, q_scratch, out, STREAM(stream), ks,
                                        (size_t)num_tokens * n);
}

int llmi_causal_mask(void* mask, int dtype, const int32_t* q_lens, const int32_t* k_lens, int batch,
                     int max_q_len, int max_k_len, llmi_stream_t stream) {
    return causal_mask_launch(mask, dtype, q_lens, k_lens, batch, max_q_len, max_k_len, STREAM(stream));
}

int llmi_masked_softmax(const void* qk, const void* mask, void* score, int dtype, int batch, int heads, int q_len,
                        int k_len, float scale, llmi_stream_t stream) {
    return masked_softmax_launch(qk, mask, score, dtype, batch, heads, q_len, k_len, scale, STREAM(stream));
}

int llmi_batched_matmul(const void* a, const void* b, void* c, int dtype, int batch, int m, int n, int k, int trans_a,
                        int trans_b, llmi_stream_t stream) {
    return batched_matmul_launch(a, b, c, dtype, batch, m, n, k, trans_a, trans_b, STREAM(stream));
}

int llmi_transpose_remove_pad(const void* src, const int32_t* padding_offset, void* dst, int dtype, int num_tokens,
                              int batch, int seq_len, int heads, int head_dim, llmi_stream_t stream) {
    return transpose_remove_pad_launch(src, padding_offset, dst, dtype, num_tokens, batch, seq_len, heads, head_dim,
                                       STREAM(stream));
}

int llmi_argmax(const float* logits, int n, int32_t* out_id, llmi_stream_t stream) {
    // 256 x 8 B of scratch for the partial keys: a per-process device buffer
    static unsigned long long* scratch = nullptr;
    if (!scratch) LLMI_HIP(hipMalloc(&scratch, 256 * sizeof(unsigned long long)));
    return argmax_launch(logits, n, out_id, scratch, STREAM(stream));
}

int llmi_synth_fill(void* out, int out_dtype, int kind, uint64_t seed, uint32_t tid, int rows, int cols, int row0,
                    int col0, int ld, llmi_stream_t stream) {
    return synth_fill_launch(out, out_dtype, kind, seed, tid, rows, cols, row0, col0, ld, STREAM(stream));
}

int llmi_synth_fill_host(void* out, int out_dtype, int kind, uint64_t seed, uint32_t tid, int rows, int cols,
                         int row0, int col0, int ld) {
    return synth_fill_host(out, out_dtype, kind, seed, tid, rows, cols, row0, col0, ld);
}

int llmi_device_alloc(void** ptr, size_t bytes) {
    LLMI_REQUIRE(ptr != nullptr, "device_alloc: null out pointer");
    const hipError_t e = hipMalloc(ptr, bytes);
    if (e != hipSuccess) {
        // clear HIP's sticky last error: the caching allocator retries after releasing
        // blocks, and the next launcher's hipGetLastError must not report this failure
        (void)hipGetLastError();
        *ptr = nullptr;
        llmi::set_last_error(std::string("hipMalloc: ") + hipGetErrorString(e) + " (" + std::to_string(bytes) +
                             " bytes)");
        return LLMI_EHIP - (int)e;
    }
    return LLMI_OK;
}

int llmi_device_free(void* ptr) {
    if (ptr) LLMI_HIP(hipFree(ptr));
    return LLMI_OK;
}

int llmi_device_memset(void* ptr, int value, size_t bytes) {
    LLMI_REQUIRE(ptr != nullptr || bytes == 0, "device_memset: null pointer");
    if (bytes) LLMI_HIP(hipMemset(ptr, value, bytes));
    return LLMI_OK;
}

int llmi_device_memset_async(void* ptr, int value, size_t bytes, llmi_stream_t stream) {
    LLMI_REQUIRE(ptr != nullptr || bytes == 0, "device_memset_async: null pointer");
    if (bytes) LLMI_HIP(hipMemsetAsync(ptr, value, bytes, STREAM(stream)));
    return LLMI_OK;
}

int llmi_memcpy(void* dst, const void* src, size_t bytes, int kind) {
    LLMI_REQUIRE(kind >= 0 && kind <= 2, "memcpy: kind must be 0 (H2D), 1 (D2H) or 2 (D2D)");
    const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost
                                                                           : hipMemcpyDeviceToDevice;
    LLMI_HIP(hipMemcpy(dst, src, bytes, k));
    return LLMI_OK;
}

int llmi_device_sync(void) {
    LLMI_HIP(hipDeviceSynchronize());
    return LLMI_OK;
}

int llmi_hbm_read_bench(size_t bytes, int iters, float* us, float* gbps, size_t* bytes_read) {
    return hbm_read_bench(bytes, iters, us, gbps, bytes_read);
}

int llmi_synth_prompt(uint64_t seed, int n, int vocab, int32_t* out) {
    LLMI_REQUIRE(out && n >= 0 && vocab > 0, "synth_prompt: bad arguments");
    const uint64_t key = prng::tensor_key(seed, prng::PROMPT);
    for (int i = 0; i < n; ++i) out[i] = (int32_t)(prng::bits(key, (uint64_t)i) % (uint64_t)vocab);
    return LLMI_OK;
}

}  // extern "C"
