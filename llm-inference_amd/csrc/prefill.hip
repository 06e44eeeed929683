// Prefill (context) attention for M prompt rows at positions p0 .. p0+M-1
// (SURVEY.md §8 a15, config 3). Replaces LLaMAContextAttentionLayer's middle
// (context_attention.cpp:108-161): launchAddFusedQKVBiasTransposeAndRoPE
// (qkv_bias_and_RoPE.cu:49-144), launchConcatKVCache (concat_past_kv.cu:16-143),
// the QK^T strided-batched GEMM, launchScaleMaskAndSoftmax with
// launchBuildCausalMasks (attn_softmax_kernel.cu:79-377, build_causal_mask.cu:29),
// the PV GEMM and launchTransposeOutRemovePadding -- as two kernels:
//
//   rope_kv_prefill: rotate q (in place) and k of every row with the engine's
//     cos/sin table, write k, v into cache slots p0 + m (the decode kernel's
//     exact arithmetic, so a prefilled slot equals a decoded one);
//   attn_prefill: causal flash attention, one workgroup per (head, 32 query
//     rows), 32-key chunks of the cache staged in LDS, online softmax in fp32;
//     the causal mask is the index test key <= p0 + row (never materialised).
//
// Roofline: the attention is ~2.1 GFLOP per 7B layer at M = 512 (4 * heads *
// d * M^2 / 2), bound by LDS operand traffic in this fp32 form; the GEMMs
// around it dominate prefill (gemm.hip).
#include "kernels.h"

namespace llmi {
namespace {

constexpr int D = 128;
constexpr int kThreads = 256;
constexpr int QB = 32;   // query rows per workgroup
constexpr int KC = 32;   // keys per LDS chunk
constexpr int kLdq = D + 4;  // padded fp32 row stride (conflict-free float4 reads)

__device__ __forceinline__ void store_c(__half* p, float v) { *p = __float2half(v); }
__device__ __forceinline__ void store_c(float* p, float v) { *p = v; }
__device__ __forceinline__ float load_c(const __half* p) { return __half2float(*p); }
__device__ __forceinline__ float load_c(const float* p) { return *p; }

// grid (M), block 256: row m of qkv [M, (heads + 2 kv) * D]
template <typename KT>
__global__ void rope_kv_prefill_kernel(float* qkv, int ld, int p0, int heads, int kv_heads, const float* rope_tab,
                                       KT* k_cache, KT* v_cache, int max_seq) {
    const int m = blockIdx.x, pos = p0 + m;
    float* row = qkv + (size_t)m * ld;
    const float2* cs = reinterpret_cast<const float2*>(rope_tab) + (size_t)pos * (D / 2);
    // q heads then k heads: pairs (i, i + D/2), same expression as attn_decode_kernel
    for (int e = threadIdx.x; e < (heads + kv_heads) * (D / 2); e += blockDim.x) {
        const int hh = e / (D / 2), i = e % (D / 2);
        const float c = cs[i].x, s = cs[i].y;
        float* p = row + (size_t)hh * D;
        const float x0 = p[i], x1 = p[i + D / 2];
        const float r0 = x0 * c - x1 * s, r1 = x1 * c + x0 * s;
        if (hh < heads) {
            p[i] = r0;
            p[i + D / 2] = r1;
        } else {
            KT* kc = k_cache + ((size_t)(hh - heads) * max_seq + pos) * D;
            store_c(kc + i, r0);
            store_c(kc + i + D / 2, r1);
        }
    }
    const float* v = row + (size_t)(heads + kv_heads) * D;
    for (int e = threadIdx.x; e < kv_heads * D; e += blockDim.x) {
        const int hh = e / D, d = e % D;
        store_c(v_cache + ((size_t)hh * max_seq + pos) * D + d, v[e]);
    }
}

// grid (ceil(M / QB), heads), block 256. Thread t: query row qi = t >> 3 of the
// block; for scores keys kg + 8 c (kg = t & 7, c < 4) of the chunk; for the
// output dims 4 kg + 32 r + {0..3} (r < 4).
template <typename KT>
__global__ __launch_bounds__(kThreads) void attn_prefill_kernel(const float* qkv, int ld, int m_rows, int p0,
                                                                int heads, int kv_heads, const KT* k_cache,
                                                                const KT* v_cache, int max_seq, float* out,
                                                                int ldo) {
    __shared__ float q_s[QB * kLdq];
    __shared__ float k_s[KC * kLdq];
    __shared__ float v_s[KC * D];
    __shared__ float p_s[QB * (KC + 1)];

    const int t = threadIdx.x;
    const int qb = gridDim.x - 1 - blockIdx.x;  // longest (latest) query blocks first
    const int h = blockIdx.y;
    const int kvh = h / (heads / kv_heads);
    const int qi = t >> 3, kg = t & 7;
    const int q_first = qb * QB;
    const int q_row = min(q_first + qi, m_rows - 1);  // clamp: rows past M compute, never store
    const float qscale = 1.0f / sqrtf((float)D);

    // stage q (already rotated), scaled as in the decode kernel
    for (int e = t; e < QB * D; e += kThreads) {
        const int r = e / D, d = e % D;
        const int qr = min(q_first + r, m_rows - 1);
        q_s[r * kLdq + d] = qkv[(size_t)qr * ld + (size_t)h * D + d] * qscale;
    }

    const KT* kc = k_cache + (size_t)kvh * max_seq * D;
    const KT* vc = v_cache + (size_t)kvh * max_seq * D;
    const int my_pos = p0 + q_row;
    const int kend = p0 + min(q_first + QB, m_rows);  // keys [0, kend)

    float m_run = -INFINITY, l_run = 0.f;
    float o[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) o[i] = 0.f;

    for (int k0 = 0; k0 < kend; k0 += KC) {
        __syncthreads();
        for (int e = t; e < KC * D; e += kThreads) {
            const int r = e / D, d = e % D;
            const int j = min(k0 + r, kend - 1);
            k_s[r * kLdq + d] = load_c(kc + (size_t)j * D + d);
            v_s[r * D + d] = load_c(vc + (size_t)j * D + d);
        }
        __syncthreads();

        float s[4] = {0.f, 0.f, 0.f, 0.f};
        const float* qp = q_s + qi * kLdq;
#pragma unroll 4
        for (int d = 0; d < D; d += 4) {
            const float4 qv = *reinterpret_cast<const float4*>(qp + d);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float4 kv = *reinterpret_cast<const float4*>(k_s + (kg + 8 * c) * kLdq + d);
                s[c] = fmaf(qv.x, kv.x, s[c]);
                s[c] = fmaf(qv.y, kv.y, s[c]);
                s[c] = fmaf(qv.z, kv.z, s[c]);
                s[c] = fmaf(qv.w, kv.w, s[c]);
            }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int j = k0 + kg + 8 * c;
            if (j > my_pos || j >= kend) s[c] = -INFINITY;  // causal (build_causal_mask.cu:29)
            mx = fmaxf(mx, s[c]);
        }
        mx = fmaxf(mx, __shfl_xor(mx, 1));
        mx = fmaxf(mx, __shfl_xor(mx, 2));
        mx = fmaxf(mx, __shfl_xor(mx, 4));
        const float m_new = fmaxf(m_run, mx);  // finite: key 0 is always visible
        const float alpha = expf(m_run - m_new);
        float ps = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const float p = expf(s[c] - m_new);
            ps += p;
            p_s[qi * (KC + 1) + kg + 8 * c] = p;
        }
        ps += __shfl_xor(ps, 1);
        ps += __shfl_xor(ps, 2);
        ps += __shfl_xor(ps, 4);
        l_run = l_run * alpha + ps;
        m_run = m_new;
        __builtin_amdgcn_wave_barrier();  // p_s row is written and read by the same 8 lanes

#pragma unroll
        for (int i = 0; i < 16; ++i) o[i] *= alpha;
        const float* pr = p_s + qi * (KC + 1);
#pragma unroll 4
        for (int j = 0; j < KC; ++j) {
            const float p = pr[j];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float4 vv = *reinterpret_cast<const float4*>(v_s + j * D + 4 * kg + 32 * r);
                o[4 * r + 0] = fmaf(p, vv.x, o[4 * r + 0]);
                o[4 * r + 1] = fmaf(p, vv.y, o[4 * r + 1]);
                o[4 * r + 2] = fmaf(p, vv.z, o[4 * r + 2]);
                o[4 * r + 3] = fmaf(p, vv.w, o[4 * r + 3]);
            }
        }
    }

    if (q_first + qi < m_rows) {
        const float inv = 1.0f / l_run;
        float* orow = out + (size_t)(q_first + qi) * ldo + (size_t)h * D;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float4 v;
            v.x = o[4 * r + 0] * inv;
            v.y = o[4 * r + 1] * inv;
            v.z = o[4 * r + 2] * inv;
            v.w = o[4 * r + 3] * inv;
            *reinterpret_cast<float4*>(orow + 4 * kg + 32 * r) = v;
        }
    }
}

__global__ void prefill_finish_kernel(DecodeState* st, const int32_t* prompt, int32_t* tokens, int p0, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) tokens[p0 + i] = prompt[p0 + i];
    if (threadIdx.x == 0) {
        st->next_pos = p0 + n;
        st->cur_pos = p0 + n - 1;
    }
}

}  // namespace

int prefill_finish_launch(DecodeState* st, const int32_t* prompt, int32_t* tokens, int p0, int n, hipStream_t s) {
    LLMI_REQUIRE(st && prompt && tokens && n > 0 && p0 >= 0, "prefill_finish: bad arguments");
    hipLaunchKernelGGL(prefill_finish_kernel, dim3(1), dim3(256), 0, s, st, prompt, tokens, p0, n);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

int prefill_attn_launch(const PrefillAttnArgs& a, hipStream_t s) {
    LLMI_REQUIRE(a.qkv && a.k_cache && a.v_cache && a.out && a.rope_tab, "prefill attention: null argument");
    LLMI_REQUIRE(a.head_dim == D, "prefill attention: head_dim must be 128");
    LLMI_REQUIRE(a.m > 0 && a.p0 >= 0 && a.p0 + a.m <= a.max_seq, "prefill attention: rows past max_seq");
    LLMI_REQUIRE(a.heads > 0 && a.kv_heads > 0 && a.heads % a.kv_heads == 0, "prefill attention: bad head counts");
    const int ld = (a.heads + 2 * a.kv_heads) * D;
    const dim3 ga((a.m + QB - 1) / QB, a.heads);
    if (a.cache_dtype == LLMI_F16) {
        hipLaunchKernelGGL(rope_kv_prefill_kernel<__half>, dim3(a.m), dim3(kThreads), 0, s, a.qkv, ld, a.p0, a.heads,
                           a.kv_heads, a.rope_tab, (__half*)a.k_cache, (__half*)a.v_cache, a.max_seq);
        hipLaunchKernelGGL(attn_prefill_kernel<__half>, ga, dim3(kThreads), 0, s, a.qkv, ld, a.m, a.p0, a.heads,
                           a.kv_heads, (const __half*)a.k_cache, (const __half*)a.v_cache, a.max_seq, a.out,
                           a.heads * D);
    } else if (a.cache_dtype == LLMI_F32) {
        hipLaunchKernelGGL(rope_kv_prefill_kernel<float>, dim3(a.m), dim3(kThreads), 0, s, a.qkv, ld, a.p0, a.heads,
                           a.kv_heads, a.rope_tab, (float*)a.k_cache, (float*)a.v_cache, a.max_seq);
        hipLaunchKernelGGL(attn_prefill_kernel<float>, ga, dim3(kThreads), 0, s, a.qkv, ld, a.m, a.p0, a.heads,
                           a.kv_heads, (const float*)a.k_cache, (const float*)a.v_cache, a.max_seq, a.out,
                           a.heads * D);
    } else {
        LLMI_REQUIRE(false, "prefill attention: cache dtype must be f16 or f32");
    }
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

}  // namespace llmi
