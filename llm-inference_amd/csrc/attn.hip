// Fused decode attention for one token: RoPE(q, k) + KV-cache write + split-KV
// softmax(q K^T / sqrt(d)) V with a log-sum-exp merge by the last-arriving
// workgroup of each head.
//
// Replaces launchRoPE + launchDecoderMaskedMHA (src/kernels/qkv_bias_and_RoPE.cu:322-451,
// src/kernels/fused_decoder_self_attention.cu:97-385; layer call sites
// src/layers/attention/masked_self_attention.cpp:76-80). Semantics follow
// modeling_llama.py:351-437 (HF eager attention, fp32 softmax, no +1e-6 in the
// denominator); none of the reference kernel's defects (SURVEY App. A #1-#6:
// kv-head 0 for every head, missing kv_head in the layer offset, softmax capped at
// 128 positions, empty fp16 path) are carried over.
//
// Roofline: HBM. Algorithmic bytes per launch = 2 * ctx * kv_heads * d * sizeof(cache)
// (K and V read) + 2 * kv_heads * d * sizeof(cache) (current slot write).
//
// Work split (MI355X): grid (heads, max_seq / 64). A workgroup (256 threads = 16
// groups of 16 lanes) owns 64 cached positions of one head; a 16-lane group reads a
// 256-byte fp16 K/V row with one 16-B load per lane (4 rows per wave instruction).
// 32 heads alone would use 32 of 256 CUs; at ctx 2048 the split gives 1024
// workgroups. Partial (m, l, o) go to a workspace; an agent-scope release +
// relaxed ticket per head selects the last arriver, which acquires and merges
// (cdna_hip_programming.md §6 Guideline 16, split-K recipe). The counters are left
// at zero for the next launch.
#include "kernels.h"

namespace llmi {
namespace {

constexpr int kThreads = 256;
constexpr int D = 128;         // head_dim
constexpr int CH = kAttnChunk;  // positions per workgroup
constexpr int LPR = 16;        // lanes per cached row (8 dims per lane)

__device__ __forceinline__ void load8(const __half* p, float* v) {
    uint4 u = *reinterpret_cast<const uint4*>(p);
    const __half2* h = reinterpret_cast<const __half2*>(&u);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float2 f = __half22float2(h[i]);
        v[2 * i] = f.x;
        v[2 * i + 1] = f.y;
    }
}
__device__ __forceinline__ void load8(const float* p, float* v) {
    float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void store_cache(__half* p, float v) { *p = __float2half(v); }
__device__ __forceinline__ void store_cache(float* p, float v) { *p = v; }
// value as the cache holds it (the current position must read exactly what later
// steps will read back from an fp16 cache)
template <typename KT> __device__ __forceinline__ float cache_round(float v);
template <> __device__ __forceinline__ float cache_round<__half>(float v) { return __half2float(__float2half(v)); }
template <> __device__ __forceinline__ float cache_round<float>(float v) { return v; }

// HF rotary angle (modeling_llama.py:130-141): inv_freq = 1 / fp32(base^(2i/d)) with
// the power correctly rounded (== torch's fp32 pow), angle = fp32(pos * inv_freq),
// cos/sin correctly rounded from double.
__device__ __forceinline__ void rope_cs(int pos, int i, int d, float base, float* c, float* s) {
    const float p = (float)pow((double)base, (double)(2 * i) / (double)d);
    const float inv = __fdiv_rn(1.0f, p);
    const float ang = __fmul_rn((float)pos, inv);
    double sd, cd;
    sincos((double)ang, &sd, &cd);
    *c = (float)cd;
    *s = (float)sd;
}

struct Ws {
    unsigned* counters;  // [heads]
    float* ml;           // [heads][nsplit][2]
    float* o;            // [heads][nsplit][D]
};
__host__ __device__ inline size_t ws_bytes(int heads, int max_seq) {
    const int ns = (max_seq + CH - 1) / CH;
    size_t c = ((size_t)heads * 4 + 255) / 256 * 256;
    return c + (size_t)heads * ns * 2 * 4 + (size_t)heads * ns * D * 4;
}
__device__ inline Ws ws_carve(void* base, int heads, int ns) {
    Ws w;
    char* p = reinterpret_cast<char*>(base);
    w.counters = reinterpret_cast<unsigned*>(p);
    p += ((size_t)heads * 4 + 255) / 256 * 256;
    w.ml = reinterpret_cast<float*>(p);
    p += (size_t)heads * ns * 2 * 4;
    w.o = reinterpret_cast<float*>(p);
    return w;
}

template <typename KT>
__global__ __launch_bounds__(kThreads) void attn_decode_kernel(AttnArgs a) {
    __shared__ __attribute__((aligned(16))) float q_s[D];
    __shared__ __attribute__((aligned(16))) float kcur_s[D];
    __shared__ __attribute__((aligned(16))) float vcur_s[D];
    __shared__ float p_s[CH];
    __shared__ __attribute__((aligned(16))) float o_red[kThreads / LPR][D];  // [groups][D]
    __shared__ float ml_s[2];
    __shared__ int last_s;

    const int pos = a.pos_dev ? *a.pos_dev : a.pos_host;
    if (pos < 0 || pos >= a.max_seq) return;  // host validates; guard against a stale state
    const int ctx = pos + 1;
    const int h = blockIdx.x, split = blockIdx.y;
    const int start = split * CH;
    if (start >= ctx) return;
    const int end = min(start + CH, ctx);
    const int nact = (ctx + CH - 1) / CH;
    const int ns = gridDim.y;
    const int group = a.heads / a.kv_heads;
    const int kvh = h / group;
    const int tid = threadIdx.x;
    const bool owns_pos = (end == ctx);

    // ---- q (and the current k, v when this block owns position `pos`)
    const float* qrow = a.qkv + (size_t)h * D;
    const float* krow = a.qkv + (size_t)(a.heads + kvh) * D;
    const float* vrow = a.qkv + (size_t)(a.heads + a.kv_heads + kvh) * D;
    const float qscale = 1.0f / sqrtf((float)D);
    if (tid < D / 2) {
        const int i = tid;
        float c = 1.f, s = 0.f;
        if (a.rope) rope_cs(pos, i, D, a.rope_base, &c, &s);
        // rotate_half pairing (i, i + d/2): modeling_llama.py:204-235
        const float q0 = qrow[i], q1 = qrow[i + D / 2];
        q_s[i] = (q0 * c - q1 * s) * qscale;
        q_s[i + D / 2] = (q1 * c + q0 * s) * qscale;
        if (owns_pos) {
            const float k0 = krow[i], k1 = krow[i + D / 2];
            kcur_s[i] = cache_round<KT>(k0 * c - k1 * s);
            kcur_s[i + D / 2] = cache_round<KT>(k1 * c + k0 * s);
        }
    } else if (owns_pos && tid >= D && tid < 2 * D) {
        vcur_s[tid - D] = cache_round<KT>(vrow[tid - D]);
    }
    __syncthreads();

    KT* kc = reinterpret_cast<KT*>(a.k_cache) + (size_t)kvh * a.max_seq * D;
    KT* vc = reinterpret_cast<KT*>(a.v_cache) + (size_t)kvh * a.max_seq * D;
    if (owns_pos && (h % group) == 0 && tid < D) {
        // KV-cache write at slot pos (concat: fused_decoder_self_attention.cu:187-193,292-295)
        store_cache(kc + (size_t)pos * D + tid, kcur_s[tid]);
        store_cache(vc + (size_t)pos * D + tid, vcur_s[tid]);
    }
    // The current position is always taken from LDS, never re-read from the cache,
    // so no other workgroup depends on the store above within this launch.

    const int grp = tid / LPR, l16 = tid % LPR;  // 16 groups x 16 lanes
    float qv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) qv[i] = q_s[l16 * 8 + i];

    // ---- scores
    for (int j = start + grp; j < end; j += kThreads / LPR) {
        float kv[8];
        if (j == pos) {
#pragma unroll
            for (int i = 0; i < 8; ++i) kv[i] = kcur_s[l16 * 8 + i];
        } else {
            load8(kc + (size_t)j * D + l16 * 8, kv);
        }
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) d = fmaf(qv[i], kv[i], d);
#pragma unroll
        for (int off = LPR / 2; off > 0; off >>= 1) d += __shfl_xor(d, off, kWave);
        if (l16 == 0) p_s[j - start] = d;
    }
    __syncthreads();

    // ---- local softmax over this block's positions (wave 0)
    if (tid < kWave) {
        const int n = end - start;
        float s = tid < n ? p_s[tid] : -INFINITY;
        const float m = wave_max(s);
        const float p = tid < n ? expf(s - m) : 0.f;
        const float l = wave_sum(p);
        if (tid < n) p_s[tid] = p;
        if (tid == 0) { ml_s[0] = m; ml_s[1] = l; }
    }
    __syncthreads();

    // ---- o = sum_j p_j v_j
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    for (int j = start + grp; j < end; j += kThreads / LPR) {
        float vv[8];
        if (j == pos) {
#pragma unroll
            for (int i = 0; i < 8; ++i) vv[i] = vcur_s[l16 * 8 + i];
        } else {
            load8(vc + (size_t)j * D + l16 * 8, vv);
        }
        const float p = p_s[j - start];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = fmaf(p, vv[i], acc[i]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) o_red[grp][l16 * 8 + i] = acc[i];
    __syncthreads();

    float o = 0.f;
    if (tid < D) {
#pragma unroll
        for (int g = 0; g < kThreads / LPR; ++g) o += o_red[g][tid];
    }
    if (nact == 1) {
        if (tid < D) a.out[(size_t)h * D + tid] = o / ml_s[1];
        return;
    }

    // ---- publish partial, last arriver merges
    Ws ws = ws_carve(a.workspace, a.heads, ns);
    if (tid < D) ws.o[((size_t)h * ns + split) * D + tid] = o;
    if (tid == 0) {
        ws.ml[((size_t)h * ns + split) * 2 + 0] = ml_s[0];
        ws.ml[((size_t)h * ns + split) * 2 + 1] = ml_s[1];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev = __hip_atomic_fetch_add(ws.counters + h, 1u, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
        last_s = (prev == (unsigned)(nact - 1));
        if (last_s) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!last_s) return;
    if (tid < D) {
        float M = -INFINITY;
        for (int s = 0; s < nact; ++s) M = fmaxf(M, ws.ml[((size_t)h * ns + s) * 2]);
        float L = 0.f, O = 0.f;
        for (int s = 0; s < nact; ++s) {
            const float w = expf(ws.ml[((size_t)h * ns + s) * 2] - M);
            L = fmaf(ws.ml[((size_t)h * ns + s) * 2 + 1], w, L);
            O = fmaf(ws.o[((size_t)h * ns + s) * D + tid], w, O);
        }
        a.out[(size_t)h * D + tid] = O / L;
    }
    if (tid == 0) __hip_atomic_store(ws.counters + h, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

size_t attn_workspace_bytes(int heads, int head_dim, int max_seq) {
    (void)head_dim;
    return ws_bytes(heads, max_seq);
}

int attn_decode_launch(const AttnArgs& a, hipStream_t s) {
    LLMI_REQUIRE(a.head_dim == D, "attn: head_dim must be 128");
    LLMI_REQUIRE(a.heads > 0 && a.kv_heads > 0 && a.heads % a.kv_heads == 0, "attn: bad head counts");
    LLMI_REQUIRE(a.max_seq > 0, "attn: max_seq must be > 0");
    LLMI_REQUIRE(a.pos_dev || (a.pos_host >= 0 && a.pos_host < a.max_seq), "attn: pos out of range");
    LLMI_REQUIRE(a.qkv && a.k_cache && a.v_cache && a.out && a.workspace, "attn: null pointer");
    const dim3 grid(a.heads, (a.max_seq + CH - 1) / CH);
    if (a.cache_dtype == LLMI_F16)
        hipLaunchKernelGGL(attn_decode_kernel<__half>, grid, dim3(kThreads), 0, s, a);
    else if (a.cache_dtype == LLMI_F32)
        hipLaunchKernelGGL(attn_decode_kernel<float>, grid, dim3(kThreads), 0, s, a);
    else
        LLMI_REQUIRE(false, "attn: cache dtype must be f16 or f32");
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

}  // namespace llmi
