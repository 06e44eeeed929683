// Decode attention for one token: RoPE(q, k) + KV-cache write + split-KV
// softmax(q K^T / sqrt(d)) V, and the two consumers of its split partials:
//   * attn_merge_kernel: log-sum-exp merge -> out[heads * d] (operator API);
//   * attn_oproj_kernel: merge fused into a split-by-head O projection whose
//     per-head partial products are summed into the residual stream with
//     int64 fixed-point atomics (engine path; exact, order-independent sums).
//
// Replaces launchRoPE + launchDecoderMaskedMHA (+ the o_proj launchLinearGemm)
// (src/kernels/qkv_bias_and_RoPE.cu:322-451, src/kernels/fused_decoder_self_attention.cu:97-385,
// src/layers/attention/masked_self_attention.cpp:76-84). Semantics follow
// modeling_llama.py:351-448 (HF eager attention, fp32 softmax, no +1e-6 in the
// denominator); none of the reference kernel's defects (SURVEY App. A #1-#6:
// kv-head 0 for every head, missing kv_head in the layer offset, softmax capped at
// 128 positions, empty fp16 path) are carried over.
//
// Roofline: HBM. Algorithmic bytes = 2 * ctx * kv_heads * d * sizeof(cache) (K and V
// read) + 2 * kv_heads * d * sizeof(cache) (current slot write); attn_oproj adds
// hidden * heads * d * sizeof(W) (the o_proj weights).
//
// Work split (MI355X): grid (heads, max_seq / 64). A workgroup (256 threads = 16
// groups of 16 lanes) owns 64 cached positions of one head; a 16-lane group reads a
// 256-byte fp16 K/V row with one 16-B load per lane (4 rows per wave instruction),
// all its rows issued before anything waits. 32 heads alone would use 32 of 256 CUs;
// at ctx 2048 the split gives 1024 workgroups. Each writes (m, l, o) partials; the
// next kernel merges them (a kernel boundary orders the hand-off -- an in-kernel
// last-arriver merge measured no faster: its store-drain + ticket + load chain costs
// as much as the boundary, profiles/).
#include <cstdlib>

#include "attn_impl.h"

namespace llmi {
namespace {

using namespace attn_detail;

template <typename KT>
__global__ __launch_bounds__(kThreads) void attn_decode_kernel(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    WgStamp ts(a.stamps);
    attn_body<KT, PlainIO>(a, blockIdx.x, blockIdx.y, gridDim.y, smem, NoSync{});
}

// attention + merge by the last-arriving split workgroup of each head (the
// split-K "last block reduces" form, cdna_hip_programming.md §5 Projection GEMM
// item 2, sc1 variant): partials are stored write-through and drained, one
// agent-scope ticket per workgroup, the workgroup that draws nact - 1 reads every
// partial of its head with sc1 loads, merges (same arithmetic as the o_proj merge)
// and writes merge_out; it re-zeroes the head's ticket for the next launch.
struct PartialSc1IO : PlainIO {
    __device__ __forceinline__ static void st(float* p, float v) { Sc1IO::st(p, v); }
};
template <typename KT>
__global__ __launch_bounds__(kThreads) void attn_decode_merge_kernel(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    WgStamp ts(a.stamps);
    const int h = blockIdx.x, split = blockIdx.y, ns = gridDim.y, tid = threadIdx.x;
    const int pos = a.pos_dev ? *a.pos_dev : a.pos_host;
    if (pos < 0 || pos >= a.max_seq) return;
    const int nact = (pos + 1 + CH - 1) / CH;
    if (split >= nact) return;
    attn_body<KT, PartialSc1IO>(a, h, split, ns, smem, NoSync{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 partials
    __syncthreads();
    int* last = reinterpret_cast<int*>(smem + kAttnLds / 4);
    Ws ws = ws_carve(a.workspace, a.heads, ns);
    unsigned* ticket = ws.counters + (size_t)h * kCntWordsPerHead + 2;
    if (tid == 0)
        *last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)nact - 1;
    __syncthreads();
    if (!*last) return;
    if (tid == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float* m_s = smem;
    float* l_s = smem + ns;
    float* o2 = smem + 2 * ns;  // [2][D]
    float* linv = o2 + 2 * D;
    const float* mlh = ws.ml + (size_t)h * ns * 2;
    const int d = tid % D, half = tid / D;
    const float* oh = ws.o + (size_t)h * ns * D + d;
    // every partial load in one round (o-partials, then m / l), as in the o_proj merge
    float ov[kMergeChunk];
#pragma unroll
    for (int i = 0; i < kMergeChunk; ++i) {
        const int sp = half + 2 * i;
        ov[i] = Sc1IO::ld(oh + (size_t)(sp < nact ? sp : 0) * D);
    }
    constexpr int kMlPer = kMaxSplits / kThreads;
    float mr[kMlPer], lr[kMlPer];
#pragma unroll
    for (int i = 0; i < kMlPer; ++i) {
        if (i * kThreads < nact) {
            const int sp = min(tid + i * kThreads, nact - 1);
            mr[i] = Sc1IO::ld(mlh + 2 * sp);
            lr[i] = Sc1IO::ld(mlh + 2 * sp + 1);
        }
    }
#pragma unroll
    for (int i = 0; i < kMlPer; ++i) {
        const int sp = tid + i * kThreads;
        if (i * kThreads < nact && sp < nact) {
            m_s[sp] = mr[i];
            l_s[sp] = lr[i];
        }
    }
    __syncthreads();
    if (tid < kWave) {
        float M = -INFINITY;
        for (int sp = tid; sp < nact; sp += kWave) M = fmaxf(M, m_s[sp]);
        M = wave_max(M);
        float lsum = 0.f;
        for (int sp = tid; sp < nact; sp += kWave) {
            const float wgt = expf(m_s[sp] - M);
            m_s[sp] = wgt;
            lsum = fmaf(l_s[sp], wgt, lsum);
        }
        lsum = wave_sum(lsum);
        if (tid == 0) *linv = 1.0f / lsum;
    }
    __syncthreads();
    float O = 0.f;
#pragma unroll
    for (int i = 0; i < kMergeChunk; ++i) {
        const int sp = half + 2 * i;
        O = fmaf(sp < nact ? ov[i] : 0.f, sp < nact ? m_s[sp] : 0.f, O);
    }
    for (int sp = half + 2 * kMergeChunk; sp < nact; sp += 2) O = fmaf(Sc1IO::ld(oh + (size_t)sp * D), m_s[sp], O);
    o2[half * D + d] = O;
    __syncthreads();
    if (tid < D) a.merge_out[(size_t)h * D + tid] = (o2[tid] + o2[D + tid]) * *linv;
}

// Log-sum-exp merge of the split-KV partials of each head (one workgroup per
// head, 2 threads per head dim). Every load it needs -- the position, (m, l) of
// every split and up to 2 * kMergeChunk o-partials per dim -- is issued in one
// round; splits past nact hold stale data and are excluded by selects, never by
// multiplying with a zero weight (stale NaN * 0 = NaN).
__global__ __launch_bounds__(kThreads) void attn_merge_kernel(AttnArgs a, int ns) {
    __shared__ float m_s[kMaxSplits];
    __shared__ float l_s[kMaxSplits];
    __shared__ float red_s[16];
    __shared__ float o_red[2][D];
    const int pos = a.pos_dev ? *a.pos_dev : a.pos_host;
    const int h = blockIdx.x, tid = threadIdx.x;
    const int d = tid % D, half = tid / D;
    Ws ws = ws_carve(a.workspace, a.heads, ns);
    const float* mlh = ws.ml + (size_t)h * ns * 2;
    const float* oh = ws.o + (size_t)h * ns * D + d;
    float ov[kMergeChunk];
#pragma unroll
    for (int i = 0; i < kMergeChunk; ++i) {
        const int sp = half + 2 * i;
        ov[i] = oh[(size_t)(sp < ns ? sp : 0) * D];
    }
    for (int sp = tid; sp < ns; sp += kThreads) {
        m_s[sp] = mlh[2 * sp];
        l_s[sp] = mlh[2 * sp + 1];
    }
    if (pos < 0 || pos >= a.max_seq) return;
    const int nact = (pos + 1 + CH - 1) / CH;
    if (nact == 1) return;  // the attention kernel wrote the output itself (direct_out)
    __syncthreads();
    float M = -INFINITY;
    for (int sp = 0; sp < nact; ++sp) M = fmaxf(M, m_s[sp]);
    float lw = 0.f;
    for (int sp = tid; sp < nact; sp += kThreads) lw = fmaf(l_s[sp], expf(m_s[sp] - M), lw);
    const float L = block_sum(lw, red_s);
    float O = 0.f;
#pragma unroll
    for (int i = 0; i < kMergeChunk; ++i) {
        const int sp = half + 2 * i;
        const float w = sp < nact ? expf(m_s[sp] - M) : 0.f;
        O = fmaf(sp < nact ? ov[i] : 0.f, w, O);
    }
    for (int sp = half + 2 * kMergeChunk; sp < nact; sp += 2) O = fmaf(oh[(size_t)sp * D], expf(m_s[sp] - M), O);
    o_red[half][d] = O;
    __syncthreads();
    if (tid < D) a.out[(size_t)h * D + tid] = (o_red[0][tid] + o_red[1][tid]) / L;
}

// Workgroup (h, row chunk of 16 * NPL rows): see oproj_body.
template <typename WT, int NPL>
__global__ __launch_bounds__(kThreads) void attn_oproj_kernel(OprojArgs a, int ns) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    WgStamp ts(a.stamps);
    oproj_body<WT, NPL, PlainIO>(a, blockIdx.x, blockIdx.y, ns, smem, NoSync{});
}

// ---- attention + merge/o_proj co-scheduled in one launch (the engine's default).
// Workgroup (h, j) of grid (heads, max(ns, nchunk)):
//   1. issues its W_o slice (row chunk j of head h) -- it depends on nothing;
//   2. if j < nact: split j of head h's attention (K/V loads, scores, softmax, o),
//      partials stored write-through (sc1), drained, then one arrival on head h's
//      counter (cdna_hip_programming.md Guideline 16, valid form 1);
//   3. if j < nchunk: waits for head h's nact arrivals (one lane polls, bounded),
//      reads the partials with sc1 loads, merges, and adds its rows' dot products
//      into the int64 residual accumulator; the last departing workgroup of head h
//      re-zeroes the head's two counters for the next launch.
// A workgroup waits only after its own attention work, and only on workgroups of
// its own head; the host admits the fused form only when the whole grid is
// co-resident (occupancy query), so the wait can never block a producer.
// Replaces the attention -> o_proj kernel boundary: the W_o stream overlaps the
// latency-bound attention instead of starting after it.
#ifndef LLMI_POLL_SLEEP
#define LLMI_POLL_SLEEP 2
#endif
#ifndef LLMI_FUSED_NOWAIT
#define LLMI_FUSED_NOWAIT 0  // diagnostic only (wrong results): skip the per-head wait
#endif
struct StoreSc1IO : PlainIO {  // attention partials: write-through stores
    __device__ __forceinline__ static void st(float* p, float v) { Sc1IO::st(p, v); }
    __device__ __forceinline__ static void st_ll(long long* p, long long v) { Sc1IO::st_ll(p, v); }
};
struct LoadSc1IO : PlainIO {  // merge: sc1 loads of the handed-off partials
    __device__ __forceinline__ static float ld(const float* p) { return Sc1IO::ld(p); }
};
struct HeadSync {
    static constexpr bool kFlow = true;
    const unsigned* cnt;
    unsigned target;
    int* err;
    __device__ __forceinline__ void wait() const {
        if (!LLMI_FUSED_NOWAIT && threadIdx.x == 0) {
            // the clock (a scalar-memory round trip) only once the counter was seen short
            unsigned long long t0 = 0;
            for (unsigned n = 0;; ++n) {
                if (__hip_atomic_load(const_cast<unsigned*>(cnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target)
                    break;
                if (n == 0) t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
                if ((n & 63) == 63 && __builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {  // 200 ms: give up
                    if (err) atomicOr(err, 4);
                    break;
                }
                __builtin_amdgcn_s_sleep(LLMI_POLL_SLEEP);
            }
        }
        __syncthreads();
    }
};

#ifndef LLMI_OPROJ_EARLY
#define LLMI_OPROJ_EARLY 1  // issue the W_o slice before the attention work
#endif

template <typename WT, typename KT, int NPL>
__global__ __launch_bounds__(kThreads) void attn_oproj_fused_kernel(AttnArgs aa, OprojArgs oa, int ns, int nchunk,
                                                                    int* err) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    WgStamp ts(oa.stamps);
    const int h = blockIdx.x, j = blockIdx.y;
    const int pos = aa.pos_dev ? *aa.pos_dev : aa.pos_host;
    if (pos < 0 || pos >= aa.max_seq) return;  // host validates; uniform over the grid
    const int nact = (pos + 1 + CH - 1) / CH;
    Ws ws = ws_carve(aa.workspace, aa.heads, ns);
    unsigned* arrive = ws.counters + (size_t)h * kCntWordsPerHead;
    unsigned* leave = arrive + 1;
    W8<WT> wr[NPL];
    const bool has_o = j < nchunk;
    if (LLMI_OPROJ_EARLY && has_o) oproj_load_w<WT, NPL>(oa, h, j, wr);
    if (j < nact) {
        attn_body<KT, StoreSc1IO>(aa, h, j, ns, smem, NoSync{});
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ts.mark(1);
    }
    if (!has_o) return;
    if (!LLMI_OPROJ_EARLY) oproj_load_w<WT, NPL>(oa, h, j, wr);
    oproj_body<WT, NPL, LoadSc1IO, HeadSync, true>(oa, h, j, ns, smem, HeadSync{arrive, (unsigned)nact, err}, &wr);
    ts.mark(2);
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add(leave, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == (unsigned)nchunk - 1) {  // every waiter of head h has passed: reset for the next launch
            __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(leave, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

int oproj_npl(const OprojArgs& a) {
    static const int forced = [] {  // tuning override: LLMI_OPROJ_NPL = 1, 2, 4 or 8
        const char* e = std::getenv("LLMI_OPROJ_NPL");
        const int v = e ? std::atoi(e) : 0;
        return (v == 1 || v == 2 || v == 4 || v == 8) ? v : 0;
    }();
    if (forced) return forced;
    const long target = (long)a.heads * a.n_rows / (1024 * 16);  // ~1024 workgroups
    return target >= 8 ? 8 : target >= 4 ? 4 : target >= 2 ? 2 : 1;
}

template <typename WT, typename KT, int NPL>
const void* fused_fn() {
    return reinterpret_cast<const void*>(&attn_oproj_fused_kernel<WT, KT, NPL>);
}
template <typename WT, typename KT>
const void* fused_fn_npl(int npl) {
    return npl == 8 ? fused_fn<WT, KT, 8>() : npl == 4 ? fused_fn<WT, KT, 4>() : npl == 2 ? fused_fn<WT, KT, 2>()
                                                                                    : fused_fn<WT, KT, 1>();
}
const void* fused_fn_any(int wdt, int kdt, int npl) {
    const bool k16 = kdt == LLMI_F16;
    switch (wdt) {
        case LLMI_F16: return k16 ? fused_fn_npl<__half, __half>(npl) : fused_fn_npl<__half, float>(npl);
        case LLMI_F32: return k16 ? fused_fn_npl<float, __half>(npl) : fused_fn_npl<float, float>(npl);
        case LLMI_I8: return k16 ? fused_fn_npl<int8_t, __half>(npl) : fused_fn_npl<int8_t, float>(npl);
    }
    return nullptr;
}
size_t fused_lds(int npl) {
    const size_t o = npl == 8 ? oproj_lds<8>() : npl == 4 ? oproj_lds<4>() : npl == 2 ? oproj_lds<2>() : oproj_lds<1>();
    return o > kAttnLds ? o : kAttnLds;
}

template <typename WT>
int oproj_launch_w(const OprojArgs& a, hipStream_t s) {
    // ~1024 workgroups: rows per workgroup = 16 * NPL
    const int ns = (a.max_seq + CH - 1) / CH;
    const int npl = oproj_npl(a);
    const dim3 grid(a.heads, (a.n_rows + 16 * npl - 1) / (16 * npl));
    switch (npl) {
        case 8: hipLaunchKernelGGL((attn_oproj_kernel<WT, 8>), grid, dim3(kThreads), oproj_lds<8>(), s, a, ns); break;
        case 4: hipLaunchKernelGGL((attn_oproj_kernel<WT, 4>), grid, dim3(kThreads), oproj_lds<4>(), s, a, ns); break;
        case 2: hipLaunchKernelGGL((attn_oproj_kernel<WT, 2>), grid, dim3(kThreads), oproj_lds<2>(), s, a, ns); break;
        default: hipLaunchKernelGGL((attn_oproj_kernel<WT, 1>), grid, dim3(kThreads), oproj_lds<1>(), s, a, ns); break;
    }
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

}  // namespace

size_t attn_workspace_bytes(int heads, int head_dim, int max_seq) {
    (void)head_dim;
    return ws_bytes(heads, max_seq);
}

int attn_decode_launch(const AttnArgs& a, hipStream_t s) {
    LLMI_REQUIRE(a.head_dim == D, "attn: head_dim must be 128");
    LLMI_REQUIRE(a.heads > 0 && a.kv_heads > 0 && a.heads % a.kv_heads == 0, "attn: bad head counts");
    LLMI_REQUIRE(a.max_seq > 0 && (a.max_seq + CH - 1) / CH <= kMaxSplits, "attn: max_seq out of range");
    LLMI_REQUIRE(a.pos_dev || (a.pos_host >= 0 && a.pos_host < a.max_seq), "attn: pos out of range");
    LLMI_REQUIRE(a.qkv && a.k_cache && a.v_cache && a.workspace, "attn: null pointer");
    LLMI_REQUIRE(!a.direct_out || a.out, "attn: null output");
    LLMI_REQUIRE(!a.xacc || a.resid || a.resid_fixed, "attn: xacc seeding needs resid");
    const dim3 grid(a.heads, (a.max_seq + CH - 1) / CH);  // ns = gridDim.y
    if (a.merge_out) {
        LLMI_REQUIRE(!a.direct_out && !a.xacc && a.pos_dev, "attn: merge_out needs the engine form (device position, no xacc)");
        LLMI_REQUIRE(2 * (size_t)grid.y + 2 * D + 4 <= kAttnLds / 4, "attn: max_seq too large for the in-kernel merge");
        const size_t lds = kAttnLds + 16;
        if (a.cache_dtype == LLMI_F16)
            hipLaunchKernelGGL(attn_decode_merge_kernel<__half>, grid, dim3(kThreads), lds, s, a);
        else if (a.cache_dtype == LLMI_F32)
            hipLaunchKernelGGL(attn_decode_merge_kernel<float>, grid, dim3(kThreads), lds, s, a);
        else
            LLMI_REQUIRE(false, "attn: cache dtype must be f16 or f32");
        LLMI_HIP(hipGetLastError());
        return LLMI_OK;
    }
    if (a.cache_dtype == LLMI_F16)
        hipLaunchKernelGGL(attn_decode_kernel<__half>, grid, dim3(kThreads), kAttnLds, s, a);
    else if (a.cache_dtype == LLMI_F32)
        hipLaunchKernelGGL(attn_decode_kernel<float>, grid, dim3(kThreads), kAttnLds, s, a);
    else
        LLMI_REQUIRE(false, "attn: cache dtype must be f16 or f32");
    LLMI_HIP(hipGetLastError());
    if (a.direct_out) {
        hipLaunchKernelGGL(attn_merge_kernel, dim3(a.heads), dim3(kThreads), 0, s, a, (int)grid.y);
        LLMI_HIP(hipGetLastError());
    }
    return LLMI_OK;
}

// grid shape of the fused launch; 0 if the arguments do not fit it
static dim3 fused_grid(const AttnArgs& aa, const OprojArgs& oa, int* ns, int* nchunk, int* npl) {
    *npl = oproj_npl(oa);
    *ns = (aa.max_seq + CH - 1) / CH;
    *nchunk = (oa.n_rows + 16 * *npl - 1) / (16 * *npl);
    return dim3(aa.heads, *ns > *nchunk ? *ns : *nchunk);
}

int attn_oproj_fused_check(const AttnArgs& aa, const OprojArgs& oa, int device) {
    if (aa.direct_out || aa.xacc || aa.heads != oa.heads || aa.max_seq != oa.max_seq || !aa.pos_dev ||
        aa.pos_dev != oa.pos_dev || aa.workspace != oa.workspace || aa.head_dim != D || oa.head_dim != D)
        return LLMI_EUNSUPPORTED;
    int ns, nchunk, npl;
    const dim3 grid = fused_grid(aa, oa, &ns, &nchunk, &npl);
    const void* fn = fused_fn_any(oa.w_dtype, aa.cache_dtype, npl);
    if (!fn) return LLMI_EUNSUPPORTED;
    int per_cu = 0, cus = 0;
    LLMI_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kThreads, fused_lds(npl)));
    LLMI_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    // every workgroup co-resident: a waiting workgroup can never hold the slot a producer needs
    return (long)grid.x * grid.y <= (long)per_cu * cus ? LLMI_OK : LLMI_EUNSUPPORTED;
}

int attn_oproj_fused_launch(const AttnArgs& aa, const OprojArgs& oa, int* err, hipStream_t s) {
    LLMI_REQUIRE(aa.qkv && aa.k_cache && aa.v_cache && aa.workspace && oa.w && oa.xacc, "attn_oproj_fused: null pointer");
    LLMI_REQUIRE(aa.max_seq > 0 && (aa.max_seq + CH - 1) / CH <= kMaxSplits, "attn_oproj_fused: max_seq out of range");
    LLMI_REQUIRE(aa.heads > 0 && aa.kv_heads > 0 && aa.heads % aa.kv_heads == 0, "attn_oproj_fused: bad head counts");
    LLMI_REQUIRE(oa.ldw >= oa.heads * D && oa.n_rows > 0, "attn_oproj_fused: bad W_o shape");
    LLMI_REQUIRE(oa.w_dtype != LLMI_I8 || oa.scales, "attn_oproj_fused: int8 weights need scales");
    int ns, nchunk, npl;
    const dim3 grid = fused_grid(aa, oa, &ns, &nchunk, &npl);
    const void* fn = fused_fn_any(oa.w_dtype, aa.cache_dtype, npl);
    LLMI_REQUIRE(fn != nullptr, "attn_oproj_fused: weight dtype must be f16, f32 or i8; cache f16 or f32");
    void* args[] = {const_cast<AttnArgs*>(&aa), const_cast<OprojArgs*>(&oa), &ns, &nchunk, &err};
    LLMI_HIP(hipLaunchKernel(fn, grid, dim3(kThreads), args, fused_lds(npl), s));
    return LLMI_OK;
}

int attn_oproj_launch(const OprojArgs& a, hipStream_t s) {
    LLMI_REQUIRE(a.head_dim == D, "attn_oproj: head_dim must be 128");
    LLMI_REQUIRE(a.w && a.workspace && a.xacc && a.heads > 0 && a.n_rows > 0, "attn_oproj: bad arguments");
    LLMI_REQUIRE(a.ldw >= a.heads * D, "attn_oproj: ldw < heads * head_dim");
    LLMI_REQUIRE(a.max_seq > 0 && (a.max_seq + CH - 1) / CH <= kMaxSplits, "attn_oproj: max_seq out of range");
    switch (a.w_dtype) {
        case LLMI_F16: return oproj_launch_w<__half>(a, s);
        case LLMI_F32: return oproj_launch_w<float>(a, s);
        case LLMI_I8:
            LLMI_REQUIRE(a.scales != nullptr, "attn_oproj: int8 weights need scales");
            return oproj_launch_w<int8_t>(a, s);
    }
    LLMI_REQUIRE(false, "attn_oproj: weight dtype must be f16, f32 or i8");
}

}  // namespace llmi
