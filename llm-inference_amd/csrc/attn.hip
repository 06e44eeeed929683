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
// Work split (MI355X): grid (heads, active splits ceil(ctx / 64)) when the caller knows
// the position on the host (the engine: one token graph per split count), else
// (heads, max_seq / 64) with the inactive splits exiting. A workgroup (256 threads = 16
// groups of 16 lanes) owns 64 cached positions of one head; a 16-lane group reads a
// 256-byte fp16 K/V row with one 16-B load per lane (4 rows per wave instruction),
// all its rows issued before anything waits. 32 heads alone would use 32 of 256 CUs;
// at ctx 2048 the split gives 1024 workgroups. Each writes (m, l, o) partials; the
// next kernel merges them (a kernel boundary orders the hand-off -- an in-kernel
// last-arriver merge measured no faster: its store-drain + ticket + load chain costs
// as much as the boundary, profiles/).
#include <cstdlib>

#include "attn_impl.h"
#include "xchg_impl.h"

namespace llmi {
namespace {

using namespace attn_detail;

// ns: the workspace's split stride (max_seq / 64); the grid holds ns splits, or only
// the a.nact active ones (HOST_SIZED)
template <typename KT, bool HOST_SIZED>
__global__ __launch_bounds__(kThreads) void attn_decode_kernel(AttnArgs a, int ns) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    WgStamp ts(a.stamps);
    attn_body<KT, PlainIO, HOST_SIZED>(a, blockIdx.x, blockIdx.y, ns, smem, &ts);
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
    oproj_body<WT, NPL, PlainIO>(a, blockIdx.x, blockIdx.y, ns, smem);
    xchg_detail::xchg_tail(a.xt, a.xt_cnt, reinterpret_cast<int*>(smem));  // TP: push xacc from this launch
}

// two heads per workgroup (oproj_body2)
template <typename WT, int NPL>
__global__ __launch_bounds__(kThreads) void attn_oproj2_kernel(OprojArgs a, int ns) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    WgStamp ts(a.stamps);
    oproj_body2<WT, NPL, PlainIO>(a, blockIdx.x, blockIdx.y, ns, smem);
    xchg_detail::xchg_tail(a.xt, a.xt_cnt, reinterpret_cast<int*>(smem));  // TP: push xacc from this launch
}

#ifndef LLMI_OPROJ_HG
#define LLMI_OPROJ_HG 2  // heads per fp16 o_proj workgroup when the head count is even (1: one head, A/B)
#endif

int oproj_npl(const OprojArgs& a) {
    const long target = (long)a.heads * a.n_rows / (1024 * 16);  // ~1024 workgroups
#ifdef LLMI_OPROJ_NPL
    if (target >= 8) return LLMI_OPROJ_NPL;
#endif
    return target >= 8 ? 8 : target >= 4 ? 4 : target >= 2 ? 2 : 1;
}

template <typename WT>
int oproj_launch_w(const OprojArgs& a, hipStream_t s) {
    // ~1024 workgroups: rows per workgroup = 16 * NPL
    const int ns = (a.max_seq + CH - 1) / CH;
    const int npl = oproj_npl(a);
    // fp16 weights only: the int8 form needs 92 VGPRs with two heads (68 with one), so 13B's
    // 1,600 workgroups no longer fit in one round and it measured 0.7-0.9 us slower (r06q); fp32
    // weights (the parity instantiation) would need 140
    if (LLMI_OPROJ_HG == 2 && sizeof(WT) == 2 && a.heads % 2 == 0 && !a.head_major && npl == 8) {
        const dim3 grid2(a.heads / 2, (a.n_rows + 8 * npl - 1) / (8 * npl));
        hipLaunchKernelGGL((attn_oproj2_kernel<WT, 8>), grid2, dim3(kThreads), oproj2_lds<8>(), s, a, ns);
        LLMI_HIP(hipGetLastError());
        return LLMI_OK;
    }
    const dim3 grid(a.heads, (a.n_rows + 16 * npl - 1) / (16 * npl));
    switch (npl) {
#if LLMI_OPROJ_NPL == 16
        case 16: hipLaunchKernelGGL((attn_oproj_kernel<WT, 16>), grid, dim3(kThreads), oproj_lds<16>(), s, a, ns); break;
#endif
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
    const int ns = (a.max_seq + CH - 1) / CH;
    LLMI_REQUIRE(a.nact >= 0 && a.nact <= ns, "attn: nact out of range");
    LLMI_REQUIRE(a.pos_dev || a.nact == 0 || a.nact == a.pos_host / CH + 1, "attn: nact != ceil((pos + 1) / 64)");
    LLMI_REQUIRE(a.nact == 0 || a.pos_dev, "attn: nact > 0 needs the device position");
    const bool hs = a.nact > 0;
    const dim3 grid(a.heads, hs ? a.nact : ns);
    if (a.cache_dtype == LLMI_F16) {
        if (hs)
            hipLaunchKernelGGL((attn_decode_kernel<__half, true>), grid, dim3(kThreads), kAttnLds, s, a, ns);
        else
            hipLaunchKernelGGL((attn_decode_kernel<__half, false>), grid, dim3(kThreads), kAttnLds, s, a, ns);
    } else if (a.cache_dtype == LLMI_F32) {
        if (hs)
            hipLaunchKernelGGL((attn_decode_kernel<float, true>), grid, dim3(kThreads), kAttnLds, s, a, ns);
        else
            hipLaunchKernelGGL((attn_decode_kernel<float, false>), grid, dim3(kThreads), kAttnLds, s, a, ns);
    } else {
        LLMI_REQUIRE(false, "attn: cache dtype must be f16 or f32");
    }
    LLMI_HIP(hipGetLastError());
    if (a.direct_out) {
        hipLaunchKernelGGL(attn_merge_kernel, dim3(a.heads), dim3(kThreads), 0, s, a, ns);
        LLMI_HIP(hipGetLastError());
    }
    return LLMI_OK;
}

int attn_oproj_launch(const OprojArgs& a, hipStream_t s) {
    LLMI_REQUIRE(a.head_dim == D, "attn_oproj: head_dim must be 128");
    LLMI_REQUIRE(a.w && a.workspace && a.xacc && a.heads > 0 && a.n_rows > 0, "attn_oproj: bad arguments");
    LLMI_REQUIRE(a.ldw >= a.heads * D, "attn_oproj: ldw < heads * head_dim");
    LLMI_REQUIRE(a.max_seq > 0 && (a.max_seq + CH - 1) / CH <= kMaxSplits, "attn_oproj: max_seq out of range");
    LLMI_REQUIRE(a.nact >= 0 && a.nact <= (a.max_seq + CH - 1) / CH, "attn_oproj: nact out of range");
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
