// Dataflow decode layer: one launch per transformer layer (batch 1) whose
// workgroups are laid out in phase order
//
//   [ q/k/v GEMV | split-KV attention | merge + o_proj | gate_up GEMV | down GEMV ]
//
// (the same device bodies as the five standalone kernels, gemv_impl.h and
// attn_impl.h, with identical arithmetic). Each workgroup first issues the loads
// that do not depend on the previous phase -- its first weight batch, its K/V
// chunk, its W_o slice -- then waits for the previous phase's completion counter,
// then reads the handed-off activations. Workgroups are dispatched in index order,
// so the next phase's workgroups start streaming into the slots the previous
// phase frees while its tail drains: the per-launch fill/drain of five separate
// kernels (profiles/r01: ~18 us of a 85 us layer below the 6.3 TB/s copy rate)
// becomes overlapped weight streaming. Hand-offs follow handoff.h (write-through
// stores, sharded counters, sc1 loads); a wait can only target lower-indexed
// workgroups, which in-order dispatch has already placed, and every spin is bounded.
//
// Replaces, per layer, LlamaSelfDecoder<T>::forward's launch sequence
// (self_decoder.cpp:23-89: rmsnorm, qkv linear, rope, masked MHA, o linear,
// fused add+rmsnorm, gate_up linear, act, down linear, add residual).
#include <algorithm>
#include <type_traits>

#include "attn_impl.h"
#include "gemv_impl.h"

namespace llmi {
namespace {

using namespace gemv_detail;
using namespace attn_detail;

// phase-specific access: loads of bytes made by the previous phase of this launch
// and stores of bytes the next phase reads are sc1; everything else plain
template <bool LOAD_SC1, bool STORE_SC1>
struct MixIO {
    using L = typename std::conditional<LOAD_SC1, Sc1IO, PlainIO>::type;
    using S = typename std::conditional<STORE_SC1, Sc1IO, PlainIO>::type;
    __device__ __forceinline__ static float ld(const float* p) { return L::ld(p); }
    __device__ __forceinline__ static float4 ld4(const float4* p) { return L::ld4(p); }
    __device__ __forceinline__ static longlong2 ld_ll2(const longlong2* p) { return L::ld_ll2(p); }
    __device__ __forceinline__ static long long ld_ll(const long long* p) { return L::ld_ll(p); }
    __device__ __forceinline__ static void st(float* p, float v) { S::st(p, v); }
    __device__ __forceinline__ static void st_ll(long long* p, long long v) { S::st_ll(p, v); }
    __device__ __forceinline__ static void st4(float4* p, float4 v) { S::st4(p, v); }
};

enum Phase { PH_QKV = 0, PH_ATTN, PH_O, PH_GU, PH_DOWN, PH_COUNT };
constexpr int kLayerThreads = 256;
#ifndef LLMI_LAYER_WAVES
#define LLMI_LAYER_WAVES 4  // waves per SIMD the register budget must admit (4 workgroups / CU)
#endif
static_assert(kLayerThreads == gemv_detail::kThreads && kLayerThreads == attn_detail::kThreads,
              "the bodies share one workgroup shape");

// PLAIN (diagnostic, one phase per launch only): the same bodies with plain
// loads/stores and no hand-off, to separate the hand-off cost from the bodies'
// code generation inside this kernel
template <bool PLAIN, bool LD, bool ST>
using PhIO = typename std::conditional<PLAIN, MixIO<false, false>, MixIO<LD, ST>>::type;
struct PlainSync : NoSync {
    const unsigned* wait_cnt = nullptr;
    unsigned wait_target = 0;
    unsigned* pub_cnt = nullptr;
    int* err = nullptr;
    unsigned long long* stamp = nullptr;
};

template <typename WT, typename KT, int XH, int XI, int NPL, int UQ, int UG, int UD, bool PLAIN = false>
__global__ __launch_bounds__(kLayerThreads, LLMI_LAYER_WAVES) void layer_kernel(LayerArgs L) {
    extern __shared__ __attribute__((aligned(16))) float4 smem[];
    int b = blockIdx.x;
    typename std::conditional<PLAIN, PlainSync, FlowSync>::type s;
    s.err = L.err;
    unsigned long long t_start = 0;
    if (L.stamps) {  // debug timeline: {start, wait passed, end} per workgroup (100 MHz clock)
        t_start = __builtin_amdgcn_s_memrealtime();
        s.stamp = L.stamps + 3 * (size_t)blockIdx.x;
    }
    struct EndStamp {
        unsigned long long* p;
        unsigned long long t0;
        __device__ ~EndStamp() {
            if (p && threadIdx.x == 0) {
                p[0] = t0;
                p[2] = __builtin_amdgcn_s_memrealtime();
            }
        }
    } end_stamp{s.stamp, t_start};
    auto cnt = [&](int ph) { return L.cnt + ph * kPhaseCntWords; };
    if (b < L.nb[PH_QKV]) {
        s.pub_cnt = cnt(PH_QKV);
        gemv_body<WT, kRows, EPI_STORE, true, __half, XH, UQ, true, PhIO<PLAIN, false, true>>(L.qkv, b, L.nb[PH_QKV],
                                                                                       smem, s);
        s.publish();
        return;
    }
    b -= L.nb[PH_QKV];
    if (b < L.nb[PH_ATTN]) {
        s.wait_cnt = cnt(PH_QKV);
        s.wait_target = L.nb[PH_QKV];
        s.pub_cnt = cnt(PH_ATTN);
        attn_body<KT, PhIO<PLAIN, true, true>>(L.attn, b % L.attn.heads, b / L.attn.heads, L.ns,
                                         reinterpret_cast<float*>(smem), s);
        s.publish();
        return;
    }
    b -= L.nb[PH_ATTN];
    if (b < L.nb[PH_O]) {
        s.wait_cnt = cnt(PH_ATTN);
        s.wait_target = L.nb[PH_ATTN];
        s.pub_cnt = cnt(PH_O);
        oproj_body<WT, NPL, PhIO<PLAIN, true, true>>(L.o, b % L.o.heads, b / L.o.heads, L.ns,
                                               reinterpret_cast<float*>(smem), s);
        s.publish();
        return;
    }
    b -= L.nb[PH_O];
    if (b < L.nb[PH_GU]) {
        s.wait_cnt = cnt(PH_O);
        s.wait_target = L.nb[PH_O];
        s.pub_cnt = cnt(PH_GU);
        gemv_body<WT, 2, EPI_SILU_MUL, true, __half, XH, UG, true, PhIO<PLAIN, true, true>>(L.gu, b, L.nb[PH_GU], smem,
                                                                                      s);
        s.publish();
        return;
    }
    b -= L.nb[PH_GU];
    if (b < L.nb[PH_DOWN]) {
        s.wait_cnt = cnt(PH_GU);
        s.wait_target = L.nb[PH_GU];
        s.pub_cnt = cnt(PH_DOWN);
        // split-K, int64 atomics into the layer output (read by the next launch)
        gemv_body<WT, kRows, EPI_ATOMIC, false, float, XI, UD, false, PhIO<PLAIN, true, false>>(L.down, b, L.nb[PH_DOWN],
                                                                                          smem, s);
    }
}

template <typename WT, typename KT, int XH, int XI, int NPL, int UQ, int UG, int UD>
int launch_cfg(const LayerArgs& L, size_t lds, hipStream_t s) {
    int total = 0, phases = 0;
    for (int p = 0; p < PH_COUNT; ++p) {
        total += L.nb[p];
        phases += L.nb[p] > 0;
    }
    if (L.plain_diag && phases == 1)
        hipLaunchKernelGGL((layer_kernel<WT, KT, XH, XI, NPL, UQ, UG, UD, true>), dim3(total), dim3(kLayerThreads),
                           lds, s, L);
    else
        hipLaunchKernelGGL((layer_kernel<WT, KT, XH, XI, NPL, UQ, UG, UD>), dim3(total), dim3(kLayerThreads), lds, s,
                           L);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

template <typename WT, typename KT>
int launch_kt(const LayerArgs& L, int xh, int xi, int npl, int uq, int ug, int ud, size_t lds, hipStream_t s) {
    // instantiated: Llama-2-7B (x staging 4 x 4 x 256 floats, down K-slice 2752),
    // Llama-2-13B (hidden 5120, K-slice 3456), the tiny test model
    // (unroll 4 throughout: 2 rows x 4 x 16 B in flight per lane keeps the body at
    // <= 128 VGPRs, i.e. 4 workgroups per CU, with 4 waves each streaming 8 KiB)
    (void)uq; (void)ug; (void)ud;
    if (xh == 4 && xi == 4 && npl == 8) return launch_cfg<WT, KT, 4, 4, 8, 4, 4, 4>(L, lds, s);
    if (xh == 5 && xi == 4 && npl == 8) return launch_cfg<WT, KT, 5, 4, 8, 4, 4, 4>(L, lds, s);
    if (xh == 4 && xi == 4 && npl == 1) return launch_cfg<WT, KT, 4, 4, 1, 4, 4, 4>(L, lds, s);
    return LLMI_EUNSUPPORTED;
}

}  // namespace

int layer_cnt_words() { return PH_COUNT * kPhaseCntWords; }

int layer_launch(LayerArgs L, hipStream_t s) { return layer_launch_probe(L, s, 0, nullptr); }

int layer_launch_phases(LayerArgs L, int first, int last, hipStream_t s) {
    return layer_launch_probe(L, s, 0, nullptr, first, last);
}

int layer_launch_probe(LayerArgs L, hipStream_t s, int max_wg, int* phase_wgs, int first, int last) {
    LLMI_REQUIRE(first >= 0 && first <= last && last < PH_COUNT, "layer: bad phase range");
    const int hidden = L.qkv.k;
    if (L.qkv.w_dtype != L.gu.w_dtype || L.qkv.w_dtype != L.down.w_dtype || L.qkv.w_dtype != L.o.w_dtype)
        return LLMI_EUNSUPPORTED;
    if (L.qkv.g_dtype != LLMI_F16 || L.gu.g_dtype != LLMI_F16) return LLMI_EUNSUPPORTED;
    if (L.qkv.x_fixed == nullptr || L.gu.x_fixed == nullptr || L.down.epi != EPI_ATOMIC || L.down.x == nullptr)
        return LLMI_EUNSUPPORTED;
    const int kl = L.down.k / L.down.ksplit;  // down K-slice staged per workgroup
    auto xpt = [](int k) { const int k4 = k / 4; return k4 <= 4 * kLayerThreads ? 4 : k4 <= 5 * kLayerThreads ? 5 : 0; };
    const int xh = xpt(hidden), xi = xpt(kl);
    LLMI_REQUIRE(L.cnt && L.err, "layer: counters and error word are required");
    // grids exactly as the standalone launches would use them
    L.nb[PH_QKV] = gemv_grid(L.qkv);
    L.ns = (L.attn.max_seq + kAttnChunk - 1) / kAttnChunk;
    L.nb[PH_ATTN] = L.attn.heads * L.ns;
    const long target = (long)L.o.heads * L.o.n_rows / (1024 * 16);
    const int npl = target >= 8 ? 8 : target >= 4 ? 4 : target >= 2 ? 2 : 1;
    L.nb[PH_O] = L.o.heads * ((L.o.n_rows + 16 * npl - 1) / (16 * npl));
    L.nb[PH_GU] = gemv_grid(L.gu);
    L.nb[PH_DOWN] = gemv_grid(L.down);
    for (int p = 0; p < PH_COUNT; ++p)  // phases outside [first, last] run as their own launches
        if (p < first || p > last) L.nb[p] = 0;
    auto unroll = [](const GemvArgs& a, bool silu) {
        const int groups = silu ? a.pair_off : (a.n_rows + kRows - 1) / kRows;
        return (groups >= 4096 && groups <= 12288 && kUnrollMax >= 4) ? 4 : kUnrollMax;
    };
    const int uq = unroll(L.qkv, false), ug = unroll(L.gu, true), ud = unroll(L.down, false);
    size_t lds = gemv_lds_bytes(hidden);
    lds = std::max(lds, gemv_lds_bytes(kl));
    lds = std::max(lds, kAttnLds);
    lds = std::max(lds, npl == 8 ? oproj_lds<8>() : npl == 4 ? oproj_lds<4>() : npl == 2 ? oproj_lds<2>() : oproj_lds<1>());
    if (phase_wgs) {
        int total = 0;
        for (int p = 0; p < PH_COUNT; ++p) total += (phase_wgs[p] = L.nb[p]);
        LLMI_REQUIRE(!L.stamps || total <= max_wg, "layer: stamp buffer too small");
    }
    const bool kv16 = L.attn.cache_dtype == LLMI_F16;
    switch (L.qkv.w_dtype) {
        case LLMI_F16:
            return kv16 ? launch_kt<__half, __half>(L, xh, xi, npl, uq, ug, ud, lds, s)
                        : launch_kt<__half, float>(L, xh, xi, npl, uq, ug, ud, lds, s);
        case LLMI_I8:
            return kv16 ? launch_kt<int8_t, __half>(L, xh, xi, npl, uq, ug, ud, lds, s)
                        : launch_kt<int8_t, float>(L, xh, xi, npl, uq, ug, ud, lds, s);
    }
    return LLMI_EUNSUPPORTED;
}

}  // namespace llmi
