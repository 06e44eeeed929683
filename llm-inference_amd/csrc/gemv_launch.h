// GEMV launchers (templates) shared by the per-weight-dtype translation units
// gemv_f16.hip / gemv_f32.hip / gemv_i8.hip, which instantiate launch_epi<WT>
// (split so the build compiles the dtypes in parallel).
#pragma once
#include "gemv_impl.h"
#include "xchg_impl.h"

namespace llmi {
namespace gemv_detail {


#ifndef LLMI_GEMV_MAX_GRID
#define LLMI_GEMV_MAX_GRID 1024
#endif
#ifndef LLMI_GEMV_MIN_WAVES
#define LLMI_GEMV_MIN_WAVES 1  // min waves per SIMD (launch-bounds 2nd arg): caps VGPRs
#endif

#ifndef LLMI_GEMV_MIN_WAVES_I8
// int8 at unroll <= 5: 4 waves per SIMD. The 13B-width q/k/v / gate_up / lm_head kernels need 130-135
// VGPRs (3 waves) for a prologue peak (the 5 x 16-B x-staging loads with gammas beside the first
// weight batch); capped at 128 they spill 2-4 VGPRs there and run 0.5 % faster a 13B token (same
// box, alternating libraries: 3,133 -> 3,115 us, profiles/r07i_int8_minwaves_ab.jsonl)
#define LLMI_GEMV_MIN_WAVES_I8 4
#endif
template <typename WT, int U> constexpr int min_waves() {
    return sizeof(WT) == 1 && U <= 5 ? LLMI_GEMV_MIN_WAVES_I8 : LLMI_GEMV_MIN_WAVES;
}

template <typename WT, int ROWS, int EPI, bool NORM, typename GT, int XPT, int kUnroll, bool XFIX, int KPT = 1>
__global__ __launch_bounds__(kThreads, (min_waves<WT, kUnroll>())) void gemv_kernel(GemvArgs a) {
    // all LDS in one 16-B aligned dynamic region (cdna_hip_programming.md G17):
    // [PK][nc] float4 x image, then 16 floats of reduction scratch, then keys
    extern __shared__ __attribute__((aligned(16))) float4 xs[];
    WgStamp ts(a.stamps);
    gemv_body<WT, ROWS, EPI, NORM, GT, XPT, kUnroll, XFIX, PlainIO, KPT>(a, blockIdx.x, gridDim.x, xs);
    if constexpr (EPI == EPI_ATOMIC || EPI == EPI_ARGMAX) {  // TP: push yacc / the argmax keys from this launch
        const int k4 = (EPI == EPI_ATOMIC ? a.k / a.ksplit : a.k) / 4;
        xchg_detail::xchg_tail(a.xt, a.xt_cnt, reinterpret_cast<int*>(xs + k4) + 15);  // red[15]: free by now
    }
}

// Workgroups of one instantiation that fit the chip at once (occupancy x CUs),
// cached per instantiation and LDS size.
inline int device_cus() {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 0;
    }
    return cus;
}
template <typename WT, int ROWS, int EPI, bool NORM, typename GT, int XPT, int U, bool XF, int KPT = 1>
int launch_k(const GemvArgs& a, int grid, size_t lds, hipStream_t s) {
    auto kern = gemv_kernel<WT, ROWS, EPI, NORM, GT, XPT, U, XF, KPT>;
    // An automatic grid larger than what is resident leaves the excess workgroups to
    // start only when early ones retire -- a second, latency-bound round at the tail
    // (profiles/r01c: int8 13B q/k/v and down). Clamp it to the resident count
    // (argmax grids stay: their partial count is fixed by gemv_grid for step_start).
    if (EPI != EPI_ARGMAX && a.grid == 0 && a.kpar <= 1) {  // (kpar: one group per wave, no loop: never clamped)
        static size_t occ_lds = ~(size_t)0;
        static int occ_blocks = 0;
        if (lds != occ_lds) {
            int n = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(kern), kThreads, lds) !=
                hipSuccess)
                n = 0;
            occ_blocks = n * device_cus();
            occ_lds = lds;
        }
        const int S = (EPI == EPI_ATOMIC) ? a.ksplit : 1;
        if (occ_blocks >= S && grid > occ_blocks) grid = occ_blocks / S * S;
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, s, a);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

template <typename WT, int ROWS, int EPI, bool NORM, typename GT, int U, bool XF>
int launch_u(const GemvArgs& a, int grid, hipStream_t s) {
    const int kl = (EPI == EPI_ATOMIC) ? a.k / a.ksplit : a.k;  // x extent one workgroup stages
    const size_t lds = gemv_lds_bytes(kl);
    const int k4 = kl / 4;
    if constexpr ((EPI == EPI_STORE || EPI == EPI_SILU_MUL) && NORM && XF && U == 4) {
        // kpar (a TP rank's q/k/v and gate_up): the engine's normed fixed-point projections,
        // hidden <= 5120
        if (a.kpar > 1) {
            LLMI_REQUIRE(k4 <= 5 * kThreads, "gemv: kpar needs k <= 5120");
            if (a.kpar == 2)
                return k4 <= 4 * kThreads ? launch_k<WT, ROWS, EPI, NORM, GT, 4, U, XF, 2>(a, grid, lds, s)
                                          : launch_k<WT, ROWS, EPI, NORM, GT, 5, U, XF, 2>(a, grid, lds, s);
            return k4 <= 4 * kThreads ? launch_k<WT, ROWS, EPI, NORM, GT, 4, U, XF, 4>(a, grid, lds, s)
                                      : launch_k<WT, ROWS, EPI, NORM, GT, 5, U, XF, 4>(a, grid, lds, s);
        }
    }
    LLMI_REQUIRE(a.kpar <= 1, "gemv: kpar only for the engine's normed fixed-point q/k/v and gate_up");
    if (k4 <= 4 * kThreads) return launch_k<WT, ROWS, EPI, NORM, GT, 4, U, XF>(a, grid, lds, s);
    if (k4 <= 5 * kThreads) return launch_k<WT, ROWS, EPI, NORM, GT, 5, U, XF>(a, grid, lds, s);    // 13B hidden
    if (k4 <= 11 * kThreads) return launch_k<WT, ROWS, EPI, NORM, GT, 11, U, XF>(a, grid, lds, s);  // 7B inter
    if (k4 <= 14 * kThreads) return launch_k<WT, ROWS, EPI, NORM, GT, 14, U, XF>(a, grid, lds, s);  // 13B inter
    return launch_k<WT, ROWS, EPI, NORM, GT, 0, U, XF>(a, grid, lds, s);
}

// Loads in flight per wave: measured on MI355X (tools/tune_gemv.sh, profiles/):
// with many row groups per CU (q/k/v, gate_up) 2 rows x 4 loads per wave win
// (more waves resident); with few groups (o, down: 2048 pairs; lm_head argmax)
// 2 rows x 8 loads per wave win.
// Unroll (16-B loads per row in flight per lane; a batch covers 64 * U chunks of a
// row). Preference measured on MI355X (tools/tune_gemv.sh, profiles/): with many
// row groups per CU (q/k/v, gate_up) U = 4 (more waves resident), otherwise U = 8.
// A U that pads the row's chunk count to fewer batch slots wins over the
// preference: masked slots cost load issue and VALU (13B rows: 320 int8 / 640
// fp16 chunks waste 37.5 % / 25 % of their slots at U = 8, none at U = 5).
template <typename WT, int EPI>
int pick_unroll(const GemvArgs& a, int groups) {
    const int kl = (EPI == EPI_ATOMIC) ? a.k / a.ksplit : a.k;
    const int nc = kl / WT_<WT>::EPL / (a.kpar > 1 ? a.kpar : 1);  // chunks one wave streams
    auto slots = [&](int u) { const int b = kWave * u; return (nc + b - 1) / b * b; };
    // kpar: only U = 4 is instantiated for the K-parted kernel (launch_u), so it is taken
    // whatever the slot count (13B fp16 at kpar 2: 320 chunks a part would pick U = 5 and
    // fail the launch)
    if (a.kpar > 1) return 4;
    int best = (EPI != EPI_ARGMAX && groups >= 4096 && groups <= 12288 && kUnrollMax >= 4) ? 4 : kUnrollMax;
    for (int u : {4, 5, 8})
        if (u <= kUnrollMax && slots(u) < slots(best)) best = u;
    return best;
}

template <typename WT, int ROWS, int EPI, bool NORM, typename GT, bool XF>
int launch_x(const GemvArgs& a, int grid, int u, hipStream_t s) {
    if (u == 4) return launch_u<WT, ROWS, EPI, NORM, GT, 4, XF>(a, grid, s);
    if (u == 5) return launch_u<WT, ROWS, EPI, NORM, GT, 5, XF>(a, grid, s);
    return launch_u<WT, ROWS, EPI, NORM, GT, kUnrollMax, XF>(a, grid, s);
}

template <typename WT, int ROWS, int EPI, bool NORM, typename GT>
int launch_t(const GemvArgs& a, int grid, hipStream_t s) {
    const int groups = (EPI == EPI_SILU_MUL) ? a.pair_off : (a.n_rows + ROWS - 1) / ROWS;
    const int u = pick_unroll<WT, EPI>(a, groups);
    if (a.x_fixed) {
        // the engine's residual stream is int64 fixed point: the normed projections read it
        if constexpr (NORM && EPI != EPI_ADD && EPI != EPI_ATOMIC) {
            return launch_x<WT, ROWS, EPI, NORM, GT, true>(a, grid, u, s);
        }
        LLMI_REQUIRE(false, "gemv: a fixed-point x needs rmsnorm and a store/silu/argmax epilogue");
    }
    return launch_x<WT, ROWS, EPI, NORM, GT, false>(a, grid, u, s);
}

template <typename WT, int ROWS, int EPI>
int launch_norm(const GemvArgs& a, int grid, hipStream_t s) {
    if (a.gamma == nullptr) return launch_t<WT, ROWS, EPI, false, float>(a, grid, s);
    if (a.g_dtype == LLMI_F16) return launch_t<WT, ROWS, EPI, true, __half>(a, grid, s);
    if (a.g_dtype == LLMI_F32) return launch_t<WT, ROWS, EPI, true, float>(a, grid, s);
    LLMI_REQUIRE(false, "gemv: gamma dtype must be f16 or f32");
}

template <typename WT>
int launch_epi(const GemvArgs& a, int grid, hipStream_t s) {
    switch (a.epi) {
        case EPI_STORE: return launch_norm<WT, kRows, EPI_STORE>(a, grid, s);
        case EPI_ADD: return launch_norm<WT, kRows, EPI_ADD>(a, grid, s);
        case EPI_SILU_MUL: return launch_norm<WT, 2, EPI_SILU_MUL>(a, grid, s);
        case EPI_ARGMAX: return launch_norm<WT, kRows, EPI_ARGMAX>(a, grid, s);
        case EPI_ATOMIC:
            LLMI_REQUIRE(a.gamma == nullptr, "gemv: the split-K atomic epilogue takes no rmsnorm");
            return launch_t<WT, kRows, EPI_ATOMIC, false, float>(a, grid, s);
    }
    LLMI_REQUIRE(false, "gemv: bad epilogue");
}


}  // namespace gemv_detail
}  // namespace llmi
