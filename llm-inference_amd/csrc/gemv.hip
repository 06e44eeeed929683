// HBM-streaming GEMV for batch-1 decode: y = W x, W [n_rows, k] row-major
// (fp16 / fp32 / int8+row-scale), x fp32, fp32 accumulate.
//
// Replaces launchLinearGemm -> cublasGemmEx with m = 1 (src/kernels/linear.cu:38-104,
// src/kernels/cublas_utils.cc:32-71) for the q/k/v, o, gate_up, down and lm_head
// projections.
//
// Roofline: HBM. Algorithmic bytes per launch = n_rows * k * sizeof(W) (+ scales);
// x (<= 55 KB) is L2-resident and re-read by every workgroup.
//
// Design (MI355X, wave64):
//  * one workgroup = 4 waves; x is staged once per workgroup into LDS in a
//    packet-major layout (packet p of chunk c at [p][c]) so that 64 lanes reading
//    consecutive chunks hit consecutive 16-byte slots (conflict-free ds_read_b128);
//  * a wave owns ROWS weight rows at a time and streams them with 16-byte
//    nontemporal loads, 8 loads per row in flight per lane (1 KiB per wave
//    instruction, coalesced), then a 6-step xor-shuffle reduction;
//  * prologue fusion: RMSNorm of x (modeling_llama.py:112-117) computed by every
//    workgroup from the L2-resident x -- removes the separate launchRMSNorm /
//    launchFusedAddBiasResidualRMSNorm kernels of self_decoder.cpp:59-70;
//  * epilogue fusion: residual add (add_residual.cu), SiLU*mul with the gate/up
//    row pair owned by one wave (act_kernel.cu:17-31), or logits + per-workgroup
//    argmax key for greedy sampling (topK.cu + sampling.cu with K = 1).
#include "gemv_impl.h"

namespace llmi {
namespace {

using namespace gemv_detail;

#ifndef LLMI_GEMV_MAX_GRID
#define LLMI_GEMV_MAX_GRID 1024
#endif
#ifndef LLMI_GEMV_MIN_WAVES
#define LLMI_GEMV_MIN_WAVES 1  // min waves per SIMD (launch-bounds 2nd arg): caps VGPRs
#endif

template <typename WT, int ROWS, int EPI, bool NORM, typename GT, int XPT, int kUnroll, bool XFIX>
__global__ __launch_bounds__(kThreads, LLMI_GEMV_MIN_WAVES) void gemv_kernel(GemvArgs a) {
    // all LDS in one 16-B aligned dynamic region (cdna_hip_programming.md G17):
    // [PK][nc] float4 x image, then 16 floats of reduction scratch, then keys
    extern __shared__ __attribute__((aligned(16))) float4 xs[];
    gemv_body<WT, ROWS, EPI, NORM, GT, XPT, kUnroll, XFIX, PlainIO>(a, blockIdx.x, gridDim.x, xs, NoSync{});
}

template <typename WT, int ROWS, int EPI, bool NORM, typename GT, int U, bool XF>
int launch_u(const GemvArgs& a, int grid, hipStream_t s) {
    const int kl = (EPI == EPI_ATOMIC) ? a.k / a.ksplit : a.k;  // x extent one workgroup stages
    const size_t lds = gemv_lds_bytes(kl);
    const int k4 = kl / 4;
    if (k4 <= 4 * kThreads)
        hipLaunchKernelGGL((gemv_kernel<WT, ROWS, EPI, NORM, GT, 4, U, XF>), dim3(grid), dim3(kThreads), lds, s, a);
    else if (k4 <= 5 * kThreads)  // 13B hidden (5120)
        hipLaunchKernelGGL((gemv_kernel<WT, ROWS, EPI, NORM, GT, 5, U, XF>), dim3(grid), dim3(kThreads), lds, s, a);
    else if (k4 <= 11 * kThreads)  // 7B inter (11008)
        hipLaunchKernelGGL((gemv_kernel<WT, ROWS, EPI, NORM, GT, 11, U, XF>), dim3(grid), dim3(kThreads), lds, s, a);
    else if (k4 <= 14 * kThreads)  // 13B inter (13824)
        hipLaunchKernelGGL((gemv_kernel<WT, ROWS, EPI, NORM, GT, 14, U, XF>), dim3(grid), dim3(kThreads), lds, s, a);
    else
        hipLaunchKernelGGL((gemv_kernel<WT, ROWS, EPI, NORM, GT, 0, U, XF>), dim3(grid), dim3(kThreads), lds, s, a);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

// Loads in flight per wave: measured on MI355X (tools/tune_gemv.sh, profiles/):
// with many row groups per CU (q/k/v, gate_up) 2 rows x 4 loads per wave win
// (more waves resident); with few groups (o, down: 2048 pairs; lm_head argmax)
// 2 rows x 8 loads per wave win.
template <typename WT, int ROWS, int EPI, bool NORM, typename GT>
int launch_t(const GemvArgs& a, int grid, hipStream_t s) {
    const int groups = (EPI == EPI_SILU_MUL) ? a.pair_off : (a.n_rows + ROWS - 1) / ROWS;
    const bool u4 = EPI != EPI_ARGMAX && groups >= 4096 && groups <= 12288 && kUnrollMax >= 4;
    if (a.x_fixed) {
        // the engine's residual stream is int64 fixed point: the normed projections read it
        if constexpr (NORM && EPI != EPI_ADD && EPI != EPI_ATOMIC) {
            return u4 ? launch_u<WT, ROWS, EPI, NORM, GT, 4, true>(a, grid, s)
                      : launch_u<WT, ROWS, EPI, NORM, GT, kUnrollMax, true>(a, grid, s);
        }
        LLMI_REQUIRE(false, "gemv: a fixed-point x needs rmsnorm and a store/silu/argmax epilogue");
    }
    return u4 ? launch_u<WT, ROWS, EPI, NORM, GT, 4, false>(a, grid, s)
              : launch_u<WT, ROWS, EPI, NORM, GT, kUnrollMax, false>(a, grid, s);
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

int epl_of(int dt) { return dt == LLMI_F16 ? 8 : dt == LLMI_F32 ? 4 : dt == LLMI_I8 ? 16 : 0; }

}  // namespace

int gemv_grid(const GemvArgs& a) {
    if (a.grid > 0) return a.grid;
    const int groups = (a.epi == EPI_SILU_MUL) ? a.pair_off : (a.n_rows + kRows - 1) / kRows;
    int blocks = (groups + kWavesPerBlock - 1) / kWavesPerBlock;
    // cap (default ~4 workgroups per CU on 256 CUs); waves then loop over several row groups
    const int S = (a.epi == EPI_ATOMIC) ? a.ksplit : 1;  // split-K: S workgroups per row-group block
    const int cap = LLMI_GEMV_MAX_GRID / S > 0 ? LLMI_GEMV_MAX_GRID / S : 1;
    return (blocks < cap ? blocks : cap) * S;
}

int gemv_launch(const GemvArgs& a, hipStream_t s) {
    const int epl = epl_of(a.w_dtype);
    LLMI_REQUIRE(epl > 0, "gemv: weight dtype must be f16, f32 or i8");
    LLMI_REQUIRE(a.k > 0 && a.k % epl == 0, "gemv: k must be a positive multiple of 16 bytes of weights");
    LLMI_REQUIRE((size_t)a.k * 4 <= 150 * 1024, "gemv: k too large for LDS staging");
    LLMI_REQUIRE(a.w && (a.x || a.x_fixed) && (a.y || a.epi == EPI_ATOMIC), "gemv: null pointer");
    LLMI_REQUIRE(a.w_dtype != LLMI_I8 || a.scales, "gemv: int8 weights need per-row scales");
    LLMI_REQUIRE(a.epi != EPI_ADD || a.resid, "gemv: EPI_ADD needs resid");
    LLMI_REQUIRE(a.epi != EPI_ARGMAX || a.partials, "gemv: EPI_ARGMAX needs partials");
    LLMI_REQUIRE(a.epi != EPI_SILU_MUL || (a.pair_off > 0 && a.n_rows == 2 * a.pair_off),
                 "gemv: EPI_SILU_MUL needs n_rows == 2 * pair_off");
    LLMI_REQUIRE(a.n_rows > 0, "gemv: n_rows must be > 0");
    LLMI_REQUIRE(a.epi != EPI_ATOMIC || (a.yacc && a.x && !a.x_fixed && a.ksplit >= 1 &&
                                         a.k % (a.ksplit * epl) == 0),
                 "gemv: EPI_ATOMIC needs yacc, an fp32 x and k divisible into ksplit 16-B slices");
    LLMI_REQUIRE(a.epi == EPI_ATOMIC || a.ksplit == 1, "gemv: ksplit only with EPI_ATOMIC");
    LLMI_REQUIRE(a.ldw == 0 || a.ldw >= a.k, "gemv: ldw < k");
    const int grid = gemv_grid(a);
    switch (a.w_dtype) {
        case LLMI_F16: return launch_epi<__half>(a, grid, s);
        case LLMI_F32: return launch_epi<float>(a, grid, s);
        case LLMI_I8: return launch_epi<int8_t>(a, grid, s);
    }
    return LLMI_EINVAL;
}

}  // namespace llmi
