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
namespace gemv_detail {
#ifndef LLMI_GEMV_MAX_GRID
#define LLMI_GEMV_MAX_GRID 1024
#endif
template <typename WT>
int launch_epi(const GemvArgs& a, int grid, hipStream_t s);  // gemv_{f16,f32,i8}.hip
}  // namespace gemv_detail

namespace {
using namespace gemv_detail;
int epl_of(int dt) { return dt == LLMI_F16 ? 8 : dt == LLMI_F32 ? 4 : dt == LLMI_I8 ? 16 : 0; }

}  // namespace

int gemv_grid(const GemvArgs& a) {
    if (a.grid > 0) return a.grid;
    const int groups = (a.epi == EPI_SILU_MUL) ? a.pair_off : (a.n_rows + kRows - 1) / kRows;
    if (a.kpar > 1) return (groups + kWavesPerBlock / a.kpar - 1) / (kWavesPerBlock / a.kpar);  // a group per wave
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
    LLMI_REQUIRE(a.kpar <= 1 || ((a.kpar == 2 || a.kpar == 4) && (a.epi == EPI_STORE || a.epi == EPI_SILU_MUL) &&
                                 a.grid == 0 && (a.k / epl) % a.kpar == 0),
                 "gemv: kpar 2 / 4 needs a store or silu epilogue, an automatic grid and k / kpar whole 16-B chunks");
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
