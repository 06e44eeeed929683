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
#include "kernels.h"

namespace llmi {
namespace {

constexpr int kThreads = 256;
constexpr int kWavesPerBlock = kThreads / kWave;
constexpr int kUnroll = 8;  // 16-B loads per row in flight per lane

template <typename WT> struct WT_ { };
template <> struct WT_<__half> { static constexpr int EPL = 8; };
template <> struct WT_<float> { static constexpr int EPL = 4; };
template <> struct WT_<int8_t> { static constexpr int EPL = 16; };

__device__ __forceinline__ float dot_packet(const uint4& w, const float4* xp, int nc, __half*) {
    const __half2* h = reinterpret_cast<const __half2*>(&w);
    float4 x0 = xp[0], x1 = xp[nc];
    float2 a = __half22float2(h[0]), b = __half22float2(h[1]);
    float2 c = __half22float2(h[2]), d = __half22float2(h[3]);
    float s = a.x * x0.x;
    s = fmaf(a.y, x0.y, s);
    s = fmaf(b.x, x0.z, s);
    s = fmaf(b.y, x0.w, s);
    s = fmaf(c.x, x1.x, s);
    s = fmaf(c.y, x1.y, s);
    s = fmaf(d.x, x1.z, s);
    s = fmaf(d.y, x1.w, s);
    return s;
}
__device__ __forceinline__ float dot_packet(const uint4& w, const float4* xp, int nc, float*) {
    float4 x0 = xp[0];
    float s = __uint_as_float(w.x) * x0.x;
    s = fmaf(__uint_as_float(w.y), x0.y, s);
    s = fmaf(__uint_as_float(w.z), x0.z, s);
    s = fmaf(__uint_as_float(w.w), x0.w, s);
    return s;
}
__device__ __forceinline__ float i8(uint32_t v, int j) { return (float)(int8_t)((v >> (8 * j)) & 0xff); }
__device__ __forceinline__ float dot_packet(const uint4& w, const float4* xp, int nc, int8_t*) {
    const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        float4 x = xp[p * nc];
        s = fmaf(i8(ws[p], 0), x.x, s);
        s = fmaf(i8(ws[p], 1), x.y, s);
        s = fmaf(i8(ws[p], 2), x.z, s);
        s = fmaf(i8(ws[p], 3), x.w, s);
    }
    return s;
}

template <typename GT>
__device__ __forceinline__ float gamma_at(const void* g, int i) {
    return to_f32(reinterpret_cast<const GT*>(g)[i]);
}

__device__ __forceinline__ float silu(float v) { return v / (1.0f + expf(-v)); }

template <typename WT, int ROWS, int EPI, bool NORM, typename GT>
__global__ __launch_bounds__(kThreads) void gemv_kernel(GemvArgs a) {
    constexpr int EPL = WT_<WT>::EPL;
    constexpr int PK = EPL / 4;                 // float4 packets per 16-B weight load
    // all LDS in one 16-B aligned dynamic region (cdna_hip_programming.md G17):
    // [PK][nc] float4 x image, then 16 floats of reduction scratch, then keys
    extern __shared__ __attribute__((aligned(16))) float4 xs[];
    const int k = a.k;
    const int nc = k / EPL;                     // 16-B chunks per row
    float* red = reinterpret_cast<float*>(xs + k / 4);
    unsigned long long* best_s = reinterpret_cast<unsigned long long*>(red + 16);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    // ---- stage x (packet-major), optional RMSNorm prologue
    const float4* x4 = reinterpret_cast<const float4*>(a.x);
    float ss = 0.f;
    for (int j = tid; j < k / 4; j += kThreads) {
        float4 v = x4[j];
        if (NORM) ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
        xs[(j % PK) * nc + j / PK] = v;
    }
    if (NORM) {
        ss = block_sum(ss, red);  // includes __syncthreads
        const float rstd = 1.0f / sqrtf(ss / (float)k + a.eps);
        for (int j = tid; j < k / 4; j += kThreads) {
            const int slot = (j % PK) * nc + j / PK;
            float4 v = xs[slot];
            v.x = gamma_at<GT>(a.gamma, 4 * j + 0) * (v.x * rstd);
            v.y = gamma_at<GT>(a.gamma, 4 * j + 1) * (v.y * rstd);
            v.z = gamma_at<GT>(a.gamma, 4 * j + 2) * (v.z * rstd);
            v.w = gamma_at<GT>(a.gamma, 4 * j + 3) * (v.w * rstd);
            xs[slot] = v;
        }
    }
    __syncthreads();

    const int n_groups = (EPI == EPI_SILU_MUL) ? a.pair_off : (a.n_rows + ROWS - 1) / ROWS;
    const char* wbase = reinterpret_cast<const char*>(a.w);
    const size_t row_bytes = (size_t)k * sizeof(WT);
    unsigned long long best = 0ull;

    for (int g = blockIdx.x * kWavesPerBlock + wave; g < n_groups; g += gridDim.x * kWavesPerBlock) {
        int rows[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; ++r)
            rows[r] = (EPI == EPI_SILU_MUL) ? g + r * a.pair_off : g * ROWS + r;
        float acc[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) acc[r] = 0.f;

        for (int base = 0; base < nc; base += kWave * kUnroll) {
            uint4 wv[ROWS][kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int c = base + u * kWave + lane;
#pragma unroll
                for (int r = 0; r < ROWS; ++r) {
                    if (c < nc && rows[r] < a.n_rows)
                        wv[r][u] = ld_nt16(wbase + (size_t)rows[r] * row_bytes + (size_t)c * 16);
                    else
                        wv[r][u] = make_uint4(0, 0, 0, 0);
                }
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int c = base + u * kWave + lane;
                if (c < nc) {
                    const float4* xp = xs + c;
#pragma unroll
                    for (int r = 0; r < ROWS; ++r) acc[r] += dot_packet(wv[r][u], xp, nc, (WT*)nullptr);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            acc[r] = wave_sum(acc[r]);
            if (a.scales != nullptr && rows[r] < a.n_rows) acc[r] *= __half2float(a.scales[rows[r]]);
        }
        if (EPI == EPI_SILU_MUL) {
            if (lane == 0) a.y[g] = silu(acc[0]) * acc[1];
        } else {
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                const int row = rows[r];
                if (row >= a.n_rows) continue;
                if (lane == r) {
                    float v = acc[r];
                    if (EPI == EPI_ADD) v += a.resid_scale * a.resid[row];
                    a.y[row] = v;
                }
                if (EPI == EPI_ARGMAX) {
                    unsigned long long kk = argmax_key(acc[r], a.idx_base + (uint32_t)row);
                    best = kk > best ? kk : best;
                }
            }
        }
    }
    if (EPI == EPI_ARGMAX) {
        if (lane == 0) best_s[wave] = best;
        __syncthreads();
        if (tid == 0) {
            unsigned long long b = best_s[0];
            for (int i = 1; i < kWavesPerBlock; ++i) b = best_s[i] > b ? best_s[i] : b;
            a.partials[blockIdx.x] = b;
        }
    }
}

template <typename WT, int ROWS, int EPI, bool NORM, typename GT>
int launch_t(const GemvArgs& a, int grid, hipStream_t s) {
    const size_t lds = (size_t)a.k * sizeof(float) + 16 * sizeof(float) + kWavesPerBlock * 8;
    hipLaunchKernelGGL((gemv_kernel<WT, ROWS, EPI, NORM, GT>), dim3(grid), dim3(kThreads), lds, s, a);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
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
        case EPI_STORE: return launch_norm<WT, 2, EPI_STORE>(a, grid, s);
        case EPI_ADD: return launch_norm<WT, 2, EPI_ADD>(a, grid, s);
        case EPI_SILU_MUL: return launch_norm<WT, 2, EPI_SILU_MUL>(a, grid, s);
        case EPI_ARGMAX: return launch_norm<WT, 2, EPI_ARGMAX>(a, grid, s);
    }
    LLMI_REQUIRE(false, "gemv: bad epilogue");
}

int epl_of(int dt) { return dt == LLMI_F16 ? 8 : dt == LLMI_F32 ? 4 : dt == LLMI_I8 ? 16 : 0; }

}  // namespace

int gemv_grid(const GemvArgs& a) {
    if (a.grid > 0) return a.grid;
    const int groups = (a.epi == EPI_SILU_MUL) ? a.pair_off : (a.n_rows + 1) / 2;
    int blocks = (groups + kWavesPerBlock - 1) / kWavesPerBlock;
    // cap: ~4 workgroups per CU on 256 CUs; waves then loop over several row groups
    return blocks < 1024 ? blocks : 1024;
}

int gemv_launch(const GemvArgs& a, hipStream_t s) {
    const int epl = epl_of(a.w_dtype);
    LLMI_REQUIRE(epl > 0, "gemv: weight dtype must be f16, f32 or i8");
    LLMI_REQUIRE(a.k > 0 && a.k % epl == 0, "gemv: k must be a positive multiple of 16 bytes of weights");
    LLMI_REQUIRE((size_t)a.k * 4 <= 150 * 1024, "gemv: k too large for LDS staging");
    LLMI_REQUIRE(a.w && a.x && a.y, "gemv: null pointer");
    LLMI_REQUIRE(a.w_dtype != LLMI_I8 || a.scales, "gemv: int8 weights need per-row scales");
    LLMI_REQUIRE(a.epi != EPI_ADD || a.resid, "gemv: EPI_ADD needs resid");
    LLMI_REQUIRE(a.epi != EPI_ARGMAX || a.partials, "gemv: EPI_ARGMAX needs partials");
    LLMI_REQUIRE(a.epi != EPI_SILU_MUL || (a.pair_off > 0 && a.n_rows == 2 * a.pair_off),
                 "gemv: EPI_SILU_MUL needs n_rows == 2 * pair_off");
    LLMI_REQUIRE(a.n_rows > 0, "gemv: n_rows must be > 0");
    const int grid = gemv_grid(a);
    switch (a.w_dtype) {
        case LLMI_F16: return launch_epi<__half>(a, grid, s);
        case LLMI_F32: return launch_epi<float>(a, grid, s);
        case LLMI_I8: return launch_epi<int8_t>(a, grid, s);
    }
    return LLMI_EINVAL;
}

}  // namespace llmi
