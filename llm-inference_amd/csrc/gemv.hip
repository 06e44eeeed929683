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
#ifndef LLMI_GEMV_UNROLL
#define LLMI_GEMV_UNROLL 8
#endif
#ifndef LLMI_GEMV_ROWS
#define LLMI_GEMV_ROWS 2
#endif
#ifndef LLMI_GEMV_MAX_GRID
#define LLMI_GEMV_MAX_GRID 1024
#endif
constexpr int kUnrollMax = LLMI_GEMV_UNROLL;  // 16-B loads per row in flight per lane
constexpr int kRows = LLMI_GEMV_ROWS;      // rows per wave (EPI_SILU_MUL always pairs 2)

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

__device__ __forceinline__ float silu(float v) { return v / (1.0f + expf(-v)); }

template <typename GT>
__device__ __forceinline__ float4 gamma4(const void* g, int j) {
    if constexpr (sizeof(GT) == 2) {
        const uint2 u = reinterpret_cast<const uint2*>(g)[j];
        const float2 a = __half22float2(*reinterpret_cast<const __half2*>(&u.x));
        const float2 b = __half22float2(*reinterpret_cast<const __half2*>(&u.y));
        return make_float4(a.x, a.y, b.x, b.y);
    } else {
        return reinterpret_cast<const float4*>(g)[j];
    }
}

// XPT: float4s of x each thread holds in registers during staging (k <= XPT*4*256);
// 0 = generic strided staging (no weight prefetch).
#ifndef LLMI_GEMV_MIN_WAVES
#define LLMI_GEMV_MIN_WAVES 1  // min waves per SIMD (launch-bounds 2nd arg): caps VGPRs
#endif
template <typename WT, int ROWS, int EPI, bool NORM, typename GT, int XPT, int kUnroll, bool XFIX>
__global__ __launch_bounds__(kThreads, LLMI_GEMV_MIN_WAVES) void gemv_kernel(GemvArgs a) {
    constexpr int EPL = WT_<WT>::EPL;
    constexpr int PK = EPL / 4;                 // float4 packets per 16-B weight load
    // all LDS in one 16-B aligned dynamic region (cdna_hip_programming.md G17):
    // [PK][nc] float4 x image, then 16 floats of reduction scratch, then keys
    extern __shared__ __attribute__((aligned(16))) float4 xs[];
    const int k = a.k;
    const int k4 = k / 4;
    const int nc = k / EPL;                     // 16-B chunks per row
    float* red = reinterpret_cast<float*>(xs + k4);
    unsigned long long* best_s = reinterpret_cast<unsigned long long*>(red + 16);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n_groups = (EPI == EPI_SILU_MUL) ? a.pair_off : (a.n_rows + ROWS - 1) / ROWS;
    const char* wbase = reinterpret_cast<const char*>(a.w);
    const size_t row_bytes = (size_t)k * sizeof(WT);
    const float4* x4 = reinterpret_cast<const float4*>(a.x);

    auto rows_of = [&](int g, int* rows) {
#pragma unroll
        for (int r = 0; r < ROWS; ++r) rows[r] = (EPI == EPI_SILU_MUL) ? g + r * a.pair_off : g * ROWS + r;
    };
    // Branch-free streaming: every lane always issues its ROWS x kUnroll loads; out of
    // range chunks/rows are clamped to a valid address and zeroed by a mask. A
    // predicated load makes hipcc branch around each load and wait vmcnt(0) per load
    // (cdna_hip_programming.md §5 "three .s-level traps" (c)), serialising the stream.
    auto load_batch = [&](uint4 (&wv)[ROWS][kUnroll], const int* rows, int base) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int c = base + u * kWave + lane;
            const int cc = c < nc ? c : nc - 1;
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                const int rr = rows[r] < a.n_rows ? rows[r] : a.n_rows - 1;
                const unsigned m = (c < nc && rows[r] < a.n_rows) ? 0xFFFFFFFFu : 0u;
                uint4 v = ld_nt16(wbase + (size_t)rr * row_bytes + (size_t)cc * 16);
                v.x &= m; v.y &= m; v.z &= m; v.w &= m;
                wv[r][u] = v;
            }
        }
    };
    auto dot_batch = [&](const uint4 (&wv)[ROWS][kUnroll], int base, float* acc) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int c = base + u * kWave + lane;
            const float4* xp = xs + (c < nc ? c : nc - 1);  // masked chunks have zero weights
#pragma unroll
            for (int r = 0; r < ROWS; ++r) acc[r] += dot_packet(wv[r][u], xp, nc, (WT*)nullptr);
        }
    };

    // ---- prologue. Issue order matters: vmcnt retires loads in issue order, so x
    // (and gamma) go first, then this wave's first weight batch; the weight stream is
    // then in flight while x is staged and the norm is reduced.
    const int g0 = blockIdx.x * kWavesPerBlock + wave;
    int rows0[ROWS];
    rows_of(g0, rows0);
    uint4 w0[ROWS][kUnroll];
    float ss = 0.f;
    const bool wb = XFIX && blockIdx.x == 0 && a.x_out != nullptr;  // one block writes x back
    if constexpr (XPT > 0) {
        // branch-free: clamp the index, load, and predicate only the LDS store
        float4 xv[XPT], gv[XPT];
        longlong2 xf[XFIX ? XPT : 1][2];
#pragma unroll
        for (int i = 0; i < XPT; ++i) {
            int j = tid + i * kThreads;
            j = j < k4 ? j : k4 - 1;
            if constexpr (XFIX) {
                xf[i][0] = reinterpret_cast<const longlong2*>(a.x_fixed)[2 * j];
                xf[i][1] = reinterpret_cast<const longlong2*>(a.x_fixed)[2 * j + 1];
            } else {
                xv[i] = x4[j];
            }
            if (NORM) gv[i] = gamma4<GT>(a.gamma, j);
        }
        load_batch(w0, rows0, 0);
        // RMSNorm (modeling_llama.py:112-117) as gamma*x staged + one scalar rsqrt per
        // dot product in the epilogue: sum_k W[r,k] gamma_k x_k * rstd.
#pragma unroll
        for (int i = 0; i < XPT; ++i) {
            const int j = tid + i * kThreads;
            if (j < k4) {
                float4 v;
                if constexpr (XFIX) {
                    v = make_float4(from_fixed(xf[i][0].x), from_fixed(xf[i][0].y),
                                    from_fixed(xf[i][1].x), from_fixed(xf[i][1].y));
                    if (wb) reinterpret_cast<float4*>(a.x_out)[j] = v;
                } else {
                    v = xv[i];
                }
                if (NORM) {
                    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
                    v.x *= gv[i].x; v.y *= gv[i].y; v.z *= gv[i].z; v.w *= gv[i].w;
                }
                xs[(j % PK) * nc + j / PK] = v;
            }
        }
    } else {
        for (int j = tid; j < k4; j += kThreads) {
            float4 v;
            if constexpr (XFIX) {
                const long long* f = a.x_fixed + 4 * j;
                v = make_float4(from_fixed(f[0]), from_fixed(f[1]), from_fixed(f[2]), from_fixed(f[3]));
                if (wb) reinterpret_cast<float4*>(a.x_out)[j] = v;
            } else {
                v = x4[j];
            }
            if (NORM) {
                const float4 gg = gamma4<GT>(a.gamma, j);
                ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
                v.x *= gg.x; v.y *= gg.y; v.z *= gg.z; v.w *= gg.w;
            }
            xs[(j % PK) * nc + j / PK] = v;
        }
        load_batch(w0, rows0, 0);
    }
    float rstd = 1.f;
    if (NORM) {
        ss = block_sum(ss, red);  // its barriers also publish xs
        rstd = 1.0f / sqrtf(ss / (float)k + a.eps);
    } else {
        __syncthreads();
    }

    unsigned long long best = 0ull;
    auto finish = [&](int g, const int* rows, float* acc) {
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            acc[r] = wave_sum(acc[r]) * rstd;
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
    };

    // ---- first group (its first batch is already in flight)
    if (g0 < n_groups) {
        float acc[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) acc[r] = 0.f;
        dot_batch(w0, 0, acc);
        for (int base = kWave * kUnroll; base < nc; base += kWave * kUnroll) {
            uint4 wv[ROWS][kUnroll];
            load_batch(wv, rows0, base);
            dot_batch(wv, base, acc);
        }
        finish(g0, rows0, acc);
    }
    // ---- remaining groups
    for (int g = g0 + gridDim.x * kWavesPerBlock; g < n_groups; g += gridDim.x * kWavesPerBlock) {
        int rows[ROWS];
        rows_of(g, rows);
        float acc[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) acc[r] = 0.f;
        for (int base = 0; base < nc; base += kWave * kUnroll) {
            uint4 wv[ROWS][kUnroll];
            load_batch(wv, rows, base);
            dot_batch(wv, base, acc);
        }
        finish(g, rows, acc);
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

template <typename WT, int ROWS, int EPI, bool NORM, typename GT, int U, bool XF>
int launch_u(const GemvArgs& a, int grid, hipStream_t s) {
    const size_t lds = (size_t)a.k * sizeof(float) + 16 * sizeof(float) + kWavesPerBlock * 8;
    const int k4 = a.k / 4;
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
    if constexpr (EPI == EPI_SILU_MUL && NORM) {
        // the engine's gate_up reads the residual from the fixed-point accumulator
        if (a.x_fixed) {
            if (groups >= 4096 && groups <= 12288 && kUnrollMax >= 4)
                return launch_u<WT, ROWS, EPI, NORM, GT, 4, true>(a, grid, s);
            return launch_u<WT, ROWS, EPI, NORM, GT, kUnrollMax, true>(a, grid, s);
        }
    }
    LLMI_REQUIRE(a.x_fixed == nullptr, "gemv: fixed-point x only with rmsnorm + silu_mul");
    if (EPI != EPI_ARGMAX && groups >= 4096 && groups <= 12288 && kUnrollMax >= 4)
        return launch_u<WT, ROWS, EPI, NORM, GT, 4, false>(a, grid, s);
    return launch_u<WT, ROWS, EPI, NORM, GT, kUnrollMax, false>(a, grid, s);
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
    return blocks < LLMI_GEMV_MAX_GRID ? blocks : LLMI_GEMV_MAX_GRID;
}

int gemv_launch(const GemvArgs& a, hipStream_t s) {
    const int epl = epl_of(a.w_dtype);
    LLMI_REQUIRE(epl > 0, "gemv: weight dtype must be f16, f32 or i8");
    LLMI_REQUIRE(a.k > 0 && a.k % epl == 0, "gemv: k must be a positive multiple of 16 bytes of weights");
    LLMI_REQUIRE((size_t)a.k * 4 <= 150 * 1024, "gemv: k too large for LDS staging");
    LLMI_REQUIRE(a.w && (a.x || a.x_fixed) && a.y, "gemv: null pointer");
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
