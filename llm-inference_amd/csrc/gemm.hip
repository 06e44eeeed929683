// Prefill linear layers on the matrix cores:
//   Y[m, n] = sum_k A[m, k] * W[n, k]        (nn.Linear, W row-major [out, in])
// the M = prompt-rows case of launchLinearGemm (linear.cu:38-99 -> cublasGemmEx
// with trans_b, as called from context_attention.cpp:99,166 and ffn.cpp:72,89).
//
// Numerics. W is fp16 (or int8 with a per-row fp16 scale), so it enters the
// f16 MFMA exactly. The fp32 activations are split while they are staged:
// a = hi + lo with hi = fp16(a), lo = fp16(a - hi), and both halves are
// multiplied against the same W fragment (SPLIT = 2), accumulating in fp32.
// That keeps the product fp32-faithful (|a - hi - lo| <= 2^-22 |a|) for twice
// the MFMA work; SPLIT = 1 (plain fp16 activations) measured 2.3e-3 logits
// rel-L2 over 32 layers vs the fp32 reference -- over the 1e-3 bar -- so it is
// kept only as the throughput variant.
//
// Fusions: the RMSNorm of x is folded in (NORM): gamma * x is staged and the
// per-row sum of squares is accumulated from the same loads, so the row's rstd
// is applied to the accumulator in the epilogue, like the decode GEMV. The
// epilogue stores, adds into the residual stream in place (o_proj, down), or
// pairs gate/up columns of one tile into silu(gate) * up (gate_up).
//
// Tiling for gfx950: BM x 128 output tile per 256-thread workgroup (4 waves,
// 2 x 2, each (BM/2) x 64 = (BM/32) x 4 tiles of v_mfma_f32_16x16x32_f16),
// BK = 64, register-staged double-step pipeline (tile k+1 is loaded into
// registers while tile k is multiplied out of LDS), rows padded by 16 B so the
// ds_read_b128 fragment reads are bank-conflict free. Workgroup ids are
// remapped so each XCD works on one row band of A (kept in its 4 MiB L2) while
// the weight tiles stream.
// Roofline: MFMA (fp16 dense 2.5 PFLOP/s); FLOPs per launch 2 * M * N * K
// (the SPLIT = 2 variant issues 2x that on the matrix cores).
#include "kernels.h"

namespace llmi {

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kBN = 128;
constexpr int kBK = 64;
constexpr int kLd = kBK + 8;  // LDS row stride in halves (144 B)

__device__ __forceinline__ float silu_f(float v) { return v / (1.0f + expf(-v)); }

__device__ __forceinline__ f4 load_gamma4(const void* g, int g_dt, int k) {
    if (g_dt == LLMI_F32) return *reinterpret_cast<const f4*>(static_cast<const float*>(g) + k);
    const h4 h = *reinterpret_cast<const h4*>(static_cast<const _Float16*>(g) + k);
    return f4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
}

// SILU epilogue pairing: tile row tr of the B tile holds W row
//   gate g0 + 32*(tr>>6) + (tr&31)           for (tr & 32) == 0
//   up   pair_off + (same gate column)        for (tr & 32) != 0
// so wave column wc sees gate columns in its n-fragments 0,1 and the matching
// up columns in fragments 2,3 (same lane, same register).
__device__ __forceinline__ int b_src_row(int epi, int n0, int tr, int pair_off) {
    if (epi != EPI_SILU_MUL) return n0 + tr;
    const int gc = n0 + 32 * (tr >> 6) + (tr & 31);
    return (tr & 32) ? pair_off + gc : gc;
}

template <int BM, int SPLIT, int WT, int EPI, bool NORM>
__global__ __launch_bounds__(kThreads) void gemm_kernel(GemmArgs a) {
    constexpr int MI = BM / 32;            // 16-row fragments per wave
    constexpr int A_LOADS = BM * kBK / 4 / kThreads;   // float4 per thread
    constexpr int B_CHUNK = (WT == LLMI_I8) ? 16 : 8;  // elements per 16-B load
    constexpr int B_LOADS = kBN * kBK / B_CHUNK / kThreads;
    constexpr int A_ROWS_PER_PASS = kThreads / (kBK / 4);  // 16

    __shared__ _Float16 lds[(SPLIT * BM + kBN) * kLd];
    __shared__ float rs_lds[BM];
    _Float16* a_hi = lds;
    _Float16* a_lo = lds + BM * kLd;  // SPLIT == 2 only
    _Float16* b_t = lds + SPLIT * BM * kLd;

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wr = w >> 1, wc = w & 1;

    // XCD-aware tile order: consecutive remapped ids share an XCD (bid % 8).
    const int nwg = gridDim.x;
    int id = blockIdx.x;
    if ((nwg & 7) == 0) id = (id & 7) * (nwg >> 3) + (id >> 3);
    const int rt = id / a.n_tiles, ct = id - rt * a.n_tiles;
    const int m0 = rt * BM;
    const int n0 = (EPI == EPI_SILU_MUL) ? ct * (kBN / 2) : ct * kBN;
    const int K = a.k;

    // per-thread staging coordinates
    const int a_c4 = t & 15, a_r0 = t >> 4;   // row a_r0 + 16 i, k offset 4 * a_c4
    const float* a_src[A_LOADS];
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
        const int row = min(m0 + a_r0 + A_ROWS_PER_PASS * i, a.m - 1);
        a_src[i] = a.a + (size_t)row * a.lda + 4 * a_c4;
    }
    const char* b_src[B_LOADS];
    int b_row[B_LOADS], b_col[B_LOADS];
#pragma unroll
    for (int i = 0; i < B_LOADS; ++i) {
        const int idx = t + kThreads * i;
        constexpr int CPR = kBK / B_CHUNK;  // chunks per row
        b_row[i] = idx / CPR;
        b_col[i] = (idx % CPR) * B_CHUNK;
        const int src = b_src_row(EPI, n0, b_row[i], a.pair_off);
        const size_t ldb = a.w_kblock ? a.w_kblock : K;
        b_src[i] = static_cast<const char*>(a.w) + ((size_t)src * ldb + b_col[i]) * (WT == LLMI_I8 ? 1 : 2);
    }

    f4 ra[A_LOADS];
    u32x4 rb[B_LOADS];
    float ss[A_LOADS];
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) ss[i] = 0.f;

    auto load = [&](int k0) {
        // head-major W: K block k0 / w_kblock is an [n][w_kblock] slab
        const size_t koff = a.w_kblock ? (size_t)(k0 / a.w_kblock) * a.n * a.w_kblock + k0 % a.w_kblock : (size_t)k0;
#pragma unroll
        for (int i = 0; i < A_LOADS; ++i) ra[i] = *reinterpret_cast<const f4*>(a_src[i] + k0);
#pragma unroll
        for (int i = 0; i < B_LOADS; ++i)
            rb[i] = *reinterpret_cast<const u32x4*>(b_src[i] + koff * (WT == LLMI_I8 ? 1 : 2));
    };
    auto stage = [&](int k0) {
        f4 g = f4{1.f, 1.f, 1.f, 1.f};
        if (NORM) g = load_gamma4(a.gamma, a.g_dtype, k0 + 4 * a_c4);
#pragma unroll
        for (int i = 0; i < A_LOADS; ++i) {
            f4 v = ra[i];
            if (NORM) {
                ss[i] += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
                v = v * g;
            }
            const h4 hi = __builtin_convertvector(v, h4);
            const int off = (a_r0 + A_ROWS_PER_PASS * i) * kLd + 4 * a_c4;
            *reinterpret_cast<h4*>(a_hi + off) = hi;
            if (SPLIT == 2) {
                const f4 rem = v - __builtin_convertvector(hi, f4);
                *reinterpret_cast<h4*>(a_lo + off) = __builtin_convertvector(rem, h4);
            }
        }
#pragma unroll
        for (int i = 0; i < B_LOADS; ++i) {
            _Float16* dst = b_t + b_row[i] * kLd + b_col[i];
            if (WT == LLMI_I8) {
                h8 lo8, hi8;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    lo8[j] = (_Float16)(float)(signed char)((rb[i][j >> 2] >> (8 * (j & 3))) & 0xff);
                    hi8[j] = (_Float16)(float)(signed char)((rb[i][2 + (j >> 2)] >> (8 * (j & 3))) & 0xff);
                }
                *reinterpret_cast<h8*>(dst) = lo8;
                *reinterpret_cast<h8*>(dst + 8) = hi8;
            } else {
                *reinterpret_cast<u32x4*>(dst) = rb[i];
            }
        }
    };

    f4 acc[MI][4];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

    const int fr = lane & 15, fk = 8 * (lane >> 4);
    const int a_base = (wr * (BM / 2) + fr) * kLd + fk;
    const int b_base = (wc * 64 + fr) * kLd + fk;

    const int KT = K / kBK;
    load(0);
    for (int kt = 0; kt < KT; ++kt) {
        if (kt) __syncthreads();
        stage(kt * kBK);
        __syncthreads();
        if (kt + 1 < KT) load((kt + 1) * kBK);
#pragma unroll
        for (int kk = 0; kk < kBK / 32; ++kk) {
            h8 bf[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const h8*>(b_t + b_base + j * 16 * kLd + kk * 32);
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                const h8 ah = *reinterpret_cast<const h8*>(a_hi + a_base + i * 16 * kLd + kk * 32);
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bf[j], acc[i][j], 0, 0, 0);
                if (SPLIT == 2) {
                    const h8 al = *reinterpret_cast<const h8*>(a_lo + a_base + i * 16 * kLd + kk * 32);
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bf[j], acc[i][j], 0, 0, 0);
                }
            }
        }
    }

    // per-row rstd: the 16 threads of a staging row are 16 consecutive lanes
    if (NORM) {
#pragma unroll
        for (int i = 0; i < A_LOADS; ++i) {
            float v = ss[i];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            if (a_c4 == 0) rs_lds[a_r0 + A_ROWS_PER_PASS * i] = 1.0f / sqrtf(v / (float)K + a.eps);
        }
        __syncthreads();
    }

    // epilogue: C fragment (i, j) register r is row 16 i + 4 (lane >> 4) + r, column 16 j + (lane & 15)
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int lr = wr * (BM / 2) + 16 * i + 4 * (lane >> 4) + r;
            const int m = m0 + lr;
            if (m >= a.m) continue;
            const float rsc = NORM ? rs_lds[lr] : 1.f;
            float* yrow = a.y + (size_t)m * a.ldy;
            if (EPI == EPI_SILU_MUL) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int gc = n0 + 32 * wc + 16 * j + fr;
                    float g = acc[i][j][r] * rsc, u = acc[i][j + 2][r] * rsc;
                    if (WT == LLMI_I8) {
                        g *= __half2float(a.scales[gc]);
                        u *= __half2float(a.scales[a.pair_off + gc]);
                    }
                    yrow[gc] = silu_f(g) * u;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int n = n0 + wc * 64 + 16 * j + fr;
                    float v = acc[i][j][r] * rsc;
                    if (WT == LLMI_I8) v *= __half2float(a.scales[n]);
                    if (EPI == EPI_ADD)
                        yrow[n] += v;
                    else
                        yrow[n] = v;
                }
            }
        }
    }
}

template <int BM, int SPLIT, int WT>
int dispatch_epi(const GemmArgs& a, dim3 grid, hipStream_t s) {
    if (a.epi == EPI_STORE && a.gamma)
        hipLaunchKernelGGL((gemm_kernel<BM, SPLIT, WT, EPI_STORE, true>), grid, dim3(kThreads), 0, s, a);
    else if (a.epi == EPI_STORE)
        hipLaunchKernelGGL((gemm_kernel<BM, SPLIT, WT, EPI_STORE, false>), grid, dim3(kThreads), 0, s, a);
    else if (a.epi == EPI_ADD && !a.gamma)
        hipLaunchKernelGGL((gemm_kernel<BM, SPLIT, WT, EPI_ADD, false>), grid, dim3(kThreads), 0, s, a);
    else if (a.epi == EPI_SILU_MUL && a.gamma)
        hipLaunchKernelGGL((gemm_kernel<BM, SPLIT, WT, EPI_SILU_MUL, true>), grid, dim3(kThreads), 0, s, a);
    else
        LLMI_REQUIRE(false, "gemm: unsupported epilogue/norm combination");
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

template <int BM>
int dispatch_bm(const GemmArgs& a, dim3 grid, hipStream_t s) {
    if (a.split == 2) {
        return a.w_dtype == LLMI_I8 ? dispatch_epi<BM, 2, LLMI_I8>(a, grid, s)
                                    : dispatch_epi<BM, 2, LLMI_F16>(a, grid, s);
    }
    return a.w_dtype == LLMI_I8 ? dispatch_epi<BM, 1, LLMI_I8>(a, grid, s) : dispatch_epi<BM, 1, LLMI_F16>(a, grid, s);
}

}  // namespace

bool gemm_supported(int w_dtype, int n, int k, int epi) {
    if (w_dtype != LLMI_F16 && w_dtype != LLMI_I8) return false;
    const int ncols = (epi == EPI_SILU_MUL) ? n / 2 : n;
    const int tile = (epi == EPI_SILU_MUL) ? kBN / 2 : kBN;
    return n > 0 && k > 0 && ncols % tile == 0 && k % kBK == 0;
}

int gemm_bm(const GemmArgs& a) {
    const int ncols = (a.epi == EPI_SILU_MUL) ? a.n / 2 : a.n;
    const int nt = ncols / ((a.epi == EPI_SILU_MUL) ? kBN / 2 : kBN);
    // 128-row tiles unless that leaves most of the 256 CUs idle
    return ((a.m + 127) / 128) * nt >= 256 ? 128 : 64;
}

int gemm_launch(GemmArgs a, hipStream_t s) {
    LLMI_REQUIRE(a.a && a.w && a.y && a.m > 0, "gemm: null operand or empty M");
    LLMI_REQUIRE(gemm_supported(a.w_dtype, a.n, a.k, a.epi),
                 "gemm: needs f16/i8 weights, N a multiple of 128 (gate_up: 2 x 64) and K of 64");
    LLMI_REQUIRE(a.w_dtype != LLMI_I8 || a.scales, "gemm: int8 weights need per-row scales");
    LLMI_REQUIRE(a.lda % 4 == 0 && (reinterpret_cast<uintptr_t>(a.a) & 15) == 0, "gemm: A rows must be 16-B aligned");
    LLMI_REQUIRE((reinterpret_cast<uintptr_t>(a.w) & 15) == 0, "gemm: W must be 16-B aligned");
    LLMI_REQUIRE(a.split == 1 || a.split == 2, "gemm: split must be 1 or 2");
    LLMI_REQUIRE(a.w_kblock == 0 || (a.w_kblock % kBK == 0 && a.k % a.w_kblock == 0 && a.epi != EPI_SILU_MUL),
                 "gemm: w_kblock must be a multiple of 64 dividing K (not with the gate_up pairing)");
    LLMI_REQUIRE(a.epi != EPI_SILU_MUL || a.pair_off == a.n / 2, "gemm: gate_up pair offset must be N / 2");
    const int ncols = (a.epi == EPI_SILU_MUL) ? a.n / 2 : a.n;
    a.n_tiles = ncols / ((a.epi == EPI_SILU_MUL) ? kBN / 2 : kBN);
    const int bm = gemm_bm(a);
    const int mt = (a.m + bm - 1) / bm;
    const dim3 grid(mt * a.n_tiles);
    return bm == 128 ? dispatch_bm<128>(a, grid, s) : dispatch_bm<64>(a, grid, s);
}

}  // namespace llmi
