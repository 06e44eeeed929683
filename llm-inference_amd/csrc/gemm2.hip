// Prefill linear layers, fp16 weights, on the matrix cores with LDS-DMA staging
// (SURVEY.md §8 a15, config 3):
//   Y[m, n] (op)= sum_p sum_k A_p[m, k] * W[n, k]      (nn.Linear, W row-major [out, in])
// the M = prompt-rows case of launchLinearGemm (linear.cu:38-99 -> cublasGemmEx with
// trans_b, called from context_attention.cpp:99,166 and ffn.cpp:72,89).
//
// Numerics. W is fp16, so it enters the f16 MFMA exactly. The fp32 activations
// arrive as P fp16 planes written by the producer (rows_split_kernel below, or the
// gate_up epilogue): P = 2 is hi = fp16(a), lo = fp16(a - hi), both multiplied
// against the same W fragment and accumulated in fp32 -- fp32-faithful
// (|a - hi - lo| <= 2^-22 |a|); P = 1 is plain fp16 activations (the throughput
// mode; 2.3e-3 logits rel-L2 over 32 layers vs the fp32 reference).
// The RMSNorm of x (modeling_llama.py:112-117: x * rsqrt(mean(x^2) + eps), then
// * gamma) is applied by rows_split_kernel while it writes the planes.
//
// Structure for gfx950 (cdna_hip_programming.md §5 "Async global->LDS copy" and
// the 128^2 "step-3" structure): a BM x 128 output tile per 256-thread workgroup
// (4 waves, 2 x 2, each (BM/2) x 64 = (BM/32) x 4 v_mfma_f32_16x16x32_f16 tiles),
// BK = 64, operands staged global -> LDS by global_load_lds_dwordx4 (no VGPRs,
// no ds_write pass) into two LDS stages: stage k+1 is in flight while stage k is
// multiplied. The LDS image is lane-linear (the DMA writes wave base + 16 * lane)
// with an XOR swizzle (swz below) applied on the global SOURCE address, so the fragment
// ds_read_b128s spread over the banks. Workgroup
// ids are remapped (bijectively) so consecutive tiles share an XCD.
// Roofline: MFMA (fp16 dense 2.5 PFLOP/s); FLOPs per launch 2 * M * N * K
// (P = 2 issues 2x that on the matrix cores).
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <utility>

#include "kernels.h"

namespace llmi {

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
// LLMI_RN256=1: the row kernels (rows_split, resid_norm) at 256 threads a row instead of 1024 (A/B)
inline bool noexp_rn() {
    static const bool v = [] {
        const char* e = std::getenv("LLMI_RN256");
        return e && e[0] == '1';
    }();
    return v;
}
constexpr int kBN = 128;
constexpr int kBK = 64;
constexpr int kRowB = kBK * 2;  // 128-B LDS rows

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) const void* glb_ptr_t;

// LDS image swizzle (an involution on 2-KB blocks): 16-B chunk c of 128-B row r is stored at
// chunk c ^ ((r >> 1) & 7) -- gemm3's swz3, under which the 16 lanes of each fragment
// ds_read_b128 lane group hit 16 distinct 16-B bank slots. (The st_16x32 XOR, byte bit 5 ^=
// bit 9, that this kernel used before left them 2-way conflicted: 4 bank-conflict cycles per
// LDS instruction on the prefill o_proj, profiles/r07k_prefill_lds_pmc.json.) LLMI_GEMM2_SWZ=0:
// the old XOR (A/B builds).
#ifndef LLMI_GEMM2_SWZ
#define LLMI_GEMM2_SWZ 1
#endif
__device__ __forceinline__ int swz(int b) {
    return LLMI_GEMM2_SWZ ? b ^ (((b >> 8) & 7) << 4) : b ^ (((b >> 9) & 1) << 5);
}

#ifndef LLMI_GEMM2_STAGES
#define LLMI_GEMM2_STAGES 3
#endif
constexpr int kStages = LLMI_GEMM2_STAGES;  // LDS stages: kStages - 1 in flight while one is multiplied

// 16-B LDS-DMA as inline asm (M0 saved/restored): hipcc neither counts it nor waits
// for it, so the K-loop's counted vmcnt keeps kStages - 1 stages in flight across the
// raw barrier (cdna_hip_programming.md §5 "Pipelining across barriers")
__device__ __forceinline__ void glds16(const void* g, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(lds)
                 : "memory");
}
__device__ __forceinline__ float silu_f(float v) { return v / (1.0f + expf(-v)); }

// SILU pairing (as gemm.hip): tile row tr of the B tile holds gate column
// g0 + 32 (tr >> 6) + (tr & 31) for (tr & 32) == 0, its up row (+ pair_off) otherwise,
// so a lane's n-fragments 0, 1 hold gate columns and 2, 3 the matching up columns.
__device__ __forceinline__ int b_src_row(int epi, int n0, int tr, int pair_off) {
    if (epi != EPI_SILU_MUL) return n0 + tr;
    const int gc = n0 + 32 * (tr >> 6) + (tr & 31);
    return (tr & 32) ? pair_off + gc : gc;
}

template <int BM, int P, int EPI>
__global__ __launch_bounds__(kThreads) void gemm2_kernel(Gemm2Args a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int A_BYTES = BM * kRowB;          // one plane of one stage
    constexpr int B_BYTES = kBN * kRowB;
    constexpr int STAGE = P * A_BYTES + B_BYTES;
    constexpr int A_GL = A_BYTES / (kThreads * 16);  // DMA instructions per thread per plane
    constexpr int B_GL = B_BYTES / (kThreads * 16);
    constexpr int MI = BM / 32;                  // 16-row fragments per wave

    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wr = w >> 1, wc = w & 1;

    // bijective XCD remap: blocks sharing bid % 8 get consecutive tile ids
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    const int S = (EPI == EPI_SLAB) ? a.ksplit : 1;  // split-K: slices of one tile are consecutive ids
    const int tile = id / S, slice = id - tile * S;
    const int rt = tile / a.n_tiles, ct = tile - rt * a.n_tiles;
    const int m0 = rt * BM;
    const int n0 = (EPI == EPI_SILU_MUL) ? ct * (kBN / 2) : ct * kBN;
    const int K = a.k / S;                            // this slice's K extent, from k_begin
    const int k_begin = slice * K;
    const size_t ldb = a.w_kblock ? (size_t)a.w_kblock : (size_t)a.k;  // W row stride (full K)

    // per-thread DMA sources: instruction j of this thread fills LDS bytes
    // j * 4096 + 16 t (lane-linear); that slot holds logical byte swz(.) of the tile
    const char* a_src[P][A_GL];
    const char* b_src[B_GL];
#pragma unroll
    for (int j = 0; j < A_GL; ++j) {
        const int b = swz(j * kThreads * 16 + t * 16);
        const int row = min(m0 + (b >> 7), a.m - 1);
#pragma unroll
        for (int p = 0; p < P; ++p)
            a_src[p][j] = reinterpret_cast<const char*>(a.a[p]) + ((size_t)row * a.lda) * 2 + (b & 127);
    }
#pragma unroll
    for (int j = 0; j < B_GL; ++j) {
        const int b = swz(j * kThreads * 16 + t * 16);
        const int src = b_src_row(EPI, n0, b >> 7, a.pair_off);
        b_src[j] = reinterpret_cast<const char*>(a.w) + (size_t)src * ldb * 2 + (b & 127);
    }
    const unsigned lds_base = (unsigned)(uintptr_t)lds;
    auto issue = [&](int stage, int kl) {
        const int k0 = k_begin + kl;
        const unsigned base = __builtin_amdgcn_readfirstlane(lds_base + stage * STAGE + w * 1024);  // wave-uniform
        const size_t koff =
            (a.w_kblock ? (size_t)(k0 / a.w_kblock) * a.n * a.w_kblock + k0 % a.w_kblock : (size_t)k0) * 2;
#pragma unroll
        for (int p = 0; p < P; ++p)
#pragma unroll
            for (int j = 0; j < A_GL; ++j) glds16(a_src[p][j] + (size_t)k0 * 2, base + p * A_BYTES + j * kThreads * 16);
#pragma unroll
        for (int j = 0; j < B_GL; ++j) glds16(b_src[j] + koff, base + P * A_BYTES + j * kThreads * 16);
    };
    constexpr int GL = P * A_GL + B_GL;  // DMA instructions per stage per thread

    f4 acc[MI][4];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

    const int fr = lane & 15, fq = lane >> 4;
    const int KT = K / kBK;
#pragma unroll
    for (int st = 0; st < kStages - 1; ++st)
        if (st < KT) issue(st, st * kBK);
    for (int kt = 0; kt < KT; ++kt) {
        // stage kt landed in every wave (counted vmcnt: later stages stay in flight), then
        // the raw barrier publishes it; every wave has also finished reading stage kt - 1,
        // whose buffer the next issue refills
        if (kt + kStages - 2 < KT) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"(GL * (kStages - 2)) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        if (kt + kStages - 1 < KT) issue((kt + kStages - 1) % kStages, (kt + kStages - 1) * kBK);
        const char* As = lds + (kt % kStages) * STAGE;
        const char* Bs = As + P * A_BYTES;
#pragma unroll
        for (int kk = 0; kk < kBK / 32; ++kk) {
            const int kb = kk * 64 + fq * 16;
            h8 bf[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                bf[j] = *reinterpret_cast<const h8*>(Bs + swz((wc * 64 + j * 16 + fr) * kRowB + kb));
#pragma unroll
            for (int i = 0; i < MI; ++i) {
                const int ab = swz((wr * (BM / 2) + i * 16 + fr) * kRowB + kb);
#pragma unroll
                for (int p = 0; p < P; ++p) {
                    const h8 af = *reinterpret_cast<const h8*>(As + p * A_BYTES + ab);
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf[j], acc[i][j], 0, 0, 0);
                }
            }
        }
    }

    // epilogue: C fragment (i, j) register r is row 16 i + 4 (lane >> 4) + r, column 16 j + (lane & 15)
#pragma unroll
    for (int i = 0; i < MI; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + wr * (BM / 2) + 16 * i + 4 * fq + r;
            if (m >= a.m) continue;
            if (EPI == EPI_SILU_MUL) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int gc = n0 + 32 * wc + 16 * j + fr;
                    const float v = silu_f(acc[i][j][r]) * acc[i][j + 2][r];
                    const size_t o = (size_t)m * a.ldy + gc;
                    if (a.y_hi) {  // the down GEMM's input planes, written directly
                        const _Float16 hi = (_Float16)v;
                        a.y_hi[o] = hi;
                        if (a.y_lo) a.y_lo[o] = (_Float16)(v - (float)hi);
                    } else {
                        a.y[o] = v;
                    }
                }
            } else {
                float* yrow = (EPI == EPI_SLAB ? a.slab + (size_t)slice * a.m * a.ldy : a.y) + (size_t)m * a.ldy;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int n = n0 + wc * 64 + 16 * j + fr;
                    if (EPI == EPI_ADD)
                        yrow[n] += acc[i][j][r];
                    else
                        yrow[n] = acc[i][j][r];
                }
            }
        }
    }
}

// RMSNorm (optional) + split of fp32 rows into fp16 planes: one workgroup per row.
// v = x * rsqrt(mean(x^2) + eps) * gamma (the reference's order, modeling_llama.py:
// 112-117); hi = fp16(v), lo = fp16(v - hi). The row stays in registers (NPT float4s
// per thread, k <= NPT * 1024): x and the slab slices are read once, x written once.
// KS > 0: the slice count is a constant and every slice's loads are issued before the
// first add (one memory round trip instead of one per slice); KS = 0: runtime ksplit.
template <int NPT, int KS, int BS = kThreads>
__global__ __launch_bounds__(BS) void rows_split_kernel(float* x, int ldx, int k, const void* gamma,
                                                       int g_dtype, float eps, _Float16* hi, _Float16* lo,
                                                       int ldh, const float* slab, int ksplit, int m, int lo8) {
    __shared__ float red[16];
    float* xr = x + (size_t)blockIdx.x * ldx;
    const int k4 = k / 4;
    float4 v[NPT];
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
        const int j = threadIdx.x + i * BS;
        v[i] = j < k4 ? reinterpret_cast<const float4*>(xr)[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (KS > 0 && slab) {  // split-K combine: x += slice 0 + slice 1 + ... (fixed order)
        float4 p[KS > 0 ? KS : 1][NPT];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const float4* sl = reinterpret_cast<const float4*>(slab + ((size_t)s * m + blockIdx.x) * ldx);
#pragma unroll
            for (int i = 0; i < NPT; ++i) {
                const int j = threadIdx.x + i * BS;
                p[s][i] = j < k4 ? sl[j] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int i = 0; i < NPT; ++i) {
                v[i].x += p[s][i].x; v[i].y += p[s][i].y; v[i].z += p[s][i].z; v[i].w += p[s][i].w;
            }
    } else if (slab) {
        for (int s = 0; s < ksplit; ++s) {
            const float4* sl = reinterpret_cast<const float4*>(slab + ((size_t)s * m + blockIdx.x) * ldx);
#pragma unroll
            for (int i = 0; i < NPT; ++i) {
                const int j = threadIdx.x + i * BS;
                if (j < k4) {
                    const float4 p = sl[j];
                    v[i].x += p.x; v[i].y += p.y; v[i].z += p.z; v[i].w += p.w;
                }
            }
        }
    }
    if (slab) {  // x written back
#pragma unroll
        for (int i = 0; i < NPT; ++i) {
            const int j = threadIdx.x + i * BS;
            if (j < k4) reinterpret_cast<float4*>(xr)[j] = v[i];
        }
        if (!hi) return;
    }
    float rstd = 1.f;
    if (gamma) {
        float ss = 0.f;
#pragma unroll
        for (int i = 0; i < NPT; ++i) ss += v[i].x * v[i].x + v[i].y * v[i].y + v[i].z * v[i].z + v[i].w * v[i].w;
        ss = block_sum(ss, red);
        rstd = 1.0f / sqrtf(ss / (float)k + eps);
    }
    if (!hi) return;
    _Float16* hr = hi + (size_t)blockIdx.x * ldh;
    _Float16* lr = lo ? lo + (size_t)blockIdx.x * ldh : nullptr;
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
        const int j = threadIdx.x + i * BS;
        if (j >= k4) continue;
        float e[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
        if (gamma) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float g = g_dtype == LLMI_F16 ? __half2float(static_cast<const __half*>(gamma)[4 * j + q])
                                                    : static_cast<const float*>(gamma)[4 * j + q];
                e[q] = (e[q] * rstd) * g;
            }
        }
        h4 h, l;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            h[q] = (_Float16)e[q];
            l[q] = (_Float16)(e[q] - (float)h[q]);
        }
        reinterpret_cast<h4*>(hr)[j] = h;
        if (lr && lo8)  // e4m3 bytes of the exact fp32 remainder
            reinterpret_cast<uint32_t*>(lr)[j] =
                lo8_pack4(e[0] - (float)h[0], e[1] - (float)h[1], e[2] - (float)h[2], e[3] - (float)h[3]);
        else if (lr)
            reinterpret_cast<h4*>(lr)[j] = l;
    }
}

template <int BM, int P, int EPI>
int launch3(const Gemm2Args& a, int grid, hipStream_t s) {
    constexpr size_t lds = kStages * (size_t)(P * BM * kRowB + kBN * kRowB);
    static const bool attr = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm2_kernel<BM, P, EPI>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
    }();
    LLMI_REQUIRE(attr, "gemm2: cannot raise the dynamic LDS limit");
    hipLaunchKernelGGL((gemm2_kernel<BM, P, EPI>), dim3(grid), dim3(kThreads), lds, s, a);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

template <int BM, int P>
int launch2(const Gemm2Args& a, int grid, hipStream_t s) {
    switch (a.epi) {
        case EPI_STORE: return launch3<BM, P, EPI_STORE>(a, grid, s);
        case EPI_ADD: return launch3<BM, P, EPI_ADD>(a, grid, s);
        case EPI_SILU_MUL: return launch3<BM, P, EPI_SILU_MUL>(a, grid, s);
        case EPI_SLAB: return launch3<BM, P, EPI_SLAB>(a, grid, s);
    }
    LLMI_REQUIRE(false, "gemm2: epilogue must be store, add, silu_mul or slab");
}

}  // namespace

bool gemm2_supported(int n, int k, int epi) {
    const int ncols = (epi == EPI_SILU_MUL) ? n / 2 : n;
    const int tile = (epi == EPI_SILU_MUL) ? kBN / 2 : kBN;
    return n > 0 && k > 0 && ncols % tile == 0 && k % kBK == 0;
}

int gemm2_bm(const Gemm2Args& a) {
    if (a.epi == EPI_SLAB) return 128;  // split-K supplies the workgroups
    const int ncols = (a.epi == EPI_SILU_MUL) ? a.n / 2 : a.n;
    const int nt = ncols / ((a.epi == EPI_SILU_MUL) ? kBN / 2 : kBN);
    // 128-row tiles unless that leaves CUs idle
    return ((a.m + 127) / 128) * nt >= 256 ? 128 : 64;
}

int gemm2_launch(Gemm2Args a, hipStream_t s) {
    LLMI_REQUIRE(a.a[0] && a.w && a.m > 0, "gemm2: null operand or empty M");
    LLMI_REQUIRE(a.planes == 1 || (a.planes == 2 && a.a[1]), "gemm2: planes must be 1 or 2 (with a[1])");
    LLMI_REQUIRE(gemm2_supported(a.n, a.k, a.epi), "gemm2: N a multiple of 128 (gate_up: 2 x 64), K of 64");
    LLMI_REQUIRE(a.epi == EPI_SILU_MUL ? (a.y || a.y_hi) : a.y != nullptr, "gemm2: null output");
    LLMI_REQUIRE(a.lda % 8 == 0 && (reinterpret_cast<uintptr_t>(a.a[0]) & 15) == 0 &&
                     (a.planes == 1 || (reinterpret_cast<uintptr_t>(a.a[1]) & 15) == 0),
                 "gemm2: A planes must be 16-B aligned with lda % 8 == 0");
    LLMI_REQUIRE((reinterpret_cast<uintptr_t>(a.w) & 15) == 0, "gemm2: W must be 16-B aligned");
    LLMI_REQUIRE(a.w_kblock == 0 || (a.w_kblock % kBK == 0 && a.k % a.w_kblock == 0 && a.epi != EPI_SILU_MUL),
                 "gemm2: w_kblock must be a multiple of 64 dividing K (not with the gate_up pairing)");
    LLMI_REQUIRE(a.epi != EPI_SILU_MUL || a.pair_off == a.n / 2, "gemm2: gate_up pair offset must be N / 2");
    const int ncols = (a.epi == EPI_SILU_MUL) ? a.n / 2 : a.n;
    a.n_tiles = ncols / ((a.epi == EPI_SILU_MUL) ? kBN / 2 : kBN);
    if (a.epi == EPI_SLAB) {
        LLMI_REQUIRE(a.slab && a.ksplit >= 1 && a.k % (a.ksplit * kBK) == 0 &&
                         (a.w_kblock == 0 || (a.k / a.ksplit) % a.w_kblock == 0),
                     "gemm2: split-K needs a slab and K / ksplit a multiple of 64 (and of w_kblock)");
    } else {
        a.ksplit = 1;
    }
    const int bm = gemm2_bm(a);
    const int grid = ((a.m + bm - 1) / bm) * a.n_tiles * a.ksplit;
    if (bm == 128) return a.planes == 2 ? launch2<128, 2>(a, grid, s) : launch2<128, 1>(a, grid, s);
    return a.planes == 2 ? launch2<64, 2>(a, grid, s) : launch2<64, 1>(a, grid, s);
}

int rows_split_launch(float* x, int ldx, int m, int k, const void* gamma, int g_dtype, float eps, _Float16* hi,
                      _Float16* lo, int ldh, hipStream_t s, const float* slab, int ksplit, bool lo8) {
    LLMI_REQUIRE(x && (hi || slab) && m > 0 && k > 0 && k % 4 == 0 && ldx % 4 == 0 && ldh % 4 == 0,
                 "rows_split: bad arguments");
    LLMI_REQUIRE(!slab || (ksplit >= 1 && ldx == k), "rows_split: slab rows must be dense (ldx == k)");
    LLMI_REQUIRE(k <= 8 * 4 * kThreads, "rows_split: rows longer than 8192 are not supported");
    const int npt = (k / 4 + kThreads - 1) / kThreads;
    // slice counts the prefill uses get the all-loads-first instance (o_proj 2, down 8)
    const int ks = !slab ? 0 : (ksplit == 2 || (ksplit == 8 && npt <= 5)) ? ksplit : 0;
#define RS_LAUNCH(N, S) \
    hipLaunchKernelGGL((rows_split_kernel<N, S>), dim3(m), dim3(kThreads), 0, s, x, ldx, k, gamma, g_dtype, eps, hi, lo, \
                       ldh, slab, ksplit, m, lo8 ? 1 : 0)
#define RS_KS(N) \
    do {                                  \
        if (ks == 2)                      \
            RS_LAUNCH(N, 2);              \
        else if (ks == 8 && (N) <= 5)     \
            RS_LAUNCH(N, ((N) <= 5 ? 8 : 0)); \
        else                              \
            RS_LAUNCH(N, 0);              \
    } while (0)
    if (k / 4 <= 1024 && !noexp_rn()) {  // one float4 per thread: 16 waves a row (resid_norm's A/B)
        if (ks == 2)
            hipLaunchKernelGGL((rows_split_kernel<1, 2, 1024>), dim3(m), dim3(1024), 0, s, x, ldx, k, gamma, g_dtype, eps,
                               hi, lo, ldh, slab, ksplit, m, lo8 ? 1 : 0);
        else if (ks == 8)
            hipLaunchKernelGGL((rows_split_kernel<1, 8, 1024>), dim3(m), dim3(1024), 0, s, x, ldx, k, gamma, g_dtype, eps,
                               hi, lo, ldh, slab, ksplit, m, lo8 ? 1 : 0);
        else
            hipLaunchKernelGGL((rows_split_kernel<1, 0, 1024>), dim3(m), dim3(1024), 0, s, x, ldx, k, gamma, g_dtype, eps,
                               hi, lo, ldh, slab, ksplit, m, lo8 ? 1 : 0);
    } else if (npt <= 4)
        RS_KS(4);
    else if (npt <= 5)
        RS_KS(5);
    else
        RS_KS(8);
#undef RS_KS
#undef RS_LAUNCH
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

// ------------------------------------------------ llmi_linear on the prefill GEMMs
// The layer API's projections (launchLinearGemm, linear.cu:38-104: cublasGemmEx over
// [num_tokens, k] x [n, k]^T) for fp16 weights: the fp32 input split into hi/lo planes
// (fp32-faithful, as the engine's prefill), then the 256 x 256 ping-pong GEMM (gemm3)
// when the rows fill its tiles, else gemm2; split-K slices when the tiles alone would
// leave CUs idle, summed in slice order by slab_sum_kernel (deterministic). Workspace:
// one growing device buffer per stream (a grow waits for the stream first).
namespace {
__global__ __launch_bounds__(kThreads) void planes_kernel(const float4* x, _Float16* hi, _Float16* lo, size_t n4) {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < n4; i += (size_t)gridDim.x * kThreads) {
        const float4 v = x[i];
        const float e[4] = {v.x, v.y, v.z, v.w};
        h4 h, l;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            h[q] = (_Float16)e[q];
            l[q] = (_Float16)(e[q] - (float)h[q]);
        }
        reinterpret_cast<h4*>(hi)[i] = h;
        reinterpret_cast<h4*>(lo)[i] = l;
    }
}
__global__ __launch_bounds__(kThreads) void slab_sum_kernel(const float4* slab, float4* y, int ks, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < n4; i += (size_t)gridDim.x * kThreads) {
        float4 a = slab[i];
        for (int s = 1; s < ks; ++s) {
            const float4 b = slab[(size_t)s * n4 + i];
            a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        }
        y[i] = a;
    }
}
// ResidEpi (kernels.h), one workgroup per row: t = slice 0 + slice 1 + ... (slab_sum_kernel's
// order), r = resid + t (add_resid_rmsnorm_kernel's / add_resid_kernel's order), then the
// row's RMSNorm * gamma -- the launchLinearGemm + launchFusedAddBiasResidualRMSNorm pair
// (or + launchAddResidual + the next layer's launchRMSNorm) in one pass over the slices.
template <int NPT, int BS = kThreads>
__global__ __launch_bounds__(BS) void resid_norm_kernel(float* resid, const float* slab, int ks, int m, int n,
                                                        float* out, const void* gamma, int g_dtype, float eps) {
    __shared__ float red[16];
    const size_t row = blockIdx.x;
    const int n4 = n / 4;
    const size_t plane4 = (size_t)m * n4;
    const float4* sl = reinterpret_cast<const float4*>(slab) + row * n4;
    float4* rr = reinterpret_cast<float4*>(resid) + row * n4;
    float4 v[NPT];
    float ss = 0.f;
    // (an instance with the 8 slices' loads all issued first measured 22.8 vs 20.1 us at
    // 512 x 4096: the slice-at-a-time loop below keeps more rows in flight per CU)
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
        const int j = threadIdx.x + i * BS;
        v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (j >= n4) continue;
        float4 t = sl[j];
        for (int s = 1; s < ks; ++s) {
            const float4 b = sl[(size_t)s * plane4 + j];
            t.x += b.x; t.y += b.y; t.z += b.z; t.w += b.w;
        }
        const float4 r = rr[j];
        v[i] = make_float4(r.x + t.x, r.y + t.y, r.z + t.z, r.w + t.w);
        rr[j] = v[i];
        ss += v[i].x * v[i].x + v[i].y * v[i].y + v[i].z * v[i].z + v[i].w * v[i].w;
    }
    if (!out) return;
    float rstd = 1.f;
    if (gamma) {
        ss = block_sum(ss, red);
        rstd = 1.0f / sqrtf(ss / (float)n + eps);
    }
    float4* o = reinterpret_cast<float4*>(out) + row * n4;
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
        const int j = threadIdx.x + i * BS;
        if (j >= n4) continue;
        float e[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
        if (gamma) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float g = g_dtype == LLMI_F16 ? __half2float(static_cast<const __half*>(gamma)[4 * j + q])
                                                    : static_cast<const float*>(gamma)[4 * j + q];
                e[q] = g * (e[q] * rstd);
            }
        }
        o[j] = make_float4(e[0], e[1], e[2], e[3]);
    }
}
int resid_norm_launch(const ResidEpi& re, const float* slab, int ks, int m, int n, hipStream_t s) {
    const int npt = (n / 4 + kThreads - 1) / kThreads;
    if (n / 4 <= 1024 && !noexp_rn())  // one float4 per thread: 16 waves a row keep more loads in flight
        hipLaunchKernelGGL((resid_norm_kernel<1, 1024>), dim3(m), dim3(1024), 0, s, re.resid, slab, ks, m, n, re.out,
                           re.gamma, re.g_dtype, re.eps);
    else if (npt <= 4)
        hipLaunchKernelGGL(resid_norm_kernel<4>, dim3(m), dim3(kThreads), 0, s, re.resid, slab, ks, m, n, re.out,
                           re.gamma, re.g_dtype, re.eps);
    else
        hipLaunchKernelGGL(resid_norm_kernel<8>, dim3(m), dim3(kThreads), 0, s, re.resid, slab, ks, m, n, re.out,
                           re.gamma, re.g_dtype, re.eps);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}
bool resid_epi_ok(const ResidEpi* re, int n) {
    return !re || (re->resid && n % 4 == 0 && n <= 8 * 4 * kThreads &&
                   (reinterpret_cast<uintptr_t>(re->resid) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(re->out) & 15) == 0 &&
                   (re->g_dtype == LLMI_F16 || re->g_dtype == LLMI_F32));
}
// keyed by (device, stream): the null stream is the same handle on every device
std::mutex g_ws_mu;
std::map<std::pair<int, hipStream_t>, std::pair<void*, size_t>> g_ws;
int linear_workspace(hipStream_t s, size_t bytes, char** out) {
    int dev = 0;
    LLMI_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lock(g_ws_mu);
    auto& e = g_ws[{dev, s}];
    if (bytes > e.second) {
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        LLMI_HIP(hipStreamIsCapturing(s, &cap));
        LLMI_REQUIRE(cap == hipStreamCaptureStatusNone,
                     "linear_mfma: the workspace must grow, which cannot happen while the stream is capturing "
                     "(run the same shapes once before capture)");
        if (e.first) {  // earlier launches on this stream may still read it
            LLMI_HIP(hipStreamSynchronize(s));
            LLMI_HIP(hipFree(e.first));
            e = {nullptr, 0};
        }
        LLMI_HIP(hipMalloc(&e.first, bytes));
        e.second = bytes;
    }
    *out = static_cast<char*>(e.first);
    return LLMI_OK;
}
int grid_of(size_t n4) { return (int)std::min<size_t>((n4 + kThreads - 1) / kThreads, 4096); }
// gemm3 stream-K state per (device, stream): partial slots, and the control words (epoch,
// finished count: 256 B) followed by the flags, all zeroed when allocated; grown like the
// linear workspace
std::map<std::pair<int, hipStream_t>, std::pair<std::pair<void*, size_t>, std::pair<unsigned*, size_t>>> g_sk;
constexpr size_t kSkCtlBytes = kSkCtlWords * sizeof(unsigned);
int sk_workspace(hipStream_t s, size_t slab_bytes, size_t flag_bytes, float** slab, unsigned** flags, unsigned** ctl) {
    flag_bytes += kSkCtlBytes;
    int dev = 0;
    LLMI_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lock(g_ws_mu);
    auto& e = g_sk[{dev, s}];
    if (slab_bytes > e.first.second || flag_bytes > e.second.second) {
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        LLMI_HIP(hipStreamIsCapturing(s, &cap));
        LLMI_REQUIRE(cap == hipStreamCaptureStatusNone,
                     "gemm3 stream-K: the workspace must grow, which cannot happen while the stream is capturing "
                     "(run the same shapes once before capture)");
        LLMI_HIP(hipStreamSynchronize(s));
        const size_t sb = std::max(slab_bytes, e.first.second), fb = std::max(std::max(flag_bytes, e.second.second), (size_t)4);
        if (e.first.first) LLMI_HIP(hipFree(e.first.first));
        if (e.second.first) LLMI_HIP(hipFree(e.second.first));
        e = {{nullptr, 0}, {nullptr, 0}};
        LLMI_HIP(hipMalloc(&e.first.first, sb));
        LLMI_HIP(hipMalloc(reinterpret_cast<void**>(&e.second.first), fb));
        LLMI_HIP(hipMemset(e.second.first, 0, fb));
        e.first.second = sb;
        e.second.second = fb;
    }
    *slab = static_cast<float*>(e.first.first);
    *ctl = e.second.first;
    *flags = e.second.first + kSkCtlBytes / sizeof(unsigned);
    return LLMI_OK;
}
// sticky device error bits per (device, stream) for launches whose caller passes no error
// word (the layer API): allocated once and zeroed, read and cleared by stream_errors()
std::map<std::pair<int, hipStream_t>, int*> g_err;
int stream_error_word(hipStream_t s, int** out) {
    int dev = 0;
    LLMI_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lock(g_ws_mu);
    int*& e = g_err[{dev, s}];
    if (!e) {
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        LLMI_HIP(hipStreamIsCapturing(s, &cap));
        LLMI_REQUIRE(cap == hipStreamCaptureStatusNone,
                     "stream error word: first use cannot happen while the stream is capturing");
        LLMI_HIP(hipMalloc(reinterpret_cast<void**>(&e), sizeof(int)));
        LLMI_HIP(hipMemsetAsync(e, 0, sizeof(int), s));
    }
    *out = e;
    return LLMI_OK;
}
int cu_count() {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    return n;
}
// stream-K for a gemm3 launch of these shapes when it keeps at most 3 partial slots per tile
// (q/k/v and gate_up at 512 rows; o_proj / down, whose tiles would split 8 ways, keep the
// split-K slices summed by their consumer). LLMI_SK=0 turns it off.
bool sk_setup(Gemm2Args& g, hipStream_t s) {
    static const bool off = [] {
        const char* e = std::getenv("LLMI_SK");
        return e && std::string(e) == "0";
    }();
    if (off) return false;
    // one fp16 plane (the fp16-activation prefill): since the plain kernel's steady tiles run
    // paired (gemm3.hip, round 6) it is the faster form -- 512-row prefill 9.37-9.41 -> 9.17-9.18
    // ms on one box, while two planes and fp8 lo planes stay faster on stream-K (r06m)
    if (g.planes == 1 && !g.lo8) return false;
    const int n_cu = cu_count();
    const Gemm3SkPlan p = gemm3_sk_plan(g.m, g.n, g.k, g.epi, g.planes, g.lo8, n_cu);
    if (p.pmax < 1 || p.pmax > 3) return false;
    if (sk_workspace(s, p.slab_bytes, p.flag_bytes, &g.sk_slab, &g.sk_flags, &g.sk_ctl) != LLMI_OK) return false;
    // a partial that never arrives sets bit 16 somewhere the caller can read (stream_errors)
    if (!g.err && stream_error_word(s, &g.err) != LLMI_OK) return false;
    g.sk_grid = n_cu;
    return true;
}
}  // namespace

bool gemm3_sk_attach(Gemm2Args& g, hipStream_t s) { return sk_setup(g, s); }

int stream_errors(hipStream_t s, int* flags) {
    LLMI_REQUIRE(flags, "stream_errors: flags must not be null");
    *flags = 0;
    int dev = 0;
    LLMI_HIP(hipGetDevice(&dev));
    int* e = nullptr;
    {
        std::lock_guard<std::mutex> lock(g_ws_mu);
        auto it = g_err.find({dev, s});
        if (it != g_err.end()) e = it->second;
    }
    if (!e) return LLMI_OK;  // nothing on this stream could have set one
    LLMI_HIP(hipMemcpyAsync(flags, e, sizeof(int), hipMemcpyDeviceToHost, s));
    LLMI_HIP(hipMemsetAsync(e, 0, sizeof(int), s));
    LLMI_HIP(hipStreamSynchronize(s));
    return LLMI_OK;
}

bool linear_mfma_supported(int m, int n, int k) {
    return m >= 16 && k % 64 == 0 && gemm2_supported(n, k, EPI_STORE);
}

int linear_mfma_launch(const float* x, const void* w, float* y, int m, int n, int k, hipStream_t s,
                       const ResidEpi* re, const float** slab_out, int* ks_out) {
    LLMI_REQUIRE(x && w && (y || re || (slab_out && ks_out)) && linear_mfma_supported(m, n, k),
                 "linear_mfma: N a multiple of 128, K of 64, M >= 16");
    LLMI_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0,
                 "linear_mfma: x and y must be 16-B aligned");
    LLMI_REQUIRE(resid_epi_ok(re, n), "linear_mfma: residual epilogue needs n <= 8192 (multiple of 4), 16-B aligned "
                                      "residual / out and an fp16 or fp32 gamma");
    const bool g3 = m >= 256 && gemm3_supported(n, k, EPI_STORE, 1);
    const int tiles = g3 ? ((m + 255) / 256) * (n / 256) : ((m + 127) / 128) * (n / kBN);
    // (stream-K measured slower here than the 2-slice split: q/k/v 112 vs ~108 us with the
    // slices' sum, its 256-KB partial slots being on the critical path; gate_up gains.
    // LLMI_SK_LINEAR=1 turns it on for these projections, for A/B)
    static const bool sk_lin = [] {
        const char* e = std::getenv("LLMI_SK_LINEAR");
        return e && e[0] == '1';
    }();
    Gemm2Args skg;
    skg.m = m; skg.n = n; skg.k = k; skg.planes = 2; skg.epi = EPI_STORE;
    const bool sk = sk_lin && g3 && sk_setup(skg, s);
    int ks = 1;  // K slices while the tiles leave more than a third of the 256 CUs idle
    while (!sk && tiles * ks < 160 && ks < 8) {
        const int nk = ks * 2;
        if (g3 ? !gemm3_supported(n, k, EPI_SLAB, nk) : k % (nk * kBK) != 0) break;
        ks = nk;
    }
    const size_t plane = ((size_t)m * k * 2 + 255) / 256 * 256;
    const bool raw = slab_out != nullptr;  // the slices themselves, for a consumer that sums them
    const size_t slab = ks > 1 || re || raw ? (size_t)ks * m * n * 4 : 0;  // residual / raw forms: >= 1 slice
    char* ws = nullptr;
    LLMI_TRY(linear_workspace(s, 2 * plane + slab, &ws));
    _Float16* hi = reinterpret_cast<_Float16*>(ws);
    _Float16* lo = reinterpret_cast<_Float16*>(ws + plane);
    const size_t n4x = (size_t)m * k / 4;
    hipLaunchKernelGGL(planes_kernel, dim3(grid_of(n4x)), dim3(kThreads), 0, s, reinterpret_cast<const float4*>(x), hi,
                       lo, n4x);
    LLMI_HIP(hipGetLastError());
    Gemm2Args g;
    g.a[0] = hi; g.a[1] = lo; g.planes = 2; g.lda = k;
    g.w = w; g.m = m; g.n = n; g.k = k; g.ldy = n;
    if (sk) { g.sk_slab = skg.sk_slab; g.sk_flags = skg.sk_flags; g.sk_ctl = skg.sk_ctl; g.sk_grid = skg.sk_grid; g.err = skg.err; }
    float* sl = reinterpret_cast<float*>(ws + 2 * plane);
    if (ks > 1) {
        g.epi = EPI_SLAB; g.ksplit = ks; g.slab = sl; g.y = re || raw ? sl : y;
    } else {
        g.epi = EPI_STORE; g.y = re || raw ? sl : y;
    }
    LLMI_TRY(g3 ? gemm3_launch(g, s) : gemm2_launch(g, s));
    if (raw) {
        *slab_out = sl;
        *ks_out = ks;
        return LLMI_OK;
    }
    if (re) return resid_norm_launch(*re, sl, ks, m, n, s);
    if (ks > 1) {
        const size_t n4y = (size_t)m * n / 4;
        hipLaunchKernelGGL(slab_sum_kernel, dim3(grid_of(n4y)), dim3(kThreads), 0, s,
                           reinterpret_cast<const float4*>(g.slab), reinterpret_cast<float4*>(y), ks, n4y);
        LLMI_HIP(hipGetLastError());
    }
    return LLMI_OK;
}

// LLaMAFFNLayer::forward (ffn.cpp:52-93) for the context phase in three launches on the
// matrix cores: x -> fp16 hi/lo planes; gate_up whose epilogue writes silu(g) * u straight
// as the down GEMM's input planes (gemm3 / gemm2 EPI_SILU_MUL, the engine prefill's
// form: no fp32 [m, 2 I] product and no separate SiLU pass); down with the K slices of
// llmi_linear summed in slice order. fp16 weights; fp32 x and y.
bool ffn_mfma_supported(int m, int hidden, int inter) {
    const bool g3 = m >= 256 && gemm3_supported(2 * inter, hidden, EPI_SILU_MUL, 1);
    return m >= 16 && hidden % 64 == 0 && inter % 64 == 0 &&
           (g3 || gemm2_supported(2 * inter, hidden, EPI_SILU_MUL)) && linear_mfma_supported(m, hidden, inter);
}

int ffn_mfma_launch(const float* x, const void* w_gu, const void* w_down, float* y, int m, int hidden, int inter,
                    hipStream_t s, const ResidEpi* re) {
    LLMI_REQUIRE(x && w_gu && w_down && (y || re) && ffn_mfma_supported(m, hidden, inter),
                 "ffn_mfma: unsupported shape (M >= 16, hidden and inter multiples of 64 the GEMMs tile)");
    LLMI_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0,
                 "ffn_mfma: x and y must be 16-B aligned");
    LLMI_REQUIRE(resid_epi_ok(re, hidden), "ffn_mfma: residual epilogue needs hidden <= 8192 (multiple of 4), 16-B "
                                           "aligned residual / out and an fp16 or fp32 gamma");
    const bool g3gu = m >= 256 && gemm3_supported(2 * inter, hidden, EPI_SILU_MUL, 1);
    const bool g3d = m >= 256 && gemm3_supported(hidden, inter, EPI_STORE, 1);
    const int tiles = g3d ? ((m + 255) / 256) * (hidden / 256) : ((m + 127) / 128) * (hidden / kBN);
    int ks = 1;
    while (tiles * ks < 160 && ks < 8) {
        const int nk = ks * 2;
        if (g3d ? !gemm3_supported(hidden, inter, EPI_SLAB, nk) : inter % (nk * kBK) != 0) break;
        ks = nk;
    }
    const size_t xplane = ((size_t)m * hidden * 2 + 255) / 256 * 256;
    const size_t aplane = ((size_t)m * inter * 2 + 255) / 256 * 256;
    const size_t slab = ks > 1 || re ? (size_t)ks * m * hidden * 4 : 0;
    char* ws = nullptr;
    LLMI_TRY(linear_workspace(s, 2 * xplane + 2 * aplane + slab, &ws));
    _Float16* xh = reinterpret_cast<_Float16*>(ws);
    _Float16* xl = reinterpret_cast<_Float16*>(ws + xplane);
    _Float16* ah = reinterpret_cast<_Float16*>(ws + 2 * xplane);
    _Float16* al = reinterpret_cast<_Float16*>(ws + 2 * xplane + aplane);
    const size_t n4x = (size_t)m * hidden / 4;
    hipLaunchKernelGGL(planes_kernel, dim3(grid_of(n4x)), dim3(kThreads), 0, s, reinterpret_cast<const float4*>(x), xh,
                       xl, n4x);
    LLMI_HIP(hipGetLastError());
    Gemm2Args g;
    g.a[0] = xh; g.a[1] = xl; g.planes = 2; g.lda = hidden;
    g.w = w_gu; g.m = m; g.n = 2 * inter; g.k = hidden;
    g.epi = EPI_SILU_MUL; g.pair_off = inter; g.y = nullptr; g.y_hi = ah; g.y_lo = al; g.ldy = inter;
    if (g3gu) sk_setup(g, s);  // stream-K when its tiles leave CUs idle
    LLMI_TRY(g3gu ? gemm3_launch(g, s) : gemm2_launch(g, s));
    Gemm2Args d;
    d.a[0] = ah; d.a[1] = al; d.planes = 2; d.lda = inter;
    d.w = w_down; d.m = m; d.n = hidden; d.k = inter; d.ldy = hidden;
    float* sl = reinterpret_cast<float*>(ws + 2 * xplane + 2 * aplane);
    if (ks > 1) {
        d.epi = EPI_SLAB; d.ksplit = ks; d.slab = sl; d.y = re ? sl : y;
    } else {
        d.epi = EPI_STORE; d.y = re ? sl : y;
    }
    LLMI_TRY(g3d ? gemm3_launch(d, s) : gemm2_launch(d, s));
    if (re) return resid_norm_launch(*re, sl, ks, m, hidden, s);
    if (ks > 1) {
        const size_t n4y = (size_t)m * hidden / 4;
        hipLaunchKernelGGL(slab_sum_kernel, dim3(grid_of(n4y)), dim3(kThreads), 0, s,
                           reinterpret_cast<const float4*>(d.slab), reinterpret_cast<float4*>(y), ks, n4y);
        LLMI_HIP(hipGetLastError());
    }
    return LLMI_OK;
}

}  // namespace llmi
