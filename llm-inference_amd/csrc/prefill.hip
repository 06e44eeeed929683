// Prefill (context) attention for M prompt rows at positions p0 .. p0+M-1
// (SURVEY.md §8 a15, config 3). Replaces LLaMAContextAttentionLayer's middle
// (context_attention.cpp:108-161): launchAddFusedQKVBiasTransposeAndRoPE
// (qkv_bias_and_RoPE.cu:49-144), launchConcatKVCache (concat_past_kv.cu:16-143),
// the QK^T strided-batched GEMM, launchScaleMaskAndSoftmax with
// launchBuildCausalMasks (attn_softmax_kernel.cu:79-377, build_causal_mask.cu:29),
// the PV GEMM and launchTransposeOutRemovePadding -- as two kernels:
//
//   rope_kv_prefill: rotate q (in place) and k of every row with the engine's
//     cos/sin table, write k, v into cache slots p0 + m (the decode kernel's
//     exact arithmetic, so a prefilled slot equals a decoded one);
//   attn_prefill: causal flash attention, one workgroup per (head, 32 query
//     rows), 32-key chunks of the cache staged in LDS, online softmax in fp32;
//     the causal mask is the index test key <= p0 + row (never materialised).
//
// Roofline: the attention is ~2.1 GFLOP per 7B layer at M = 512 (4 * heads *
// d * M^2 / 2), bound by LDS operand traffic in this fp32 form; the GEMMs
// around it dominate prefill (gemm.hip).
#include <algorithm>
#include <atomic>

#include <cstdlib>

#include "kernels.h"

namespace llmi {
namespace {

constexpr int D = 128;
constexpr int kThreads = 256;
constexpr int QB = 32;   // query rows per workgroup
constexpr int KC = 32;   // keys per LDS chunk
constexpr int kLdq = D + 4;  // padded fp32 row stride (conflict-free float4 reads)

__device__ __forceinline__ void store_c(__half* p, float v) { *p = __float2half(v); }
__device__ __forceinline__ void store_c(float* p, float v) { *p = v; }
__device__ __forceinline__ float load_c(const __half* p) { return __half2float(*p); }
__device__ __forceinline__ float load_c(const float* p) { return *p; }

// grid (M), block 256: row m of qkv [M, (heads + 2 kv) * D]; with qkv2 (the second
// K slice of the qkv GEMM) each element is qkv + qkv2 first, and the summed, rotated q
// is what stays in qkv. Thread work item e: head e / 16, dims 4 (e % 16) .. + 3 and
// their RoPE partners + 64, as float4s (the pair expression is the decode kernel's).
template <typename KT>
__global__ void rope_kv_prefill_kernel(float* qkv, const float* qkv2, int ld, int p0, int heads, int kv_heads,
                                       const float* rope_tab, KT* k_cache, KT* v_cache, int max_seq) {
    const int m = blockIdx.x, pos = p0 + m;
    float* row = qkv + (size_t)m * ld;
    const float* row2 = qkv2 ? qkv2 + (size_t)m * ld : nullptr;
    const float4* cs4 = reinterpret_cast<const float4*>(rope_tab + (size_t)pos * D);  // (cos, sin) pairs
    for (int e = threadIdx.x; e < (heads + kv_heads) * (D / 8); e += blockDim.x) {
        const int hh = e / (D / 8), i = 4 * (e % (D / 8));
        float* p = row + (size_t)hh * D;
        float4 x0 = *reinterpret_cast<const float4*>(p + i), x1 = *reinterpret_cast<const float4*>(p + i + D / 2);
        if (row2) {
            const float* p2 = row2 + (size_t)hh * D;
            const float4 y0 = *reinterpret_cast<const float4*>(p2 + i), y1 = *reinterpret_cast<const float4*>(p2 + i + D / 2);
            x0.x += y0.x; x0.y += y0.y; x0.z += y0.z; x0.w += y0.w;
            x1.x += y1.x; x1.y += y1.y; x1.z += y1.z; x1.w += y1.w;
        }
        const float4 c01 = cs4[i / 2], c23 = cs4[i / 2 + 1];  // (c, s) of dims i .. i + 3
        const float c[4] = {c01.x, c01.z, c23.x, c23.z}, sn[4] = {c01.y, c01.w, c23.y, c23.w};
        const float a0[4] = {x0.x, x0.y, x0.z, x0.w}, a1[4] = {x1.x, x1.y, x1.z, x1.w};
        float r0[4], r1[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            r0[j] = a0[j] * c[j] - a1[j] * sn[j];
            r1[j] = a1[j] * c[j] + a0[j] * sn[j];
        }
        if (hh < heads) {
            *reinterpret_cast<float4*>(p + i) = make_float4(r0[0], r0[1], r0[2], r0[3]);
            *reinterpret_cast<float4*>(p + i + D / 2) = make_float4(r1[0], r1[1], r1[2], r1[3]);
        } else {
            KT* kc = k_cache + ((size_t)(hh - heads) * max_seq + pos) * D;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                store_c(kc + i + j, r0[j]);
                store_c(kc + i + j + D / 2, r1[j]);
            }
        }
    }
    const size_t vo = (size_t)(heads + kv_heads) * D;
    for (int e = threadIdx.x; e < kv_heads * (D / 4); e += blockDim.x) {
        const int hh = e / (D / 4), d = 4 * (e % (D / 4));
        float4 v = *reinterpret_cast<const float4*>(row + vo + 4 * e);
        if (row2) {
            const float4 y = *reinterpret_cast<const float4*>(row2 + vo + 4 * e);
            v.x += y.x; v.y += y.y; v.z += y.z; v.w += y.w;
        }
        KT* vc = v_cache + ((size_t)hh * max_seq + pos) * D + d;
        store_c(vc, v.x);
        store_c(vc + 1, v.y);
        store_c(vc + 2, v.z);
        store_c(vc + 3, v.w);
    }
}

// grid (ceil(M / QB), heads), block 256. Thread t: query row qi = t >> 3 of the
// block; for scores keys kg + 8 c (kg = t & 7, c < 4) of the chunk; for the
// output dims 4 kg + 32 r + {0..3} (r < 4).
template <typename KT>
__global__ __launch_bounds__(kThreads) void attn_prefill_kernel(const float* qkv, int ld, int m_rows, int p0,
                                                                int heads, int kv_heads, const KT* k_cache,
                                                                const KT* v_cache, int max_seq, float* out,
                                                                int ldo) {
    __shared__ float q_s[QB * kLdq];
    __shared__ float k_s[KC * kLdq];
    __shared__ float v_s[KC * D];
    __shared__ float p_s[QB * (KC + 1)];

    const int t = threadIdx.x;
    const int qb = gridDim.x - 1 - blockIdx.x;  // longest (latest) query blocks first
    const int h = blockIdx.y;
    const int kvh = h / (heads / kv_heads);
    const int qi = t >> 3, kg = t & 7;
    const int q_first = qb * QB;
    const int q_row = min(q_first + qi, m_rows - 1);  // clamp: rows past M compute, never store
    const float qscale = 1.0f / sqrtf((float)D);

    // stage q (already rotated), scaled as in the decode kernel
    for (int e = t; e < QB * D; e += kThreads) {
        const int r = e / D, d = e % D;
        const int qr = min(q_first + r, m_rows - 1);
        q_s[r * kLdq + d] = qkv[(size_t)qr * ld + (size_t)h * D + d] * qscale;
    }

    const KT* kc = k_cache + (size_t)kvh * max_seq * D;
    const KT* vc = v_cache + (size_t)kvh * max_seq * D;
    const int my_pos = p0 + q_row;
    const int kend = p0 + min(q_first + QB, m_rows);  // keys [0, kend)

    float m_run = -INFINITY, l_run = 0.f;
    float o[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) o[i] = 0.f;

    for (int k0 = 0; k0 < kend; k0 += KC) {
        __syncthreads();
        for (int e = t; e < KC * D; e += kThreads) {
            const int r = e / D, d = e % D;
            const int j = min(k0 + r, kend - 1);
            k_s[r * kLdq + d] = load_c(kc + (size_t)j * D + d);
            v_s[r * D + d] = load_c(vc + (size_t)j * D + d);
        }
        __syncthreads();

        float s[4] = {0.f, 0.f, 0.f, 0.f};
        const float* qp = q_s + qi * kLdq;
#pragma unroll 4
        for (int d = 0; d < D; d += 4) {
            const float4 qv = *reinterpret_cast<const float4*>(qp + d);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float4 kv = *reinterpret_cast<const float4*>(k_s + (kg + 8 * c) * kLdq + d);
                s[c] = fmaf(qv.x, kv.x, s[c]);
                s[c] = fmaf(qv.y, kv.y, s[c]);
                s[c] = fmaf(qv.z, kv.z, s[c]);
                s[c] = fmaf(qv.w, kv.w, s[c]);
            }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int j = k0 + kg + 8 * c;
            if (j > my_pos || j >= kend) s[c] = -INFINITY;  // causal (build_causal_mask.cu:29)
            mx = fmaxf(mx, s[c]);
        }
        mx = fmaxf(mx, __shfl_xor(mx, 1));
        mx = fmaxf(mx, __shfl_xor(mx, 2));
        mx = fmaxf(mx, __shfl_xor(mx, 4));
        const float m_new = fmaxf(m_run, mx);  // finite: key 0 is always visible
        const float alpha = expf(m_run - m_new);
        float ps = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const float p = expf(s[c] - m_new);
            ps += p;
            p_s[qi * (KC + 1) + kg + 8 * c] = p;
        }
        ps += __shfl_xor(ps, 1);
        ps += __shfl_xor(ps, 2);
        ps += __shfl_xor(ps, 4);
        l_run = l_run * alpha + ps;
        m_run = m_new;
        __builtin_amdgcn_wave_barrier();  // p_s row is written and read by the same 8 lanes

#pragma unroll
        for (int i = 0; i < 16; ++i) o[i] *= alpha;
        const float* pr = p_s + qi * (KC + 1);
#pragma unroll 4
        for (int j = 0; j < KC; ++j) {
            const float p = pr[j];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float4 vv = *reinterpret_cast<const float4*>(v_s + j * D + 4 * kg + 32 * r);
                o[4 * r + 0] = fmaf(p, vv.x, o[4 * r + 0]);
                o[4 * r + 1] = fmaf(p, vv.y, o[4 * r + 1]);
                o[4 * r + 2] = fmaf(p, vv.z, o[4 * r + 2]);
                o[4 * r + 3] = fmaf(p, vv.w, o[4 * r + 3]);
            }
        }
    }

    if (q_first + qi < m_rows) {
        const float inv = 1.0f / l_run;
        float* orow = out + (size_t)(q_first + qi) * ldo + (size_t)h * D;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float4 v;
            v.x = o[4 * r + 0] * inv;
            v.y = o[4 * r + 1] * inv;
            v.z = o[4 * r + 2] * inv;
            v.w = o[4 * r + 3] * inv;
            *reinterpret_cast<float4*>(orow + 4 * kg + 32 * r) = v;
        }
    }
}

// ---- MFMA form for the fp16 cache (engine prefill): attn_prefill_tr_kernel below. P = 2
// (hi + lo fp16 planes of q and of p against the exact fp16 K, V) is fp32-faithful; P = 1
// is the fp16 throughput mode. Output: fp32 rows, or the o_proj GEMM's fp16 input planes.
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int QM = 64;  // query rows per workgroup
constexpr int KB = 64;  // keys per block

// Split keys: the causal range of query block qb (key blocks [0, nkb(qb))) can be cut into
// chunks of cb key blocks, one workgroup each -- used when whole query blocks leave CUs
// idle (few rows after a long history: one chunk of 64 rows at p0 = 1984 is 32 workgroups
// of 32 dependent blocks). A query block with one chunk writes its output directly;
// otherwise every chunk writes its unnormalised (O, m, l) to ws[head][qb][chunk] and
// attn_prefill_merge_kernel combines them in chunk order. blockIdx.x enumerates
// (qb, chunk), longest query blocks first.
// workgroup size of rope_kv_prefill_kernel (LLMI_ROPE_THREADS, A/B; default 1024)
inline int pf_rope_threads() {
    static const int v = [] {
        const char* e = std::getenv("LLMI_ROPE_THREADS");
        const int n = e ? std::atoi(e) : 1024;
        return (n == 256 || n == 512 || n == 1024) ? n : 1024;
    }();
    return v;
}
__host__ __device__ inline int pf_nkb(int qb, int p0, int m_rows) {
    const int kend = p0 + (qb * QM + QM < m_rows ? qb * QM + QM : m_rows);
    return (kend + KB - 1) / KB;
}
constexpr int kPartFloats = QM * D + 2 * QM;  // one chunk's O rows, then m, then l

// ---- Transposed form (round 5; it replaced a 4-wave register-staged kernel that put P
// and a transposed V through LDS writes: 27.3 us + a 7.3-us merge launch per 7B layer at
// M = 512, r05p). Workgroup = (64 query rows, head, key chunk), 8 waves: wave w owns query rows 16 (w & 3) .. + 15 and the
// key HALF kp = w >> 2 (keys 32 kp .. 32 kp + 31) of every 64-key block, with its own online
// softmax state; the two halves are combined once, in LDS, at the end. The two products are
// oriented so that neither P nor V needs an LDS rewrite:
//   S^T = K Q^T   A = K rows from the LDS image, B = the Q fragments: the accumulator holds
//                 ONE query per lane (column lane & 15) and 8 keys, so a softmax row
//                 reduction is 7 register ops + 2 cross-group shuffles;
//   O^T = V^T P^T B = P^T straight from the S^T accumulators (the two 16-key tiles of the
//                 wave's half, converted to fp16 planes in registers), A = V^T read from a
//                 ROW-major V image with ds_read_b64_tr_b16 (the hardware transpose).
// K and V are copied HBM -> LDS by global_load_lds_dwordx4 (no register staging) through a
// ring of kStages = 4 32-KB stages worked in pairs: the pair being computed and the next pair
// in flight, one barrier per pair (r05p: 22.2 us / layer with a single block of look-ahead;
// the copies never gate the loop now, r05t). The swizzles are applied by
// permuting each lane's SOURCE chunk (the DMA writes lane-linear 1 KB spans).
// Key order inside a 16-key tile: the A-operand lane of row i reads key kperm(i) =
// 4 ksig(i >> 2) + (i & 3) (ksig = 0 2 1 3), so accumulator group fq holds keys
// 4 ksig(fq) + r and a transposed read's 32-lane half takes two 4-row blocks 8 rows apart
// in the V image (conflict-free, guide T10; PMC SQ_LDS_BANK_CONFLICT = 0); the PV k order
// uses the same map. Scores are kept in log2 units (q pre-scaled by log2(e) / sqrt(d),
// v_exp_f32 in the softmax); the partial m written for the merge is in those units too.
typedef short s4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int ksig(int g) { return ((g & 1) << 1) | (g >> 1); }
// V image: 16-B chunk ch of 256-B row r at chunk ch ^ vtr_swz(r) (guide T10 layout (b))
__device__ __forceinline__ int vtr_swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ s4v tr_read(const char* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(p));
}
// butterfly reductions over lane ^ 16 / lane ^ 32 with the gfx950 row swaps (no LDS trip):
// after v_permlane{16,32}_swap of x with itself the pair holds x[l] and x[l ^ 16 / 32], the
// lower lane's value first, so every lane computes the same sum bit for bit
__device__ __forceinline__ float xmax16(float x) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xmax32(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xsum16(float x) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xsum32(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// global_load_lds_dwordx4 with a uniform base (SGPRs) and a per-lane 32-bit byte offset:
// the wave's 64 lanes fill 1 KB of LDS from `lds` on, lane-linear
__device__ __forceinline__ void pf_glds(const void* sbase, unsigned voff, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(sbase), "s"(lds)
                 : "memory");
}
constexpr int kTrThreads = 512;
constexpr int kStages = 4;
constexpr int kImg = KB * D * 2;  // one 64-key image (K or V): 16 KB

template <int P>
__global__ __launch_bounds__(kTrThreads) void attn_prefill_tr_kernel(const float* qkv, int ld, int m_rows, int p0,
                                                                     int heads, int kv_heads, const __half* k_cache,
                                                                     const __half* v_cache, int max_seq, float* out,
                                                                     _Float16* out_hi, _Float16* out_lo, int ldo, int cb,
                                                                     float* ws, int maxc, int lo8,
                                                                     unsigned long long* stamps) {
    __shared__ __attribute__((aligned(16))) char smem[kStages * 2 * kImg];  // [stage][K | V]
    WgStamp ts(stamps);
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int qt = w & 3, kp = w >> 2;  // query tile, key half

    const int nqb = (m_rows + QM - 1) / QM;
    // XCD-aware 1-D grid (workgroup id % 8 = its XCD): every (query block, chunk) of one head
    // runs on the same XCD, whose L2 then serves the head's K / V blocks to all of them
    const int xcd = blockIdx.x & 7, r = blockIdx.x >> 3;
    const int per = (heads - xcd + 7) / 8;
    int items = 0;
    for (int q = 0; q < nqb; ++q) items += (pf_nkb(q, p0, m_rows) + cb - 1) / cb;
    if (r >= per * items) return;
    const int h = xcd + 8 * (r % per);
    int qb = nqb - 1, chunk = 0, nch = 1;
    for (int idx = r / per; qb >= 0; --qb) {
        nch = (pf_nkb(qb, p0, m_rows) + cb - 1) / cb;
        if (idx < nch) {
            chunk = idx;
            break;
        }
        idx -= nch;
    }
    const int kvh = h / (heads / kv_heads);
    const int q_first = qb * QM;
    const float qscale = 1.4426950408889634f / sqrtf((float)D);  // log2(e) / sqrt(d)

    h8 qa[P][4];
    const int kend = p0 + min(q_first + QM, m_rows);
    const int nkb = (kend + KB - 1) / KB;
    const int kb0 = chunk * cb, kb1 = min(kb0 + cb, nkb);
    const void* kc = k_cache + (size_t)kvh * max_seq * D;
    const void* vc = v_cache + (size_t)kvh * max_seq * D;
    const unsigned lds0 = (unsigned)(uintptr_t)smem;
    // iteration i computes key block kb0 + i (a descending order measured the same, r05u)
    const int nit = kb1 - kb0;
    auto kb_of = [&](int i) { return kb0 + i; };
    // wave w fills 1-KB spans n = 8 i + w (image rows 4 n .. 4 n + 3) of both images: lane ->
    // row 4 n + lane / 16, physical chunk lane % 16 = logical chunk ^ swizzle. 4 copies per wave
    auto issue = [&](int it) {
        const int kb = kb_of(it);
        const unsigned sb = lds0 + (unsigned)(it % kStages) * 2 * kImg;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int n = 8 * i + w, row = 4 * n + fq;
            const unsigned src = (unsigned)min(kb * KB + row, kend - 1) * (unsigned)(D * 2);
            const unsigned dst = __builtin_amdgcn_readfirstlane(sb + n * 1024);
            pf_glds(kc, src + ((fr ^ (row & 15)) << 4), dst);
            pf_glds(vc, src + ((fr ^ vtr_swz(row)) << 4), dst + kImg);
        }
    };
    // the workgroup's 64 fp32 q rows (32 KB) go through the LDS of the last stage, which the
    // first pair of blocks leaves free: 512-B rows, 16-B chunk ch at ch ^ (row & 31), two
    // rows per 1-KB span, 4 copies per wave. Every global read of the kernel is then a copy
    // whose completion the kernel counts itself (a plain load's compiler-placed vmcnt wait
    // would also wait for the K/V copies issued behind it)
    char* qimg = smem + (kStages - 1) * 2 * kImg;
    {
        const unsigned qb0 = lds0 + (unsigned)(kStages - 1) * 2 * kImg;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int n = 8 * i + w, row = 2 * n + (lane >> 5), cp = lane & 31;
            const unsigned src = (unsigned)min(q_first + row, m_rows - 1) * (unsigned)ld * 4u + (unsigned)h * D * 4u +
                                 (unsigned)((cp ^ (row & 31)) << 4);
            pf_glds(qkv, src, __builtin_amdgcn_readfirstlane(qb0 + n * 1024));
        }
    }
    for (int i = 0; i < 2; ++i)
        if (i < nit) issue(i);

    float m_run = -INFINITY, l_run = 0.f;  // this lane's query (column fr), log2 units
    f4 o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f4{0.f, 0.f, 0.f, 0.f};
    const int qpos = p0 + q_first + 16 * qt + fr;
    const int arow = 32 * kp + 4 * ksig(fr >> 2) + (fr & 3);        // K image row of this A lane (tile 0)
    // S^T tile pair of iteration it: s[j][e] = score of key kb * KB + 32 kp + 16 j + 4 ksig(fq) + e
    auto qk = [&](int it, f4 (&s)[2]) {
        const char* Ks = smem + (it % kStages) * 2 * kImg;
        s[0] = s[1] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int row = 16 * j + arow;
                const h8 ak = *reinterpret_cast<const h8*>(Ks + row * 256 + (((4 * ks + fq) ^ (row & 15)) << 4));
#pragma unroll
                for (int p = 0; p < P; ++p) s[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ak, qa[p][ks], s[j], 0, 0, 0);
            }
        }
    };

    // q and blocks 0, 1 landed, for every wave
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ts.mark(1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
        const int row = 16 * qt + fr;
        const float* qr = reinterpret_cast<const float*>(qimg + row * 512);
        const float4 x0 = *reinterpret_cast<const float4*>(qr + 4 * ((8 * ks + 2 * fq) ^ (row & 31)));
        const float4 x1 = *reinterpret_cast<const float4*>(qr + 4 * ((8 * ks + 2 * fq + 1) ^ (row & 31)));
        const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float x = v[e] * qscale;
            const _Float16 hi = (_Float16)x;
            qa[0][ks][e] = hi;
            if (P == 2) qa[P - 1][ks][e] = (_Float16)(x - (float)hi);
        }
    }
    if (ts.p && t == 0) {
        ts.p[5] = (unsigned long long)qb | (unsigned long long)h << 16;
        ts.p[6] = (unsigned long long)nit;
    }
    __syncthreads();  // every wave read its q: the last stage is free for block 3
    const int tq = fr >> 2, tp = fr & 3;
    const int qpos_max = p0 + q_first + 16 * qt + 15;  // the wave's last query
    for (int it = 0; it < nit; ++it) {
        // two key blocks per barrier (r05ai: −0.4 µs a layer against one): at an even
        // iteration blocks it, it + 1 have landed (issued one pair earlier) and every wave is
        // done with it - 2, it - 1, whose stages take the next pair
        if ((it & 1) == 0) {
            if (it > 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
            }
            if (it + 2 < nit) issue(it + 2);
            if (it + 3 < nit) issue(it + 3);
        }
        const int kbase = kb_of(it) * KB + 32 * kp;
        if (kbase > qpos_max) continue;  // the half has no key visible to the wave's queries
        f4 s[2];
        qk(it, s);
        // causal mask (build_causal_mask.cu:29: key <= query position), only where the half
        // reaches past the wave's first query or the keys' end (wave-uniform test)
        if (kbase + 31 > p0 + q_first + 16 * qt || kbase + 31 >= kend) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int key = kbase + 16 * j + 4 * ksig(fq) + e;
                    if (key > qpos || key >= kend) s[j][e] = -INFINITY;
                }
        }
        // Online softmax with a lazy reference: p = 2^(s - m_run) and m_run is raised (O, l
        // rescaled) only when a score exceeds it by more than kTau = 8, so p <= 256 (exact in
        // the fp16 planes' range) and the rescale -- a pass over the 32 accumulators -- is
        // skipped by the whole wave on almost every block after the first
        float mx = fmaxf(fmaxf(fmaxf(s[0][0], s[0][1]), fmaxf(s[0][2], s[0][3])),
                         fmaxf(fmaxf(s[1][0], s[1][1]), fmaxf(s[1][2], s[1][3])));
        mx = xmax16(mx);
        mx = xmax32(mx);
        constexpr float kTau = 8.f;
        if (__builtin_amdgcn_ballot_w64(mx > m_run + kTau) != 0) {
            const float m_new = mx > m_run + kTau ? mx : m_run;
            // 0 from -inf, 1 if unchanged -- including a lane whose query still has every key
            // masked (m_run = m_new = -inf) while another query of the wave fired the ballot:
            // exp2(-inf - -inf) would be NaN there
            const float alpha = m_new == m_run ? 1.f : __builtin_amdgcn_exp2f(m_run - m_new);
            m_run = m_new;
            l_run *= alpha;
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] *= alpha;
        }
        const float m_use = m_run == -INFINITY ? 0.f : m_run;  // every key so far masked: p = 0
        float ps = 0.f;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float pv = __builtin_amdgcn_exp2f(s[j][e] - m_use);
                s[j][e] = pv;
                ps += pv;
            }
        ps = xsum16(ps);
        ps = xsum32(ps);
        l_run += ps;

        // O^T += V^T P^T over the half's 32 keys: P^T element e = s[e / 4][e % 4]; the V^T
        // fragment's elements 0-3 / 4-7 are the transposed reads of image rows
        // 32 kp + 4 ksig(fq) + (0..3) and the same + 16, columns 16 dt + fr
        h8 pb[P];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float x = s[e >> 2][e & 3];
            const _Float16 hi = (_Float16)x;
            pb[0][e] = hi;
            if (P == 2) pb[P - 1][e] = (_Float16)(x - (float)hi);
        }
        const char* Vs = smem + (it % kStages) * 2 * kImg + kImg;
        const int row0 = 32 * kp + 4 * ksig(fq) + tq;  // row0 + 16 has the same swizzle
        const char* vrow0 = Vs + row0 * 256 + 8 * (tp & 1);
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
            const int cofs = ((2 * dt + (tp >> 1)) ^ vtr_swz(row0)) << 4;
            const s4v v0 = tr_read(vrow0 + cofs);
            const s4v v1 = tr_read(vrow0 + 16 * 256 + cofs);
            const h8 av = __builtin_bit_cast(h8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
            for (int p = 0; p < P; ++p) o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, pb[p], o[dt], 0, 0, 0);
        }
    }

    // epilogue. o[dt][e] = O[query 16 qt + fr][dim 16 dt + 4 fq + e] of this key half.
    // Half 1 leaves (O, m, l) in LDS; half 0 combines: M = max, a_i = 2^(m_i - M),
    // L = l_0 a_0 + l_1 a_1, O = O_0 a_0 + O_1 a_1 (/ L for a direct output), into the padded
    // fp32 image that the 16-B row stores below read (32 lanes per row).
    constexpr int kIs = D + 4;
    __syncthreads();  // every wave is done with the stages (no copy is in flight)
    ts.mark(2);
    float* img1 = reinterpret_cast<float*>(smem);   // half 1's O rows [64][kIs]
    float* ml1 = img1 + QM * kIs;                   // half 1's m, l [2][64]
    float* img = ml1 + 2 * QM;                      // the combined rows [64][kIs]
    const int lr = 16 * qt + fr;
    if (kp == 1) {
#pragma unroll
        for (int dt = 0; dt < 8; ++dt)
            *reinterpret_cast<f4*>(img1 + lr * kIs + 16 * dt + 4 * fq) = o[dt];
        if (fq == 0) {
            ml1[lr] = m_run;
            ml1[QM + lr] = l_run;
        }
    }
    __syncthreads();
    if (kp == 0) {
        const float m1 = ml1[lr], l1 = ml1[QM + lr];
        const float M = fmaxf(m_run, m1);
        const float M_use = M == -INFINITY ? 0.f : M;
        const float a0 = __builtin_amdgcn_exp2f(m_run - M_use), a1 = __builtin_amdgcn_exp2f(m1 - M_use);
        const float L = l_run * a0 + l1 * a1;
        const float sc = nch > 1 ? 1.f : 1.0f / L;
        const float s0 = a0 * sc, s1 = a1 * sc;
#pragma unroll
        for (int dt = 0; dt < 8; ++dt) {
            const f4 o1 = *reinterpret_cast<const f4*>(img1 + lr * kIs + 16 * dt + 4 * fq);
            *reinterpret_cast<f4*>(img + lr * kIs + 16 * dt + 4 * fq) = o[dt] * s0 + o1 * s1;
        }
        if (nch > 1 && fq == 0) {
            float* part = ws + ((size_t)(h * nqb + qb) * maxc + chunk) * kPartFloats;
            part[QM * D + lr] = M;
            part[QM * D + QM + lr] = L;
        }
    }
    __syncthreads();
    if (nch > 1) {  // partial: unnormalised O rows of this chunk (m, l written above)
        float* part = ws + ((size_t)(h * nqb + qb) * maxc + chunk) * kPartFloats;
#pragma unroll
        for (int i = 0; i < QM * D / 4 / kTrThreads; ++i) {
            const int f = i * kTrThreads + t, rr = f >> 5, c4 = f & 31;
            reinterpret_cast<float4*>(part)[f] = *reinterpret_cast<const float4*>(img + rr * kIs + 4 * c4);
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < QM * D / 8 / kTrThreads; ++i) {
        const int f = i * kTrThreads + t, rr = f >> 4, c8 = f & 15;
        const int row = q_first + rr;
        if (row >= m_rows) continue;
        const float4 x0 = *reinterpret_cast<const float4*>(img + rr * kIs + 8 * c8);
        const float4 x1 = *reinterpret_cast<const float4*>(img + rr * kIs + 8 * c8 + 4);
        const size_t idx = (size_t)row * ldo + (size_t)h * D + 8 * c8;
        if (out_hi) {
            const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            h8 hv, lv;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                hv[e] = (_Float16)v[e];
                lv[e] = (_Float16)(v[e] - (float)hv[e]);
            }
            *reinterpret_cast<h8*>(out_hi + idx) = hv;
            if (out_lo && lo8)
                *reinterpret_cast<uint2*>(reinterpret_cast<char*>(out_lo + (size_t)row * ldo) + (size_t)h * D + 8 * c8) =
                    make_uint2(lo8_pack4(v[0] - (float)hv[0], v[1] - (float)hv[1], v[2] - (float)hv[2], v[3] - (float)hv[3]),
                               lo8_pack4(v[4] - (float)hv[4], v[5] - (float)hv[5], v[6] - (float)hv[6], v[7] - (float)hv[7]));
            else if (out_lo)
                *reinterpret_cast<h8*>(out_lo + idx) = lv;
        } else {
            *reinterpret_cast<float4*>(out + idx) = x0;
            *reinterpret_cast<float4*>(out + idx + 4) = x1;
        }
    }
}

// grid (nqb, heads), block 256: the chunks of a split query block, combined in chunk
// order: M = max m_c, L = sum l_c e^(m_c - M), O = sum O_c e^(m_c - M) / L. Four passes
// of 16 rows; thread t: row 16 pass + t / 16, dims 8 (t % 16) .. + 8, so 16 lanes cover a
// row with 16-B loads and stores. Every chunk's loads are issued before any is used
// (MAXC slots, clamped chunk index, unused slots weighted 0): one memory round trip.
template <int MAXC>  // the partials' m are in log2 units (attn_prefill_tr_kernel)
__global__ __launch_bounds__(kThreads) void attn_prefill_merge_kernel(const float* ws, int maxc, int cb, int m_rows,
                                                                      int p0, float* out, _Float16* out_hi,
                                                                      _Float16* out_lo, int ldo, int lo8) {
    const int qb = blockIdx.x, h = blockIdx.y, nqb = gridDim.x;
    const int nch = (pf_nkb(qb, p0, m_rows) + cb - 1) / cb;
    if (nch <= 1) return;  // written directly by the attention kernel
    const float* base = ws + (size_t)(h * nqb + qb) * maxc * kPartFloats;
    const int d0 = (threadIdx.x & 15) * 8;
    for (int pass = 0; pass < QM / 16; ++pass) {
        const int lr = pass * 16 + (threadIdx.x >> 4);
        const int row = qb * QM + lr;
        if (row >= m_rows) break;
        float mc[MAXC], lc[MAXC];
        float4 oc[MAXC][2];
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            const float* part = base + (size_t)min(c, nch - 1) * kPartFloats;
            mc[c] = part[QM * D + lr];
            lc[c] = part[QM * D + QM + lr];
            const float4* o4 = reinterpret_cast<const float4*>(part + lr * D + d0);
            oc[c][0] = o4[0];
            oc[c][1] = o4[1];
        }
        float M = -INFINITY;
#pragma unroll
        for (int c = 0; c < MAXC; ++c) M = fmaxf(M, mc[c]);  // clamped slots repeat a real chunk
        float L = 0.f, acc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = 0.f;
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            const float wgt = c < nch ? exp2f(mc[c] - M) : 0.f;  // 0 for a fully masked chunk (m = -inf)
            L += lc[c] * wgt;
            const float v[8] = {oc[c][0].x, oc[c][0].y, oc[c][0].z, oc[c][0].w,
                                oc[c][1].x, oc[c][1].y, oc[c][1].z, oc[c][1].w};
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[i] += v[i] * wgt;
        }
        const float inv = 1.0f / L;
        const size_t idx = (size_t)row * ldo + (size_t)h * D + d0;
        if (out_hi) {
            h8 hv, lv;
            float r[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float v = acc[i] * inv;
                hv[i] = (_Float16)v;
                r[i] = v - (float)hv[i];
                lv[i] = (_Float16)r[i];
            }
            *reinterpret_cast<h8*>(out_hi + idx) = hv;
            if (out_lo && lo8)
                *reinterpret_cast<uint2*>(reinterpret_cast<char*>(out_lo + (size_t)row * ldo) + (size_t)h * D + d0) =
                    make_uint2(lo8_pack4(r[0], r[1], r[2], r[3]), lo8_pack4(r[4], r[5], r[6], r[7]));
            else if (out_lo)
                *reinterpret_cast<h8*>(out_lo + idx) = lv;
        } else {
            *reinterpret_cast<float4*>(out + idx) = make_float4(acc[0] * inv, acc[1] * inv, acc[2] * inv, acc[3] * inv);
            *reinterpret_cast<float4*>(out + idx + 4) = make_float4(acc[4] * inv, acc[5] * inv, acc[6] * inv, acc[7] * inv);
        }
    }
}

__global__ void prefill_finish_kernel(DecodeState* st, const int32_t* prompt, int32_t* tokens, int p0, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) tokens[p0 + i] = prompt[p0 + i];
    if (threadIdx.x == 0) {
        st->next_pos = p0 + n;
        st->cur_pos = p0 + n - 1;
    }
}

}  // namespace

int prefill_finish_launch(DecodeState* st, const int32_t* prompt, int32_t* tokens, int p0, int n, hipStream_t s) {
    LLMI_REQUIRE(st && prompt && tokens && n > 0 && p0 >= 0, "prefill_finish: bad arguments");
    hipLaunchKernelGGL(prefill_finish_kernel, dim3(1), dim3(256), 0, s, st, prompt, tokens, p0, n);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

static std::atomic<unsigned long long*> g_pf_stamps{nullptr};
void prefill_stamps_debug(unsigned long long* stamps) { g_pf_stamps.store(stamps); }

int prefill_attn_launch(const PrefillAttnArgs& a, hipStream_t s) {
    LLMI_REQUIRE(a.qkv && a.k_cache && a.v_cache && a.rope_tab, "prefill attention: null argument");
    LLMI_REQUIRE(a.head_dim == D, "prefill attention: head_dim must be 128");
    LLMI_REQUIRE(a.m > 0 && a.p0 >= 0 && a.p0 + a.m <= a.max_seq, "prefill attention: rows past max_seq");
    LLMI_REQUIRE(a.heads > 0 && a.kv_heads > 0 && a.heads % a.kv_heads == 0, "prefill attention: bad head counts");
    LLMI_REQUIRE(a.mfma_planes == 0 || ((a.mfma_planes == 1 || a.mfma_planes == 2) && a.cache_dtype == LLMI_F16 &&
                                        (a.out || a.out_hi)),
                 "prefill attention: the MFMA form needs the fp16 cache, 1 or 2 planes and an output");
    LLMI_REQUIRE(a.mfma_planes != 0 || a.out, "prefill attention: null output");
    const int ld = (a.heads + 2 * a.kv_heads) * D;
    const dim3 ga((a.m + QB - 1) / QB, a.heads);
    if (a.cache_dtype == LLMI_F16) {
        hipLaunchKernelGGL(rope_kv_prefill_kernel<__half>, dim3(a.m), dim3(pf_rope_threads()), 0, s, a.qkv, a.qkv2, ld, a.p0, a.heads,
                           a.kv_heads, a.rope_tab, (__half*)a.k_cache, (__half*)a.v_cache, a.max_seq);
        if (a.mfma_planes) {
            // split keys: chunks of cb key blocks
            const int nqb = (a.m + QM - 1) / QM;
            int blocks = 0, max_nkb = 0;
            for (int qb = 0; qb < nqb; ++qb) {
                blocks += pf_nkb(qb, a.p0, a.m);
                max_nkb = std::max(max_nkb, pf_nkb(qb, a.p0, a.m));
            }
            // one 8-wave workgroup per CU (128 KB of LDS): whole query blocks when they give
            // every CU one; otherwise chunks of cb key blocks sized for ~one workgroup per CU
            static const int n_cu = [] {
                int dev = 0, n = 256;
                if (hipGetDevice(&dev) == hipSuccess)
                    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
                return n > 0 ? n : 256;
            }();
            int cb = max_nkb;
            if (a.split_ws && nqb * a.heads < n_cu) cb = std::max(1, (blocks * a.heads + n_cu - 1) / n_cu);
            static const int cb_env = [] {  // tuning knob: key blocks per chunk (LLMI_PF_CHUNK)
                const char* e = std::getenv("LLMI_PF_CHUNK");
                return e ? std::atoi(e) : 0;
            }();
            if (a.split_ws && cb_env > 0) cb = cb_env;
            int maxc = (max_nkb + cb - 1) / cb;
            if (a.split_ws && (maxc > 8 || (size_t)a.heads * nqb * maxc * kPartFloats > a.split_ws_floats)) {
                cb = max_nkb;  // no room: one chunk per query block
                maxc = 1;
            }
            if (!a.split_ws) cb = max_nkb, maxc = 1;
            int grid = 0;
            for (int qb = 0; qb < nqb; ++qb) grid += (pf_nkb(qb, a.p0, a.m) + cb - 1) / cb;
            // 1-D, XCD-interleaved: 8 x ceil(heads / 8) x (items per head) workgroups
            const dim3 gm(8 * ((a.heads + 7) / 8) * grid);
            unsigned long long* st = g_pf_stamps.load(std::memory_order_relaxed);
#define PF_ATTN(PL)                                                                                            \
    hipLaunchKernelGGL(attn_prefill_tr_kernel<PL>, gm, dim3(kTrThreads), 0, s, a.qkv, ld, a.m, a.p0, a.heads,  \
                       a.kv_heads, (const __half*)a.k_cache, (const __half*)a.v_cache, a.max_seq, a.out, a.out_hi, \
                       a.out_lo, a.heads * D, cb, a.split_ws, maxc, a.out_lo8, st)
            if (a.mfma_planes == 2)
                PF_ATTN(2);
            else
                PF_ATTN(1);
#undef PF_ATTN
            if (maxc > 1) {
#define PF_MERGE(C)                                                                                              \
    hipLaunchKernelGGL(attn_prefill_merge_kernel<C>, dim3(nqb, a.heads), dim3(kThreads), 0, s, a.split_ws, maxc, cb, \
                       a.m, a.p0, a.out, a.out_hi, a.out_lo, a.heads * D, a.out_lo8)
                if (maxc <= 2)
                    PF_MERGE(2);
                else if (maxc <= 4)
                    PF_MERGE(4);
                else
                    PF_MERGE(8);
#undef PF_MERGE
            }
        } else {
            hipLaunchKernelGGL(attn_prefill_kernel<__half>, ga, dim3(kThreads), 0, s, a.qkv, ld, a.m, a.p0, a.heads,
                               a.kv_heads, (const __half*)a.k_cache, (const __half*)a.v_cache, a.max_seq, a.out,
                               a.heads * D);
        }
    } else if (a.cache_dtype == LLMI_F32) {
        hipLaunchKernelGGL(rope_kv_prefill_kernel<float>, dim3(a.m), dim3(pf_rope_threads()), 0, s, a.qkv, a.qkv2, ld, a.p0, a.heads,
                           a.kv_heads, a.rope_tab, (float*)a.k_cache, (float*)a.v_cache, a.max_seq);
        hipLaunchKernelGGL(attn_prefill_kernel<float>, ga, dim3(kThreads), 0, s, a.qkv, ld, a.m, a.p0, a.heads,
                           a.kv_heads, (const float*)a.k_cache, (const float*)a.v_cache, a.max_seq, a.out,
                           a.heads * D);
    } else {
        LLMI_REQUIRE(false, "prefill attention: cache dtype must be f16 or f32");
    }
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

}  // namespace llmi
