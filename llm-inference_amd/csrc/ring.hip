// Persistent ring layer: the post-attention half of decode layer l plus the next
// layer's q/k/v projection as ONE launch (cdna_hip_programming.md §5.6;
// MI355X_MICROARCH.md price rows ldsdma-fill, prefetch-credit, nt-weights,
// engine-vs-launches):
//
//   O  xmid   = x_l + W_o . merge(attention partials)   by head: CU (h, row block)
//   G  act    = silu(g) * u, [g; u] = W_gu . RMSNorm(xmid) rows of W_gu, whole
//   D  x_l+1  = xmid + W_d . act                         K split: each CU its act slice
//   Q  qkv    = W_qkv(l+1) . RMSNorm(x_l+1)               rows of W_qkv, whole
//
// Replaces, per layer, the launches o_proj / gate_up / down / next q/k/v and their
// boundaries (masked_self_attention.cpp:84, self_decoder.cpp:59-85, ffn.cpp:72-89,
// masked_self_attention.cpp:62). One workgroup per CU: waves 0..kLoaders-1 are LOADERS,
// the next kCons waves CONSUMERS. Each CU owns a fixed slice of every phase; its
// loaders stream that slice's weights -- O, G, D, Q back to back -- into a ring of
// 8-KB LDS slots by non-temporal LDS-DMA (global_load_lds_dwordx4 nt; an asm
// statement, so hipcc adds no waits), kDepth pieces in flight each, publishing a
// landed piece with a FULL word. Consumers read a slot into registers, count
// themselves out of it (FREE), and compute. Weights never depend on activations, so
// the loaders run ahead across both in-launch hand-offs: while the consumers wait for
// every CU's o_proj (or down) sums, HBM keeps streaming the next phase into the ring.
//
// The two hand-offs need no all-gather of activations: o_proj and down both finish by
// adding fp32 partial sums into int64 fixed-point accumulators with device-scope
// atomics (exact, so the result is independent of order: deterministic, graph =
// eager), then one lane adds to a counter sharded over 8 lines after every consumer
// wave drained its atomics (vmcnt(0) + consumer barrier). The waiting CU polls the 8
// shards with sc1 loads from one lane group, then reads the accumulators with 8-byte
// agent-scope (sc1) loads -- the "8-B agent atomics both sides" form of
// MI355X_MICROARCH.md § inter-workgroup visibility. The down projection is split over
// K by CU (each CU multiplies ITS act slice by the matching rows of W_down^T and adds
// a 4096-wide partial), so gate_up -> down stays inside the CU: no act hand-off.
// Every spin is bounded (error bit 32, wrong tokens, never a hang).
//
// Roofline: HBM. Algorithmic bytes per launch = (H * Q + 2 I H + I H + n_qkv H) * 2
// (fp16 W_o, W_gu, W_d, next W_qkv) + partials + gammas.
#include "attn_impl.h"
#include "kernels.h"

namespace llmi {
namespace {

constexpr int kH = 4096;                    // hidden: one weight row = one 8-KB piece
constexpr int kPiece = 8192;                // bytes per piece / ring slot
constexpr int kSlots = 16;                  // 128 KB ring
constexpr int kLoaders = 2;
constexpr int kCons = 4;
constexpr int kThreads = 64 * (kLoaders + kCons);
constexpr int kCT = 64 * kCons;             // consumer threads
#ifndef LLMI_RING_EXP
#define LLMI_RING_EXP 0
#endif
#ifndef LLMI_RING_DEPTH
#define LLMI_RING_DEPTH 6
#endif
constexpr int kDepth = LLMI_RING_DEPTH;     // pieces in flight per loader (8 DMA each: vmcnt <= 48)
static_assert(kDepth >= 1 && kDepth <= 7, "vmcnt holds at most 63 DMAs per loader wave");
constexpr int kMaxPairs = 64;               // gate/up pairs (= W_d^T rows) per CU
constexpr int kChunks = kH * 2 / 16;        // 16-B chunks per row (512)
constexpr int kRowPL = kChunks / 64;        // chunks of a row per lane when one wave reads it (8)
constexpr int kXOff = kSlots * kPiece;      // fp32 x image [kH]
constexpr int kCtl = kXOff + kH * 4;        // control words, act, merged head, scratch
constexpr int kLds = kCtl + 4096;
constexpr unsigned long long kSpinLimit = 20000000ull;  // 200 ms of the 100 MHz clock
#ifndef LLMI_RING_PROF
#define LLMI_RING_PROF 0  // 1: the 8 stamp words of a workgroup hold wait-time totals instead (tools/ring_timeline.py --prof)
#endif

struct Plan {
    int h, r0, s_o;     // O: head, first W_o row, pieces (32 rows each)
    int p0, np;         // G/D: gate/up pairs [p0, p0 + np) = W_d^T rows
    int q0, nq;         // Q: next layer's rows [q0, q0 + nq)
    int b_g, b_d, b_q, n;  // first piece of G, D, Q; total pieces
};
__device__ __forceinline__ void part(int n, int b, int g, int& beg, int& cnt) {
    beg = (int)((long)n * b / g);
    cnt = (int)((long)n * (b + 1) / g) - beg;
}
__device__ __forceinline__ Plan make_plan(const RingArgs& a, int b, int g) {
    Plan p;
    const int rb_n = g / a.heads;  // row blocks per head
    p.h = b / rb_n;
    const int rows = a.hidden / rb_n;
    p.r0 = (b % rb_n) * rows;
    p.s_o = rows / 32;
    part(a.inter, b, g, p.p0, p.np);
    if (a.w_qkv) part(a.n_qkv, b, g, p.q0, p.nq);
    else p.q0 = p.nq = 0;
    p.b_g = p.s_o;
    p.b_d = p.b_g + 2 * p.np;
    p.b_q = p.b_d + p.np;
    p.n = p.b_q + p.nq;
    return p;
}
// consumer waves that read piece seq (D: all of them, O, G and Q: its owner)
__device__ __forceinline__ int cons_of(const Plan& p, int seq) {
    return (seq >= p.b_d && seq < p.b_q) ? kCons : 1;
}
// lane's 16-B source of piece seq for its first DMA instruction, and the byte step to
// each of the next seven (8 per piece, 1 KB each): computed once per piece, so the
// loader spends two VALU ops per DMA instead of re-deriving the phase and row
__device__ __forceinline__ const char* piece_base(const RingArgs& a, const Plan& p, int seq, int lane, size_t& step) {
    if (seq < p.b_g) {  // 32 rows x 256 B of W_o: row p.r0 + 32 seq + 4 j + lane / 16, head p.h
        const int row = p.r0 + seq * 32 + (lane >> 4);
        step = (size_t)4 * a.heads * 128 * 2;
        return reinterpret_cast<const char*>(a.w_o) +
               ((size_t)row * (a.heads * 128) + (size_t)p.h * 128 + (lane & 15) * 8) * 2;
    }
    step = 1024;
    const char* row;
    if (seq < p.b_d) {
        const int k = seq - p.b_g;
        row = reinterpret_cast<const char*>(a.w_gu) + (size_t)(((k & 1) ? a.inter : 0) + p.p0 + (k >> 1)) * kPiece;
    } else if (seq < p.b_q) {
        row = reinterpret_cast<const char*>(a.w_dt) + (size_t)(p.p0 + seq - p.b_d) * kPiece;
    } else {
        row = reinterpret_cast<const char*>(a.w_qkv) + (size_t)(p.q0 + seq - p.b_q) * kPiece;
    }
    return row + lane * 16;
}

__device__ __forceinline__ void glds16_nt(const void* gsrc, unsigned lds_dst) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off nt\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_dst)
        : "memory");
}
__device__ __forceinline__ int lds_ld(const int* p) {
    return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ bool err_set(const int* err, int bit) {
    return __hip_atomic_load(const_cast<int*>(err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit;
}
// bounded spin on an LDS word; the clock is read only once the word was seen unready.
// Once any wave of the launch (or an earlier launch) timed out, every later slow-path wait
// gives up at once: a hand-off that cannot complete (e.g. a workgroup that never became
// resident) costs one spin limit, not one per wait.
template <typename F>
__device__ __forceinline__ bool spin_until(F&& ready, int* err, int bit) {
    if (ready()) return true;
    if (err_set(err, bit)) return false;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned n = 1;; ++n) {
        __builtin_amdgcn_s_sleep(1);
        if (ready()) return true;
        if ((n & 63) == 0 && (__builtin_amdgcn_s_memrealtime() - t0 > kSpinLimit || err_set(err, bit))) {
            if ((threadIdx.x & 63) == 0) atomicOr(err, bit);
            return false;
        }
    }
}
__device__ __forceinline__ long long ld_sc1(const long long* p) {
    return (long long)__hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<long long*>(p)),
                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void add_fixed(long long* p, float v) {
    atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)to_fixed(v));
}
__device__ __forceinline__ float silu(float v) { return v / (1.0f + expf(-v)); }
__device__ __forceinline__ float dot8(const uint4& w, const float4& x0, const float4& x1) {
    const __half2* h = reinterpret_cast<const __half2*>(&w);
    const float2 a = __half22float2(h[0]), b = __half22float2(h[1]);
    const float2 c = __half22float2(h[2]), d = __half22float2(h[3]);
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
__device__ __forceinline__ float4 gamma4(const void* g, int j) {  // fp16 gamma elements 4j .. 4j + 3
    const uint2 u = reinterpret_cast<const uint2*>(g)[j];
    const float2 a = __half22float2(*reinterpret_cast<const __half2*>(&u.x));
    const float2 b = __half22float2(*reinterpret_cast<const __half2*>(&u.y));
    return make_float4(a.x, a.y, b.x, b.y);
}

__global__ __launch_bounds__(kThreads, 1) void ring_layer_kernel(RingArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    int* full = reinterpret_cast<int*>(smem + kCtl);   // [kSlots] piece that landed in the slot
    int* freec = full + kSlots;                          // [kSlots] consumer waves done with it (cumulative)
    int* expect = freec + kSlots;                        // [kSlots] loader: consumers of pieces issued so far
    int* cbar = expect + kSlots;                         // consumer-wave barrier counter
    float* act_s = reinterpret_cast<float*>(cbar + 4);   // [kMaxPairs]
    float* oh_s = act_s + kMaxPairs;                     // [128] merged attention output of head h
    float* red_s = oh_s + 128;                           // [2][kCons] reductions
    float* wm_s = red_s + 16;                            // [kMaxSplits] merge weights (uses the rest)
    float* ximg = reinterpret_cast<float*>(smem + kXOff);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int G = gridDim.x, b = blockIdx.x;
    const Plan p = make_plan(a, b, G);
    unsigned long long* ts = a.stamps ? a.stamps + 8 * (size_t)b : nullptr;
    auto stamp = [&](int i) {
        if (!LLMI_RING_PROF && ts && lane == 0) ts[i] = __builtin_amdgcn_s_memrealtime();
    };
    // LLMI_RING_PROF 2: consumer wave 0's marks through the O phase and the first seam
    auto ostamp = [&](int i) {
        if (LLMI_RING_PROF == 2 && ts && wave == kLoaders && lane == 0) ts[i] = __builtin_amdgcn_s_memrealtime();
    };
    // LLMI_RING_PROF: 100 MHz ticks a wave spent waiting, [2 lw] loader lw on a free slot,
    // [2 lw + 1] loader lw on its oldest piece landing, [4 + phase] consumer wave 0 on a
    // piece landing in phase O / G / D / Q
    unsigned long long t_a = 0, t_b = 0, t_c = 0, t_cur = 0;
    auto now = [&]() { return LLMI_RING_PROF == 1 ? __builtin_amdgcn_s_memrealtime() : 0ull; };
    if (tid < kSlots) {
        full[tid] = -1;
        freec[tid] = 0;
        expect[tid] = 0;
    }
    if (tid == 0) {
        cbar[0] = 0;
        cbar[1] = 0;  // G: next gate/up pair to take
        cbar[2] = 0;  // Q: next q/k/v row to take
    }
    __syncthreads();  // the only full-workgroup barrier: loaders never join another one

    if (wave < kLoaders) {
        // ---------------------------------------------------------------- loaders
        // loader lw issues pieces lw, lw + kLoaders, ... (its slots keep that parity);
        // a landed piece is published once kDepth - 1 newer ones are in flight, or
        // while the loader waits for a free slot (so a full ring never hides a landed piece)
        if (tid == 0) stamp(0);
        const int lw = wave;
        const unsigned ring = (unsigned)(uintptr_t)smem;
        int inflight = 0, pub = lw;
        auto publish_oldest = [&]() {
            const unsigned long long q0 = now();
            switch (inflight) {  // vmcnt needs an immediate: the oldest piece has landed
                case 1: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
                case 2: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
                case 3: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
                case 4: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
                case 5: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
                case 6: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
                default: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
            }
            t_b += now() - q0;
            if (lane == 0) lds_st(full + pub % kSlots, pub);
            pub += kLoaders;
            --inflight;
        };
        for (int seq = lw; seq < p.n; seq += kLoaders) {
            const int slot = seq % kSlots;
            if (seq >= kSlots) {
                const int want = lds_ld(expect + slot);
                bool ok = true;
                if (lds_ld(freec + slot) < want) {
                    const unsigned long long q0 = now();
                    while (inflight > 0 && lds_ld(freec + slot) < want) publish_oldest();
                    ok = spin_until([&]() { return lds_ld(freec + slot) >= want; }, a.err, 32);
                    t_a += now() - q0;
                }
                if (!ok) break;
            }
            if (lane == 0) lds_st(expect + slot, lds_ld(expect + slot) + cons_of(p, seq));
            const unsigned dst = __builtin_amdgcn_readfirstlane(ring + slot * kPiece);
            size_t step;
            const char* src = piece_base(a, p, seq, lane, step);
#pragma unroll
            for (int j = 0; j < 8; ++j) glds16_nt(src + j * step, dst + j * 1024);
            if (++inflight == kDepth) publish_oldest();
        }
        while (inflight > 0) publish_oldest();
        if (tid == 0) stamp(7);
        if (LLMI_RING_PROF == 1 && ts && lane == 0) {
            ts[2 * lw] = t_a;
            ts[2 * lw + 1] = t_b;
        }
        return;
    }

    // ------------------------------------------------------------------ consumers
    const int cw = wave - kLoaders, ct = tid - 64 * kLoaders;
    int gen = 0;
    auto cbarrier = [&]() {  // the consumer waves only
        gen += kCons;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_fetch_add(cbar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        spin_until([&]() { return lds_ld(cbar) >= gen; }, a.err, 32);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    auto wait_full = [&](int seq) {
        const int slot = seq % kSlots;
        if (LLMI_RING_PROF == 1 && lds_ld(full + slot) != seq) {
            const unsigned long long q0 = now();
            spin_until([&]() { return lds_ld(full + slot) == seq; }, a.err, 32);
            t_cur += now() - q0;
        } else {
            spin_until([&]() { return lds_ld(full + slot) == seq; }, a.err, 32);
        }
        return smem + slot * kPiece;
    };
    auto release = [&](int seq) {  // after this wave's reads of the slot completed
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_add(freec + seq % kSlots, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    // one lane per shard adds this CU's arrival, after every consumer wave drained its atomics
    auto arrive = [&](unsigned* cnt) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        cbarrier();
        if (ct == 0)
            __hip_atomic_fetch_add(cnt + (b & (kRingShards - 1)) * kRingShardWords, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    };
    auto wait_all = [&](const unsigned* cnt) {  // every CU arrived (wave 0 polls, the others wait at the barrier)
        if (cw == 0) {
            auto ready = [&]() {
                unsigned v = lane < kRingShards ? __hip_atomic_load(const_cast<unsigned*>(cnt) + lane * kRingShardWords,
                                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                : 0u;
                v += __shfl_xor(v, 1);
                v += __shfl_xor(v, 2);
                v += __shfl_xor(v, 4);
                return __shfl(v, 0) >= (unsigned)G;
            };
            if (!ready() && !err_set(a.err, 32)) {
                const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                for (unsigned n = 1;; ++n) {
                    __builtin_amdgcn_s_sleep(2);
                    if (ready()) break;
                    if ((n & 63) == 0 && (__builtin_amdgcn_s_memrealtime() - t0 > kSpinLimit || err_set(a.err, 32))) {
                        if (lane == 0) atomicOr(a.err, 32);
                        break;
                    }
                }
            }
        }
        cbarrier();
    };
    // the accumulator acc (fixed point, published by wait_all) into the LDS x image as
    // gamma * x, returning rstd = 1 / sqrt(mean x^2 + eps) (modeling_llama.py:112-117);
    // seed (may be null): this CU's slice of acc is added into it (exact integers)
    float gv[kH / kCT];  // this thread's gamma, loaded ahead of the wait
    auto load_gamma = [&](const void* g) {
#pragma unroll
        for (int i = 0; i < kH / kCT / 4; ++i) {
            const float4 v = gamma4(g, ct + i * kCT);
            gv[4 * i + 0] = v.x;
            gv[4 * i + 1] = v.y;
            gv[4 * i + 2] = v.z;
            gv[4 * i + 3] = v.w;
        }
    };
    int e0, en;
    part(a.hidden, b, G, e0, en);
    auto gather = [&](const long long* acc, long long* seed) -> float {
        long long v[kH / kCT];
#pragma unroll
        for (int i = 0; i < kH / kCT / 4; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q) v[4 * i + q] = ld_sc1(acc + 4 * (ct + i * kCT) + q);
        float ss = 0.f;
#pragma unroll
        for (int i = 0; i < kH / kCT / 4; ++i) {
            const int e = 4 * (ct + i * kCT);
            float4 f;
            f.x = from_fixed(v[4 * i + 0]);
            f.y = from_fixed(v[4 * i + 1]);
            f.z = from_fixed(v[4 * i + 2]);
            f.w = from_fixed(v[4 * i + 3]);
            ss += f.x * f.x + f.y * f.y + f.z * f.z + f.w * f.w;
            reinterpret_cast<float4*>(ximg)[e / 4] =
                make_float4(f.x * gv[4 * i], f.y * gv[4 * i + 1], f.z * gv[4 * i + 2], f.w * gv[4 * i + 3]);
            if (seed) {
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (e + q >= e0 && e + q < e0 + en)
                        atomicAdd(reinterpret_cast<unsigned long long*>(seed + e + q), (unsigned long long)v[4 * i + q]);
            }
        }
        ss = wave_sum(ss);
        if (lane == 0) red_s[cw] = ss;
        cbarrier();  // image and partial sums complete
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < kCons; ++w) t += red_s[w];
        return 1.0f / sqrtf(t / (float)a.hidden + a.eps);
    };
    // x registers of the row phases: lane holds elements (i * 64 + lane) * 8 + [0, 8)
    float4 xr[kRowPL][2];
    auto image_to_regs = [&]() {
#pragma unroll
        for (int i = 0; i < kRowPL; ++i) {
            const float4* s = reinterpret_cast<const float4*>(ximg + (i * 64 + lane) * 8);
            xr[i][0] = s[0];
            xr[i][1] = s[1];
        }
    };
    // one whole row piece by this wave: its dot with xr
    auto dot_row = [&](int seq) -> float {
        const char* sp = wait_full(seq);
        uint4 w[kRowPL];
#pragma unroll
        for (int i = 0; i < kRowPL; ++i) w[i] = *reinterpret_cast<const uint4*>(sp + (i * 64 + lane) * 16);
        release(seq);
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < kRowPL; ++i) acc += dot8(w[i], xr[i][0], xr[i][1]);
        return wave_sum(acc);
    };

    auto cstamp = [&](int i) {
        if (cw == 0) stamp(i);
    };
    ostamp(0);
    // ---- housekeeping for the next launches (their accumulators / counters), and the
    // residual seed of the o_proj sum: acc_mid[slice] += x_l[slice]
    for (int i = e0 + ct; i < e0 + en; i += kCT) {
        if (a.zero0) a.zero0[i] = 0;
        if (a.zero1) a.zero1[i] = 0;
        atomicAdd(reinterpret_cast<unsigned long long*>(a.acc_mid + i), (unsigned long long)a.acc_x[i]);
    }
    if (b == 0 && a.cnt_zero)
        for (int i = ct; i < kRingCntWords; i += kCT) a.cnt_zero[i] = 0u;
    load_gamma(a.g_ffn);

    // ---- O: merge head h's split partials (attn_impl.h workspace), then its W_o slice
    {
        const int ns = (a.max_seq + attn_detail::CH - 1) / attn_detail::CH, nact = a.nact;
        const attn_detail::Ws ws = attn_detail::ws_carve(const_cast<void*>(a.attn_ws), a.heads, ns);
        const float* mlh = ws.ml + (size_t)p.h * ns * 2;
        const int d = ct & 127, half = ct >> 7;
        const float* oh = ws.o + (size_t)p.h * ns * attn_detail::D + d;
        constexpr int kOv = 16;
        float ov[kOv];
        // one round trip: the partial outputs and every split's (m, l), all issued together
#pragma unroll
        for (int i = 0; i < kOv; ++i) {
            const int s = half + 2 * i;
            ov[i] = oh[(size_t)(s < nact ? s : 0) * attn_detail::D];
        }
        const float2* ml2 = reinterpret_cast<const float2*>(mlh);
        const float2 ml0 = ml2[lane < nact ? lane : 0];  // splits 0..63 (max_seq <= 4096: all of them)
        float M = lane < nact ? ml0.x : -INFINITY;
        for (int s = lane + 64; s < nact; s += 64) M = fmaxf(M, ml2[s].x);
        M = wave_max(M);  // every wave the same
        ostamp(1);
        float L = 0.f;
        if (lane < nact) {
            const float w = expf(ml0.x - M);
            L = ml0.y * w;
            if (cw == 0) wm_s[lane] = w;
        }
        for (int s = lane + 64; s < nact; s += 64) {
            const float w = expf(ml2[s].x - M);
            L = fmaf(ml2[s].y, w, L);
            if (cw == 0) wm_s[s] = w;
        }
        L = wave_sum(L);
        cbarrier();
        float O = 0.f;
#pragma unroll
        for (int i = 0; i < kOv; ++i) {
            const int s = half + 2 * i;
            O = fmaf(s < nact ? ov[i] : 0.f, s < nact ? wm_s[s] : 0.f, O);
        }
        for (int s = half + 2 * kOv; s < nact; s += 2) O = fmaf(oh[(size_t)s * attn_detail::D], wm_s[s], O);
        if (half) ximg[d] = O;  // scratch: the image is free until the gather
        cbarrier();
        if (!half) oh_s[d] = (O + ximg[d]) * (1.0f / L);  // attn_oproj_kernel's arithmetic, bit for bit
        cbarrier();
        ostamp(2);
    }
    {
        // a whole 32-row piece per consumer wave: lane reads chunk (lane & 15) of rows
        // lane / 16 + 4 i (i < 8), the 16 lanes of a row group reduce by xor shuffles
        const int c16 = lane & 15, g4 = lane >> 4;
        const float4 x0 = reinterpret_cast<const float4*>(oh_s)[2 * c16];
        const float4 x1 = reinterpret_cast<const float4*>(oh_s)[2 * c16 + 1];
        for (int k = cw; k < p.s_o; k += kCons) {
            const char* sp = wait_full(k);
            uint4 w[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) w[i] = *reinterpret_cast<const uint4*>(sp + (lane + 64 * i) * 16);
            release(k);
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = dot8(w[i], x0, x1);
#pragma unroll
            for (int off = 8; off > 0; off >>= 1)
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] += __shfl_xor(v[i], off);
            if (c16 == 0)  // the row sums wait in the x image (free until the gather)
#pragma unroll
                for (int i = 0; i < 8; ++i) ximg[k * 32 + g4 + 4 * i] = v[i];
        }
        ostamp(3);
        cbarrier();  // then one wave instruction adds 64 consecutive rows (512 contiguous bytes)
        for (int i = ct; i < p.s_o * 32; i += kCT) add_fixed(a.acc_mid + p.r0 + i, ximg[i]);
        ostamp(4);
    }
    arrive(a.cnt);
    ostamp(5);
    cstamp(1);
    t_a = t_cur;
    t_cur = 0;

    // ---- G: xmid from every CU; this CU's gate/up pairs; SiLU * up into act_s
    wait_all(a.cnt);
    ostamp(6);
    cstamp(2);
    float rstd = gather(a.acc_mid, a.acc_out);  // + seeds acc_out[slice] with xmid (the down sum adds to it)
    ostamp(7);
    if (a.w_qkv) load_gamma(a.g_attn);
    image_to_regs();
    // pairs are taken in ring order by whichever consumer wave is free (an LDS ticket), so
    // one slow wave never holds the ring's oldest slots while the others starve
    auto take = [&](int* ctr) {
        int j = 0;
        if (lane == 0) j = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return __shfl(j, 0);
    };
    for (int j = take(cbar + 1); j < p.np; j = take(cbar + 1)) {
        const float g = dot_row(p.b_g + 2 * j) * rstd;
        const float u = dot_row(p.b_g + 2 * j + 1) * rstd;
        if (lane == 0) act_s[j] = silu(g) * u;
    }
    cbarrier();
    cstamp(3);
    t_b = t_cur;
    t_cur = 0;

    // ---- D: x_{l+1} += W_d[:, slice] . act[slice] (this CU's rows of W_d^T); every
    // consumer thread owns 16 outputs: elements 8 ct + [0, 8) and 8 (ct + 256) + [0, 8)
    {
        float acc[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 0.f;
        // kDB pieces per step: their FULL polls, LDS reads and FREE counts overlap, so the
        // per-piece LDS round trips are paid once per step
        constexpr int kDB = 4;
        auto dstep = [&](int k0, int nb) {
            uint4 w0[kDB], w1[kDB];
            float av[kDB];
#pragma unroll
            for (int q = 0; q < kDB; ++q) {
                if (q < nb) {
                    const char* sp = wait_full(p.b_d + k0 + q);
                    w0[q] = *reinterpret_cast<const uint4*>(sp + ct * 16);
                    w1[q] = *reinterpret_cast<const uint4*>(sp + (ct + kCT) * 16);
                    av[q] = act_s[k0 + q];
                }
            }
#pragma unroll
            for (int q = 0; q < kDB; ++q)
                if (q < nb) release(p.b_d + k0 + q);
#pragma unroll
            for (int q = 0; q < kDB; ++q) {
                if (q < nb) {
                    const __half2* h0 = reinterpret_cast<const __half2*>(&w0[q]);
                    const __half2* h1 = reinterpret_cast<const __half2*>(&w1[q]);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const float2 f0 = __half22float2(h0[i]), f1 = __half22float2(h1[i]);
                        acc[2 * i] = fmaf(av[q], f0.x, acc[2 * i]);
                        acc[2 * i + 1] = fmaf(av[q], f0.y, acc[2 * i + 1]);
                        acc[8 + 2 * i] = fmaf(av[q], f1.x, acc[8 + 2 * i]);
                        acc[8 + 2 * i + 1] = fmaf(av[q], f1.y, acc[8 + 2 * i + 1]);
                    }
                }
            }
        };
        int k = 0;
        for (; k + kDB <= p.np; k += kDB) dstep(k, kDB);
        if (k < p.np) dstep(k, p.np - k);
        // through the (now free) x image, so that one wave's atomics cover 64 consecutive
        // int64 words: 512 contiguous bytes per instruction instead of 64 lanes each in its
        // own 64-B line (the scattered shape runs ~17x below the chip's atomic rate)
        float4* st = reinterpret_cast<float4*>(ximg);
        st[2 * ct] = make_float4(acc[0], acc[1], acc[2], acc[3]);
        st[2 * ct + 1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
        st[2 * (ct + kCT)] = make_float4(acc[8], acc[9], acc[10], acc[11]);
        st[2 * (ct + kCT) + 1] = make_float4(acc[12], acc[13], acc[14], acc[15]);
        cbarrier();
#if LLMI_RING_EXP != 1  // EXP 1 (timing only, wrong output): no down atomics
#pragma unroll
        for (int j = 0; j < kH / kCT; ++j) add_fixed(a.acc_out + j * kCT + ct, ximg[j * kCT + ct]);
#endif
    }
    arrive(a.cnt + kRingShards * kRingShardWords);
    cstamp(4);
    t_c = t_cur;
    t_cur = 0;
    auto prof_out = [&]() {
        if (LLMI_RING_PROF == 1 && ts && cw == 0 && lane == 0) {
            ts[4] = t_a;
            ts[5] = t_b;
            ts[6] = t_c;
            ts[7] = t_cur;
        }
    };
    if (!a.w_qkv) {
        cstamp(6);
        prof_out();
        return;
    }

    // ---- Q: x_{l+1} from every CU; the next layer's q/k/v rows
    wait_all(a.cnt + kRingShards * kRingShardWords);
    cstamp(5);
    rstd = gather(a.acc_out, nullptr);
    image_to_regs();
    for (int r = take(cbar + 2); r < p.nq; r = take(cbar + 2)) {
        const float v = dot_row(p.b_q + r) * rstd;
        if (lane == 0) a.qkv_out[p.q0 + r] = v;
    }
    cstamp(6);
    prof_out();
}

}  // namespace

bool ring_supported(int hidden, int heads, int head_dim, int inter, int n_qkv, int n_cu) {
    if (hidden != kH || head_dim != 128 || heads * head_dim != hidden || n_cu <= 0 || n_cu % heads) return false;
    const int rb = n_cu / heads;
    if (hidden % rb || (hidden / rb) % 32) return false;
    return (inter + n_cu - 1) / n_cu <= kMaxPairs && n_qkv > 0;
}

int ring_layer_launch(const RingArgs& a, int grid, hipStream_t s) {
    LLMI_REQUIRE(a.w_o && a.w_gu && a.w_dt && a.g_ffn && a.attn_ws && a.acc_x && a.acc_mid && a.acc_out && a.cnt &&
                     a.err && grid > 0,
                 "ring_layer: null argument");
    LLMI_REQUIRE(!a.w_qkv || (a.g_attn && a.qkv_out), "ring_layer: q/k/v phase without gamma or output");
    LLMI_REQUIRE(ring_supported(a.hidden, a.heads, 128, a.inter, a.w_qkv ? a.n_qkv : 1, grid),
                 "ring_layer: unsupported shape (hidden 4096, heads dividing the CU count)");
    const int ns = (a.max_seq + attn_detail::CH - 1) / attn_detail::CH;
    LLMI_REQUIRE(a.nact >= 1 && a.nact <= ns && a.nact <= (kLds - kCtl) / 4 - 256,
                 "ring_layer: bad active split count");
    static bool attr = false;
    if (!attr) {
        LLMI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&ring_layer_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
        attr = true;
    }
    hipLaunchKernelGGL(ring_layer_kernel, dim3(grid), dim3(kThreads), kLds, s, a);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

int ring_residency(int* per_cu) {
    LLMI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&ring_layer_kernel),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
    LLMI_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, reinterpret_cast<const void*>(&ring_layer_kernel),
                                                          kThreads, kLds));
    return LLMI_OK;
}

int transpose_f16_launch(const void* src, void* dst, int rows, int cols, hipStream_t s) {
    return transpose_launch(src, dst, rows, cols, 2, s);
}

}  // namespace llmi
