// Post-attention half of a decode layer as ONE persistent launch with a weight
// loader ring (cdna_hip_programming.md §5.6, MI355X_MICROARCH.md rows
// ldsdma-fill / prefetch-credit / engine-vs-launches):
//
//   O: xmid = resid + W_o attn            (rows of W_o, full K)         -> all-gather
//   G: act  = silu(g) * u, [g; u] = W_gu RMSNorm(xmid)                  -> all-gather
//   D: resid' = xmid + W_d act            (rows of W_d, full K)
//
// Replaces, per layer, the o_proj / fused add+RMSNorm / gate_up / SiLU / down /
// add-residual launches (masked_self_attention.cpp:84, self_decoder.cpp:59-81,
// ffn.cpp:72-89). One 256-thread workgroup per CU (the ring's LDS admits one):
// wave 0 is the LOADER, waves 1-3 CONSUMERS. Each workgroup owns a fixed slice
// of every phase (rows of W_o, gate/up row pairs, rows of W_d); the loader streams
// that slice's weights, phase after phase, through a ring of 8-KB LDS slots with
// non-temporal LDS-DMA (global_load_lds_dwordx4 ... nt, inline asm so hipcc adds
// no waits), keeping kDepth slots in flight and publishing each landed slot with
// a FULL word; consumers read a slot into registers, hand it back with a FREE
// word, and compute. Weights never depend on activations, so the loader runs
// ahead across the phase seams: while consumers wait for an all-gather (every
// workgroup's xmid or act), HBM keeps streaming into the ring -- the fill/drain
// of separate launches and their tails disappear.
//
// Hand-offs between workgroups follow handoff.h (write-through sc1 stores, every
// storing wave drained, sharded agent-scope counters, sc1 loads; spins bounded,
// errors set bits of DecodeState::error). Inside the workgroup the three consumer
// waves synchronise through an LDS counter (the loader never joins a barrier).
// Every output row is computed whole by one wave, chunks in order, so results are
// deterministic; the residual stays int64 fixed point.
//
// Roofline: HBM. Algorithmic bytes per launch = (H*Q + 2*I*H + H*I) * 2 (fp16 W_o,
// W_gu, W_d) + gamma.
#include "handoff.h"
#include "kernels.h"

namespace llmi {
namespace {

#ifndef LLMI_RING_LOADERS
#define LLMI_RING_LOADERS 2
#endif
constexpr int kSlotElems = 4096;               // fp16 weights per ring slot
constexpr int kSlotBytes = kSlotElems * 2;     // 8 KB
constexpr int kSlots = 16;                     // ring depth (128 KB); x lives in the consumers' registers
constexpr int kXImgBytes = 4096 * 4;           // one fp32 chunk of x, staged once for all consumer waves
constexpr int kLoaders = LLMI_RING_LOADERS;    // waves 0 .. kLoaders - 1: each streams every kLoaders-th piece
constexpr int kConsumers = 3;                  // the next three waves
constexpr int kThreads = 64 * (kLoaders + kConsumers);
#ifndef LLMI_RING_PREFETCH
#define LLMI_RING_PREFETCH 32  // pieces past the ring that idle consumers touch at each all-gather
#endif
#ifndef LLMI_RING_DEPTH
#define LLMI_RING_DEPTH 6
#endif
constexpr int kDepth = LLMI_RING_DEPTH;        // pieces in flight: 8 DMA instructions each, vmcnt <= 63
constexpr int kMaxChunks = 1;                  // x registers: one 4096-chunk (8 x 2 float4 per lane)
constexpr int kFlagBytes = 2048;               // FULL / FREE words, consumer counter, xmid rows, down partials
#ifndef LLMI_RING_DIAG
#define LLMI_RING_DIAG 0  // diagnostics only (wrong results): 1 consumers skip the dot, 2 loader ignores FREE, 3 loader alone
#endif               // FULL / FREE words, consumer counters, scratch

struct Plan {
    int o_b, o_n, co;  // O rows [o_b, o_b + o_n), chunks per row
    int g_b, g_n, cg;  // G pairs, chunks per row (2 rows per pair)
    int d_b, d_n, cd;  // D rows, chunks per row
    int s_o, s_g, s_d; // pieces per phase
};

__device__ __forceinline__ Plan make_plan(const RingArgs& a, int b, int nwg) {
    Plan p;
    auto part = [&](int n, int& beg, int& cnt) {
        beg = (int)((long)n * b / nwg);
        cnt = (int)((long)n * (b + 1) / nwg) - beg;
    };
    part(a.hidden, p.o_b, p.o_n);
    part(a.inter, p.g_b, p.g_n);
    p.d_b = p.o_b;  // D rows = O rows: the workgroup keeps its xmid rows
    p.d_n = p.o_n;
    p.co = (a.q_dim + kSlotElems - 1) / kSlotElems;
    p.cg = (a.hidden + kSlotElems - 1) / kSlotElems;
    p.cd = (a.inter + kSlotElems - 1) / kSlotElems;
    p.s_o = p.o_n * p.co;
    p.s_g = p.g_n * 2 * p.cg;
    p.s_d = p.d_n * p.cd;
    return p;
}

// piece seq -> global source and length (elements); item / chunk for the consumer
struct Piece {
    const char* src;
    int len;
};
__device__ __forceinline__ Piece piece(const RingArgs& a, const Plan& p, int seq) {
    if (seq < p.s_o) {
        const int r = p.o_b + seq / p.co, c = seq % p.co;
        return {reinterpret_cast<const char*>(a.w_o) + ((size_t)r * a.q_dim + (size_t)c * kSlotElems) * 2,
                min(kSlotElems, a.q_dim - c * kSlotElems)};
    }
    seq -= p.s_o;
    if (seq < p.s_g) {
        const int pr = p.g_b + seq / (2 * p.cg), half = (seq % (2 * p.cg)) / p.cg, c = seq % p.cg;
        const int row = half ? a.inter + pr : pr;
        return {reinterpret_cast<const char*>(a.w_gu) + ((size_t)row * a.hidden + (size_t)c * kSlotElems) * 2,
                min(kSlotElems, a.hidden - c * kSlotElems)};
    }
    seq -= p.s_g;
    const int r = p.d_b + seq / p.cd, c = seq % p.cd;
    return {reinterpret_cast<const char*>(a.w_d) + ((size_t)r * a.inter + (size_t)c * kSlotElems) * 2,
            min(kSlotElems, a.inter - c * kSlotElems)};
}

// bounded LDS poll: spin until *w == want (values are piece numbers, never reused)
// The clock (s_memrealtime, a scalar-memory round trip) is read only once the
// word has been seen unready, and then once per 64 polls: reading it up front cost
// every ready hand-off that round trip.
#ifndef LLMI_RING_SLEEP
#define LLMI_RING_SLEEP 1
#endif
__device__ __forceinline__ bool lds_wait_eq(const int* w, int want, int* err, int bit) {
    auto ready = [&]() {
        return __hip_atomic_load(const_cast<int*>(w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == want;
    };
    if (ready()) return true;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned n = 1;; ++n) {
        __builtin_amdgcn_s_sleep(LLMI_RING_SLEEP);
        if (ready()) return true;
        if ((n & 63) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {  // 200 ms: give up, flag it
            if ((threadIdx.x & 63) == 0) atomicOr(err, bit);
            return false;
        }
    }
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

__device__ __forceinline__ float silu(float v) { return v / (1.0f + expf(-v)); }

// consumer-side dot of one piece against the lane's x registers
__device__ __forceinline__ float dot_piece(const uint4 (&w)[8], const float4 (&xr)[8][2], int lane, int nch) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float d = dot8(w[i], xr[i][0], xr[i][1]);
        acc += (i * 64 + lane < nch) ? d : 0.f;
    }
    return acc;
}

__global__ __launch_bounds__(kThreads, 1) void ring_layer_kernel(RingArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* ring = smem;
    int* full = reinterpret_cast<int*>(smem + kSlots * kSlotBytes);
    int* freew = full + 32;
    int* csync_ctr = freew + 32;  // consumer-wave barrier counter
    long long* xmid_loc = reinterpret_cast<long long*>(smem + kSlots * kSlotBytes + 512);  // <= 64 rows
    float* ximg = reinterpret_cast<float*>(smem + kSlots * kSlotBytes + kFlagBytes);  // [4096] fp32

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nwg = gridDim.x, b = blockIdx.x;
    WgStamp ts(a.stamps);  // [1] O published, [2] xmid gathered, [5] G published, [6] act gathered, [7] loader done
    auto mark = [&](int i) {
        if (ts.p && lane == 0) ts.p[i] = __builtin_amdgcn_s_memrealtime();
    };
    const Plan p = make_plan(a, b, nwg);
    const int S = p.s_o + p.s_g + p.s_d;

    static_assert(kSlots % kLoaders == 0, "each loader keeps its own slots");
    if (threadIdx.x < kSlots) {
        full[threadIdx.x] = -1;
        freew[threadIdx.x] = -1;
    }
    if (threadIdx.x == 0) *csync_ctr = 0;
    __syncthreads();  // the only full-workgroup barrier

    if (wave < kLoaders) {
        // ------------------------------------------------------------ loaders
        // loader lw streams pieces lw, lw + kLoaders, ... (its slots keep one parity)
        const int lw = wave;
        const unsigned ring_base = (unsigned)(uintptr_t)ring;
        unsigned long long* dbg = (ts.p && b == 0) ? a.stamps + 8 * (size_t)nwg : nullptr;
        int k = 0;
        for (int seq = lw; seq < S; seq += kLoaders, ++k) {
            const int slot = seq % kSlots;
            if (LLMI_RING_DIAG < 2 && seq >= kSlots && !lds_wait_eq(freew + slot, seq - kSlots, a.err, 16)) break;
            if (dbg && lane == 0) dbg[3 * seq] = __builtin_amdgcn_s_memrealtime();
            const Piece pc = piece(a, p, seq);
            const int last = pc.len * 2 - 16;  // clamp: a short last piece re-reads its final 16 B
            const unsigned dst = __builtin_amdgcn_readfirstlane(ring_base + slot * kSlotBytes);
#pragma unroll
            for (int j = 0; j < 8; ++j) glds16_nt(pc.src + min(j * 1024 + lane * 16, last), dst + j * 1024);
            if (k >= kDepth - 1) {
                asm volatile("s_waitcnt vmcnt(%0)" ::"i"(8 * (kDepth - 1)) : "memory");
                const int ps = seq - kLoaders * (kDepth - 1);
                if (lane == 0) {
                    __hip_atomic_store(full + ps % kSlots, ps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (dbg) dbg[3 * ps + 1] = __builtin_amdgcn_s_memrealtime();
                }
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lw == 0) mark(7);
        if (lane == 0) {
            const int first = lw + kLoaders * (k - (kDepth - 1) > 0 ? k - (kDepth - 1) : 0);
            for (int ps = first; ps < S; ps += kLoaders)
                __hip_atomic_store(full + ps % kSlots, ps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        return;
    }

    // ---------------------------------------------------------------- consumers
    if (LLMI_RING_DIAG == 3) return;  // diagnostics: the loader alone (it ignores FREE then)
    const int cw = wave - kLoaders;  // 0 .. kConsumers - 1
    int gen = 0;
    auto csync = [&]() {  // the consumer waves
        gen += kConsumers;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_fetch_add(csync_ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__hip_atomic_load(csync_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < gen) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            for (unsigned n = 1;; ++n) {
                __builtin_amdgcn_s_sleep(1);
                if (__hip_atomic_load(csync_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= gen) break;
                if ((n & 63) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {
                    if (lane == 0) atomicOr(a.err, 64);
                    break;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    // x of the current phase, in registers: lane holds elements c * 4096 + (i * 64 + lane) * 8 + [0, 8)
    float4 xr[8][2];
    // one piece: weights LDS -> registers, FREE, dot against chunk c of xr
    auto consume = [&](int seq, int len) -> float {
        const int slot = seq % kSlots;
        lds_wait_eq(full + slot, seq, a.err, 8);
        const char* sp = ring + slot * kSlotBytes;
        const int nch = len / 8;
        uint4 w[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int cc = i * 64 + lane;
            w[i] = *reinterpret_cast<const uint4*>(sp + (cc < nch ? cc : 0) * 16);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) {
            __hip_atomic_store(freew + slot, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (ts.p && b == 0) a.stamps[8 * (size_t)nwg + 3 * seq + 2] = __builtin_amdgcn_s_memrealtime();
        }
        if (LLMI_RING_DIAG == 1) return 0.f;
        return dot_piece(w, xr, lane, nch);
    };
    auto gather_wait = [&](const unsigned* cnt) {  // the 8 counter shards sum to nwg
        if (cw == 0) {
            unsigned long long t0 = 0;
            for (unsigned n = 0;; ++n) {
                unsigned v = lane < kCntShards ? __hip_atomic_load(const_cast<unsigned*>(cnt) + lane * kCntStride,
                                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                               : 0u;
                v += __shfl_xor(v, 1);
                v += __shfl_xor(v, 2);
                v += __shfl_xor(v, 4);
                if (__shfl(v, 0) >= (unsigned)nwg) break;
                if (n == 0) t0 = __builtin_amdgcn_s_memrealtime();
                if ((n & 63) == 63 && __builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {
                    if (lane == 0) atomicOr(a.err, 32);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        csync();
    };
    auto publish = [&](unsigned* cnt) {  // after this workgroup's sc1 stores
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
        csync();
        if (cw == 0 && lane == 0)
            __hip_atomic_fetch_add(cnt + (b & (kCntShards - 1)) * kCntStride, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    };
    // While the consumers wait at an all-gather the ring is full and the loader idles:
    // consumer waves 1.. touch the pieces the loader will issue next (one dword per
    // 128-B line), so HBM keeps streaming into L2 / the Infinity Cache and the loader's
    // DMA finds them there once the ring drains. Results are folded into a value that
    // is never stored (the loads must not be dropped).
    auto prefetch = [&](int s0, int s1) {
        if (cw == 0 || LLMI_RING_PREFETCH == 0) return;
        constexpr int kB = 16;
        unsigned acc = 0;
        for (int base = s0 + (cw - 1) * kB; base < s1; base += (kConsumers - 1) * kB) {
            unsigned v[kB];
#pragma unroll
            for (int k = 0; k < kB; ++k) {
                const int sq = min(base + k, s1 - 1);
                const Piece pc = piece(a, p, sq);
                v[k] = *reinterpret_cast<const unsigned*>(pc.src + min(lane * 128, pc.len * 2 - 4));
            }
#pragma unroll
            for (int k = 0; k < kB; ++k) acc ^= v[k];
        }
        if (acc == 0x9e3779b9u && lane == 64) a.err[0] |= 0;  // never true for lane < 64: keeps the loads
    };
    // lane's elements of chunk c: c * 4096 + (i * 64 + lane) * 8 + [0, 8), as 2 float4 (zeros past K)
    auto elem0 = [&](int c, int i) { return c * kSlotElems + (i * 64 + lane) * 8; };
    float* part = reinterpret_cast<float*>(smem + kSlots * kSlotBytes + 1024);  // D partials [48 rows][kConsumers]

    // x of one chunk for every consumer wave: staged once into the LDS image by all
    // consumer threads, then each lane copies its 64 values into registers
    const int ct = threadIdx.x - 64 * kLoaders;  // 0 .. 64 * kConsumers - 1
    auto image_to_regs = [&](int k) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int e = elem0(0, i);
            const bool in = e < k;
            const float4* src = reinterpret_cast<const float4*>(ximg + (in ? e : 0));
            xr[i][0] = in ? src[0] : make_float4(0.f, 0.f, 0.f, 0.f);
            xr[i][1] = in ? src[1] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    // ---- O: attn (fp32 [q_dim <= 4096], previous launch) into registers; rows of W_o
    {
        for (int j = ct; j < a.q_dim / 4; j += 64 * kConsumers)
            reinterpret_cast<float4*>(ximg)[j] = reinterpret_cast<const float4*>(a.attn)[j];
        csync();
        image_to_regs(a.q_dim);
        for (int r = cw; r < p.o_n; r += kConsumers) {
            const float acc = wave_sum(consume(r, a.q_dim));
            if (lane == 0) {
                const int row = p.o_b + r;
                const long long v = (a.resid_keep ? a.resid[row] : 0ll) + to_fixed(acc);
                xmid_loc[r] = v;
                Sc1IO::st(a.x_out + row, from_fixed(v));  // the all-gather carries fp32 xmid (= x)
            }
        }
        publish(a.cnt);
        if (cw == 0) mark(1);
    }
    // ---- G: all-gather xmid into registers (x and sum x^2), gamma, gate/up pairs
    prefetch(p.s_o + kSlots, min(p.s_o + kSlots + LLMI_RING_PREFETCH, S));
    gather_wait(a.cnt);
    if (cw == 0) mark(2);
    {
        csync();  // every wave is done reading the image (O phase copy) before it is refilled
        for (int j = ct; j < a.hidden / 4; j += 64 * kConsumers)
            reinterpret_cast<float4*>(ximg)[j] = Sc1IO::ld4(reinterpret_cast<const float4*>(a.x_out) + j);
        csync();
        image_to_regs(a.hidden);
        float ss = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int e = elem0(0, i);
            const bool in = e < a.hidden;
            const float4 v0 = xr[i][0], v1 = xr[i][1];
            ss += v0.x * v0.x + v0.y * v0.y + v0.z * v0.z + v0.w * v0.w;
            ss += v1.x * v1.x + v1.y * v1.y + v1.z * v1.z + v1.w * v1.w;
            const uint4 gu = *reinterpret_cast<const uint4*>(reinterpret_cast<const __half*>(a.gamma) + (in ? e : 0));
            const __half2* gh = reinterpret_cast<const __half2*>(&gu);
            const float2 g0 = __half22float2(gh[0]), g1 = __half22float2(gh[1]);
            const float2 g2 = __half22float2(gh[2]), g3 = __half22float2(gh[3]);
            xr[i][0] = make_float4(v0.x * g0.x, v0.y * g0.y, v0.z * g1.x, v0.w * g1.y);
            xr[i][1] = make_float4(v1.x * g2.x, v1.y * g2.y, v1.z * g3.x, v1.w * g3.y);
        }
        const float rstd = 1.0f / sqrtf(wave_sum(ss) / (float)a.hidden + a.eps);
        const int base = p.s_o;
        for (int q = cw; q < p.g_n; q += kConsumers) {
            const float g = wave_sum(consume(base + 2 * q, a.hidden)) * rstd;
            const float u = wave_sum(consume(base + 2 * q + 1, a.hidden)) * rstd;
            if (lane == 0) Sc1IO::st(a.act + p.g_b + q, silu(g) * u);
        }
        publish(a.cnt + kPhaseCntWords);
        if (cw == 0) mark(5);
    }
    // ---- D: all-gather act into registers, down rows, resid' = xmid + W_d act
    prefetch(p.s_o + p.s_g + kSlots, min(p.s_o + p.s_g + kSlots + LLMI_RING_PREFETCH, S));
    gather_wait(a.cnt + kPhaseCntWords);
    if (cw == 0) mark(6);
    // chunk-owner: consumer wave cw takes chunk cw of every down row (x = that chunk of
    // act, 64 floats per lane); the row sums chunk partials in chunk order
    {
        const int c = cw;
        if (c < p.cd) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int e = elem0(c, i);
                const bool in = e < a.inter;
                const float4* src = reinterpret_cast<const float4*>(a.act + (in ? e : 0));
                const float4 v0 = Sc1IO::ld4(src), v1 = Sc1IO::ld4(src + 1);
                xr[i][0] = in ? v0 : make_float4(0.f, 0.f, 0.f, 0.f);
                xr[i][1] = in ? v1 : make_float4(0.f, 0.f, 0.f, 0.f);
            }
            const int base = p.s_o + p.s_g;
            const int len = min(kSlotElems, a.inter - c * kSlotElems);
            for (int r = 0; r < p.d_n; ++r) {
                const float acc = wave_sum(consume(base + r * p.cd + c, len));
                if (lane == 0) part[r * kConsumers + c] = acc;
            }
        }
        csync();
        if (cw == 0 && lane < p.d_n) {
            float acc = 0.f;
            for (int k = 0; k < p.cd; ++k) acc += part[lane * kConsumers + k];
            a.resid_out[p.d_b + lane] = xmid_loc[lane] + to_fixed(acc);
        }
    }
}

}  // namespace

size_t ring_lds_bytes(const RingArgs& a) {
    (void)a;
    return (size_t)kSlots * kSlotBytes + kFlagBytes + kXImgBytes;
}

int ring_grid(int device) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return 0;
    return cus;
}

int ring_check(const RingArgs& a, int device) {
    if (a.hidden % 8 || a.inter % 8 || a.q_dim % 8) return LLMI_EUNSUPPORTED;
    if (a.q_dim > kSlotElems || a.hidden > kSlotElems || a.inter > kConsumers * kSlotElems)
        return LLMI_EUNSUPPORTED;  // x registers hold one 4096-chunk; down rows <= one chunk per consumer wave
    const size_t lds = ring_lds_bytes(a);
    if (lds > 160 * 1024) return LLMI_EUNSUPPORTED;
    const int grid = ring_grid(device);
    if (grid <= 0 || (a.hidden + grid - 1) / grid > 48) return LLMI_EUNSUPPORTED;  // xmid_loc / part rows
    LLMI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&ring_layer_kernel),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int per_cu = 0;
    LLMI_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&ring_layer_kernel),
                                                          kThreads, lds));
    return per_cu >= 1 ? LLMI_OK : LLMI_EUNSUPPORTED;  // one workgroup per CU, all resident
}

int ring_layer_launch(const RingArgs& a, int grid, hipStream_t s) {
    LLMI_REQUIRE(a.w_o && a.w_gu && a.w_d && a.gamma && a.attn && a.resid && a.x_out && a.act && a.resid_out && a.cnt &&
                     a.err && grid > 0,
                 "ring: null argument");
    hipLaunchKernelGGL(ring_layer_kernel, dim3(grid), dim3(kThreads), ring_lds_bytes(a), s, a);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

}  // namespace llmi
