// Decode attention bodies of the kernels in attn.hip: split-KV attention with the
// KV-cache write, and the fused log-sum-exp merge + o_proj. See attn.hip for the
// design notes.
#pragma once
#include "io.h"
#include "kernels.h"

namespace llmi {
namespace attn_detail {


constexpr int kThreads = 256;
constexpr int D = 128;         // head_dim
#ifndef LLMI_ATTN_CH
#define LLMI_ATTN_CH 64
#endif
constexpr int CH = LLMI_ATTN_CH;  // positions per workgroup (<= kAttnChunk sizes the workspace)
static_assert(CH % 64 == 0 && CH >= kAttnChunk, "chunk must be a multiple of 64");
constexpr int LPR = 16;        // lanes per cached row (8 dims per lane)

constexpr int NPG = CH / (kThreads / LPR);  // cached rows per 16-lane group
constexpr int kMaxSplits = 1024;            // max_seq <= 64 Ki positions
constexpr int kMergeChunk = 16;             // o-partials per thread in the first merge round
static_assert(kThreads == 2 * D, "merge maps two threads to each head dim");

__device__ __forceinline__ float block_max(float v, float* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_max(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float t = -INFINITY;
    for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
    return t;
}

// 8 cache elements of one row, as loaded (16 B for fp16, 32 B for fp32)
template <typename KT> struct Raw { uint4 v[sizeof(KT) / 2]; };
// K/V cache rows: non-temporal loads -- the cache (up to 1 GB at ctx 2048) is streamed once
// per token and never fits the Infinity Cache. A/B on the 8-layer 7B loop (tools/ab_variants.sh,
// profiles/r03m_attn_nt_ab.jsonl): 2-5 us per 8-layer token lower in 4 of 4 alternating pairs
// (ctx 512 and 2048), though the attention kernel alone, layers cycled, reads 0.1-0.6 us slower
__device__ __forceinline__ Raw<__half> ld_raw(const __half* p) {
    Raw<__half> r;
    r.v[0] = ld_nt16(p);
    return r;
}
__device__ __forceinline__ Raw<float> ld_raw(const float* p) {
    Raw<float> r;
    r.v[0] = ld_nt16(p);
    r.v[1] = ld_nt16(p + 4);
    return r;
}
__device__ __forceinline__ void unpack8(const Raw<__half>& r, float* v) {
    const __half2* h = reinterpret_cast<const __half2*>(&r.v[0]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float2 f = __half22float2(h[i]);
        v[2 * i] = f.x;
        v[2 * i + 1] = f.y;
    }
}
__device__ __forceinline__ void unpack8(const Raw<float>& r, float* v) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        v[4 * i + 0] = __uint_as_float(r.v[i].x);
        v[4 * i + 1] = __uint_as_float(r.v[i].y);
        v[4 * i + 2] = __uint_as_float(r.v[i].z);
        v[4 * i + 3] = __uint_as_float(r.v[i].w);
    }
}
__device__ __forceinline__ void store_cache(__half* p, float v) { *p = __float2half(v); }
__device__ __forceinline__ void store_cache(float* p, float v) { *p = v; }
// value as the cache holds it (the current position must read exactly what later
// steps will read back from an fp16 cache)
template <typename KT> __device__ __forceinline__ float cache_round(float v);
template <> __device__ __forceinline__ float cache_round<__half>(float v) { return __half2float(__float2half(v)); }
template <> __device__ __forceinline__ float cache_round<float>(float v) { return v; }

// HF rotary angle (modeling_llama.py:130-141): inv_freq = 1 / fp32(base^(2i/d)) with
// the power correctly rounded (== torch's fp32 pow), angle = fp32(pos * inv_freq),
// cos/sin correctly rounded from double.
__device__ __forceinline__ void rope_cs(int pos, int i, int d, float base, float* c, float* s) {
    const float p = (float)pow((double)base, (double)(2 * i) / (double)d);
    const float inv = __fdiv_rn(1.0f, p);
    const float ang = __fmul_rn((float)pos, inv);
    double sd, cd;
    sincos((double)ang, &sd, &cd);
    *c = (float)cd;
    *s = (float)sd;
}

constexpr int kCntWordsPerHead = 64;  // 256 B: heads' counters never share a line
struct Ws {
    unsigned* counters;  // [heads][kCntWordsPerHead]: fused attention + o_proj arrivals (word 0) and
                         // departures (word 1), self-resetting; one 256-B line per head
    float* ml;           // [heads][nsplit][2]
    float* o;            // [heads][nsplit][D]
};
__host__ __device__ inline size_t ws_bytes(int heads, int max_seq) {
    const int ns = (max_seq + CH - 1) / CH;
    size_t c = (size_t)heads * kCntWordsPerHead * 4;
    return c + (size_t)heads * ns * 2 * 4 + (size_t)heads * ns * D * 4;
}
__device__ inline Ws ws_carve(void* base, int heads, int ns) {
    Ws w;
    char* p = reinterpret_cast<char*>(base);
    w.counters = reinterpret_cast<unsigned*>(p);
    p += (size_t)heads * kCntWordsPerHead * 4;
    w.ml = reinterpret_cast<float*>(p);
    p += (size_t)heads * ns * 2 * 4;
    w.o = reinterpret_cast<float*>(p);
    return w;
}

// 8 weights of one W_o row slice as loaded: 16 B (f16), 32 B (f32) or 8 B (i8)
template <typename WT> struct W8 { uint4 v[sizeof(WT) == 4 ? 2 : 1]; };
template <typename WT>
__device__ __forceinline__ W8<WT> ld_w8(const WT* p) {
    W8<WT> r;
    if constexpr (sizeof(WT) == 1) {
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 u = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
        r.v[0] = make_uint4(u.x, u.y, 0, 0);
    } else {
        r.v[0] = ld_nt16(p);
        if constexpr (sizeof(WT) == 4) r.v[1] = ld_nt16(p + 4);
    }
    return r;
}
template <typename WT>
__device__ __forceinline__ void unpack_w8(const W8<WT>& r, float* v) {
    if constexpr (sizeof(WT) == 1) {
        const uint32_t w[2] = {r.v[0].x, r.v[0].y};
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = (float)(int8_t)((w[i / 4] >> (8 * (i % 4))) & 0xff);
    } else if constexpr (sizeof(WT) == 2) {
        Raw<__half> h;
        h.v[0] = r.v[0];
        unpack8(h, v);
    } else {
        Raw<float> f;
        f.v[0] = r.v[0];
        f.v[1] = r.v[1];
        unpack8(f, v);
    }
}

// LDS carve of the attention body (16-B aligned pieces)
constexpr size_t kAttnLds = (3 * D + CH + (kThreads / LPR) * D + 4) * sizeof(float);

// One (head h, split) workgroup of the split-KV decode attention. ns = number of
// splits (workspace stride).
// HOST_SIZED (a.nact > 0): the grid holds only the active splits, so the K/V row
// loads are issued from the kernel arguments alone, before the device position (a
// scalar load from memory another kernel just wrote) has arrived; rows past the
// position are loaded (valid cache memory below max_seq) and ignored.
// agent-scope (sc1: L1 bypassed) 8-byte granule load, the fused q/k/v launch's hand-off
__device__ __forceinline__ unsigned long long ld_granule(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// TAGGED (fused q/k/v + attention launch, qkv_attn.hip; HOST_SIZED only): q, k, v are the
// granules a.qkv_tag the same launch's GEMV workgroups publish. Wave 0 holds them: it first
// polls one granule of the head's v row from one address (one line per poll, s_sleep between
// -- 1,024 pollers beside the weight stream), then every granule it needs until all carry this
// layer's tag; the K/V rows are in flight meanwhile.
template <typename KT, typename IO, bool HOST_SIZED = false, bool TAGGED = false>
__device__ __forceinline__ void attn_body(const AttnArgs& a, int h, int split, int ns, float* smem,
                                          const WgStamp* ts = nullptr) {
    static_assert(!TAGGED || HOST_SIZED, "the fused launch sizes the attention grid on the host");
    float* q_s = smem;
    float* kcur_s = q_s + D;
    float* vcur_s = kcur_s + D;
    float* p_s = vcur_s + D;
    float (*o_red)[D] = reinterpret_cast<float (*)[D]>(p_s + CH);  // [groups][D]
    float* ml_s = p_s + CH + (kThreads / LPR) * D;

    const int group = a.heads / a.kv_heads;
    const int kvh = h / group;
    const int tid = threadIdx.x;
    const int grp = tid / LPR, l16 = tid % LPR;  // 16 groups x 16 lanes, 8 dims per lane
    const int start = split * CH;
    KT* kc = reinterpret_cast<KT*>(a.k_cache) + (size_t)kvh * a.max_seq * D;
    KT* vc = reinterpret_cast<KT*>(a.v_cache) + (size_t)kvh * a.max_seq * D;
    const float* qrow = a.qkv + (size_t)h * D;
    const float* krow = a.qkv + (size_t)(a.heads + kvh) * D;
    const float* vrow = a.qkv + (size_t)(a.heads + a.kv_heads + kvh) * D;
    const int seed_per = (a.hidden + a.heads - 1) / a.heads;  // residual slice split 0 seeds
    Raw<KT> kr[NPG], vr[NPG];
    // HOST_SIZED prologue: every load that does not need the position goes out before
    // anything waits (vmcnt retires in issue order, so the position is issued first --
    // the RoPE table read depends on it): K/V rows, the q row, the current k/v rows,
    // the residual slice split 0 seeds. Each is one round trip in parallel instead of
    // the position -> K/V -> q -> table chain (4 serial round trips).
    float pq0 = 0.f, pq1 = 0.f, pk0 = 0.f, pk1 = 0.f, pv = 0.f;
    long long psd = 0;
    int pos;
    unsigned want = 0;  // TAGGED: this layer's tag
    unsigned long long gq0 = 0, gq1 = 0, gk0 = 0, gk1 = 0, gv0 = 0, gv1 = 0;
    const unsigned long long* qt = nullptr;
    const unsigned long long* kt = nullptr;
    const unsigned long long* vt = nullptr;
    if constexpr (TAGGED) {
        want = *a.tag_epoch * 128u + a.tag_layer;
        qt = a.qkv_tag + (size_t)h * D;
        kt = a.qkv_tag + (size_t)(a.heads + kvh) * D;
        vt = a.qkv_tag + (size_t)(a.heads + a.kv_heads + kvh) * D;
    }
    if constexpr (HOST_SIZED) {
        // the launcher requires a device position here. The load goes through a per-lane
        // (opaque zero) index so the compiler keeps it in a VGPR: as a uniform value it was
        // moved to an SGPR right after the load, with a vmcnt wait in front of the K/V issue
        int z = 0;
        asm volatile("" : "+v"(z));
        pos = a.pos_dev[z];
#pragma unroll
        for (int t = 0; t < NPG; ++t) {
            const int j = start + grp + t * (kThreads / LPR);
            const int jj = j < a.max_seq ? j : start;
            kr[t] = ld_raw(kc + (size_t)jj * D + l16 * 8);
            vr[t] = ld_raw(vc + (size_t)jj * D + l16 * 8);
        }
        const int i = tid & (D / 2 - 1);
        if constexpr (TAGGED) {
            if (tid < kWave) {  // wave 0's first look at its granules (almost never ready yet)
                gq0 = ld_granule(qt + i); gq1 = ld_granule(qt + i + D / 2);
                gk0 = ld_granule(kt + i); gk1 = ld_granule(kt + i + D / 2);
                gv0 = ld_granule(vt + i); gv1 = ld_granule(vt + i + D / 2);
            }
        } else {
        pq0 = IO::ld(qrow + i);
        pq1 = IO::ld(qrow + i + D / 2);
        // the current k and v (used by the split owning the position; loaded by every
        // split: a branch here made the compiler convert them, and so wait, early)
        pk0 = IO::ld(krow + i);
        pk1 = IO::ld(krow + i + D / 2);
        pv = IO::ld(vrow + (tid & (D - 1)));
        }
        if (a.xacc != nullptr && split == 0 && a.resid_fixed != nullptr)
            psd = a.resid_fixed[min(h * seed_per + tid, a.hidden - 1)];
    } else {
        pos = a.pos_dev ? *a.pos_dev : a.pos_host;
    }

    // an error exit still arrives on the head's counter (publish), so the fused o_proj blocks
    // never wait out their bound behind a workgroup that reported an error already
    auto arrive_on_error = [&]() {
        if (a.publish && tid == 0)
            atomicAdd(ws_carve(a.workspace, a.heads, ns).counters + (size_t)h * kCntWordsPerHead, 1u);
    };
    if (pos < 0 || pos >= a.max_seq) {  // host validates; guard against a stale state
        arrive_on_error();
        return;
    }
    if constexpr (HOST_SIZED) {
        // the grid (and the o_proj's merge count) came from the host's position: if the
        // device state disagrees, keys past nact * CH would be dropped or stale partials
        // merged -- report it (tokens_out raises) instead of computing a wrong token
        if (pos / CH + 1 != a.nact) {
            if (a.err != nullptr && tid == 0 && split == 0) atomicOr(a.err, 4);
            arrive_on_error();
            return;
        }
    }
    const int ctx = pos + 1;
    if (start >= ctx) {
        arrive_on_error();
        return;
    }
    const int end = min(start + CH, ctx);
    const int nact = (ctx + CH - 1) / CH;
    const bool owns_pos = (end == ctx);

    // ---- issue every K and V row load of this block first: they do not depend on
    // q, so their HBM latency overlaps the q/RoPE prologue (NPG rows per lane each)
    // branch-free: rows past `end` or at `pos` load a valid row (start) and are ignored
    // later -- a predicated load would serialise the stream on vmcnt(0) waits
    if constexpr (!HOST_SIZED) {
#pragma unroll
        for (int t = 0; t < NPG; ++t) {
            const int j = start + grp + t * (kThreads / LPR);
            const int jj = (j < end && j != pos) ? j : start;
            kr[t] = ld_raw(kc + (size_t)jj * D + l16 * 8);
            vr[t] = ld_raw(vc + (size_t)jj * D + l16 * 8);
        }
    }

    // ---- q (and the current k, v when this block owns position `pos`)
    const float qscale = 1.0f / sqrtf((float)D);
    if constexpr (TAGGED) {
        if (tid < kWave) {
            auto rdy = [&](unsigned long long g) { return (unsigned)(g >> 32) == want; };
            auto all6 = [&]() { return rdy(gq0) && rdy(gq1) && rdy(gk0) && rdy(gk1) && rdy(gv0) && rdy(gv1); };
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            bool dead = false;
            if (!__all(all6())) {
                // phase 1: one granule (the head's last v element), one line per poll
                int z = 0;
                asm volatile("" : "+v"(z));  // a per-lane address: never a scalar-cache load
                while (!a.tag_poll_all && (unsigned)(ld_granule(vt + (D - 1) + z) >> 32) != want) {
                    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) { dead = true; break; }
                    __builtin_amdgcn_s_sleep(8);
                }
                // phase 2: every granule, re-loading the ones still stale
                while (!dead && !__all(all6())) {
                    if (!rdy(gq0)) gq0 = ld_granule(qt + tid);
                    if (!rdy(gq1)) gq1 = ld_granule(qt + tid + D / 2);
                    if (!rdy(gk0)) gk0 = ld_granule(kt + tid);
                    if (!rdy(gk1)) gk1 = ld_granule(kt + tid + D / 2);
                    if (!rdy(gv0)) gv0 = ld_granule(vt + tid);
                    if (!rdy(gv1)) gv1 = ld_granule(vt + tid + D / 2);
                    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) dead = true;
                    if (a.tag_poll_all) __builtin_amdgcn_s_sleep(4);
                }
            }
            if (dead && tid == 0 && a.err != nullptr) atomicOr(a.err, 64);
            if (tid == 0) ml_s[2] = dead ? 1.f : 0.f;
            pq0 = __uint_as_float((unsigned)gq0); pq1 = __uint_as_float((unsigned)gq1);
            pk0 = __uint_as_float((unsigned)gk0); pk1 = __uint_as_float((unsigned)gk1);
            if (owns_pos) {
                vcur_s[tid] = cache_round<KT>(__uint_as_float((unsigned)gv0));
                vcur_s[tid + D / 2] = cache_round<KT>(__uint_as_float((unsigned)gv1));
            }
        }
    }
    if (tid < D / 2) {
        const int i = tid;
        float c = 1.f, s = 0.f;
        if (a.rope_tab) {
            const float2 cs = reinterpret_cast<const float2*>(a.rope_tab)[(size_t)pos * (D / 2) + i];
            c = cs.x;
            s = cs.y;
        } else if (a.rope) {
            rope_cs(pos, i, D, a.rope_base, &c, &s);
        }
        // rotate_half pairing (i, i + d/2): modeling_llama.py:204-235
        const float q0 = HOST_SIZED ? pq0 : IO::ld(qrow + i), q1 = HOST_SIZED ? pq1 : IO::ld(qrow + i + D / 2);
        q_s[i] = (q0 * c - q1 * s) * qscale;
        q_s[i + D / 2] = (q1 * c + q0 * s) * qscale;
        if (owns_pos) {
            const float k0 = HOST_SIZED ? pk0 : IO::ld(krow + i), k1 = HOST_SIZED ? pk1 : IO::ld(krow + i + D / 2);
            kcur_s[i] = cache_round<KT>(k0 * c - k1 * s);
            kcur_s[i + D / 2] = cache_round<KT>(k1 * c + k0 * s);
        }
    } else if (!TAGGED && owns_pos && tid >= D && tid < 2 * D) {
        vcur_s[tid - D] = cache_round<KT>(HOST_SIZED ? pv : IO::ld(vrow + tid - D));
    }
    __syncthreads();
    if constexpr (TAGGED) {
        if (ml_s[2] != 0.f) {  // rows never arrived (error bit 64): no partials
            arrive_on_error();
            return;
        }
    }
    if (ts) ts->mark(1);  // timeline: q rotated, this split's K/V rows in registers

    if (owns_pos && (h % group) == 0 && tid < D) {
        // KV-cache write at slot pos (concat: fused_decoder_self_attention.cu:187-193,292-295)
        store_cache(kc + (size_t)pos * D + tid, kcur_s[tid]);
        store_cache(vc + (size_t)pos * D + tid, vcur_s[tid]);
    }
    // The current position is always taken from LDS, never re-read from the cache,
    // so no other workgroup depends on the store above within this launch.

    float qv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) qv[i] = q_s[l16 * 8 + i];

    // ---- scores
#pragma unroll
    for (int t = 0; t < NPG; ++t) {
        const int j = start + grp + t * (kThreads / LPR);
        float kv[8];
        if (j == pos) {
#pragma unroll
            for (int i = 0; i < 8; ++i) kv[i] = kcur_s[l16 * 8 + i];
        } else {
            unpack8(kr[t], kv);
        }
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) d = fmaf(qv[i], kv[i], d);
        d = row16_sum(d);  // LPR = 16: the group's lanes are one DPP row
        if (l16 == 0 && j < end) p_s[j - start] = d;
    }
    __syncthreads();

    // ---- local softmax over this block's positions (wave 0)
    if (tid < kWave) {
        const int n = end - start;
        float s = tid < n ? p_s[tid] : -INFINITY;
        const float m = wave_max(s);
        const float p = tid < n ? expf(s - m) : 0.f;
        const float l = wave_sum(p);
        if (tid < n) p_s[tid] = p;
        if (tid == 0) { ml_s[0] = m; ml_s[1] = l; }
    }
    __syncthreads();

    // ---- o = sum_j p_j v_j
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
#pragma unroll
    for (int t = 0; t < NPG; ++t) {
        const int j = start + grp + t * (kThreads / LPR);
        if (j >= end) break;
        float vv[8];
        if (j == pos) {
#pragma unroll
            for (int i = 0; i < 8; ++i) vv[i] = vcur_s[l16 * 8 + i];
        } else {
            unpack8(vr[t], vv);
        }
        const float p = p_s[j - start];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = fmaf(p, vv[i], acc[i]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) o_red[grp][l16 * 8 + i] = acc[i];
    __syncthreads();

    float o = 0.f;
    if (tid < D) {
#pragma unroll
        for (int g = 0; g < kThreads / LPR; ++g) o += o_red[g][tid];
    }
    if (a.direct_out && nact == 1) {  // operator API, one split: no merge needed
        if (tid < D) a.out[(size_t)h * D + tid] = o / ml_s[1];
        return;
    }
    if (ts) ts->mark(2);  // timeline: scores, softmax and P V done
    Ws ws = ws_carve(a.workspace, a.heads, ns);
    if (a.publish) {
        // the o_proj blocks of the same launch read these: every store write-through (sc1), each
        // storing wave drained, then ONE arrival per workgroup (microarch guide, hand-off table row 1)
        auto st_wt = [](float* p, float v) {
            __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        };
        if (tid < D) st_wt(ws.o + ((size_t)h * ns + split) * D + tid, o);
        if (tid == 0) {
            st_wt(ws.ml + ((size_t)h * ns + split) * 2 + 0, ml_s[0]);
            st_wt(ws.ml + ((size_t)h * ns + split) * 2 + 1, ml_s[1]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) atomicAdd(ws.counters + (size_t)h * kCntWordsPerHead, 1u);
        return;  // (no residual seed: the fused launch runs only where xacc is seeded before it)
    }
    if (tid < D) IO::st(ws.o + ((size_t)h * ns + split) * D + tid, o);
    if (tid == 0) {
        IO::st(ws.ml + ((size_t)h * ns + split) * 2 + 0, ml_s[0]);
        IO::st(ws.ml + ((size_t)h * ns + split) * 2 + 1, ml_s[1]);
    }
    // engine path: split 0 of head h seeds the fixed-point residual accumulator of
    // the next kernel (attn_oproj) with its 128-element slice: fixed(resid) on the
    // rank that carries the residual (TP rank 0), zero elsewhere
    if (a.xacc != nullptr && split == 0) {
        const int per = seed_per;
        for (int i = h * per + tid; i < min((h + 1) * per, a.hidden); i += kThreads) {
            const bool pre = HOST_SIZED && a.resid_fixed && i == h * per + (int)tid;  // prefetched in the prologue
            IO::st_ll(a.xacc + i, a.resid_scale == 0.f ? 0ll
                                  : pre            ? psd
                                  : a.resid_fixed  ? a.resid_fixed[i]
                                                   : to_fixed(a.resid[i]));
        }
    }
}


// Workgroup (h, row chunk of 16 * NPL rows). Prologue issues, before anything waits:
// its W_o slice loads (NPL rows per 16-lane group, independent of the position),
// the position, and head h's split partials (one round). Then: log-sum-exp merge
// (every row chunk of a head repeats it from L2: ~nact * 0.5 KB), 16-lane dot
// products, and one int64 fixed-point atomic add per output row.
// LDS carve of the o_proj body
template <int NPL>
constexpr size_t oproj_lds() { return (2 * kMaxSplits + 4 + D + 2 * D + 16 * NPL) * sizeof(float); }

template <typename WT, int NPL>
__device__ __forceinline__ void oproj_load_w(const OprojArgs& a, int h, int chunk, W8<WT> (&wr)[NPL]) {
    const int grp = threadIdx.x / LPR, l16 = threadIdx.x % LPR;
    const int row0 = chunk * 16 * NPL;
    const WT* w = reinterpret_cast<const WT*>(a.w);
#pragma unroll
    for (int t = 0; t < NPL; ++t) {
        int row = row0 + grp + 16 * t;
        row = row < a.n_rows ? row : a.n_rows - 1;
        const size_t off = a.head_major ? ((size_t)h * a.n_rows + row) * D : (size_t)row * a.ldw + (size_t)h * D;
        if constexpr (sizeof(WT) == 1 && NPL >= 2) {
            // int8: 16-B loads, 8 lanes per 128-column head slice, the two halves of a
            // 16-lane group on rows t = 2u and 2u + 1 (wr[u], u < NPL / 2)
            if (t < NPL / 2) {
                int r2 = row0 + grp + 16 * (2 * t + (l16 >> 3));
                r2 = r2 < a.n_rows ? r2 : a.n_rows - 1;
                const size_t off2 =
                    a.head_major ? ((size_t)h * a.n_rows + r2) * D : (size_t)r2 * a.ldw + (size_t)h * D;
                wr[t].v[0] = ld_nt16(w + off2 + (l16 & 7) * 16);
            }
        } else {
            wr[t] = ld_w8<WT>(w + off + l16 * 8);
        }
    }
}

template <typename WT, int NPL, typename IO>
__device__ __forceinline__ void oproj_body(const OprojArgs& a, int h, int chunk, int ns, float* smem) {
    float* m_s = smem;
    float* l_s = m_s + kMaxSplits;
    float& linv_s = l_s[kMaxSplits];
    float* o_s = l_s + kMaxSplits + 4;
    float (*o_red)[D] = reinterpret_cast<float (*)[D]>(o_s + D);
    float* y_s = o_s + 3 * D;
    const int tid = threadIdx.x;
    const int grp = tid / LPR, l16 = tid % LPR;
    const int row0 = chunk * 16 * NPL;
    const WT* w = reinterpret_cast<const WT*>(a.w);

    Ws ws = ws_carve(const_cast<void*>(a.workspace), a.heads, ns);
    const int d = tid % D, half = tid / D;
    const float* mlh = ws.ml + (size_t)h * ns * 2;
    const float* oh = ws.o + (size_t)h * ns * D + d;
    float ov[kMergeChunk];
    // splits to load: the host-known active count, else every split (the position
    // decides which are used)
    const int nl = a.nact > 0 ? min(a.nact, ns) : ns;
    W8<WT> wr[NPL];
    auto load_w = [&]() { oproj_load_w<WT, NPL>(a, h, chunk, wr); };
    (void)w;
    // issue order: partials first (needed first), then the W_o slice, all into
    // registers before anything waits (a load stored straight to LDS makes the compiler
    // wait for it -- and for every load issued before it -- right there, which had
    // serialised the partials' latency in front of the W_o stream)
    {
#pragma unroll
    for (int i = 0; i < kMergeChunk; ++i) {
        const int sp = half + 2 * i;
        ov[i] = IO::ld(oh + (size_t)(sp < nl ? sp : 0) * D);
    }
    constexpr int kMlPer = kMaxSplits / kThreads;
    float mr[kMlPer], lr[kMlPer];
#pragma unroll
    for (int i = 0; i < kMlPer; ++i) {
        if (i * kThreads < nl) {  // uniform branch: no per-lane predication of the loads
            const int sp = min(tid + i * kThreads, nl - 1);
            mr[i] = IO::ld(mlh + 2 * sp);
            lr[i] = IO::ld(mlh + 2 * sp + 1);
        }
    }
    load_w();
#pragma unroll
    for (int i = 0; i < kMlPer; ++i) {
        const int sp = tid + i * kThreads;
        if (i * kThreads < nl && sp < nl) {
            m_s[sp] = mr[i];
            l_s[sp] = lr[i];
        }
    }
    int nact = nl;
    if (a.nact <= 0) {  // position-derived split count (its load waits here, after the W_o issue)
        const int pos = a.pos_dev ? *a.pos_dev : a.pos_host;
        if (pos < 0 || pos >= a.max_seq) return;
        nact = (pos + 1 + CH - 1) / CH;
    }
    __syncthreads();
    // log-sum-exp weights by wave 0 (one expf per split), into LDS
    if (tid < kWave) {
        float M = -INFINITY;
        for (int sp = tid; sp < nact; sp += kWave) M = fmaxf(M, m_s[sp]);
        M = wave_max(M);
        float lsum = 0.f;
        for (int sp = tid; sp < nact; sp += kWave) {
            const float wgt = expf(m_s[sp] - M);
            m_s[sp] = wgt;
            lsum = fmaf(l_s[sp], wgt, lsum);
        }
        lsum = wave_sum(lsum);
        if (tid == 0) linv_s = 1.0f / lsum;
    }
    __syncthreads();
    float O = 0.f;
#pragma unroll
    for (int i = 0; i < kMergeChunk; ++i) {
        const int sp = half + 2 * i;
        O = fmaf(sp < nact ? ov[i] : 0.f, sp < nact ? m_s[sp] : 0.f, O);
    }
    for (int sp = half + 2 * kMergeChunk; sp < nact; sp += 2) O = fmaf(IO::ld(oh + (size_t)sp * D), m_s[sp], O);
    o_red[half][d] = O;
    __syncthreads();
    if (tid < D) o_s[tid] = (o_red[0][tid] + o_red[1][tid]) * linv_s;
    __syncthreads();
    }

    if constexpr (sizeof(WT) == 1 && NPL >= 2) {
        float x16[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) x16[i] = o_s[(l16 & 7) * 16 + i];
#pragma unroll
        for (int u = 0; u < NPL / 2; ++u) {
            const uint32_t q[4] = {wr[u].v[0].x, wr[u].v[0].y, wr[u].v[0].z, wr[u].v[0].w};
            float acc = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) acc = fmaf((float)(int8_t)((q[i / 4] >> (8 * (i % 4))) & 0xff), x16[i], acc);
            acc = oct8_sum(acc);
            if ((l16 & 7) == 0) y_s[grp + 16 * (2 * u + (l16 >> 3))] = acc;
        }
    } else {
    float xv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) xv[i] = o_s[l16 * 8 + i];
#pragma unroll
    for (int t = 0; t < NPL; ++t) {
        float wv[8];
        unpack_w8<WT>(wr[t], wv);
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) acc = fmaf(wv[i], xv[i], acc);
        acc = row16_sum(acc);
        if (l16 == 0) y_s[grp + 16 * t] = acc;
    }
    }
    __syncthreads();
    if (tid < 16 * NPL) {
        const int row = row0 + tid;
        if (row < a.n_rows) {
            float v = y_s[tid];
            if (a.scales) v *= __half2float(a.scales[row]);
            atomicAdd(reinterpret_cast<unsigned long long*>(a.xacc + row), (unsigned long long)to_fixed(v));
        }
    }
}


// Two heads per workgroup (LLMI_OPROJ_HG 2, an even head count): workgroup (head pair hp,
// row chunk of 8 * NPL rows). 16-lane groups 0-7 take head 2 hp, 8-15 head 2 hp + 1, each on
// the same NPL rows (row0 + (grp & 7) + 8 t), so a row's two head products meet in LDS and go
// out as ONE atomic of fixed(y_a) + fixed(y_b): the integer sum of the two atomics it replaces,
// so xacc is bitwise that of oproj_body, with half the atomic write traffic (512 KB at 7B).
// W_o bytes per workgroup (32 KB at NPL 8) and the workgroup count stay those of oproj_body;
// the merge is one thread per (head, dim) over every split.
template <int NPL>
constexpr size_t oproj2_lds() { return (4 * kMaxSplits + 4 + 2 * D + 2 * 8 * NPL) * sizeof(float); }

// FUSED (the o_proj part of the fused q/k/v + attention + o_proj launch, qkv_attn.hip): the W_o
// slices are issued first (they do not depend on this token), then one lane polls the two heads'
// arrival counters until all a.nact splits have published, and every partial is read with sc1
// loads after the workgroup barrier; the pair's last departing workgroup re-zeroes the counters
// for the next launch (counters word 0 of head 2 hp and 2 hp + 1: arrivals; word 1 of head 2 hp:
// departures).
__device__ __forceinline__ float ld_wt(const float* p) {
    return __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT));
}

template <typename WT, int NPL, typename IO, bool FUSED = false>
__device__ __forceinline__ void oproj_body2(const OprojArgs& a, int hp, int chunk, int ns, float* smem) {
    float* m_s = smem;                      // [2][kMaxSplits]
    float* l_s = m_s + 2 * kMaxSplits;      // [2][kMaxSplits]
    float* linv_s = l_s + 2 * kMaxSplits;   // [2] (+2 pad)
    float* o_s = linv_s + 4;                // [2][D] merged outputs
    float* y_s = o_s + 2 * D;               // [2][8 * NPL] per-head row products
    const int tid = threadIdx.x;
    const int grp = tid / LPR, l16 = tid % LPR;
    const int hs = grp >> 3, g8 = grp & 7;  // this group's head (of the pair) and row lane
    const int h = 2 * hp + hs;
    const int row0 = chunk * 8 * NPL;
    const WT* w = reinterpret_cast<const WT*>(a.w);

    Ws ws = ws_carve(const_cast<void*>(a.workspace), a.heads, ns);
    const int mh = tid >> 7, d = tid & (D - 1);  // merge: thread (head mh of the pair, dim d)
    const float* mlh = ws.ml + (size_t)(2 * hp + mh) * ns * 2;
    const float* oh = ws.o + (size_t)(2 * hp + mh) * ns * D + d;
    constexpr int kOv = 2 * kMergeChunk;
    float ov[kOv];
    const int nl = a.nact > 0 ? min(a.nact, ns) : ns;
    constexpr int kMlPer = kMaxSplits / (kThreads / 2);
    float mr[kMlPer], lr[kMlPer];
    W8<WT> wr[NPL];
    auto load_w = [&]() {
#pragma unroll
        for (int t = 0; t < NPL; ++t) {
            int row = row0 + g8 + 8 * t;
            row = row < a.n_rows ? row : a.n_rows - 1;
            if constexpr (sizeof(WT) == 1 && NPL >= 2) {
                if (t < NPL / 2) {  // int8: two rows per 16-lane group, 8 lanes each (as oproj_load_w)
                    int r2 = row0 + g8 + 8 * (2 * t + (l16 >> 3));
                    r2 = r2 < a.n_rows ? r2 : a.n_rows - 1;
                    wr[t].v[0] = ld_nt16(w + (size_t)r2 * a.ldw + (size_t)h * D + (l16 & 7) * 16);
                }
            } else {
                wr[t] = ld_w8<WT>(w + (size_t)row * a.ldw + (size_t)h * D + l16 * 8);
            }
        }
    };
    auto ld_p = [&](const float* p) { return FUSED ? ld_wt(p) : IO::ld(p); };
    if constexpr (FUSED) {
        load_w();
        unsigned* arr0 = ws.counters + (size_t)(2 * hp) * kCntWordsPerHead;
        unsigned* arr1 = arr0 + kCntWordsPerHead;
        if (tid == 0) {
            const unsigned want = (unsigned)nl;
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            bool dead = false;
            while (__hip_atomic_load(arr0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want ||
                   __hip_atomic_load(arr1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) { dead = true; break; }
                __builtin_amdgcn_s_sleep(8);
            }
            if (dead && a.err) atomicOr(a.err, 64);
            linv_s[2] = dead ? 1.f : 0.f;
        }
        __syncthreads();
        if (linv_s[2] != 0.f) return;
    }
    // issue order as oproj_body: partials, (m, l), then the W_o slices, before any wait
#pragma unroll
    for (int i = 0; i < kOv; ++i) ov[i] = ld_p(oh + (size_t)(i < nl ? i : 0) * D);
#pragma unroll
    for (int i = 0; i < kMlPer; ++i) {
        if (i * (kThreads / 2) < nl) {
            const int sp = min(d + i * (kThreads / 2), nl - 1);
            mr[i] = ld_p(mlh + 2 * sp);
            lr[i] = ld_p(mlh + 2 * sp + 1);
        }
    }
    if constexpr (!FUSED) load_w();
#pragma unroll
    for (int i = 0; i < kMlPer; ++i) {
        const int sp = d + i * (kThreads / 2);
        if (i * (kThreads / 2) < nl && sp < nl) {
            m_s[mh * kMaxSplits + sp] = mr[i];
            l_s[mh * kMaxSplits + sp] = lr[i];
        }
    }
    int nact = nl;
    if (a.nact <= 0) {
        const int pos = a.pos_dev ? *a.pos_dev : a.pos_host;
        if (pos < 0 || pos >= a.max_seq) return;
        nact = (pos + 1 + CH - 1) / CH;
    }
    __syncthreads();
    // log-sum-exp weights: wave 0 for head 0 of the pair, wave 2 for head 1
    if ((tid & (D - 1)) < kWave) {
        float* mw = m_s + mh * kMaxSplits;
        const float* lw = l_s + mh * kMaxSplits;
        const int ln = tid & (kWave - 1);
        float M = -INFINITY;
        for (int sp = ln; sp < nact; sp += kWave) M = fmaxf(M, mw[sp]);
        M = wave_max(M);
        float lsum = 0.f;
        for (int sp = ln; sp < nact; sp += kWave) {
            const float wgt = expf(mw[sp] - M);
            mw[sp] = wgt;
            lsum = fmaf(lw[sp], wgt, lsum);
        }
        lsum = wave_sum(lsum);
        if (ln == 0) linv_s[mh] = 1.0f / lsum;
    }
    __syncthreads();
    {
        // the same two interleaved partial sums (even / odd splits) oproj_body's two
        // threads per dim form, added in the same order: bitwise its merged output
        const float* mw = m_s + mh * kMaxSplits;
        float O0 = 0.f, O1 = 0.f;
#pragma unroll
        for (int i = 0; i < kMergeChunk; ++i) {
            const int s0 = 2 * i, s1 = 2 * i + 1;
            O0 = fmaf(s0 < nact ? ov[s0] : 0.f, s0 < nact ? mw[s0] : 0.f, O0);
            O1 = fmaf(s1 < nact ? ov[s1] : 0.f, s1 < nact ? mw[s1] : 0.f, O1);
        }
        for (int sp = kOv; sp < nact; sp += 2) {
            O0 = fmaf(ld_p(oh + (size_t)sp * D), mw[sp], O0);
            if (sp + 1 < nact) O1 = fmaf(ld_p(oh + (size_t)(sp + 1) * D), mw[sp + 1], O1);
        }
        o_s[mh * D + d] = (O0 + O1) * linv_s[mh];
    }
    __syncthreads();
    if constexpr (FUSED) {
        // every partial of this workgroup is read (the barrier above): depart; the pair's last
        // workgroup re-zeroes both arrival counters and the departure counter
        if (tid == 0) {
            unsigned* arr0 = ws.counters + (size_t)(2 * hp) * kCntWordsPerHead;
            const int n_chunks = (a.n_rows + 8 * NPL - 1) / (8 * NPL);
            if (atomicAdd(arr0 + 1, 1u) == (unsigned)(n_chunks - 1)) {
                __hip_atomic_store(arr0, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(arr0 + kCntWordsPerHead, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(arr0 + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    float* yh = y_s + hs * 8 * NPL;
    const float* oh_s = o_s + hs * D;
    if constexpr (sizeof(WT) == 1 && NPL >= 2) {
        float x16[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) x16[i] = oh_s[(l16 & 7) * 16 + i];
#pragma unroll
        for (int u = 0; u < NPL / 2; ++u) {
            const uint32_t q[4] = {wr[u].v[0].x, wr[u].v[0].y, wr[u].v[0].z, wr[u].v[0].w};
            float acc = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) acc = fmaf((float)(int8_t)((q[i / 4] >> (8 * (i % 4))) & 0xff), x16[i], acc);
            acc = oct8_sum(acc);
            if ((l16 & 7) == 0) yh[g8 + 8 * (2 * u + (l16 >> 3))] = acc;
        }
    } else {
        float xv[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) xv[i] = oh_s[l16 * 8 + i];
#pragma unroll
        for (int t = 0; t < NPL; ++t) {
            float wv[8];
            unpack_w8<WT>(wr[t], wv);
            float acc = 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i) acc = fmaf(wv[i], xv[i], acc);
            acc = row16_sum(acc);
            if (l16 == 0) yh[g8 + 8 * t] = acc;
        }
    }
    __syncthreads();
    if (tid < 8 * NPL) {
        const int row = row0 + tid;
        if (row < a.n_rows) {
            float va = y_s[tid], vb = y_s[8 * NPL + tid];
            if (a.scales) {
                const float sc = __half2float(a.scales[row]);
                va *= sc;
                vb *= sc;
            }
            atomicAdd(reinterpret_cast<unsigned long long*>(a.xacc + row),
                      (unsigned long long)(to_fixed(va) + to_fixed(vb)));
        }
    }
}

}  // namespace attn_detail
}  // namespace llmi
