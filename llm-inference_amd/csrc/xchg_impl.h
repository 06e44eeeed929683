// Device side of the one-shot peer exchange (xchg.hip), shared by its own kernel and by
// the producer-fused form: the o_proj / down / lm_head kernels that finish with
// xchg_tail() push their finished vector from inside the launch (no exchange launch, no
// extra kernel boundary per exchange). Protocol and inbox layout: xchg.hip header.
#pragma once
#include "kernels.h"

namespace llmi {
namespace xchg_detail {

constexpr unsigned long long kTimeoutTicks = 200000000ull;  // 2 s of s_memrealtime (100 MHz)

__device__ __forceinline__ size_t data_elems(const XchgArgs& a) { return (size_t)2 * a.cap_w * a.cap_n; }
__device__ __forceinline__ long long* slot_of(const XchgArgs& a, char* base, int ph, int q) {
    return reinterpret_cast<long long*>(base) + ((size_t)ph * a.cap_w + q) * a.cap_n;
}
__device__ __forceinline__ unsigned long long* flag_of(const XchgArgs& a, char* base, int ph, int q, int g) {
    return reinterpret_cast<unsigned long long*>(reinterpret_cast<long long*>(base) + data_elems(a)) +
           ((size_t)ph * a.cap_w + q) * kXchgMaxSlices + g;
}
__device__ __forceinline__ long long ld_agent(const long long* p) {
    return (long long)__hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<long long*>(p)),
                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Write-through (system-coherent, sc0 sc1) 8-B store / load: the inboxes are uncached HBM,
// local or a peer's over xGMI, so these reach memory without any L2 write-back or invalidate
// (a system-scope release / acquire fence costs a whole-L2 wbl2 / inv per wave: with one per
// flag store and per wave, an exchange cost ~10 us on one GPU, r05a)
__device__ __forceinline__ void st_sys(long long* p, long long v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ long long ld_sys(const long long* p) {
    return (long long)__hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<long long*>(p)),
                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Push slice g (elements [g * kXchgSlice, ...) of a.buf) into slot [ph][rank] of every
// inbox, then raise flag [ph][rank][g] = e in every inbox. Block-wide (every thread calls).
// AGENT: read buf with agent-scope loads (its values were produced inside this launch by
// other workgroups' device-scope atomics / released stores).
// Ordering without fences: every payload store is write-through; each wave waits for its
// stores' acknowledgements (vmcnt 0: the data is in the target's memory), the barrier orders
// that before thread 0's flag stores, which are write-through too.
template <bool AGENT>
__device__ __forceinline__ void push_slice(const XchgArgs& a, int g, unsigned long long e) {
    const int ph = (int)(e & 1ull);
    const int i_end = min(a.n, (g + 1) * kXchgSlice);
    char* peer[kXchgMaxWorld];  // every inbox base, loaded together (one round trip, not one per rank)
#pragma unroll
    for (int q = 0; q < kXchgMaxWorld; ++q) peer[q] = a.peers[q < a.world ? q : 0];
    for (int i0 = g * kXchgSlice + 2 * (int)threadIdx.x; i0 < i_end; i0 += 2 * (int)blockDim.x) {
        longlong2 v = make_longlong2(0, 0);
        if constexpr (AGENT) {
            v.x = ld_agent(a.buf + i0);
            if (i0 + 1 < a.n) v.y = ld_agent(a.buf + i0 + 1);
        } else if (i0 + 1 < a.n) {
            v = *reinterpret_cast<const longlong2*>(a.buf + i0);
        } else {
            v.x = a.buf[i0];
        }
#pragma unroll
        for (int q = 0; q < kXchgMaxWorld; ++q) {
            if (q >= a.world) break;
            const bool zero = a.loop && q != a.rank;  // loopback: the other ranks' slots get zeros
            long long* d = slot_of(a, peer[q], ph, a.loop ? q : a.rank) + i0;
            st_sys(d, zero ? 0ll : v.x);
            st_sys(d + 1, zero ? 0ll : v.y);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's payload acknowledged
    __syncthreads();                                    // ... every wave's, before the flags
    if ((int)threadIdx.x < a.world) {  // one lane per rank raises that inbox's flag
        char* pb = peer[0];
#pragma unroll
        for (int q = 1; q < kXchgMaxWorld; ++q)
            if ((int)threadIdx.x == q) pb = peer[q];
        __hip_atomic_store(flag_of(a, pb, ph, a.loop ? (int)threadIdx.x : a.rank, g), e, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Wait until every rank's slice g of exchange e arrived in this rank's inbox, sum (op 0) /
// max (op 2) the W slots in rank order into a.buf, and record e as slice g's epoch.
// Block-wide. A peer that never arrives: error bit 8 (tokens_out raises), later waits skip.
// The W slot loads are all issued before the first is used (one memory round trip, not W).
__device__ __forceinline__ void reduce_slice(const XchgArgs& a, int g, unsigned long long e) {
    const int ph = (int)(e & 1ull);
    char* own = a.peers[a.rank];
    if ((int)threadIdx.x < a.world) {
        unsigned long long* f = flag_of(a, own, ph, threadIdx.x, g);
        const bool dead = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 8;
        if (!dead) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            for (unsigned it = 0;; ++it) {
                if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == e) break;
                if ((it & 63u) == 63u && __builtin_amdgcn_s_memrealtime() - t0 > kTimeoutTicks) {
                    atomicOr(a.err, 8);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        // The ordering this relies on, stated rather than implied: (1) the
        // inboxes are hipDeviceMallocUncached (MTYPE UC), so payload and flag accesses bypass
        // L1 / L2 on the producing and the consuming GPU alike, and each payload store is
        // acknowledged (vmcnt 0, push_slice) before the flag store is issued; (2) every slot
        // load below is a system-scope (sc0 sc1) load, issued after this poll. That is the
        // write-through form of cdna_hip_programming.md Guideline 16 (every handed-off byte
        // stored sc1 and drained, every load of it sc1), where the acquire reduces to an
        // ordering point for the compiler -- which this fence is: it keeps the slot loads
        // below the observation of the flag. A release / acquire pair at system scope would
        // cost a whole-L2 write-back / invalidate per slice (r05a: ~10 us an exchange).
        // Validated on one GPU (loopback, in-process group, two processes over IPC); the
        // first cross-GPU run is the driver's, where bench.py keeps the one-shot path only if
        // its tokens equal RCCL's on every rank.
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __syncthreads();  // the flags were seen before any slot is read (write-through loads below)
    const int i_end = min(a.n, (g + 1) * kXchgSlice);
    for (int i0 = g * kXchgSlice + 2 * (int)threadIdx.x; i0 < i_end; i0 += 2 * (int)blockDim.x) {
        long long v0[kXchgMaxWorld], v1[kXchgMaxWorld];
#pragma unroll
        for (int q = 0; q < kXchgMaxWorld; ++q) {
            const long long* sp = slot_of(a, own, ph, q < a.world ? q : 0) + i0;
            v0[q] = ld_sys(sp);
            v1[q] = ld_sys(sp + 1);
        }
        long long s0 = 0, s1 = 0;
        unsigned long long m0 = 0, m1 = 0;
#pragma unroll
        for (int q = 0; q < kXchgMaxWorld; ++q) {
            if (q < a.world) {
                s0 += v0[q];
                s1 += v1[q];
                m0 = max(m0, (unsigned long long)v0[q]);
                m1 = max(m1, (unsigned long long)v1[q]);
            }
        }
        a.buf[i0] = a.op == 0 ? s0 : (long long)m0;
        if (i0 + 1 < a.n) a.buf[i0 + 1] = a.op == 0 ? s1 : (long long)m1;
    }
    if (threadIdx.x == 0) a.ep[g] = e;
}

// The producer-fused exchange: called by EVERY thread of EVERY workgroup of a kernel whose
// workgroups produced a.buf with device-scope atomics or agent-scope (sc1) stores -- both
// land at the point of coherence, so a drained workgroup needs no release fence (an agent
// release per workgroup, i.e. an L2 write-back from each of up to ~1000 workgroups, cost
// ~18 us per launch in the first version; so did a single arrival counter, whose
// same-address atomics serialise at ~10 ns each). Arrivals are counted on kTailShards
// counters (workgroup b -> shard b % S, one 128-B line each); the workgroup that completes
// its shard re-zeroes that shard (all of its members have arrived) and takes a ticket on
// the top counter. These S shard finishers wait for the top counter to reach S, then
// finisher g pushes (a.mode & 1) and reduces (a.mode & 2) slices g, g + S, ... The last
// finisher to leave re-zeroes the top pair, so the next fused launch on the stream finds
// every word zero (they are zeroed once at allocation). lds: one int of LDS scratch.
// Waits are bounded (error bit 8), so a lost peer ends the run with an error, never a hang.
constexpr int kTailShards = 32;
constexpr int kTailStride = 32;  // words between counters (128 B)
constexpr int kTailWords = (kTailShards + 2) * kTailStride;  // shards, then top, then done
__device__ __forceinline__ void xchg_tail(const XchgArgs& a, unsigned* cnt, int* lds) {
    if (a.buf == nullptr) return;
    const int G = (int)(gridDim.x * gridDim.y * gridDim.z);
    const int b = (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
    const int S = G < kTailShards ? G : kTailShards;
    const int sh = b % S;
    const int members = G / S + (sh < G % S ? 1 : 0);
    unsigned* shard = cnt + sh * kTailStride;
    unsigned* top = cnt + kTailShards * kTailStride;
    unsigned* done = top + kTailStride;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's atomics / sc1 stores landed
    __syncthreads();
    if (threadIdx.x == 0) {
        int g = -1;
        if (__hip_atomic_fetch_add(shard, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)members - 1) {
            __hip_atomic_store(shard, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            g = (int)__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        *lds = g;
    }
    __syncthreads();
    const int g = *lds;
    if (g < 0) return;
    if (threadIdx.x == 0) {  // every shard complete (the other finishers are resident: they are running)
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        for (unsigned it = 0;; ++it) {
            if (__hip_atomic_load(top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)S) break;
            if ((it & 63u) == 63u && __builtin_amdgcn_s_memrealtime() - t0 > kTimeoutTicks) {
                atomicOr(a.err, 8);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    const int ns = (a.n + kXchgSlice - 1) / kXchgSlice;
    for (int sl = g; sl < ns; sl += S) {
        const unsigned long long e = a.ep[sl] + 1;
        if (a.mode & 1) push_slice<true>(a, sl, e);
        if (a.mode & 2) reduce_slice(a, sl, e);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const unsigned d = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d == (unsigned)S - 1) {  // every finisher is past its wait
            __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace xchg_detail
}  // namespace llmi
