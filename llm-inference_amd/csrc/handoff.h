// Memory-access and synchronisation policies shared by the standalone decode
// kernels and the dataflow layer kernel (layer.hip).
//
// Standalone kernels use PlainIO + NoSync: kernel boundaries order everything.
// Inside one launch, bytes handed from one workgroup to another follow the
// write-through form of cdna_hip_programming.md §6 Guideline 16 /
// MI355X_MICROARCH.md "Valid forms" (table row 1): every store of handed-off
// bytes is `sc1`, every storing wave drains (`s_waitcnt vmcnt(0)`) before a
// workgroup barrier, one lane then adds to the phase counter (agent scope);
// the consumer's wave 0 polls the counter with `sc1` loads, the other waves
// pass a barrier after the match, and every load of handed-off bytes is `sc1`.
// Counters are sharded 8 ways (blockIdx & 7 ~ one XCD) to spread the fan-in.
// Spins are bounded by wall time: a wait that times out sets an error bit and
// the launch still drains (wrong tokens, never a hung GPU).
#pragma once
#include "common.h"

namespace llmi {

struct PlainIO {
    static constexpr bool kSc1 = false;
    __device__ __forceinline__ static float ld(const float* p) { return *p; }
    __device__ __forceinline__ static void st(float* p, float v) { *p = v; }
    __device__ __forceinline__ static void st_ll(long long* p, long long v) { *p = v; }
    __device__ __forceinline__ static float4 ld4(const float4* p) { return *p; }
    __device__ __forceinline__ static longlong2 ld_ll2(const longlong2* p) { return *p; }
    __device__ __forceinline__ static long long ld_ll(const long long* p) { return *p; }
    __device__ __forceinline__ static void st4(float4* p, float4 v) { *p = v; }
};

struct Sc1IO {
    static constexpr bool kSc1 = true;
    __device__ __forceinline__ static float ld(const float* p) {
        return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ __forceinline__ static void st(float* p, float v) {
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ __forceinline__ static void st_ll(long long* p, long long v) {
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ __forceinline__ static unsigned long long ld_u64(const void* p) {
        return __hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<void*>(p)), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
    }
    __device__ __forceinline__ static float4 ld4(const float4* p) {
        const unsigned long long a = ld_u64(p), b = ld_u64(reinterpret_cast<const char*>(p) + 8);
        return make_float4(__uint_as_float((unsigned)a), __uint_as_float((unsigned)(a >> 32)),
                           __uint_as_float((unsigned)b), __uint_as_float((unsigned)(b >> 32)));
    }
    __device__ __forceinline__ static longlong2 ld_ll2(const longlong2* p) {
        longlong2 r;
        r.x = (long long)ld_u64(p);
        r.y = (long long)ld_u64(reinterpret_cast<const char*>(p) + 8);
        return r;
    }
    __device__ __forceinline__ static long long ld_ll(const long long* p) { return (long long)ld_u64(p); }
    __device__ __forceinline__ static void st4(float4* p, float4 v) {
        float* f = reinterpret_cast<float*>(p);
        st(f, v.x);
        st(f + 1, v.y);
        st(f + 2, v.z);
        st(f + 3, v.w);
    }
};

constexpr int kCntShards = 8;
constexpr int kCntStride = 32;  // u32 words between shards (one 128-B line each)
constexpr int kPhaseCntWords = kCntShards * kCntStride;

struct NoSync {
    static constexpr bool kFlow = false;
    __device__ __forceinline__ void wait() const {}
    __device__ __forceinline__ void publish() const {}
};

struct FlowSync {
    static constexpr bool kFlow = true;
    const unsigned* wait_cnt = nullptr;  // previous phase's sharded counter (nullptr: no wait)
    unsigned wait_target = 0;            // arrivals that complete it
    unsigned* pub_cnt = nullptr;         // this phase's sharded counter
    int* err = nullptr;                  // sticky error word (bit 4: wait timed out)
    unsigned long long* stamp = nullptr; // optional timeline: [1] = wall clock when the wait passed

    __device__ __forceinline__ void wait() const {
        wait_poll();
        if (stamp && threadIdx.x == 0) stamp[1] = __builtin_amdgcn_s_memrealtime();
    }
    __device__ __forceinline__ void wait_poll() const {
        if (wait_cnt == nullptr) return;
        if (threadIdx.x < kWave) {
            const int lane = threadIdx.x;
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
            for (;;) {
                unsigned v = lane < kCntShards
                                 ? __hip_atomic_load(const_cast<unsigned*>(wait_cnt) + lane * kCntStride,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                 : 0u;
                v += __shfl_xor(v, 1, kWave);
                v += __shfl_xor(v, 2, kWave);
                v += __shfl_xor(v, 4, kWave);
                if (__shfl(v, 0, kWave) >= wait_target) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {  // 200 ms: give up
                    if (lane == 0) atomicOr(err, 4);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __syncthreads();
    }
    __device__ __forceinline__ void publish() const {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_fetch_add(pub_cnt + (blockIdx.x & (kCntShards - 1)) * kCntStride, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    }
};

}  // namespace llmi
