// Activation access policy of the decode kernel bodies (gemv_impl.h, attn_impl.h):
// plain loads and stores -- kernel boundaries order every hand-off between kernels.
#pragma once
#include "common.h"

namespace llmi {

struct PlainIO {
    __device__ __forceinline__ static float ld(const float* p) { return *p; }
    __device__ __forceinline__ static void st(float* p, float v) { *p = v; }
    __device__ __forceinline__ static void st_ll(long long* p, long long v) { *p = v; }
    __device__ __forceinline__ static float4 ld4(const float4* p) { return *p; }
    __device__ __forceinline__ static longlong2 ld_ll2(const longlong2* p) { return *p; }
    __device__ __forceinline__ static long long ld_ll(const long long* p) { return *p; }
    __device__ __forceinline__ static void st4(float4* p, float4 v) { *p = v; }
};

}  // namespace llmi
