// Shared helpers for the llmi HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <stdexcept>

#include "../../include/llmi.h"

namespace llmi {

constexpr int kWave = 64;

// ---------------------------------------------------------------- errors
void set_last_error(const std::string& msg);

struct Status {
    int code = LLMI_OK;
};

#define LLMI_HIP(expr)                                                                 \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess) {                                                        \
            ::llmi::set_last_error(std::string(#expr) + ": " + hipGetErrorString(_e) + \
                                   " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
            return LLMI_EHIP - (int)_e;                                                \
        }                                                                              \
    } while (0)

#define LLMI_REQUIRE(cond, msg)                                                        \
    do {                                                                               \
        if (!(cond)) {                                                                 \
            ::llmi::set_last_error(std::string("[llmi][ERROR] ") + (msg) + " (" #cond ")"); \
            return LLMI_EINVAL;                                                        \
        }                                                                              \
    } while (0)

#define LLMI_TRY(expr)                  \
    do {                                \
        int _rc = (expr);               \
        if (_rc != LLMI_OK) return _rc; \
    } while (0)

inline size_t dtype_size(int dt) {
    switch (dt) {
        case LLMI_F32: return 4;
        case LLMI_F16: return 2;
        case LLMI_I8: return 1;
        case LLMI_I32: return 4;
        default: return 0;
    }
}

// ------------------------------------------------------------ device math
__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(__half v) { return __half2float(v); }
__device__ __forceinline__ float to_f32(int8_t v) { return (float)v; }

// Cross-lane butterflies without the LDS crossbar (__shfl_xor compiles to ds_bpermute_b32:
// an LDS round trip per step, on the critical path of every reduction tail). Lane ^ 32 and
// ^ 16 use the gfx950 row swaps (v_permlane32_swap / v_permlane16_swap of x with itself: the
// pair holds x[l] and x[l ^ 32 / 16]); lane ^ 8 ... ^ 1 use DPP row rotations, which equal the
// xor partner once the earlier steps made the values symmetric (rotating a 16-lane row by 8
// is ^ 8; after it, by 4 lands on a lane equal to l ^ 4, and so on). Each step adds the same
// two values as the xor butterfly (a + b == b + a), so every sum and max keeps its exact bits.
template <int N>
__device__ __forceinline__ float row_ror(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x120 + N, 0xF, 0xF,
                                                                 false));
}
__device__ __forceinline__ float swap32_add(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap16_add(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float swap32_max(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float swap16_max(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// sum over each aligned 8-lane group (the xor 4, 2, 1 butterfly's association): lane ^ 4 is
// the row shift left or right by 4, chosen by the lane's bit 2; ^ 2 and ^ 1 are quad permutes
__device__ __forceinline__ float oct8_sum(float v) {
    const float up = dpp<0x104>(v), down = dpp<0x114>(v);  // row_shl:4 / row_shr:4
    v += (threadIdx.x & 4) ? down : up;
    v += dpp<0x4E>(v);  // quad_perm [2, 3, 0, 1]
    v += dpp<0xB1>(v);  // quad_perm [1, 0, 3, 2]
    return v;
}
// lane ^ 4 within aligned 8-lane groups: the row shift left or right by 4 by the lane's bit 2
__device__ __forceinline__ float xor4(float v) {
    const float up = dpp<0x104>(v), down = dpp<0x114>(v);  // row_shl:4 / row_shr:4
    return (threadIdx.x & 4) ? down : up;
}
// the xor 1, 2, 4 butterfly over aligned 8-lane groups (quad permutes, then xor4)
__device__ __forceinline__ float oct8_sum_up(float v) {
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    return v + xor4(v);
}
__device__ __forceinline__ float oct8_max_up(float v) {
    v = fmaxf(v, dpp<0xB1>(v));
    v = fmaxf(v, dpp<0x4E>(v));
    return fmaxf(v, xor4(v));
}
// sum over each aligned 16-lane group (the xor 8, 4, 2, 1 butterfly's association)
__device__ __forceinline__ float row16_sum(float v) {
    v += row_ror<8>(v);
    v += row_ror<4>(v);
    v += row_ror<2>(v);
    v += row_ror<1>(v);
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {  // the xor 32, 16, ..., 1 butterfly
    return row16_sum(swap16_add(swap32_add(v)));
}
__device__ __forceinline__ float wave_max(float v) {
    v = swap16_max(swap32_max(v));
    v = fmaxf(v, row_ror<8>(v));
    v = fmaxf(v, row_ror<4>(v));
    v = fmaxf(v, row_ror<2>(v));
    return fmaxf(v, row_ror<1>(v));
}

// Block-wide sum for blockDim.x <= 1024; `red` needs >= 16 floats of LDS.
__device__ __forceinline__ float block_sum(float v, float* red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
    for (int i = 0; i < nw; ++i) t += red[i];
    return t;
}

// Order-preserving 64-bit key for (value, index) argmax: larger value wins,
// ties go to the lower index (torch/numpy argmax semantics).
__host__ __device__ __forceinline__ unsigned long long argmax_key(float v, uint32_t idx) {
    uint32_t b;
#ifdef __HIP_DEVICE_COMPILE__
    b = __float_as_uint(v);
#else
    std::memcpy(&b, &v, 4);
#endif
    b = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    return ((unsigned long long)b << 32) | (unsigned long long)(0xFFFFFFFFu - idx);
}
__host__ __device__ __forceinline__ uint32_t argmax_key_index(unsigned long long k) {
    return 0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFull);
}

// Nontemporal 16-byte weight load: weights are streamed once per token and
// never fit the 256 MiB Infinity Cache (MI355X_MICROARCH.md, row nt-weights).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt16(const void* p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

// fp8 lo plane of the prefill GEMMs (split mode 3, gemm3.hip): an fp32 activation
// a = hi + lo with hi = fp16(a) and |lo| <= 2^-11 |a|; lo is kept as OCP e4m3 of
// lo * 2^kLo8Exp, clamped to +-448 (an element whose scaled lo would overflow, |a| >
// ~224, keeps only its hi: the fp16-activation precision). The GEMM's block-scaled fp8
// MFMA undoes the scale through its E8M0 operand scale (127 - kLo8Exp).
constexpr int kLo8Exp = 12;
__device__ __forceinline__ uint32_t lo8_pack4(float l0, float l1, float l2, float l3) {
    auto c = [](float v) { return fminf(fmaxf(v * (float)(1 << kLo8Exp), -448.f), 448.f); };
    int r = __builtin_amdgcn_cvt_pk_fp8_f32(c(l0), c(l1), 0, false);
    r = __builtin_amdgcn_cvt_pk_fp8_f32(c(l2), c(l3), r, true);
    return (uint32_t)r;
}

// Debug timeline (diagnostics only; a null base costs one scalar compare): per
// workgroup 8 u64 at base + 8 * linear block id: [0] start, [1]/[2] kernel-defined
// marks, [3] end, [4] __smid() -- 100 MHz s_memrealtime clock.
struct WgStamp {
    unsigned long long* p;
    unsigned long long t0;
    __device__ __forceinline__ explicit WgStamp(unsigned long long* base)
        : p(base ? base + 8 * ((size_t)blockIdx.x + (size_t)gridDim.x * blockIdx.y) : nullptr),
          t0(base ? __builtin_amdgcn_s_memrealtime() : 0ull) {}
    __device__ __forceinline__ void mark(int i) const {
        if (p && threadIdx.x == 0) p[i] = __builtin_amdgcn_s_memrealtime();
    }
    __device__ __forceinline__ ~WgStamp() {
        if (p && threadIdx.x == 0) {
            p[0] = t0;
            p[3] = __builtin_amdgcn_s_memrealtime();
            p[4] = __smid();
        }
    }
};

}  // namespace llmi
