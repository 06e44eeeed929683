// llmi-prng-v1: counter-based synthetic-weight stream, bit-identical on host
// (C++ here, numpy in oracle/prng.py) and device. Spec in oracle/prng.py.
// Replaces the reference's host rand()%100/100000 dummy loader
// (src/weights/llama/layer_weights.cc:69-146, llama_weights.cc:56-88).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <cstdint>

namespace llmi {
namespace prng {

constexpr uint64_t GOLD = 0x9E3779B97F4A7C15ull;

enum Kind : uint32_t {
    Q = 0, K = 1, V = 2, O = 3, GATE = 4, UP = 5, DOWN = 6, ATTN_NORM = 7, FFN_NORM = 8,
    Q_SCALE = 16,
};
enum Global : uint32_t { EMBED = 1, LM_HEAD = 2, FINAL_NORM = 3, PROMPT = 0xFFFF };

__host__ __device__ __forceinline__ uint32_t layer_tid(int layer, uint32_t kind) {
    return ((uint32_t)(layer + 1) << 8) | kind;
}

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t tensor_key(uint64_t seed, uint32_t tid) {
    return mix64(seed * GOLD + (uint64_t)tid);
}
__host__ __device__ __forceinline__ uint64_t bits(uint64_t key, uint64_t idx) {
    return mix64(key + (idx + 1ull) * GOLD);
}
__host__ __device__ __forceinline__ int32_t i24(uint64_t r) {
    return (int32_t)(r >> 40) - (1 << 23);
}

// Value generators: exact fp32 products, one IEEE fp32 add where noted.
// Explicit __fmul_rn/__fadd_rn on device keep hipcc from contracting to FMA.
__host__ __device__ __forceinline__ float mul_rn(float a, float b) {
#ifdef __HIP_DEVICE_COMPILE__
    return __fmul_rn(a, b);
#else
    volatile float r = a * b;
    return r;
#endif
}
__host__ __device__ __forceinline__ float add_rn(float a, float b) {
#ifdef __HIP_DEVICE_COMPILE__
    return __fadd_rn(a, b);
#else
    volatile float r = a + b;
    return r;
#endif
}

__host__ __device__ __forceinline__ float linear_f32(uint64_t key, uint64_t idx) {
    return mul_rn((float)i24(bits(key, idx)), 0x1p-28f);
}
__host__ __device__ __forceinline__ float embed_f32(uint64_t key, uint64_t idx) {
    return mul_rn((float)i24(bits(key, idx)), 0x1p-23f);
}
__host__ __device__ __forceinline__ float gamma_f32(uint64_t key, uint64_t idx) {
    return add_rn(1.0f, mul_rn((float)i24(bits(key, idx)), 0x1p-26f));
}
__host__ __device__ __forceinline__ int8_t int8_w(uint64_t key, uint64_t idx) {
    return (int8_t)((int)(bits(key, idx) >> 56) - 128);
}
__host__ __device__ __forceinline__ float int8_scale_f32(uint64_t key, uint64_t idx) {
    return mul_rn(add_rn(1.0f, mul_rn((float)i24(bits(key, idx)), 0x1p-24f)), 0x1p-12f);
}

}  // namespace prng
}  // namespace llmi
