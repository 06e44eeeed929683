// The reference's sampling draw, curand_init(step, row, 0) + curand_uniform
// (/root/reference/src/kernels/sampling.cu:66-69), restated from cuRAND's published
// XORWOW (curand_kernel.h, a CUDA toolkit header that is not in the reference; the
// algorithm is unchanged since CUDA 3.2). oracle/xorwow.py is the CPU restatement.
//   seed:  s0 = lo32 ^ 0xaad26b49, s1 = hi32 ^ 0xf7dcefdd, t0 = 1099087573 s0,
//          t1 = 2591861531 s1; d = 6615241 + t1 + t0; v = (123456789 + t0,
//          362436069 ^ t0, 521288629 + t1, 88675123 ^ t1, 5783321 + t0)
//   row:   the state jumped by row * 2^67 steps: the step is GF(2)-linear on the 160-bit
//          v, so the jump is the matrix M^(2^67 2^i) per set bit i of row (a host-built
//          table, xorwow_jump_table); d moves by 2^67 * 362437 = 0 mod 2^32
//   draw:  t = v0 ^ (v0 >> 2); shift v; v4 = (v4 ^ (v4 << 4)) ^ (t ^ (t << 1));
//          d += 362437; x = v4 + d;  u = x * 2^-32 + 2^-33 (float, in (0, 1])
#pragma once
#include <cstdint>

#include "common.h"

namespace llmi {

constexpr int kXorwowJumpBits = 16;  // rows (subsequences) < 2^16

struct XorwowState {
    uint32_t v[5];
    uint32_t d;
};

__host__ __device__ __forceinline__ XorwowState xorwow_init(uint64_t seed) {
    const uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u, s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    const uint32_t t0 = 1099087573u * s0, t1 = 2591861531u * s1;
    XorwowState s;
    s.d = 6615241u + t1 + t0;
    s.v[0] = 123456789u + t0;
    s.v[1] = 362436069u ^ t0;
    s.v[2] = 521288629u + t1;
    s.v[3] = 88675123u ^ t1;
    s.v[4] = 5783321u + t0;
    return s;
}

__host__ __device__ __forceinline__ uint32_t xorwow_next(XorwowState& s) {
    const uint32_t t = s.v[0] ^ (s.v[0] >> 2);
    s.v[0] = s.v[1];
    s.v[1] = s.v[2];
    s.v[2] = s.v[3];
    s.v[3] = s.v[4];
    s.v[4] = (s.v[4] ^ (s.v[4] << 4)) ^ (t ^ (t << 1));
    s.d += 362437u;
    return s.v[4] + s.d;
}

__host__ __device__ __forceinline__ float xorwow_uniform(uint32_t x) {
    return (float)x * 0x1p-32f + 0x1p-33f;  // the product is exact: one rounding, fused or not
}

// v <- M^(2^67 * row) v with table [kXorwowJumpBits][160 columns][5 words]
__host__ __device__ inline void xorwow_jump(XorwowState& s, uint32_t row, const uint32_t* table) {
    for (int i = 0; i < kXorwowJumpBits && row; ++i, row >>= 1) {
        if (!(row & 1u)) continue;
        const uint32_t* cols = table + (size_t)i * 160 * 5;
        uint32_t r[5] = {0u, 0u, 0u, 0u, 0u};
        for (int c = 0; c < 160; ++c)
            if ((s.v[c >> 5] >> (c & 31)) & 1u)
                for (int w = 0; w < 5; ++w) r[w] ^= cols[c * 5 + w];
        for (int w = 0; w < 5; ++w) s.v[w] = r[w];
    }
}

// the device copy of the jump table for the current device (built on the host once)
const uint32_t* xorwow_jump_table();

}  // namespace llmi
