"""TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline may import this;
the product path never does).

CPU restatement of the draw the reference's SamplingKernel makes
(/root/reference/src/kernels/sampling.cu:66-69):

    curand_init((unsigned long long)step, (unsigned long long)batch_id, 0, &state);
    threshold = (float)curand_uniform(&state) * sum;

cuRAND is a third-party dependency that is not in /root/reference (the CUDA toolkit's
curand_kernel.h, default generator curandStateXORWOW_t; the algorithm has been the same
since CUDA 3.2). Its published algorithm, restated:

  * seeding (curand_init -> _curand_init_scratch): s0 = lo32(seed) ^ 0xaad26b49,
    s1 = hi32(seed) ^ 0xf7dcefdd, t0 = 1099087573 * s0, t1 = 2591861531 * s1 (mod 2^32);
    d = 6615241 + t1 + t0, v = (123456789 + t0, 362436069 ^ t0, 521288629 + t1,
    88675123 ^ t1, 5783321 + t0);
  * subsequence: the state advanced by subsequence * 2^67 steps (skipahead_sequence).
    The step is linear over GF(2) on the 160-bit v, so the jump is the matrix
    M^(2^67) (67 squarings of the one-step matrix M), applied once per set bit of the
    subsequence as M^(2^67 * 2^i); d advances by 362437 per step, and 2^67 * 362437 is
    0 mod 2^32, so the jump leaves d alone;
  * curand(): t = v0 ^ (v0 >> 2); v0..v3 = v1..v4; v4 = (v4 ^ (v4 << 4)) ^ (t ^ (t << 1));
    d += 362437; return v4 + d;
  * curand_uniform(x) = x * 2^-32 + 2^-32 / 2 in float ((float)x rounded to nearest,
    the product exact, one rounding of the sum): a float in (0, 1].

Parity unpinned: no CUDA runtime or cuRAND output exists in this image or in the
reference's files, so these values are checked against the restatement's own
properties (tests/test_sampling_oracle.py: the one-step matrix reproduces curand(), a
jump equals stepping) and the GPU kernel against this module bit for bit, not against
cuRAND itself.
"""
from functools import lru_cache

import numpy as np

M32 = 0xFFFFFFFF
D_INC = 362437
SEQ_JUMP_LOG2 = 67


def init(seed: int):
    """curand_init(seed, 0, 0): (v[5], d) before any subsequence jump."""
    s0 = (seed & M32) ^ 0xAAD26B49
    s1 = ((seed >> 32) & M32) ^ 0xF7DCEFDD
    t0 = (1099087573 * s0) & M32
    t1 = (2591861531 * s1) & M32
    d = (6615241 + t1 + t0) & M32
    v = [(123456789 + t0) & M32, 362436069 ^ t0, (521288629 + t1) & M32, 88675123 ^ t1, (5783321 + t0) & M32]
    return v, d


def step(v, d):
    """curand(): (new v, new d, output)."""
    t = v[0] ^ (v[0] >> 2)
    v4 = (v[4] ^ ((v[4] << 4) & M32)) ^ (t ^ ((t << 1) & M32))
    nv = [v[1], v[2], v[3], v[4], v4 & M32]
    nd = (d + D_INC) & M32
    return nv, nd, (nv[4] + nd) & M32


def _pack(v) -> int:
    return v[0] | (v[1] << 32) | (v[2] << 64) | (v[3] << 96) | (v[4] << 128)


def _unpack(x: int):
    return [(x >> (32 * i)) & M32 for i in range(5)]


def _v_step(x: int) -> int:
    nv, _, _ = step(_unpack(x), 0)
    return _pack(nv)


def _apply(cols, x: int) -> int:
    """GF(2) matrix (list of 160 column vectors) times the 160-bit vector x."""
    r = 0
    while x:
        low = x & -x
        r ^= cols[low.bit_length() - 1]
        x ^= low
    return r


def _square(cols):
    return [_apply(cols, c) for c in cols]


@lru_cache(maxsize=1)
def seq_jumps(n_bits: int = 16):
    """Columns of M^(2^67 * 2^i) for i < n_bits (subsequences < 2^n_bits)."""
    cols = [_v_step(1 << c) for c in range(160)]  # M: column c = step(e_c)
    for _ in range(SEQ_JUMP_LOG2):
        cols = _square(cols)
    out = [cols]
    for _ in range(1, n_bits):
        cols = _square(cols)
        out.append(cols)
    return out


def init_state(seed: int, subsequence: int = 0):
    v, d = init(seed)
    if subsequence:
        jumps = seq_jumps()
        assert subsequence < (1 << len(jumps)), "subsequence beyond the precomputed jumps"
        x = _pack(v)
        for i, cols in enumerate(jumps):
            if (subsequence >> i) & 1:
                x = _apply(cols, x)
        v = _unpack(x)
    return v, d


def uniform_of(x: int) -> np.float32:
    """curand_uniform's conversion of one 32-bit output."""
    return np.float32(np.float32(x) * np.float32(2.0 ** -32) + np.float32(2.0 ** -33))


def curand_uniform(seed: int, subsequence: int = 0) -> np.float32:
    """The first curand_uniform of curand_init(seed, subsequence, 0)."""
    v, d = init_state(seed, subsequence)
    _, _, x = step(v, d)
    return uniform_of(x)


def jump_table_u32(n_bits: int = 16) -> np.ndarray:
    """[n_bits][160 columns][5 words] uint32: the table the device kernel applies."""
    jumps = seq_jumps(n_bits)
    t = np.zeros((n_bits, 160, 5), np.uint32)
    for i, cols in enumerate(jumps):
        for c, x in enumerate(cols):
            t[i, c] = _unpack(x)
    return t
