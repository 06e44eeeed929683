// Prefill linear layers, second generation: 256 x 256 output tiles, 8 waves in two
// ping-pong groups (the M = prompt-rows case of
// launchLinearGemm, linear.cu:38-99, called from context_attention.cpp:99,166 and
// ffn.cpp:72,89). Same operands, numerics and epilogues as gemm2.hip (Gemm2Args);
// this file changes the schedule, which is what bounds gemm2 (27-32 % MFMA busy):
//
//  * bytes per FLOP. A 128 x 128 tile fetches 32 KB per 64-deep K step for 2 MFLOP;
//    256 x 256 fetches 64 KB for 8 MFLOP (half the L2 -> CU traffic per FLOP).
//  * the interleave. Each 64-deep K tile is four phases, one per 128 x 128 quadrant
//    of the workgroup tile (all 8 waves, 64 x 32 each, 16 v_mfma_f32_16x16x32_f16).
//    Waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave issues
//    its MFMAs while its partner issues the next phase's LDS reads and LDS-DMA
//    (cdna_hip_programming.md, "The 256² 8-phase template").
//  * the staging. The tile is four 16 KB half-images (A rows 0-127 / 128-255, W rows
//    0-127 / 128-255) in two 64 KB buffers, filled by global_load_lds_dwordx4. One
//    half-image is issued per phase, as soon as the previous occupant of its slot
//    was read for the last time (+1 phase), four to five phases ahead of its first read; every phase
//    waits a counted vmcnt (never 0 in the steady state) before the raw barrier.
//
// Hazard bookkeeping (phase n = 4 t + j of K tile t; group g's LDS reads of phase n
// are issued before its first barrier of the phase and retired -- lgkmcnt -- right
// after it, ahead of its MFMAs):
//   MFMAs:   j0 (A0, B0), j1 (A0, B1), j2 (A1, B1), j3 (A1, B0)
//   reads:   j0: A0 + B0 of tile t, j1: B1, j2: A1, j3: none (operands in registers)
//   issues:  j0: B1 of tile t+1, j1: A1 of t+1, j2: A0 of t+2, j3: B0 of t+2
//   each slot is re-filled two phases after its last read (by then both groups have
//   retired those reads and passed a barrier), and every half-image is retired by the
//   wait of the phase before its first read (the wait at phase n retires everything
//   issued up to phase n - 4), published by the next barrier.
// Measured alternatives that lost (tools/gemm_bench, same process A/B): the DMA issued
// between the MFMAs instead of in the load slot (-4..-9 %), reads rebalanced 8/4/8/4
// by pre-reading the next tile's B0 in j3 (-5..-8 %), the st_16x32 swizzle (2-way
// conflicted fragment reads, -5..-10 %).
// Exact mode (planes = 2): the lo plane is 2 K more K -- the K loop runs over
// [hi | lo] against [W | W], so LDS and registers are those of the fp16 mode.
// fp8 lo mode (lo8, split mode 3): the lo plane is e4m3(lo * 2^12) against an e4m3
// copy of W (w8 = e4m3(W * 2^w8_exp)); both keep the byte stride of their fp16 form
// (2 lda, 2 K per row, the first half used), so the per-thread DMA offsets serve both
// passes. One 128-deep K tile per 128-B LDS row -- the
// DMA, swizzle and fragment reads of an fp16 tile unchanged: a lane's two 16-B reads
// (kk = 0, 1) become one 32-B operand of v_mfma_scale_f32_16x16x128_f8f6f4 (A and B
// take the same lane/byte -> k map, so the sum over k is the same whatever order the
// instruction assigns), the E8M0 operand scales 2^-12 and 2^-w8_exp undo the scaling.
// At twice the fp16 MFMA rate and half the K tiles, the lo pass costs half of the
// fp16 one; |lo| <= 2^-11 |a| and e4m3's 2^-4 steps leave ~2^-15 of |a W| per product.
// Roofline: MFMA (fp16 dense 2.5 PFLOP/s); FLOPs per launch 2 * M * N * K * planes.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "kernels.h"

#ifndef LLMI_G3_PIN8
#define LLMI_G3_PIN8 1  // 0: let the compiler place the fp8 lo MFMAs (A/B builds only)
#endif
#ifndef LLMI_G3_VM2
#define LLMI_G3_VM2 1  // counted vmcnt only in j1 and j3 (0: in every phase; A/B builds only)
#endif
#ifndef LLMI_G3_STEADY
#define LLMI_G3_STEADY 1  // steady-state K tiles without issue guards / runtime wait counts (0: A/B builds only)
#endif
#ifndef LLMI_G3_SBASE
#define LLMI_G3_SBASE 1  // the copies' K offset in the scalar base, not a per-lane add (0: A/B builds only)
#endif
#ifndef LLMI_G3_PAIR
#define LLMI_G3_PAIR 1  // steady tiles in pairs with a compile-time buffer parity (0: A/B builds only)
#endif
#ifndef LLMI_G3_BFIRST
#define LLMI_G3_BFIRST 1  // j0 reads B0 before A0, a scheduling barrier between (0: A first; A/B builds only)
#endif

namespace llmi {

namespace {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef int i4v __attribute__((ext_vector_type(4)));
typedef int i8v __attribute__((ext_vector_type(8)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));


constexpr int kT = 512;              // 8 waves: (wr, wc) = (w >> 2, w & 3)
constexpr int kTile = 256;           // BM = BN
constexpr int kK = 64;               // K per tile step (128-B LDS rows)
constexpr int kHalf = 128 * 128;     // one half-image: 128 rows x 128 B
constexpr int kBuf = 4 * kHalf;      // A0 A1 B0 B1
constexpr int kEpiRowB = 272;        // gate_up epilogue image: 128 halves + 16 B pad per row
constexpr int kLds = 2 * kBuf > 2 * kTile * kEpiRowB ? 2 * kBuf : 2 * kTile * kEpiRowB;  // 136 KB


// LDS image swizzle (an involution): 16-B chunk c of 128-B row r is stored at chunk
// c ^ ((r >> 1) & 7). A fragment ds_read_b128 (lane: row fr = lane & 15, chunk
// 4 kk + (lane >> 4)) then puts the 16 lanes of each ds_read_b128 lane group on 16
// distinct 16-B bank slots -- conflict-free (the st_16x32 XOR of gemm2 leaves it 2-way).
__device__ __forceinline__ int swz3(int b) { return b ^ (((b >> 8) & 7) << 4); }


// the same with a uniform base in SGPRs and a 32-bit per-lane byte offset (saddr form):
// no 64-bit per-lane pointers to keep live across the K loop
__device__ __forceinline__ void glds_s(const void* sbase, unsigned voff, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(sbase), "s"(lds)
                 : "memory");
}

// vmcnt(c) for the counts the schedule produces (wave-uniform branch)
__device__ __forceinline__ void wait_vm(int c) {
    if (c >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (c >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (c >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (c >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void bar() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ float silu3(float v) { return v / (1.0f + expf(-v)); }

// One tile's K loop into acc: nhi 64-deep fp16 K tiles of the hi plane from tile hi0, then
// nlo tiles of the lo plane from tile lo0 (fp16 plane: 64-deep tiles; lo8: 128-deep fp8
// tiles; both 128 B per LDS row). nhi + nlo >= 2: the prologue's counted wait covers the
// first two tiles. Every wave passes the same barriers, and every LDS read has retired on
// return, so the caller may reuse the LDS.
// PAIRED: steady tiles in (even, odd) pairs with a compile-time buffer parity -- only in the
// plain gemm3_kernel: in the stream-K and balanced kernels the duplicated tile bodies push the
// allocator past 256 VGPRs (10-15 spilled)
template <int EPI, bool PAIRED = false>
__device__ __forceinline__ void g3_run(const Gemm2Args& a, char* lds, int m0, int ct, int hi0, int nhi, int lo0,
                                       int nlo, f4v (&acc)[2][2][4][2]) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wr = w >> 2, wc = w & 3;  // wr is also the ping-pong group
    const int fr = lane & 15, fq = lane >> 4;
    const bool lo8 = a.lo8 != 0;
    const int KT = nhi + nlo;  // virtual K tiles ([hi | lo])

    // per-thread DMA sources: instruction i of a half-image fills half-local bytes
    // i * 8192 + 16 t, which hold logical byte swz3(.) of the image
    // byte offsets < 4 GiB (checked by the launcher): half the VGPRs of size_t; W half 1 is
    // W half 0 + a uniform row offset (gate_up: the up rows, else 128 rows on), never clamped
    unsigned a_off[2][2], b_off[2];
    const unsigned b_half1 = (unsigned)(EPI == EPI_SILU_MUL ? a.pair_off : 128) * (unsigned)a.k * 2u;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int b = swz3(i * kT * 16 + t * 16);
        const int row = b >> 7, cb = b & 127;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int m = min(m0 + h * 128 + row, a.m - 1);
            a_off[h][i] = (unsigned)m * (unsigned)a.lda * 2u + (unsigned)cb;
        }
        // W half 0: gate columns g0 + row (gate_up) or tile rows 0-127
        const int n = (EPI == EPI_SILU_MUL) ? ct * 128 + row : ct * kTile + row;
        b_off[i] = (unsigned)n * (unsigned)a.k * 2u + (unsigned)cb;
    }
    const char* abase[2] = {reinterpret_cast<const char*>(a.a[0]),
                            reinterpret_cast<const char*>(a.planes == 2 ? a.a[1] : a.a[0])};
    const char* wbase = reinterpret_cast<const char*>(a.w);
    const char* w8base = reinterpret_cast<const char*>(a.w8);
    // E8M0 operand scales of the fp8 lo pass in one register: byte 0 for A (2^-12), byte 1 for B (2^-w8_exp)
    const int sc = (127 - kLo8Exp) | ((127 - a.w8_exp) << 8);
    const unsigned lds0 = (unsigned)(uintptr_t)lds;

    // issue the half-image `half` (0 A0, 1 A1, 2 B0, 3 B1) of virtual K tile v
    // (GUARD false: the caller knows v < KT -- the steady-state tiles, no scalar branch)
    // vpar: v & 1 when the caller knows it at compile time (std::integral_constant), else
    // an int; the LDS destination then folds to a constant
    auto issue = [&](int v, int half, auto guard, auto vpar) {
        if (decltype(guard)::value && v >= KT) return;
        const int plane = v >= nhi ? 1 : 0;
        const unsigned dst = __builtin_amdgcn_readfirstlane(lds0 + (int)vpar * kBuf + half * kHalf + w * 1024);
        // fp8 rows keep the fp16 rows' byte stride (the first half of each row is used),
        // so the per-thread offsets serve both passes -- no second set of registers
        const unsigned k0b = (unsigned)(plane ? lo0 + v - nhi : hi0 + v) * 128u;
        const char* base = half < 2 ? abase[plane] : (lo8 && plane) ? w8base : wbase;  // uniform
#if LLMI_G3_SBASE
        // the K offset (and W half 1's row offset) go into the scalar base: the per-lane
        // offsets are the loop-invariant a_off / b_off, no VALU add per copy
        const char* sb = base + k0b + (half == 3 ? b_half1 : 0u);
#pragma unroll
        for (int i = 0; i < 2; ++i) glds_s(sb, half < 2 ? a_off[half][i] : b_off[i], dst + i * kT * 16);
#else
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const unsigned off = half < 2 ? a_off[half][i] + k0b : b_off[i] + (half == 3 ? b_half1 : 0u) + k0b;
            glds_s(base, off, dst + i * kT * 16);
        }
#endif
    };
    // phase n issues: j0 B1 of t+1, j1 A1 of t+1, j2 A0 of t+2, j3 B0 of t+2 (t = n >> 2)
    const int n_last = 4 * (KT - 2) + 1;  // last phase whose issue is in range
    auto vm_count = [&](int n) {          // glds of this wave issued in phases n-3 .. n
        const int c = min(n, n_last) - (n - 4);
        return 2 * max(0, min(4, c));
    };

    h8v af[4][2], b0[2][2], b1[2][2];
    auto read_a = [&](const char* img) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
                af[i][kk] = *reinterpret_cast<const h8v*>(img + swz3((wr * 64 + i * 16 + fr) * 128 + kk * 64 + fq * 16));
    };
    auto read_b = [&](const char* img, h8v (&bf)[2][2]) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
                bf[j][kk] = *reinterpret_cast<const h8v*>(img + swz3((wc * 32 + j * 16 + fr) * 128 + kk * 64 + fq * 16));
    };
    auto mma = [&](f4v (&c)[4][2], h8v (&bf)[2][2]) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    c[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[i][kk], bf[j][kk], c[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    };
    // fp8 lo pass: the same fragment reads; a lane's two 16-B reads (kk = 0, 1) are one
    // 32-B operand (A and B alike)
    auto cat8 = [](const h8v& x, const h8v& y) {
        const i4v u = __builtin_bit_cast(i4v, x), v = __builtin_bit_cast(i4v, y);
        return __builtin_shufflevector(u, v, 0, 1, 2, 3, 4, 5, 6, 7);
    };
    auto mma8 = [&](f4v (&c)[4][2], h8v (&bf)[2][2]) {  // one 128-deep fp8 K step
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                c[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(cat8(af[i][0], af[i][1]), cat8(bf[j][0], bf[j][1]),
                                                                          c[i][j], 0, 0, 0, sc, 1, sc);
        // pin the 8 MFMAs inside this phase: they are register-only, and without a use here
        // the compiler sank 3 of every 4 quadrants' fp8 MFMAs past the phase barriers (the
        // .s had 18 of 24 set-priority windows empty and 16-MFMA bunches elsewhere), which
        // broke the two groups' read / MFMA alternation of the lo pass
#if LLMI_G3_PIN8
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(c[i][j]));
#endif
        __builtin_amdgcn_s_setprio(0);
    };
    auto sync_reads = [&](int n) {  // DMA counted, then the barrier; LDS reads retire behind it
        wait_vm(vm_count(n));
        bar();
    };

    const std::true_type G{};  // guarded issue
    const std::integral_constant<int, 0> P0{};
    const std::integral_constant<int, 1> P1{};
    // prologue: virtual phases -6 .. -1 = A0, B0, B1, A1 of tile 0, A0, B0 of tile 1
    issue(0, 0, G, P0); issue(0, 2, G, P0); issue(0, 3, G, P0); issue(0, 1, G, P0);
    issue(1, 0, G, P1); issue(1, 2, G, P1);
    if (LLMI_G3_VM2)  // A0, B0, B1 of tile 0 (j0 has no wait of its own; A1 is retired by j1's)
        wait_vm(2 * (min(1, KT - 1) * 2 + 1));
    else
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // A0, B0 of tile 0
    bar();
    if (wr == 1) bar();  // ping-pong: group 1 one barrier behind

    // steady: kt + 2 < KT - 0 and 4 kt + 3 <= n_last, i.e. kt <= KT - 3 -- every issue is in
    // range and the counted waits are the constants 8 (j1) and 6 (j3): no guards, no
    // wave-uniform branch chains in the phases (LLMI_G3_STEADY; 0 = every tile generic)
    // par: kt & 1, a compile-time constant in the paired steady loop (LLMI_G3_PAIR), so the
    // LDS read and copy addresses of the tile's buffer fold to immediate offsets
    auto ktile = [&](int kt, auto f8, auto steady, auto par) {
        constexpr bool F8 = decltype(f8)::value;
        constexpr bool ST = decltype(steady)::value && LLMI_G3_VM2;
        const std::integral_constant<bool, !ST> g{};
        auto issue_g = [&](int v, int half) {
            if constexpr (std::is_same_v<decltype(par), int>) issue(v, half, g, v & 1);
            else if ((v - kt) & 1) issue(v, half, g, std::integral_constant<int, 1 - decltype(par)::value>{});
            else issue(v, half, g, par);
        };
        const char* buf = lds + (int)par * kBuf;
        const int n = 4 * kt;
        // j0: quadrant (A0, B0)
        if (LLMI_G3_BFIRST) {
            read_b(buf + 2 * kHalf, b0);
            __builtin_amdgcn_sched_barrier(0);
            read_a(buf);
        } else {
            read_a(buf);
            read_b(buf + 2 * kHalf, b0);
        }
        issue_g(kt + 1, 3);
        if (LLMI_G3_VM2) bar(); else sync_reads(n);
        if constexpr (F8) mma8(acc[0][0], b0); else mma(acc[0][0], b0);
        bar();
        // j1: quadrant (A0, B1)
        read_b(buf + 3 * kHalf, b1);
        issue_g(kt + 1, 1);
        if (LLMI_G3_VM2) {  // retires A1 of tile kt (read in j2): 4 half-images issued after it
            if constexpr (ST) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else wait_vm(vm_count(n + 1));
            bar();
        } else {
            sync_reads(n + 1);
        }
        if constexpr (F8) mma8(acc[0][1], b1); else mma(acc[0][1], b1);
        bar();
        // j2: quadrant (A1, B1)
        read_a(buf + kHalf);
        issue_g(kt + 2, 0);
        if (LLMI_G3_VM2) bar(); else sync_reads(n + 2);
        if constexpr (F8) mma8(acc[1][1], b1); else mma(acc[1][1], b1);
        bar();
        // j3: quadrant (A1, B0)
        issue_g(kt + 2, 2);
        if (LLMI_G3_VM2) {  // retires A0 / B0 and B1 of tile kt + 1 (read in its j0 / j1): 3 issued after B1
            if constexpr (ST) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            else wait_vm(2 * max(0, min(n + 3, n_last) - n));
            bar();
        } else {
            sync_reads(n + 3);
        }
        if constexpr (F8) mma8(acc[1][0], b0); else mma(acc[1][0], b0);
        bar();
    };
    const int KTh = lo8 ? nhi : KT;  // fp16 K tiles (then the fp8 lo tiles)
    const int KTs = LLMI_G3_STEADY ? KT - 2 : 0;  // tiles [0, KTs) are steady
    const std::false_type NF{};
    const std::true_type YF{};
    int kt = 0;
    if (PAIRED) {  // steady tiles in (even, odd) pairs: static buffer parity
        for (; kt + 1 < min(KTh, KTs); kt += 2) {
            ktile(kt, NF, YF, P0);
            ktile(kt + 1, NF, YF, P1);
        }
    }
    for (; kt < min(KTh, KTs); ++kt) ktile(kt, NF, YF, kt & 1);
    for (; kt < KTh; ++kt) ktile(kt, NF, NF, kt & 1);
    if (PAIRED && (kt & 1)) {  // the fp8 pass may start on an odd tile
        if (kt < KTs) { ktile(kt, YF, YF, P1); ++kt; }
    }
    if (PAIRED) {
        for (; kt + 1 < KTs; kt += 2) {
            ktile(kt, YF, YF, P0);
            ktile(kt + 1, YF, YF, P1);
        }
    }
    for (; kt < KTs; ++kt) ktile(kt, YF, YF, kt & 1);
    for (; kt < KT; ++kt) ktile(kt, YF, NF, kt & 1);
    if (wr == 0) bar();  // equal barrier counts
}

__device__ __forceinline__ void zero_acc(f4v (&acc)[2][2][4][2]) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[x][y][i][j] = f4v{0.f, 0.f, 0.f, 0.f};
}

// the tile's epilogue (slice: the EPI_SLAB K slice)
template <int EPI>
__device__ __forceinline__ void g3_epilogue(const Gemm2Args& a, char* lds, f4v (&acc)[2][2][4][2], int m0, int ct,
                                            int slice) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wr = w >> 2, wc = w & 3;
    const int fr = lane & 15, fq = lane >> 4;
    const bool lo8 = a.lo8 != 0;
    // epilogue: acc[qa][qb][i][j] register e is tile row qa*128 + wr*64 + 16 i + 4 fq + e,
    // tile column qb*128 + wc*32 + 16 j + fr (SILU: qb 0 gate, qb 1 its up column)
    if (EPI == EPI_SILU_MUL && a.y_hi) {
        // fp16 planes through LDS (the K loop's reads and DMA are all retired here), then
        // 16-B stores: 16 lanes per 256-B row instead of 2-B stores 4 rows per instruction
        // (measured store-issue-bound: 7-10 us of a 110 us gate_up). Rows padded to 272 B:
        // the accumulator rows 4 apart land 16 banks apart.
        char* img = lds;
#pragma unroll
        for (int qa = 0; qa < 2; ++qa)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const int row = qa * 128 + wr * 64 + 16 * i + 4 * fq + e, col = wc * 32 + 16 * j + fr;
                        const float v = silu3(acc[qa][0][i][j][e]) * acc[qa][1][i][j][e];
                        const _Float16 hi = (_Float16)v;
                        *reinterpret_cast<_Float16*>(img + row * kEpiRowB + col * 2) = hi;
                        if (a.y_lo)
                            *reinterpret_cast<_Float16*>(img + (kTile + row) * kEpiRowB + col * 2) =
                                (_Float16)(v - (float)hi);
                    }
        __syncthreads();
        const int planes = a.y_lo ? 2 : 1;
        for (int c = t; c < planes * kTile * 16; c += kT) {
            const int pl = c / (kTile * 16), row = (c >> 4) & (kTile - 1), ch = c & 15;
            const int m = m0 + row;
            if (m >= a.m) continue;
            const h8v v = *reinterpret_cast<const h8v*>(img + (pl * kTile + row) * kEpiRowB + ch * 16);
            if (pl && lo8) {  // e4m3 bytes [m, ldy] of the lo plane
                uint2 q;
                q.x = lo8_pack4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
                q.y = lo8_pack4((float)v[4], (float)v[5], (float)v[6], (float)v[7]);
                *reinterpret_cast<uint2*>(reinterpret_cast<char*>(a.y_lo + (size_t)m * a.ldy) + ct * 128 + ch * 8) = q;
                continue;
            }
            _Float16* dst = (pl ? a.y_lo : a.y_hi) + (size_t)m * a.ldy + ct * 128 + ch * 8;
            *reinterpret_cast<h8v*>(dst) = v;
        }
        return;
    }
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int m = m0 + qa * 128 + wr * 64 + 16 * i + 4 * fq + e;
                if (m >= a.m) continue;
                if (EPI == EPI_SILU_MUL) {
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const int gc = ct * 128 + wc * 32 + 16 * j + fr;
                        const float v = silu3(acc[qa][0][i][j][e]) * acc[qa][1][i][j][e];
                        const size_t o = (size_t)m * a.ldy + gc;
                        if (a.y_hi) {
                            const _Float16 hi = (_Float16)v;
                            a.y_hi[o] = hi;
                            if (a.y_lo) a.y_lo[o] = (_Float16)(v - (float)hi);
                        } else {
                            a.y[o] = v;
                        }
                    }
                } else {
                    float* yrow = (EPI == EPI_SLAB ? a.slab + (size_t)slice * a.m * a.ldy : a.y) + (size_t)m * a.ldy;
#pragma unroll
                    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            const int n = ct * kTile + qb * 128 + wc * 32 + 16 * j + fr;
                            if (EPI == EPI_ADD)
                                yrow[n] += acc[qa][qb][i][j][e];
                            else
                                yrow[n] = acc[qa][qb][i][j][e];
                        }
                }
            }
}

template <int EPI>
__global__ __launch_bounds__(kT) void gemm3_kernel(Gemm2Args a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    // bijective XCD remap, then tile-major over split-K slices, row tiles fastest
    // (the row tiles of one W stripe run together on one XCD: W read once into L2)
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    const int S = (EPI == EPI_SLAB) ? a.ksplit : 1;
    const int tile = id / S, slice = id - tile * S;
    const int m_tiles = (a.m + kTile - 1) / kTile;
    const int rt = tile % m_tiles, ct = tile / m_tiles;
    const int m0 = rt * kTile;
    // slice s covers K tiles [s * KT_all / S, (s + 1) * KT_all / S) of each plane
    // (lo8: on 128-deep boundaries, so the slice's fp8 lo tiles are whole)
    const bool lo8 = a.lo8 != 0;
    const int KT_all = lo8 ? a.k / (2 * kK) : a.k / kK;
    const int kt0 = (lo8 ? 2 : 1) * (slice * KT_all / S);
    const int KTs = (lo8 ? 2 : 1) * ((slice + 1) * KT_all / S) - kt0;  // 64-deep K tiles per plane in this slice
    f4v acc[2][2][4][2];
    zero_acc(acc);
    g3_run<EPI, LLMI_G3_PAIR != 0>(a, lds, m0, ct, kt0, KTs, lo8 ? kt0 / 2 : kt0, lo8 ? KTs / 2 : (a.planes == 2 ? KTs : 0),
                                   acc);
    g3_epilogue<EPI>(a, lds, acc, m0, ct, slice);
}

// gate_up with two planes and every CU busy (gemm3_launch with bal_slab): its 172
// 256 x 256 tiles alone leave 84 of 256 CUs idle for the whole launch. Workgroups
// [0, n_lo) are lo workers: the lo pass of all tiles (fp8 or fp16), in units of two K tiles,
// is split evenly over them (contiguous ranges that cross tile boundaries; a tile is
// touched by at most two workers); each piece's fp32 partial goes to its tile's slot, then
// a release fence and an epoch flag. Workgroups [n_lo, grid) own one tile each: its fp16
// hi pass, then the tile's one or two lo partials (acquire; added in slot order, so the
// result is repeatable), then the SiLU epilogue. Workers have the lower ids and are
// dispatched first, so a waiting owner never holds a CU its producer needs; every wait is
// bounded (2 s of s_memrealtime, then error bit 16 and the epilogue without that slot).
__global__ __launch_bounds__(kT) void gemm3_silu_bal_kernel(Gemm2Args a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    WgStamp ts(a.stamps);  // [1] K loop(s) done, [2] partials in / published
    const int t = threadIdx.x;
    const int m_tiles = (a.m + kTile - 1) / kTile;
    const int n_tiles = m_tiles * a.n_tiles;
    const int n_lo = (int)gridDim.x - n_tiles;
    // a tile's first `own` pairs of 128-deep lo tiles stay with its owner (balance: an fp8
    // lo tile costs ~1.4 fp16 ones); the other P units go to the workers
    const int own = a.bal_own;
    const int P = a.k / (a.lo8 ? 256 : 128) - own;  // a unit = two lo tiles (128-deep fp8 or 64-deep fp16)
    const int U = n_tiles * P;
    auto worker_of = [&](int x) { return (int)(((long)(x + 1) * n_lo + U - 1) / U) - 1; };
    auto slot_ptr = [&](int tile, int slot) {
        return reinterpret_cast<float4*>(a.bal_slab) + (size_t)(tile * 2 + slot) * 32 * kT + t;
    };
    f4v acc[2][2][4][2];
    const int bid = blockIdx.x;
    if (bid < n_lo) {
        const int u1 = (int)((long)(bid + 1) * U / n_lo);
        for (int u = (int)((long)bid * U / n_lo); u < u1;) {
            const int tile = u / P, ue = min(u1, (tile + 1) * P);
            const int slot = bid == worker_of(tile * P) ? 0 : 1;
            zero_acc(acc);
            g3_run<EPI_SILU_MUL>(a, lds, (tile % m_tiles) * kTile, tile / m_tiles, 0, 0, 2 * (own + u - tile * P),
                                 2 * (ue - u), acc);
            float4* dst = slot_ptr(tile, slot);
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            const f4v v = acc[x][y][i][j];
                            dst[(size_t)(((x * 2 + y) * 4 + i) * 2 + j) * kT] = make_float4(v[0], v[1], v[2], v[3]);
                        }
            // every wave's stores complete, then ONE release (one L2 write-back per piece: a
            // fence in each of the 8 waves wrote the XCD's L2 back 8 times and slowed the
            // owners beside it), then the flag
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (t == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                __hip_atomic_store(a.bal_flags + tile * 2 + slot, a.bal_epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            u = ue;
        }
        ts.mark(1);
        return;
    }
    // owners: with two row tiles, bids b and b + 8 (one XCD) take the two row tiles of one
    // W stripe (W read once into that XCD's L2); the remainder runs row tiles fastest
    const int o = bid - n_lo;
    int rt, ct;
    if (m_tiles == 2 && o < (n_tiles / 16) * 16) {
        rt = (o % 16) / 8;
        ct = (o / 16) * 8 + o % 8;
    } else {
        rt = o % m_tiles;
        ct = o / m_tiles;
    }
    const int tile = ct * m_tiles + rt, m0 = rt * kTile;
    zero_acc(acc);
    g3_run<EPI_SILU_MUL>(a, lds, m0, ct, 0, a.k / kK, 0, 2 * own, acc);
    ts.mark(1);
    const int w0 = worker_of(tile * P), nslots = worker_of(tile * P + P - 1) - w0 + 1;
    __shared__ int ok_s[2];
    if (t == 0) {
        for (int sl = 0; sl < nslots; ++sl) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            int ok = 1;
            while (__hip_atomic_load(a.bal_flags + tile * 2 + sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
                   a.bal_epoch) {
                __builtin_amdgcn_s_sleep(2);
                if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s at 100 MHz
                    if (a.err) atomicOr(a.err, 16);
                    ok = 0;
                    break;
                }
            }
            ok_s[sl] = ok;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // one L2 invalidate, then the barrier
    }
    __syncthreads();
    for (int sl = 0; sl < nslots; ++sl) {
        if (!ok_s[sl]) continue;
        const float4* src = slot_ptr(tile, sl);
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const float4 p = src[(size_t)(((x * 2 + y) * 4 + i) * 2 + j) * kT];
                        acc[x][y][i][j] += f4v{p.x, p.y, p.z, p.w};
                    }
    }
    ts.mark(2);
    g3_epilogue<EPI_SILU_MUL>(a, lds, acc, m0, ct, 0);
}

// Stream-K: with fewer 256 x 256 tiles than CUs (gate_up's 172 and q/k/v's 96 at 512 rows
// left 84 / 160 CUs idle for a whole launch) the tiles' K work -- per tile nh + nl virtual K
// tiles ([hi | lo], taken in pairs: g3_run needs >= 2) -- is cut into sk_grid equal
// contiguous ranges, one per workgroup, that cross tile boundaries. The workgroup holding a
// tile's first pair owns it: that is the END of its range, so the tile's later pieces (the
// START of the next workgroups' ranges) were computed first and the owner's wait is short.
// Later pieces go to fp32 partial slots and raise a flag to the launch's epoch E; the owner
// waits for flag == E (bounded: error bit 16), adds the slots in order onto its own piece
// (repeatable sums) and runs the tile's epilogue. Flags are never reset: a piece that
// publishes after its owner timed out leaves E behind, which no later launch waits for.
// E = the last completed launch's epoch + 1, read from sk_ctl[0]; the last workgroup to
// finish (a count in sk_ctl[32]) stores E there, so eager launches and graph replays alike
// see a new value each launch. Every workgroup is resident (sk_grid <= the CU count, one
// 136-KB workgroup per CU), so waits end unless another stream or process holds CUs.
// Concurrency contract: sk_ctl / sk_flags / the slots belong to ONE
// (device, stream) workspace and assume its launches never overlap -- a graph captured on
// stream S must be replayed on S (or with S idle), never beside eager stream-K work on S's
// workspace: two overlapping launches would share the ctl[32] count and the epoch and could
// pass each other's flags silently. The engine and the layer API keep one workspace per
// stream and replay their graphs on the stream they captured them on.
#ifndef LLMI_SK_EXP
#define LLMI_SK_EXP 0  // timing-only builds: 1 = flags without the slot payload, 2 = no hand-off at all
#endif
struct SkDims {
    int m_tiles, T, NH, U2;
    long TP;
};
__host__ __device__ inline SkDims sk_dims(int m, int n_tiles, int k, int planes, int lo8) {
    SkDims d;
    d.m_tiles = (m + kTile - 1) / kTile;
    d.T = d.m_tiles * n_tiles;
    d.NH = k / kK;
    const int NL = planes == 2 ? (lo8 ? k / (2 * kK) : k / kK) : 0;
    d.U2 = (d.NH + NL) / 2;
    d.TP = (long)d.T * d.U2;
    return d;
}
__host__ __device__ inline int sk_wg_of(long x, long TP, int G) { return (int)(((x + 1) * G - 1) / TP); }

template <int EPI>
__global__ __launch_bounds__(kT) void gemm3_sk_kernel(Gemm2Args a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int t = threadIdx.x;
    const SkDims d = sk_dims(a.m, a.n_tiles, a.k, a.planes, a.lo8);
    const int G = gridDim.x, bid = blockIdx.x;
    // consecutive workgroups on one XCD; workgroup w = v * m_tiles + rt: the m_tiles row tiles
    // of a W column stripe get the SAME K ranges from sibling workgroups running side by side,
    // so each W chunk is read once into the XCD's L2 for all of them (ranges cut per tile made
    // the siblings read different K at the same time: W read twice, 179 vs ~145 us at gate_up)
    const int w = (G % 8 == 0) ? (bid & 7) * (G / 8) + (bid >> 3) : bid;
    const int MT = d.m_tiles, Gp = G / MT, v = w / MT, rt = w % MT;
    const long TPs = (long)a.n_tiles * d.U2;  // pairs of all column stripes
    const long p1 = (long)(v + 1) * TPs / Gp;
    unsigned* const ctl = a.sk_flags - kSkCtlWords;  // the control words sit just before the flags
    const int pmax = a.sk_pmax & 255, sk_test = a.sk_pmax >> 8;
    auto slot_rsrc = [&](int tile, int slot) {  // one 256 KB partial slot (wave-uniform)
        return __builtin_amdgcn_make_buffer_rsrc(a.sk_slab + ((size_t)tile * pmax + slot) * kTile * kTile, (short)0,
                                                 kTile * kTile * 4, 0x00020000);
    };
    __shared__ int ok_s[8];
    // this launch's epoch (thread 0 only: it alone publishes and waits; 0 is never used)
    auto epoch = [&]() {
        const unsigned e = __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
        return e ? e : 1u;
    };
    // a range shorter than a tile (T < G) meets at most two tiles: the piece (seg) of each
    auto seg = [&](long p) {
        f4v acc[2][2][4][2];
        const int ct = (int)(p / d.U2);
        const int s = (int)(p - (long)ct * d.U2);
        const int e = (int)min((long)d.U2, p1 - (long)ct * d.U2);
        const int vs = 2 * s, ve = 2 * e;
        const int nhi = max(0, min(ve, d.NH) - vs), lo0 = max(vs, d.NH) - d.NH, nlo = max(0, ve - max(vs, d.NH));
        const int tile = ct * MT + rt, m0 = rt * kTile;
        const int owner = sk_wg_of((long)ct * d.U2, TPs, Gp);  // in units of sibling groups
        if (s > 0) {  // a later piece of the tile: slot v - owner - 1, then its flag
            zero_acc(acc);
            g3_run<EPI>(a, lds, m0, ct, vs, nhi, lo0, nlo, acc);
            const int sl = v - owner - 1;
            // payload written through (sc1) by buffer stores: one SGPR offset per quadrant
            // instead of 32 64-bit addresses, and no release fence (guide R1 hand-off)
            const auto rs = slot_rsrc(tile, sl);
#pragma unroll
            for (int x = 0; x < 2; ++x)
#pragma unroll
                for (int y = 0; y < 2; ++y)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j < 2; ++j)
                            if (LLMI_SK_EXP == 0) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, acc[x][y][i][j]), rs, t * 16,
                                                                   (((x * 2 + y) * 4 + i) * 2 + j) * kT * 16, 16);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave, then one flag
            __syncthreads();
            if (t == 0 && LLMI_SK_EXP != 2 && sk_test != 1) {
                if (sk_test == 2) {  // fault injection: publish after the owner's 2-s bound
                    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                    while (__builtin_amdgcn_s_memrealtime() - t0 < 250000000ull) __builtin_amdgcn_s_sleep(127);
                }
                __hip_atomic_store(a.sk_flags + tile * pmax + sl, epoch(), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            zero_acc(acc);
            g3_run<EPI>(a, lds, m0, ct, 0, nhi, lo0, nlo, acc);  // a tile's head: from K tile 0
            const int np = LLMI_SK_EXP == 2 ? 0 : sk_wg_of((long)ct * d.U2 + d.U2 - 1, TPs, Gp) - v;  // later pieces
            if (np > 0) {
                if (t == 0) {
                    const unsigned E = epoch();
                    for (int sl = 0; sl < np; ++sl) {
                        unsigned* f = a.sk_flags + tile * pmax + sl;
                        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
                        int ok = 1;
                        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != E) {
                            __builtin_amdgcn_s_sleep(2);
                            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s at 100 MHz
                                if (a.err) atomicOr(a.err, 16);
                                ok = 0;
                                break;
                            }
                        }
                        ok_s[sl] = ok;
                    }
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // one L2 invalidate, then the barrier
                }
                __syncthreads();
                for (int sl = 0; sl < np; ++sl) {
                    if (!ok_s[sl] || LLMI_SK_EXP == 1) continue;
                    const auto rs = slot_rsrc(tile, sl);
#pragma unroll
                    for (int x = 0; x < 2; ++x)
#pragma unroll
                        for (int y = 0; y < 2; ++y) {
#pragma unroll
                            for (int i = 0; i < 4; ++i)
#pragma unroll
                                for (int j = 0; j < 2; ++j)
                                    acc[x][y][i][j] += __builtin_bit_cast(
                                        f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, t * 16,
                                                                                   (((x * 2 + y) * 4 + i) * 2 + j) * kT * 16, 0));
                            __builtin_amdgcn_sched_barrier(0);
                        }
                }
            }
            __builtin_amdgcn_sched_barrier(0);  // keep the epilogue's address math out of the adds
            g3_epilogue<EPI>(a, lds, acc, m0, ct, 0);
            __syncthreads();  // the epilogue's LDS image is read before the next piece's DMA
        }
        return (long)ct * d.U2 + e;
    };
    if (v < Gp) {  // G not a multiple of m_tiles: the spare workgroups only count themselves
        const long p0 = (long)v * TPs / Gp;
        if (p0 < p1) {
            const long pn = seg(p0);
            if (pn < p1) seg(pn);
        }
    }
    // every workgroup read the epoch (if at all) before counting itself here, so the last
    // one can advance it for the next launch
    if (t == 0) {
        const unsigned done = __hip_atomic_fetch_add(ctl + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (done == (unsigned)G - 1u) {
            const unsigned E = epoch();
            __hip_atomic_store(ctl + 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(ctl, E, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

template <int EPI>
int launch_g3(const Gemm2Args& a, int grid, hipStream_t s) {
    static const bool attr = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm3_kernel<EPI>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, kLds) == hipSuccess;
    }();
    LLMI_REQUIRE(attr, "gemm3: cannot raise the dynamic LDS limit");
    hipLaunchKernelGGL(gemm3_kernel<EPI>, dim3(grid), dim3(kT), kLds, s, a);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

template <int EPI>
int launch_sk(const Gemm2Args& a, hipStream_t s) {
    static const bool attr = [] {
        return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm3_sk_kernel<EPI>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, kLds) == hipSuccess;
    }();
    LLMI_REQUIRE(attr, "gemm3: cannot raise the dynamic LDS limit");
    hipLaunchKernelGGL(gemm3_sk_kernel<EPI>, dim3(a.sk_grid), dim3(kT), kLds, s, a);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

__global__ void w8_amax_kernel(const __half* w, size_t n, unsigned* amax) {  // n % 8 == 0, 16-B aligned
    float m = 0.f;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n / 8; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 u = reinterpret_cast<const uint4*>(w)[i];
        const __half2* h = reinterpret_cast<const __half2*>(&u);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float2 f = __half22float2(h[j]);
            m = fmaxf(m, fmaxf(fabsf(f.x), fabsf(f.y)));
        }
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) atomicMax(amax, __float_as_uint(m));  // non-negative floats order as uints
}
// row r of the fp16 [rows, cols] weight -> the first cols bytes of e4m3 row r (stride 2 cols bytes)
__global__ void w8_convert_kernel(const __half* w, size_t n8, int cols8, float scale, uint2* out) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 u = reinterpret_cast<const uint4*>(w)[i];
        const __half2* h = reinterpret_cast<const __half2*>(&u);
        float f[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float2 p = __half22float2(h[j]);
            f[2 * j] = fminf(fmaxf(p.x * scale, -448.f), 448.f);
            f[2 * j + 1] = fminf(fmaxf(p.y * scale, -448.f), 448.f);
        }
        uint2 q;
        q.x = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false), true);
        q.y = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false), true);
        out[i + (i / cols8) * cols8] = q;
    }
}

}  // namespace

int w8_prepare(const void* w16, int rows, int cols, void* w8, int* exp_out, hipStream_t s) {
    const size_t count = (size_t)rows * cols;
    LLMI_REQUIRE(w16 && w8 && exp_out && rows > 0 && cols > 0 && cols % 8 == 0 &&
                     (reinterpret_cast<uintptr_t>(w16) & 15) == 0 && (reinterpret_cast<uintptr_t>(w8) & 15) == 0,
                 "w8_prepare: bad arguments");
    unsigned* d = nullptr;
    LLMI_HIP(hipMallocAsync(reinterpret_cast<void**>(&d), sizeof(unsigned), s));
    LLMI_HIP(hipMemsetAsync(d, 0, sizeof(unsigned), s));
    hipLaunchKernelGGL(w8_amax_kernel, dim3(2048), dim3(256), 0, s, static_cast<const __half*>(w16), count, d);
    unsigned bits = 0;
    LLMI_HIP(hipMemcpyAsync(&bits, d, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    LLMI_HIP(hipStreamSynchronize(s));
    LLMI_HIP(hipFreeAsync(d, s));
    float amax;
    memcpy(&amax, &bits, 4);
    int e = 0;
    if (amax > 0.f && std::isfinite(amax)) {
        e = (int)std::floor(std::log2(448.0 / (double)amax));
        while (std::ldexp((double)amax, e) > 448.0) --e;
        e = std::max(-100, std::min(100, e));
    }
    hipLaunchKernelGGL(w8_convert_kernel, dim3(2048), dim3(256), 0, s, static_cast<const __half*>(w16), count / 8, cols / 8,
                       (float)std::ldexp(1.0, e), static_cast<uint2*>(w8));
    LLMI_HIP(hipGetLastError());
    *exp_out = e;
    return LLMI_OK;
}

size_t gemm3_bal_slab_bytes(int m, int n) {
    if (m <= 0 || n % 256 != 0) return 0;
    const size_t tiles = (size_t)((m + kTile - 1) / kTile) * (n / 256);
    return tiles * 2 * kTile * kTile * sizeof(float);
}

namespace {
std::atomic<int> g_sk_debug_mode{0}, g_sk_debug_left{0};
}
void gemm3_sk_debug(int mode, int launches) {
    g_sk_debug_mode = mode;
    g_sk_debug_left = mode ? launches : 0;
}

Gemm3SkPlan gemm3_sk_plan(int m, int n, int k, int epi, int planes, int lo8, int g) {
    Gemm3SkPlan p;
    if ((epi != EPI_STORE && epi != EPI_SILU_MUL) || m <= 0 || g <= 0 || !gemm3_supported(n, k, epi, 1)) return p;
    if (lo8 && k % (2 * kK) != 0) return p;
    const int n_tiles = (epi == EPI_SILU_MUL) ? (n / 2) / 128 : n / kTile;
    const SkDims d = sk_dims(m, n_tiles, k, planes, lo8);
    const int NL = planes == 2 ? (lo8 ? k / (2 * kK) : k / kK) : 0;
    const int gp = g / d.m_tiles;  // sibling groups: one workgroup per row tile
    const long tps = (long)n_tiles * d.U2;
    // pairs never straddle the hi / lo boundary; >= 2 pairs a workgroup
    if (d.T >= g || gp < 1 || tps < 2L * gp || d.NH % 2 != 0 || NL % 2 != 0) return p;
    int pmax = 0;
    for (int c = 0; c < n_tiles; ++c)
        pmax = std::max(pmax, sk_wg_of((long)c * d.U2 + d.U2 - 1, tps, gp) - sk_wg_of((long)c * d.U2, tps, gp));
    if (pmax < 1 || pmax > 8) return p;
    p.pmax = pmax;
    p.slab_bytes = (size_t)d.T * pmax * kTile * kTile * sizeof(float);
    p.flag_bytes = (size_t)d.T * pmax * sizeof(unsigned);
    return p;
}

bool gemm3_supported(int n, int k, int epi, int ksplit) {
    const int ncols = (epi == EPI_SILU_MUL) ? n / 2 : n;
    const int tile = (epi == EPI_SILU_MUL) ? 128 : kTile;
    const int s = epi == EPI_SLAB ? ksplit : 1;
    return n > 0 && k > 0 && s >= 1 && ncols % tile == 0 && k % kK == 0 && k / kK / s >= 2;  // slices may be uneven
}

int gemm3_launch(Gemm2Args a, hipStream_t s) {
    LLMI_REQUIRE(a.a[0] && a.w && a.m > 0, "gemm3: null operand or empty M");
    LLMI_REQUIRE(a.planes == 1 || (a.planes == 2 && a.a[1]), "gemm3: planes must be 1 or 2 (with a[1])");
    if (a.epi != EPI_SLAB) a.ksplit = 1;
    LLMI_REQUIRE(gemm3_supported(a.n, a.k, a.epi, a.ksplit),
                 "gemm3: N a multiple of 256 (gate_up: 2 x 128), K a multiple of 64, >= 2 K tiles of 64 per slice");
    LLMI_REQUIRE(a.w_kblock == 0, "gemm3: head-major W blocks are not supported");
    LLMI_REQUIRE((uint64_t)a.n * a.k * 2 < (1ull << 32) && (uint64_t)a.m * a.lda * 2 < (1ull << 32),
                 "gemm3: W and A planes must each be under 4 GiB (32-bit DMA offsets)");
    LLMI_REQUIRE(a.epi == EPI_SILU_MUL ? (a.y || a.y_hi) : (a.epi == EPI_SLAB ? a.slab != nullptr : a.y != nullptr),
                 "gemm3: null output");
    LLMI_REQUIRE(a.lda % 8 == 0 && (reinterpret_cast<uintptr_t>(a.a[0]) & 15) == 0 &&
                     (a.planes == 1 || (reinterpret_cast<uintptr_t>(a.a[1]) & 15) == 0),
                 "gemm3: A planes must be 16-B aligned with lda % 8 == 0");
    LLMI_REQUIRE((reinterpret_cast<uintptr_t>(a.w) & 15) == 0 && a.k % 8 == 0, "gemm3: W must be 16-B aligned");
    LLMI_REQUIRE(a.epi != EPI_SILU_MUL || a.pair_off == a.n / 2, "gemm3: gate_up pair offset must be N / 2");
    LLMI_REQUIRE(a.epi != EPI_SILU_MUL || !a.y_hi ||
                     (a.ldy % 8 == 0 && (reinterpret_cast<uintptr_t>(a.y_hi) & 15) == 0 &&
                      (!a.y_lo || (reinterpret_cast<uintptr_t>(a.y_lo) & 15) == 0)),
                 "gemm3: fp16 output planes must be 16-B aligned with ldy % 8 == 0");
    LLMI_REQUIRE(!a.lo8 || (a.planes == 2 && a.w8 && a.k % (2 * kK) == 0 && a.k / (2 * kK) >= a.ksplit &&
                            (reinterpret_cast<uintptr_t>(a.w8) & 15) == 0 &&
                            (a.epi != EPI_SILU_MUL || (a.y_hi && a.y_lo))),
                 "gemm3: the fp8 lo plane needs planes = 2, w8, K a multiple of 128, >= one 128-deep tile per slice "
                 "and (gate_up) both output planes");
    const int ncols = (a.epi == EPI_SILU_MUL) ? a.n / 2 : a.n;
    a.n_tiles = ncols / ((a.epi == EPI_SILU_MUL) ? 128 : kTile);
    const int grid = ((a.m + kTile - 1) / kTile) * a.n_tiles * a.ksplit;
    if (a.epi == EPI_SILU_MUL && a.planes == 2 && a.bal_slab && a.bal_flags) {
        // every CU busy: lo workers beside the tile owners, when the split is even enough
        // (a tile touched by at most two workers) and the slots are large enough
        // owner share `own` (units of two lo tiles) so that owner (hi tiles + own units) and
        // worker (their share of the rest) times meet. A hi tile costs 0.5 unit against fp16
        // lo tiles; against fp8 ones ~0.35 (measured: an fp8 lo tile costs ~1.4x an fp16
        // one in this kernel, 2.2 vs 1.55 us)
        const int n_lo = a.bal_grid - grid, Pall = a.k / (a.lo8 ? 256 : 128);
        const double per = (double)grid / (n_lo > 0 ? n_lo : 1);  // tiles per worker
        const double hi_units = (a.lo8 ? 0.35 : 0.5) * (a.k / kK);
        int own = (int)std::lround((Pall * per - hi_units) / (1.0 + per));
        own = std::max(0, std::min(Pall - 1, own));
        const int P = Pall - own, U = grid * P;
        a.bal_own = own;
        if (a.k % (a.lo8 ? 256 : 128) == 0 && n_lo >= 1 && U / n_lo >= P &&
            gemm3_bal_slab_bytes(a.m, a.n) > 0) {
            static std::atomic<unsigned> epoch{0};
            a.bal_epoch = ++epoch;
            if (a.bal_epoch == 0) a.bal_epoch = ++epoch;  // 0 is the flags' initial value
            static const bool attr = [] {
                return hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm3_silu_bal_kernel),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, kLds) == hipSuccess;
            }();
            LLMI_REQUIRE(attr, "gemm3: cannot raise the dynamic LDS limit");
            hipLaunchKernelGGL(gemm3_silu_bal_kernel, dim3(a.bal_grid), dim3(kT), kLds, s, a);
            LLMI_HIP(hipGetLastError());
            return LLMI_OK;
        }
    }
    if (a.sk_slab && a.sk_flags && a.sk_grid > 0 && (a.epi == EPI_STORE || a.epi == EPI_SILU_MUL)) {
        const Gemm3SkPlan p = gemm3_sk_plan(a.m, a.n, a.k, a.epi, a.planes, a.lo8, a.sk_grid);
        LLMI_REQUIRE(p.pmax > 0, "gemm3: stream-K requested for a shape it does not cover (see gemm3_sk_plan)");
        LLMI_REQUIRE(a.sk_ctl && a.sk_ctl + kSkCtlWords == a.sk_flags,
                     "gemm3: stream-K needs its control words just before the flags (sk_workspace)");
        int left = g_sk_debug_left.load();
        while (left > 0 && !g_sk_debug_left.compare_exchange_weak(left, left - 1)) {
        }
        a.sk_pmax = p.pmax | ((left > 0 ? g_sk_debug_mode.load() : 0) << 8);  // + the fault-injection mode
        if (a.epi == EPI_STORE) return launch_sk<EPI_STORE>(a, s);
        return launch_sk<EPI_SILU_MUL>(a, s);
    }
    switch (a.epi) {
        case EPI_STORE: return launch_g3<EPI_STORE>(a, grid, s);
        case EPI_ADD: return launch_g3<EPI_ADD>(a, grid, s);
        case EPI_SILU_MUL: return launch_g3<EPI_SILU_MUL>(a, grid, s);
        case EPI_SLAB: return launch_g3<EPI_SLAB>(a, grid, s);
    }
    LLMI_REQUIRE(false, "gemm3: epilogue must be store, add, silu_mul or slab");
}

}  // namespace llmi
