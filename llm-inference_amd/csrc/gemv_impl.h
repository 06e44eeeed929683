// GEMV body of gemv_kernel (gemv_launch.h; design notes in gemv.hip).
#pragma once
#include "io.h"
#include "kernels.h"

namespace llmi {
namespace gemv_detail {

constexpr int kThreads = 256;
constexpr int kWavesPerBlock = kThreads / kWave;
#ifndef LLMI_GEMV_UNROLL
#define LLMI_GEMV_UNROLL 8
#endif
#ifndef LLMI_GEMV_ROWS
#define LLMI_GEMV_ROWS 2
#endif
#ifndef LLMI_I8_PIPE
#define LLMI_I8_PIPE 0  // software-pipelined int8 gate_up stream (measured: 30.7 vs 28.2 us once grids are clamped to residency)
#endif
#ifndef LLMI_GEMV_PIPE16
#define LLMI_GEMV_PIPE16 0  // bit EPI: software-pipelined fp16 stream for that epilogue
#endif
constexpr int kUnrollMax = LLMI_GEMV_UNROLL;  // 16-B loads per row in flight per lane
constexpr int kRows = LLMI_GEMV_ROWS;      // rows per wave (EPI_SILU_MUL always pairs 2)

template <typename WT> struct WT_ { };
template <> struct WT_<__half> { static constexpr int EPL = 8; };
template <> struct WT_<float> { static constexpr int EPL = 4; };
template <> struct WT_<int8_t> { static constexpr int EPL = 16; };

__device__ __forceinline__ float dot_packet(const uint4& w, const float4* xp, int nc, __half*) {
    const __half2* h = reinterpret_cast<const __half2*>(&w);
    float4 x0 = xp[0], x1 = xp[nc];
    float2 a = __half22float2(h[0]), b = __half22float2(h[1]);
    float2 c = __half22float2(h[2]), d = __half22float2(h[3]);
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
__device__ __forceinline__ float dot_packet(const uint4& w, const float4* xp, int nc, float*) {
    float4 x0 = xp[0];
    float s = __uint_as_float(w.x) * x0.x;
    s = fmaf(__uint_as_float(w.y), x0.y, s);
    s = fmaf(__uint_as_float(w.z), x0.z, s);
    s = fmaf(__uint_as_float(w.w), x0.w, s);
    return s;
}
__device__ __forceinline__ float i8(uint32_t v, int j) { return (float)(int8_t)((v >> (8 * j)) & 0xff); }
__device__ __forceinline__ float dot_packet(const uint4& w, const float4* xp, int nc, int8_t*) {
    const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        float4 x = xp[p * nc];
        s = fmaf(i8(ws[p], 0), x.x, s);
        s = fmaf(i8(ws[p], 1), x.y, s);
        s = fmaf(i8(ws[p], 2), x.z, s);
        s = fmaf(i8(ws[p], 3), x.w, s);
    }
    return s;
}

__device__ __forceinline__ float silu(float v) { return v / (1.0f + expf(-v)); }

template <typename GT>
__device__ __forceinline__ float4 gamma4(const void* g, int j) {
    if constexpr (sizeof(GT) == 2) {
        const uint2 u = reinterpret_cast<const uint2*>(g)[j];
        const float2 a = __half22float2(*reinterpret_cast<const __half2*>(&u.x));
        const float2 b = __half22float2(*reinterpret_cast<const __half2*>(&u.y));
        return make_float4(a.x, a.y, b.x, b.y);
    } else {
        return reinterpret_cast<const float4*>(g)[j];
    }
}

// LDS bytes the body needs for a k-wide x: [PK][nc] float4 image + reduction scratch + keys
__host__ __device__ inline size_t gemv_lds_bytes(int k) {
    return (size_t)k * 4 + 16 * 4 + kWavesPerBlock * 8 + kWavesPerBlock * 2 * 4;  // + kpar partials [4][2]
}

// XPT: float4s of x each thread holds in registers during staging (k <= XPT*4*256);
// 0 = generic strided staging (standalone only).
// bid / nblk: this workgroup's index in the GEMV grid and the grid size.
// TAG (EPI_STORE only; the fused q/k/v + attention launch, qkv_attn.hip): rows go out as
// write-through {fp32 bits, tag} granules in a.y_tag instead of fp32 stores in a.y.
template <typename WT, int ROWS, int EPI, bool NORM, typename GT, int XPT, int kUnroll, bool XFIX, typename IO,
          int KPT = 1, bool TAG = false>
__device__ __forceinline__ void gemv_body(const GemvArgs& a, int bid, int nblk, float4* xs) {
    static_assert(!TAG || EPI == EPI_STORE, "granule rows: store epilogue only");
    // the tag's epoch is one scalar load, issued first (consumed in the first epilogue)
    const unsigned long long tag_hi = TAG ? (unsigned long long)(*a.tag_epoch * 128u + a.tag_layer) << 32 : 0ull;
    // residual hand-over (seed_dst <- seed_src slice)
    auto seed = [&, bid0 = bid, nblk0 = nblk]() {
        if (a.seed_dst == nullptr) return;
        const int per = (a.seed_n + nblk0 - 1) / nblk0;
        const int i0 = bid0 * per, i1 = min(i0 + per, a.seed_n);
        for (int i = i0 + (int)threadIdx.x; i < i1; i += kThreads)
            IO::st_ll(a.seed_dst + i, a.seed_keep ? IO::ld_ll(a.seed_src + i) : 0ll);
    };
    constexpr int EPL = WT_<WT>::EPL;
    constexpr int PK = EPL / 4;                 // float4 packets per 16-B weight load
    static_assert(!(XFIX && EPI == EPI_ATOMIC), "split-K reads an fp32 x");
    // split-K (EPI_ATOMIC): workgroup bid takes K slice bid % S of row-group block bid / S
    const int S = (EPI == EPI_ATOMIC) ? a.ksplit : 1;
    const int ks = bid % S;
    bid /= S;
    nblk /= S;
    const int k = a.k / S;                      // this workgroup's K extent
    const int k4 = k / 4;
    const int nc = k / EPL;                     // 16-B chunks per row
    float* red = reinterpret_cast<float*>(xs + k4);
    unsigned long long* best_s = reinterpret_cast<unsigned long long*>(red + 16);
    float* kpart = reinterpret_cast<float*>(best_s + kWavesPerBlock);  // [wave][ROWS] kpar partial dots
    const int tid = threadIdx.x, lane = tid & 63;
    const int n_groups = (EPI == EPI_SILU_MUL) ? a.pair_off : (a.n_rows + ROWS - 1) / ROWS;
    // LLMI_I8_PIPE: bit EPI enables the software-pipelined int8 stream for that epilogue
    // (4 = gate_up only); LLMI_GEMV_PIPE16 the same for fp16 (both off by default)
    constexpr bool PIPE = (sizeof(WT) == 1 && kUnroll <= 5 && ((LLMI_I8_PIPE >> EPI) & 1))
                          || (sizeof(WT) == 2 && ((LLMI_GEMV_PIPE16 >> EPI) & 1));
    // KPT (GemvArgs::kpar, a template argument so the KPT = 1 kernels are unchanged):
    // wave w takes K part w % KP of the workgroup's group slot w / KP
    constexpr bool KPOK = (EPI == EPI_STORE || EPI == EPI_SILU_MUL) && ROWS <= 2 && !PIPE;
    constexpr int KP = KPOK ? KPT : 1;
    const int wave = (tid >> 6) / KP, kq = (tid >> 6) % KP;  // group slot and K part
    constexpr int gpw = kWavesPerBlock / KP;                  // groups per workgroup
    const int c_lo = KP > 1 ? kq * (nc / KP) : 0;              // this wave's chunks [c_lo, c_hi)
    const int c_hi = KP > 1 ? c_lo + nc / KP : nc;
    const size_t row_bytes = (size_t)(a.ldw ? a.ldw : a.k) * sizeof(WT);
    const char* wbase = reinterpret_cast<const char*>(a.w) + (size_t)ks * k * sizeof(WT);
    const float4* x4 = reinterpret_cast<const float4*>(a.x + (size_t)ks * k);

    auto rows_of = [&](int g, int* rows) {
        if constexpr (TAG) {
            // head-major order (a.tag_heads > 0, MHA): group g of head h's q, k, v rows in turn,
            // so a head's rows finish together and its attention can start while later heads'
            // rows stream (64 two-row groups per 128-row head block)
            if (a.tag_heads > 0) {
                const int h = g / 192, rem = g - 192 * h, t = rem >> 6;
                g = t * a.tag_heads * 64 + h * 64 + (rem & 63);
            }
        }
#pragma unroll
        for (int r = 0; r < ROWS; ++r) rows[r] = (EPI == EPI_SILU_MUL) ? g + r * a.pair_off : g * ROWS + r;
    };
    // Branch-free streaming: every lane always issues its ROWS x kUnroll loads; out of
    // range chunks/rows are clamped to a valid address and zeroed by a mask. A
    // predicated load makes hipcc branch around each load and wait vmcnt(0) per load
    // (cdna_hip_programming.md §5 "three .s-level traps" (c)), serialising the stream.
    auto load_batch = [&](uint4 (&wv)[ROWS][kUnroll], const int* rows, int base) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int c = base + u * kWave + lane;
            const int cc = c < c_hi ? c : c_hi - 1;
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                const int rr = rows[r] < a.n_rows ? rows[r] : a.n_rows - 1;
                const unsigned m = (c < c_hi && rows[r] < a.n_rows) ? 0xFFFFFFFFu : 0u;
                uint4 v = ld_nt16(wbase + (size_t)rr * row_bytes + (size_t)cc * 16);
                v.x &= m; v.y &= m; v.z &= m; v.w &= m;
                wv[r][u] = v;
            }
        }
    };
    auto dot_batch = [&](const uint4 (&wv)[ROWS][kUnroll], int base, float* acc) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int c = base + u * kWave + lane;
            const float4* xp = xs + (c < c_hi ? c : c_hi - 1);  // masked chunks have zero weights
#pragma unroll
            for (int r = 0; r < ROWS; ++r) acc[r] += dot_packet(wv[r][u], xp, nc, (WT*)nullptr);
        }
    };

    // ---- prologue. Issue order matters: vmcnt retires loads in issue order, so x
    // (and gamma) go first, then this wave's first weight batch; the weight stream is
    // then in flight while x is staged and the norm is reduced.
    const int g0 = bid * gpw + wave;
    int rows0[ROWS];
    rows_of(g0, rows0);
    uint4 w0[ROWS][kUnroll];
    float ss = 0.f;
    const bool wb = XFIX && bid == 0 && a.x_out != nullptr;  // one block writes x back
    if constexpr (XPT > 0) {
        // branch-free: clamp the index, load, and predicate only the LDS store
        float4 xv[XPT], gv[XPT];
        longlong2 xf[XFIX ? XPT : 1][2];
#pragma unroll
        for (int i = 0; i < XPT; ++i) {
            int j = tid + i * kThreads;
            j = j < k4 ? j : k4 - 1;
            if constexpr (XFIX) {
                xf[i][0] = IO::ld_ll2(reinterpret_cast<const longlong2*>(a.x_fixed) + 2 * j);
                xf[i][1] = IO::ld_ll2(reinterpret_cast<const longlong2*>(a.x_fixed) + 2 * j + 1);
            } else {
                xv[i] = IO::ld4(x4 + j);
            }
            if (NORM) gv[i] = gamma4<GT>(a.gamma, j);
        }
        load_batch(w0, rows0, c_lo);
        // RMSNorm (modeling_llama.py:112-117) as gamma*x staged + one scalar rsqrt per
        // dot product in the epilogue: sum_k W[r,k] gamma_k x_k * rstd.
#pragma unroll
        for (int i = 0; i < XPT; ++i) {
            const int j = tid + i * kThreads;
            if (j < k4) {
                float4 v;
                if constexpr (XFIX) {
                    v = make_float4(from_fixed(xf[i][0].x), from_fixed(xf[i][0].y),
                                    from_fixed(xf[i][1].x), from_fixed(xf[i][1].y));
                    if (wb) IO::st4(reinterpret_cast<float4*>(a.x_out) + j, v);
                } else {
                    v = xv[i];
                }
                if (NORM) {
                    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
                    v.x *= gv[i].x; v.y *= gv[i].y; v.z *= gv[i].z; v.w *= gv[i].w;
                }
                xs[(j % PK) * nc + j / PK] = v;
            }
        }
    } else {
        for (int j = tid; j < k4; j += kThreads) {
            float4 v;
            if constexpr (XFIX) {
                const long long* f = a.x_fixed + 4 * j;
                v = make_float4(from_fixed(f[0]), from_fixed(f[1]), from_fixed(f[2]), from_fixed(f[3]));
                if (wb) reinterpret_cast<float4*>(a.x_out)[j] = v;
            } else {
                v = x4[j];
            }
            if (NORM) {
                const float4 gg = gamma4<GT>(a.gamma, j);
                ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
                v.x *= gg.x; v.y *= gg.y; v.z *= gg.z; v.w *= gg.w;
            }
            xs[(j % PK) * nc + j / PK] = v;
        }
        load_batch(w0, rows0, c_lo);
    }
    seed();
    float rstd = 1.f;
    if (NORM) {
        ss = block_sum(ss, red);  // its barriers also publish xs
        rstd = 1.0f / sqrtf(ss / (float)k + a.eps);
    } else {
        __syncthreads();
    }

    unsigned long long best = 0ull;
    // single-producer EPI_ATOMIC: the first group's base values, loaded with the prologue so the
    // epilogue's store does not wait for them (lane r holds row rows0[r])
    long long pre_b = 0;
    if constexpr (EPI == EPI_ATOMIC) {
        if (a.yacc_single && a.yacc_base && lane < ROWS && g0 < n_groups)
        {
            int rr = rows0[0];
#pragma unroll
            for (int r = 1; r < ROWS; ++r) rr = lane == r ? rows0[r] : rr;  // no dynamic register index
            pre_b = IO::ld_ll(a.yacc_base + min(rr, a.n_rows - 1));
        }
    }
    auto finish = [&](int g, const int* rows, float* acc) {
        if constexpr (KP > 1) {  // the K parts of one group meet in LDS; part 0 adds them in order
#pragma unroll
            for (int r = 0; r < ROWS; ++r) acc[r] = wave_sum(acc[r]);
            if (lane == 0)
#pragma unroll
                for (int r = 0; r < ROWS; ++r) kpart[(tid >> 6) * 2 + r] = acc[r];
            __syncthreads();
            if (kq != 0 || g >= n_groups) return;
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                float sum = kpart[(wave * KP) * 2 + r];
                for (int q = 1; q < KP; ++q) sum += kpart[(wave * KP + q) * 2 + r];
                acc[r] = sum * rstd;
                if (a.scales != nullptr && rows[r] < a.n_rows) acc[r] *= __half2float(a.scales[rows[r]]);
            }
        } else {
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                acc[r] = wave_sum(acc[r]) * rstd;
                if (a.scales != nullptr && rows[r] < a.n_rows) acc[r] *= __half2float(a.scales[rows[r]]);
            }
        }
        if (EPI == EPI_SILU_MUL) {
            if (lane == 0) IO::st(a.y + g, silu(acc[0]) * acc[1]);
        } else {
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                const int row = rows[r];
                if (row >= a.n_rows) continue;
                if (lane == r) {
                    float v = acc[r];
                    if (EPI == EPI_ATOMIC) {
                        if (a.yacc_single) {  // single producer: base + fixed(v), written through (sc1)
                            const long long b = !a.yacc_base ? 0ll : g == g0 ? pre_b : IO::ld_ll(a.yacc_base + row);
                            const unsigned long long nv = (unsigned long long)(b + to_fixed(v));
                            __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.yacc + row), nv,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            if (a.yacc_copy)  // this row's xmid was read above (pre_b): overwriting it is safe
                                __hip_atomic_store(reinterpret_cast<unsigned long long*>(a.yacc_copy + row), nv,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        } else {
                            atomicAdd(reinterpret_cast<unsigned long long*>(a.yacc + row),
                                      (unsigned long long)to_fixed(v));
                        }
                    } else if constexpr (TAG) {
                        __hip_atomic_store(a.y_tag + row, tag_hi | (unsigned long long)__float_as_uint(v),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    } else {
                        if (EPI == EPI_ADD) v += a.resid_scale * IO::ld(a.resid + row);
                        IO::st(a.y + row, v);
                    }
                }
                if (EPI == EPI_ARGMAX) {
                    unsigned long long kk = argmax_key(acc[r], a.idx_base + (uint32_t)row);
                    best = kk > best ? kk : best;
                }
            }
        }
    };

    // ---- int8: software-pipelined stream over (row group, batch) items -- the next
    // item's loads are issued before the current item's convert + FMA work, across
    // row-group boundaries too; two register buffers, manually unrolled by 2. The
    // item after the last one re-loads the last item (a cache hit, never used).
    // (PIPE is defined at the top of the body.)
    if constexpr (PIPE) {
        constexpr int B = kWave * kUnroll;
        const int stride = nblk * kWavesPerBlock;
        if (g0 < n_groups) {
            auto advance = [&](int& g, int& base) {
                base += B;
                if (base >= nc) {
                    base = 0;
                    g += stride;
                }
            };
            float acc[ROWS];
#pragma unroll
            for (int r = 0; r < ROWS; ++r) acc[r] = 0.f;
            int ga = g0, ba = 0;
            int rows_a[ROWS], rows_b[ROWS];
            rows_of(ga, rows_a);
            uint4 wb[ROWS][kUnroll];
            auto step = [&](const uint4 (&cur)[ROWS][kUnroll], const int* rows_c, int gc, int bc, float* ac) {
                dot_batch(cur, bc, ac);
                if (bc + B >= nc) {
                    finish(gc, rows_c, ac);
#pragma unroll
                    for (int r = 0; r < ROWS; ++r) ac[r] = 0.f;
                }
            };
            for (;;) {
                int gb = ga, bb = ba;
                advance(gb, bb);
                const bool vb = gb < n_groups;
                if (!vb) { gb = ga; bb = ba; }
                rows_of(gb, rows_b);
                load_batch(wb, rows_b, bb);
                step(w0, rows_a, ga, ba, acc);
                if (!vb) break;
                int gc = gb, bc = bb;
                advance(gc, bc);
                const bool vc = gc < n_groups;
                if (!vc) { gc = gb; bc = bb; }
                rows_of(gc, rows_a);
                load_batch(w0, rows_a, bc);
                step(wb, rows_b, gb, bb, acc);
                if (!vc) break;
                ga = gc;
                ba = bc;
            }
        }
    }
    constexpr int B = kWave * kUnroll;  // chunks per batch
    // ---- first group (its first batch is already in flight)
    if (!PIPE && (g0 < n_groups || KP > 1)) {  // kpar: every wave reaches finish's barrier
        float acc[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) acc[r] = 0.f;
        dot_batch(w0, c_lo, acc);
        for (int base = c_lo + B; base < c_hi; base += B) {
            uint4 wv[ROWS][kUnroll];
            load_batch(wv, rows0, base);
            dot_batch(wv, base, acc);
        }
        finish(g0, rows0, acc);
    }
    // ---- remaining groups (KP == 1: a wave's later groups)
    for (int g = g0 + nblk * kWavesPerBlock; !PIPE && KP == 1 && g < n_groups; g += nblk * kWavesPerBlock) {
        int rows[ROWS];
        rows_of(g, rows);
        float acc[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) acc[r] = 0.f;
        for (int base = 0; base < nc; base += kWave * kUnroll) {
            uint4 wv[ROWS][kUnroll];
            load_batch(wv, rows, base);
            dot_batch(wv, base, acc);
        }
        finish(g, rows, acc);
    }
    if (EPI == EPI_ARGMAX) {
        if (lane == 0) best_s[wave] = best;
        __syncthreads();
        if (tid == 0) {
            unsigned long long b = best_s[0];
            for (int i = 1; i < kWavesPerBlock; ++i) b = best_s[i] > b ? best_s[i] : b;
            // agent-scope (write-through) store: a fused exchange tail may read it in-launch
            __hip_atomic_store(a.partials + bid, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace gemv_detail
}  // namespace llmi
