// Prefill GEMM bench: gemm2 (128^2 tiles) vs gemm3 (256^2 ping-pong) on the
// Llama-2-7B prefill shapes at M rows (default 512) and a 4096^3 square, random
// fp16 operands, HIP-event timing; checks gemm3 against gemm2 (EPI_STORE).
//   hipcc -std=c++17 -O2 -I include -I llm-inference_amd/csrc tools/gemm_bench/gemm_bench.cpp \
//     -L llm-inference_amd/lib -lllmi -Wl,-rpath,$PWD/llm-inference_amd/lib -o tools/gemm_bench/gemm_bench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "kernels.h"

using namespace llmi;

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

__global__ void fill_kernel(_Float16* p, size_t n, unsigned seed, float scale) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
        p[i] = (_Float16)(((x & 0xffffff) / 8388608.0f - 1.0f) * scale);
    }
}

// exact-data mode: integers j / den with |j| <= 15 (e4m3-exact once scaled by a power of two)
__global__ void fill_int_kernel(_Float16* p, size_t n, unsigned seed, float den) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned x = (unsigned)i * 2654435761u ^ seed;
        x ^= x >> 15; x *= 2246822519u; x ^= x >> 13;
        p[i] = (_Float16)((float)((int)(x % 31u) - 15) / den);
    }
}
// the lo8 plane of gemm3 from fp16 lo values: e4m3(lo * 2^12) in the first lda bytes of each 2 lda-byte row
__global__ void lo8_kernel(const _Float16* lo, size_t rows, int lda, unsigned char* out) {
    const size_t n4 = rows * lda / 4;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const size_t e = 4 * i, r = e / lda, c = e % lda;
        *reinterpret_cast<uint32_t*>(out + r * 2 * lda + c) =
            lo8_pack4((float)lo[e], (float)lo[e + 1], (float)lo[e + 2], (float)lo[e + 3]);
    }
}

static void fill(_Float16* p, size_t n, unsigned seed, float scale) {
    hipLaunchKernelGGL(fill_kernel, dim3(2048), dim3(256), 0, 0, p, n, seed, scale);
    CK(hipGetLastError());
}

struct Shape {
    const char* name;
    int n, k, epi, ksplit;
};

template <typename F>
static float time_us(F f, int iters) {
    for (int i = 0; i < 3; ++i) f();
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) f();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return 1e3f * ms / iters;
}

int main(int argc, char** argv) {
    const int M = argc > 1 ? std::atoi(argv[1]) : 512;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 20;
    const int check = argc > 3 ? std::atoi(argv[3]) : 1;
    const std::string only = argc > 4 ? argv[4] : "";  // run only this shape (and planes = argv[5])
    const int only_planes = argc > 5 ? std::atoi(argv[5]) : 0;  // 3 = the fp8 lo plane (lo8)
    const int exact_data = argc > 6 ? std::atoi(argv[6]) : 0;   // 1: e4m3-exact lo and W (checks the fp8 k map)
    std::vector<Shape> shapes = {
        {"qkv", 12288, 4096, EPI_STORE, 1},   {"qkv_s2", 12288, 4096, EPI_SLAB, 2},
        {"o_s2", 4096, 4096, EPI_SLAB, 2},    {"o_s4", 4096, 4096, EPI_SLAB, 4},
        {"o_s8", 4096, 4096, EPI_SLAB, 8},    {"gate_up", 22016, 4096, EPI_SILU_MUL, 1},
        {"down_s2", 4096, 11008, EPI_SLAB, 2}, {"down_s4", 4096, 11008, EPI_SLAB, 4},
        {"down_s8", 4096, 11008, EPI_SLAB, 8}, {"qkv_s3", 12288, 4096, EPI_SLAB, 3}, {"o_s16", 4096, 4096, EPI_SLAB, 16},
        {"sq4096", 4096, 4096, EPI_STORE, 1},
    };
    size_t maxA = 0, maxW = 0, maxY = 0;
    for (auto& s : shapes) {
        const int m = std::string(s.name) == "sq4096" ? 4096 : M;
        maxA = std::max(maxA, (size_t)m * s.k);
        maxW = std::max(maxW, (size_t)s.n * s.k);
        maxY = std::max(maxY, (size_t)m * s.n * (s.epi == EPI_SLAB ? s.ksplit : 1));
    }
    _Float16 *ah, *al, *al8, *w, *w8, *yh, *yl;
    float *y2, *y3, *slab;
    CK(hipMalloc(&ah, maxA * 2));
    CK(hipMalloc(&al, maxA * 2));
    CK(hipMalloc(&w, maxW * 2));
    CK(hipMalloc(&al8, maxA * 2));
    float* bal_slab;
    unsigned* bal_flags;
    int* bal_err;
    const size_t bal_bytes = gemm3_bal_slab_bytes(M, 22016);
    CK(hipMalloc(&bal_slab, bal_bytes));
    CK(hipMalloc(&bal_flags, 4096));
    CK(hipMalloc(&bal_err, 4));
    CK(hipMemset(bal_flags, 0, 4096));
    CK(hipMemset(bal_err, 0, 4));
    CK(hipMalloc(&w8, maxW * 2));
    CK(hipMalloc(&y2, maxY * 4));
    CK(hipMalloc(&y3, maxY * 4));
    CK(hipMalloc(&slab, maxY * 4));
    CK(hipMalloc(&yh, maxY * 2));
    CK(hipMalloc(&yl, maxY * 2));
    if (exact_data == 2) {  // zero-filled operands: the kernel's schedule without the power draw of random bits
        CK(hipMemset(ah, 0, maxA * 2));
        CK(hipMemset(al, 0, maxA * 2));
        CK(hipMemset(w, 0, maxW * 2));
    } else if (exact_data) {  // hi = 0, lo = j / 4096, W = j / 64: the lo8 pass is then exact (fp32 sums of integers)
        CK(hipMemset(ah, 0, maxA * 2));
        hipLaunchKernelGGL(fill_int_kernel, dim3(2048), dim3(256), 0, 0, al, maxA, 2u, 4096.f);
        hipLaunchKernelGGL(fill_int_kernel, dim3(2048), dim3(256), 0, 0, w, maxW, 3u, 64.f);
    } else {
        fill(ah, maxA, 1, 1.0f);
        fill(al, maxA, 2, 1.0f / 2048);
        fill(w, maxW, 3, 0.05f);
    }
    CK(hipDeviceSynchronize());

    for (auto& s : shapes) {
        if (!only.empty() && only != s.name) continue;
        const int m = std::string(s.name) == "sq4096" ? 4096 : M;
        int w8e = 0;
        if (only_planes == 0 || only_planes >= 3) {
            if (w8_prepare(w, s.n, s.k, w8, &w8e, 0) != 0) return 1;
            hipLaunchKernelGGL(lo8_kernel, dim3(2048), dim3(256), 0, 0, al, (size_t)m, s.k, (unsigned char*)al8);
            CK(hipDeviceSynchronize());
        }
        for (int pm = 1; pm <= 5; ++pm) {  // 4 / 5: lo8 / fp16 lo with the balanced gate_up (every CU busy)
            if (only_planes && pm != only_planes) continue;
            if (pm >= 4 && s.epi != EPI_SILU_MUL) continue;
            const int planes = pm >= 3 ? 2 : pm;
            Gemm2Args g;
            g.a[0] = ah; g.a[1] = al; g.planes = planes; g.lda = s.k; g.w = w; g.m = m; g.n = s.n; g.k = s.k;
            g.epi = s.epi; g.ksplit = s.ksplit; g.slab = slab; g.ldy = s.epi == EPI_SILU_MUL ? s.n / 2 : s.n;
            g.pair_off = s.epi == EPI_SILU_MUL ? s.n / 2 : 0;
            g.y_hi = s.epi == EPI_SILU_MUL ? yh : nullptr;
            g.y_lo = s.epi == EPI_SILU_MUL && planes == 2 ? yl : nullptr;
            g.y = y2;
            const double flop = 2.0 * m * s.n * s.k * planes;
            float us2 = -1.f;
            Gemm2Args g8 = g;  // the lo8 form of g (gemm3 only)
            g8.a[1] = al8; g8.lo8 = 1; g8.w8 = w8; g8.w8_exp = w8e;
            if (pm == 5) {  // the fp16 two-plane gate_up, balanced: through the lo8 report path with lo8 off
                g8 = g;
            }
            if (pm >= 4) {
                int ncu = 0;
                CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
                g8.bal_slab = bal_slab; g8.bal_flags = bal_flags; g8.bal_grid = ncu; g8.err = bal_err;
            }
            if (pm >= 3) {
                float us3 = -1.f;
                if (gemm3_supported(s.n, s.k, s.epi, s.ksplit) && s.k % 128 == 0 && s.k / 128 >= s.ksplit)
                    us3 = time_us([&] { gemm3_launch(g8, 0); }, iters);
                double err = -1;
                if (check && us3 > 0) {  // vs gemm2 with both fp16 planes (EPI_STORE; SILU: fp32 output)
                    Gemm2Args c = g;
                    c.epi = s.epi == EPI_SLAB ? EPI_STORE : s.epi;
                    c.y_hi = c.y_lo = nullptr;
                    c.y = y2;
                    gemm2_launch(c, 0);
                    const size_t ny = (size_t)m * g.ldy;
                    std::vector<float> h2(ny), h3(ny, 0.f);
                    CK(hipDeviceSynchronize());
                    CK(hipMemcpy(h2.data(), y2, ny * 4, hipMemcpyDeviceToHost));
                    if (s.epi == EPI_SLAB) {
                        gemm3_launch(g8, 0);
                        CK(hipDeviceSynchronize());
                        std::vector<float> sl(ny * s.ksplit);
                        CK(hipMemcpy(sl.data(), slab, sl.size() * 4, hipMemcpyDeviceToHost));
                        for (int q = 0; q < s.ksplit; ++q)
                            for (size_t i = 0; i < ny; ++i) h3[i] += sl[q * ny + i];
                    } else if (s.epi == EPI_SILU_MUL) {  // hi plane + the e4m3 lo plane back to fp32
                        gemm3_launch(g8, 0);
                        CK(hipDeviceSynchronize());
                        std::vector<_Float16> hh(ny);
                        std::vector<unsigned char> ll(ny * 2);
                        CK(hipMemcpy(hh.data(), yh, ny * 2, hipMemcpyDeviceToHost));
                        CK(hipMemcpy(ll.data(), yl, ny * 2, hipMemcpyDeviceToHost));
                        auto e4m3 = [](unsigned char b) {
                            const int sg = b >> 7, ex = (b >> 3) & 15, mn = b & 7;
                            const double v = ex ? std::ldexp(1.0 + mn / 8.0, ex - 7) : std::ldexp(mn / 8.0, -6);
                            return sg ? -v : v;
                        };
                        const _Float16* l16 = reinterpret_cast<const _Float16*>(ll.data());
                        for (size_t i = 0; i < ny; ++i) {
                            const size_t r = i / g.ldy, cc = i % g.ldy;
                            h3[i] = g8.lo8 ? (float)((double)hh[i] + std::ldexp(e4m3(ll[r * 2 * g.ldy + cc]), -12))
                                           : (float)((double)hh[i] + (double)l16[i]);
                        }
                    } else {
                        Gemm2Args c3 = g8;
                        c3.y = y3;
                        gemm3_launch(c3, 0);
                        CK(hipDeviceSynchronize());
                        CK(hipMemcpy(h3.data(), y3, ny * 4, hipMemcpyDeviceToHost));
                    }
                    double mx = 0, ref = 0;
                    for (size_t i = 0; i < ny; ++i) {
                        mx = std::max(mx, (double)std::fabs(h2[i] - h3[i]));
                        ref = std::max(ref, (double)std::fabs(h2[i]));
                    }
                    err = mx / (ref > 0 ? ref : 1);
                }
                int herr = 0;
                CK(hipMemcpy(&herr, bal_err, 4, hipMemcpyDeviceToHost));
                if (pm >= 4) {  // one stamped launch: worker / owner timelines (us from the first start)
                    unsigned long long* st;
                    const int ng = g8.bal_grid;
                    CK(hipMalloc(&st, (size_t)ng * 64));
                    CK(hipMemset(st, 0, (size_t)ng * 64));
                    Gemm2Args gs = g8;
                    gs.stamps = st;
                    gemm3_launch(gs, 0);
                    CK(hipDeviceSynchronize());
                    std::vector<unsigned long long> h((size_t)ng * 8);
                    CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
                    const int n_lo = ng - 172;
                    unsigned long long t0 = ~0ull;
                    for (int b = 0; b < ng; ++b) t0 = std::min(t0, h[b * 8]);
                    auto us = [&](unsigned long long v) { return (v - t0) / 100.0; };
                    double wk_start_max = 0, wk_end_min = 1e9, wk_end_max = 0, ow_start_max = 0, ow_hi_min = 1e9,
                           ow_hi_max = 0, ow_wait_max = 0, ow_end_max = 0;
                    for (int b = 0; b < ng; ++b) {
                        const unsigned long long* r = &h[b * 8];
                        if (b < n_lo) {
                            wk_start_max = std::max(wk_start_max, us(r[0]));
                            wk_end_min = std::min(wk_end_min, us(r[1]));
                            wk_end_max = std::max(wk_end_max, us(r[1]));
                        } else {
                            ow_start_max = std::max(ow_start_max, us(r[0]));
                            ow_hi_min = std::min(ow_hi_min, us(r[1]));
                            ow_hi_max = std::max(ow_hi_max, us(r[1]));
                            ow_wait_max = std::max(ow_wait_max, us(r[2]));
                            ow_end_max = std::max(ow_end_max, us(r[3]));
                        }
                    }
                    std::printf("{\"timeline_us\": {\"workers\": %d, \"worker_start_max\": %.1f, \"worker_end\": [%.1f, %.1f], "
                                "\"owner_start_max\": %.1f, \"owner_hi_done\": [%.1f, %.1f], \"owner_partials_in_max\": %.1f, "
                                "\"owner_end_max\": %.1f}}\n",
                                n_lo, wk_start_max, wk_end_min, wk_end_max, ow_start_max, ow_hi_min, ow_hi_max, ow_wait_max,
                                ow_end_max);
                    CK(hipFree(st));
                }
                std::printf("{\"shape\": \"%s\", \"m\": %d, \"n\": %d, \"k\": %d, \"planes\": \"%s\", \"ksplit\": %d, "
                            "\"w8_exp\": %d, \"exact_data\": %d, \"gemm3_us\": %.2f, \"rel_err\": %.3g, \"err_word\": %d}\n",
                            s.name, m, s.n, s.k, pm == 5 ? "hi+lo fp16 balanced" : pm == 4 ? "hi+lo8 balanced" : "hi+lo8", s.ksplit, w8e, exact_data, us3, err,
                            herr);
                std::fflush(stdout);
                continue;
            }
            if (gemm2_supported(s.n, s.k, s.epi) && (s.epi != EPI_SLAB || s.k % (s.ksplit * 64) == 0) && s.ksplit <= 8)
                us2 = time_us([&] { gemm2_launch(g, 0); }, iters);
            float us3 = -1.f;
            if (gemm3_supported(s.n, s.k, s.epi, s.ksplit)) us3 = time_us([&] { gemm3_launch(g, 0); }, iters);
            double err = -1;
            if (check && us3 > 0) {
                Gemm2Args c = g;
                c.epi = s.epi == EPI_SLAB ? EPI_STORE : s.epi;
                c.y_hi = c.y_lo = nullptr;
                c.y = y2;
                gemm2_launch(c, 0);
                const size_t ny = (size_t)m * g.ldy;
                std::vector<float> h2(ny), h3(ny, 0.f);
                if (s.epi == EPI_SLAB) {  // the slices of the timed gemm3 launch, summed in order
                    gemm3_launch(g, 0);
                    CK(hipDeviceSynchronize());
                    std::vector<float> sl(ny * s.ksplit);
                    CK(hipMemcpy(sl.data(), slab, sl.size() * 4, hipMemcpyDeviceToHost));
                    for (int q = 0; q < s.ksplit; ++q)
                        for (size_t i = 0; i < ny; ++i) h3[i] += sl[q * ny + i];
                } else {
                    c.y = y3;
                    gemm3_launch(c, 0);
                    CK(hipDeviceSynchronize());
                    CK(hipMemcpy(h3.data(), y3, ny * 4, hipMemcpyDeviceToHost));
                }
                CK(hipMemcpy(h2.data(), y2, ny * 4, hipMemcpyDeviceToHost));
                double mx = 0, ref = 0;
                for (size_t i = 0; i < ny; ++i) {
                    mx = std::max(mx, (double)std::fabs(h2[i] - h3[i]));
                    ref = std::max(ref, (double)std::fabs(h2[i]));
                }
                err = mx / (ref > 0 ? ref : 1);
            }
            std::printf(
                "{\"shape\": \"%s\", \"m\": %d, \"n\": %d, \"k\": %d, \"planes\": %d, \"ksplit\": %d, \"gemm2_us\": %.2f, "
                "\"gemm3_us\": %.2f, \"gemm2_tflops\": %.1f, \"gemm3_tflops\": %.1f, \"rel_err\": %.3g}\n",
                s.name, m, s.n, s.k, planes, s.ksplit, us2, us3, us2 > 0 ? flop / us2 * 1e-6 : 0.0,
                us3 > 0 ? flop / us3 * 1e-6 : 0.0, err);
            std::fflush(stdout);
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
