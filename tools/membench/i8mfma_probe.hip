// Go/no-go probe for an int8 (W8A16) decode GEMV on the int8 matrix cores instead of the
// VALU dequantising dot (gemv_impl.h): y[r] = sum_k W[r, k] x[k] with x split into three
// int8 planes (x ~ s (q1 + q2 / 256 + q3 / 65536), exact int32 sums per plane) and
// v_mfma_i32_16x16x64_i8 taking 16 rows x 64 K of W per 16-B lane load (lane l: row l & 15,
// bytes 16 (l >> 4) of each 64-deep step; every B column holds the same x bytes, so each
// lane ends with its 4 rows' sums). 1/16 of the MFMA is used; no per-weight VALU work.
// Shape: Llama-2-13B q/k/v (15,360 x 5,120) and gate_up (27,648 x 5,120), launches cycling
// through 8 weight copies (> the 256 MiB Infinity Cache). Checked against fp64 on the host.
//   build: hipcc -O3 --offload-arch=gfx950 i8mfma_probe.hip -o i8mfma_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i4 __attribute__((ext_vector_type(4)));
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

template <int U>
__global__ __launch_bounds__(256) void gemv_i8mfma(const signed char* W, int K, const signed char* xpl, float s,
                                                   float* y, int groups) {
    extern __shared__ __attribute__((aligned(16))) signed char xs[];  // [3][K]
    for (int i = threadIdx.x * 16; i < 3 * K; i += 256 * 16)
        *reinterpret_cast<i4*>(xs + i) = *reinterpret_cast<const i4*>(xpl + i);
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, q = lane >> 4;
    const int nsteps = K / 64;
    for (int g = blockIdx.x * 4 + wave; g < groups; g += gridDim.x * 4) {
        const signed char* wr = W + (size_t)(g * 16 + r) * K + 16 * q;
        i4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0;
        for (int j0 = 0; j0 < nsteps; j0 += U) {
            i4 a[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const u4 v = __builtin_nontemporal_load(reinterpret_cast<const u4*>(wr + 64 * (j0 + u)));
                a[u] = __builtin_bit_cast(i4, v);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int off = 64 * (j0 + u) + 16 * q;
                const i4 b0 = *reinterpret_cast<const i4*>(xs + off);
                const i4 b1 = *reinterpret_cast<const i4*>(xs + K + off);
                const i4 b2 = *reinterpret_cast<const i4*>(xs + 2 * K + off);
                a0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u], b0, a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u], b1, a1, 0, 0, 0);
                a2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u], b2, a2, 0, 0, 0);
            }
        }
        if (r == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                y[g * 16 + 4 * q + i] = s * ((float)a0[i] + (float)a1[i] * (1.f / 256.f) + (float)a2[i] * (1.f / 65536.f));
        }
    }
}

// K split over the KW waves of a workgroup (one 16-row group per workgroup): KW x more
// waves than row groups, each wave's whole K slice in flight in one batch, int32 partials
// summed through LDS
template <int KW, int U>
__global__ __launch_bounds__(64 * KW) void gemv_i8mfma_ks(const signed char* W, int K, const signed char* xpl, float s,
                                                         float* y) {
    extern __shared__ __attribute__((aligned(16))) signed char xs[];  // [3][K], then [KW][3][16] int32
    int* red = reinterpret_cast<int*>(xs + 3 * K);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, q = lane >> 4;
    const int g = blockIdx.x;
    const int S = K / 64, j0 = wave * S / KW;  // this wave's steps [j0, j0 + U)
    const signed char* wr = W + (size_t)(g * 16 + r) * K + 16 * q;
    i4 a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const u4 v = __builtin_nontemporal_load(reinterpret_cast<const u4*>(wr + 64 * (j0 + u)));
        a[u] = __builtin_bit_cast(i4, v);
    }
    for (int i = threadIdx.x * 16; i < 3 * K; i += 64 * KW * 16)
        *reinterpret_cast<i4*>(xs + i) = *reinterpret_cast<const i4*>(xpl + i);
    __syncthreads();
    i4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int off = 64 * (j0 + u) + 16 * q;
        const i4 b0 = *reinterpret_cast<const i4*>(xs + off);
        const i4 b1 = *reinterpret_cast<const i4*>(xs + K + off);
        const i4 b2 = *reinterpret_cast<const i4*>(xs + 2 * K + off);
        a0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u], b0, a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u], b1, a1, 0, 0, 0);
        a2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[u], b2, a2, 0, 0, 0);
    }
    if (r == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            red[(wave * 3 + 0) * 16 + 4 * q + i] = a0[i];
            red[(wave * 3 + 1) * 16 + 4 * q + i] = a1[i];
            red[(wave * 3 + 2) * 16 + 4 * q + i] = a2[i];
        }
    }
    __syncthreads();
    if (threadIdx.x < 16) {
        int c0 = 0, c1 = 0, c2 = 0;
        for (int w = 0; w < KW; ++w) {
            c0 += red[(w * 3 + 0) * 16 + threadIdx.x];
            c1 += red[(w * 3 + 1) * 16 + threadIdx.x];
            c2 += red[(w * 3 + 2) * 16 + threadIdx.x];
        }
        y[g * 16 + threadIdx.x] = s * ((float)c0 + (float)c1 * (1.f / 256.f) + (float)c2 * (1.f / 65536.f));
    }
}

template <int KW, int U>
float run_ks(const signed char* w, size_t wbytes, int ncopies, int rows, int K, const signed char* xpl, float s, float* y,
             int iters) {
    const size_t lds = 3 * (size_t)K + KW * 3 * 16 * 4;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL((gemv_i8mfma_ks<KW, U>), dim3(rows / 16), dim3(64 * KW), lds, 0,
                           w + (size_t)(i % ncopies) * wbytes, K, xpl, s, y);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL((gemv_i8mfma_ks<KW, U>), dim3(rows / 16), dim3(64 * KW), lds, 0,
                           w + (size_t)(i % ncopies) * wbytes, K, xpl, s, y);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.f / iters;
}

template <int U>
float run(const signed char* w, size_t wbytes, int ncopies, int rows, int K, const signed char* xpl, float s, float* y,
          int grid, int iters) {
    const int groups = rows / 16;
    const size_t lds = 3 * (size_t)K;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL(gemv_i8mfma<U>, dim3(grid), dim3(256), lds, 0, w + (size_t)(i % ncopies) * wbytes, K, xpl, s,
                           y, groups);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL(gemv_i8mfma<U>, dim3(grid), dim3(256), lds, 0, w + (size_t)(i % ncopies) * wbytes, K, xpl, s,
                           y, groups);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.f / iters;
}

int main() {
    const int K = 5120;
    const int shapes[2] = {15360, 27648};
    const char* names[2] = {"qkv_13b", "gate_up_13b"};
    const int ncopies = 8;
    const size_t maxw = (size_t)27648 * K;
    signed char* w;
    CK(hipMalloc(&w, maxw * ncopies));
    std::vector<signed char> hw(maxw);
    unsigned st = 12345u;
    for (auto& v : hw) {
        st = st * 1664525u + 1013904223u;
        v = (signed char)((int)(st >> 24) - 128 == -128 ? 0 : (int)(st >> 24) - 128);
    }
    for (int c = 0; c < ncopies; ++c) CK(hipMemcpy(w + (size_t)c * maxw, hw.data(), maxw, hipMemcpyHostToDevice));
    // x and its three int8 planes
    std::vector<float> x(K);
    for (auto& v : x) {
        st = st * 1664525u + 1013904223u;
        v = ((st >> 8) / 16777216.0f - 0.5f) * 4.f;
    }
    float mx = 0.f;
    for (float v : x) mx = std::fmax(mx, std::fabs(v));
    const float s = mx / 127.f;
    std::vector<signed char> pl(3 * (size_t)K);
    for (int k = 0; k < K; ++k) {
        double rem = x[k] / s;
        for (int p = 0; p < 3; ++p) {
            double qv = std::nearbyint(rem);
            qv = std::fmax(-127.0, std::fmin(127.0, qv));
            pl[(size_t)p * K + k] = (signed char)qv;
            rem = (rem - qv) * 256.0;
        }
    }
    signed char* xpl;
    float* y;
    CK(hipMalloc(&xpl, pl.size()));
    CK(hipMalloc(&y, 27648 * 4));
    CK(hipMemcpy(xpl, pl.data(), pl.size(), hipMemcpyHostToDevice));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    for (int si = 0; si < 2; ++si) {
        const int rows = shapes[si];
        // correctness (copy 0) against fp64 with the unquantised x
        hipLaunchKernelGGL(gemv_i8mfma<8>, dim3(rows / 64), dim3(256), 3 * K, 0, w, K, xpl, s, y, rows / 16);
        CK(hipDeviceSynchronize());
        std::vector<float> hy(rows);
        CK(hipMemcpy(hy.data(), y, rows * 4, hipMemcpyDeviceToHost));
        double num = 0, den = 0;
        for (int r = 0; r < rows; ++r) {
            double ref = 0;
            for (int k = 0; k < K; ++k) ref += (double)hw[(size_t)r * K + k] * x[k];
            num += (hy[r] - ref) * (hy[r] - ref);
            den += ref * ref;
        }
        const double bytes = (double)rows * K;
        {  // K split over the waves of a workgroup (80 steps: 4 x 20 or 8 x 10 or 16 x 5)
            hipLaunchKernelGGL((gemv_i8mfma_ks<4, 20>), dim3(rows / 16), dim3(256), 3 * K + 4 * 3 * 16 * 4, 0, w, K, xpl, s,
                               y);
            CK(hipDeviceSynchronize());
            std::vector<float> hk(rows);
            CK(hipMemcpy(hk.data(), y, rows * 4, hipMemcpyDeviceToHost));
            double n2 = 0;
            for (int r2 = 0; r2 < rows; ++r2) n2 += (double)(hk[r2] - hy[r2]) * (hk[r2] - hy[r2]);
            const float k4 = run_ks<4, 20>(w, maxw, ncopies, rows, K, xpl, s, y, 50);
            const float k8 = run_ks<8, 10>(w, maxw, ncopies, rows, K, xpl, s, y, 50);
            const float k16 = run_ks<16, 5>(w, maxw, ncopies, rows, K, xpl, s, y, 50);
            std::printf("{\"shape\": \"%s\", \"ksplit_waves\": \"4/8/16\", \"vs_unsplit_rel\": %.3g, \"us\": [%.2f, %.2f, %.2f], "
                        "\"TBps\": [%.3f, %.3f, %.3f]}\n",
                        names[si], std::sqrt(n2 / den), k4, k8, k16, bytes / k4 / 1e6, bytes / k8 / 1e6, bytes / k16 / 1e6);
            std::fflush(stdout);
        }
        for (int grid : {rows / 64, 2 * ncu}) {
            const float t8 = run<8>(w, maxw, ncopies, rows, K, xpl, s, y, grid, 50);
            const float t16 = run<16>(w, maxw, ncopies, rows, K, xpl, s, y, grid, 50);
            std::printf("{\"shape\": \"%s\", \"rows\": %d, \"k\": %d, \"grid\": %d, \"rel_l2\": %.3g, \"u8_us\": %.2f, "
                        "\"u8_TBps\": %.3f, \"u16_us\": %.2f, \"u16_TBps\": %.3f}\n",
                        names[si], rows, K, grid, std::sqrt(num / den), t8, bytes / t8 / 1e6, t16, bytes / t16 / 1e6);
            std::fflush(stdout);
        }
    }
    return 0;
}
