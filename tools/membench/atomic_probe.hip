// Go/no-go probe for a hand-off-free FFN (gate_up + down in one launch, W_d stored
// K-major): every workgroup would add a 4,096-wide int64 partial of the down output
// with device-scope atomics. How long do G x 4,096 such atomics take, alone and at
// the tail of a 270 MB weight stream (the fused FFN's bytes) spread over G
// workgroups? HIP-event timed, launches cycling through regions of a 2 GiB buffer.
//   build: hipcc -O3 --offload-arch=gfx950 atomic_probe.hip -o atomic_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// mode 0: stream only; 1: stream + 4096 int64 atomics per workgroup;
// 2: stream + 4096 fp32 plain stores per workgroup into its own slot (hand-off bytes)
template <int LOADS>
__global__ __launch_bounds__(256) void ffn_like(const char* base, size_t region, int nreg, size_t per_wg, int batches,
                                                unsigned long long* acc, float* slots, int mode, int iter0, int n_out) {
    const char* src = base + (size_t)(iter0 % nreg) * region + (size_t)blockIdx.x * per_wg;
    const int t = threadIdx.x;
    float s = 0.f;
    for (int b = 0; b < batches; ++b) {
        u32x4 v[LOADS];
#pragma unroll
        for (int i = 0; i < LOADS; ++i)
            v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + ((size_t)b * LOADS + i) * 4096 + t * 16));
#pragma unroll
        for (int i = 0; i < LOADS; ++i) s += __uint_as_float(v[i].x ^ v[i].y ^ v[i].z ^ v[i].w);
    }
    if (mode == 1) {
        // thread t owns outputs j = t + 256 * i: a wave's 64 lanes hit 64 consecutive int64
        for (int i = 0; i < n_out / 256; ++i)
            atomicAdd(acc + t + 256 * i, (unsigned long long)(long long)(s * (float)(i + 1)));
    } else if (mode == 2) {
        for (int i = 0; i < n_out / 256; ++i) slots[(size_t)blockIdx.x * n_out + t + 256 * i] = s * (float)(i + 1);
    } else if (s == 1234.5f) {
        acc[t] = 1;
    }
}

template <int LOADS>
float run(const char* buf, size_t total, int grid, int nreg, unsigned long long* acc, float* slots, int mode, int iters,
          int n_out) {
    const size_t per_wg = total / grid;
    const int batches = (int)(per_wg / ((size_t)LOADS * 4096));
    const size_t region = (total + (1 << 21)) & ~((size_t)(1 << 21) - 1);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL((ffn_like<LOADS>), dim3(grid), dim3(256), 0, 0, buf, region, nreg, per_wg, batches, acc, slots, mode, i, n_out);
    hipEventRecord(e0);
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL((ffn_like<LOADS>), dim3(grid), dim3(256), 0, 0, buf, region, nreg, per_wg, batches, acc, slots, mode, i, n_out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1000.f / iters;
}

int main() {
    const size_t cap = (size_t)2 << 30;
    char* buf;
    unsigned long long* acc;
    float* slots;
    if (hipMalloc(&buf, cap) != hipSuccess || hipMalloc(&acc, 1 << 20) != hipSuccess ||
        hipMalloc(&slots, (size_t)2048 * 4096 * 4) != hipSuccess)
        return 1;
    hipMemset(buf, 1, cap);
    hipMemset(acc, 0, 1 << 20);
    hipDeviceSynchronize();
    const int grids[] = {256, 512, 768, 1024, 2048};
    // atomics alone: a tiny stream (one batch per workgroup)
    for (int g : grids) {
        const size_t tot = (size_t)g * 8 * 4096;
        printf("{\"probe\": \"atomics_only\", \"grid\": %d, \"n_out\": 4096, \"stream_us\": %.2f, \"atomic_us\": %.2f, \"store_us\": %.2f}\n", g,
               run<8>(buf, tot, g, 8, acc, slots, 0, 50, 4096), run<8>(buf, tot, g, 8, acc, slots, 1, 50, 4096),
               run<8>(buf, tot, g, 8, acc, slots, 2, 50, 4096));
    }
    // the fused FFN's weight bytes (gate_up 180 MB + down 90 MB) with the atomics at the tail
    const size_t ffn = (size_t)270 << 20;
    for (int g : grids) {
        const size_t tot = ffn / ((size_t)g * 8 * 4096) * ((size_t)g * 8 * 4096);
        const float t0 = run<8>(buf, tot, g, 6, acc, slots, 0, 30, 4096);
        const float t1 = run<8>(buf, tot, g, 6, acc, slots, 1, 30, 4096);
        const float t2 = run<8>(buf, tot, g, 6, acc, slots, 2, 30, 4096);
        printf("{\"probe\": \"ffn_stream\", \"grid\": %d, \"bytes\": %zu, \"stream_us\": %.2f, \"stream_TBps\": %.3f, "
               "\"with_atomics_us\": %.2f, \"with_slot_stores_us\": %.2f}\n",
               g, tot, t0, tot / t0 / 1e6, t1, t2);
    }
    return 0;
}
