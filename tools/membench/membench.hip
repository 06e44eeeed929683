// Read-bandwidth microbenchmark for the shapes of the decode kernels: how long
// does a launch take to read B bytes when G workgroups each read a contiguous
// B/G slab in `batches` sequential rounds of `loads` 16-B loads per lane?
// Launches cycle through regions of a 2 GiB buffer (> the 256 MiB Infinity
// Cache) so every launch streams from HBM. HIP-event timed, back to back.
//   build: hipcc -O3 --offload-arch=gfx950 membench.hip -o membench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int LOADS, bool NT>
__global__ __launch_bounds__(256) void rd(const char* base, size_t region, int nreg, size_t per_wg, int batches,
                                          unsigned* out, int iter0) {
    const char* src = base + (size_t)((iter0 + 0) % nreg) * region + (size_t)blockIdx.x * per_wg;
    unsigned acc = 0;
    const int t = threadIdx.x;
    for (int b = 0; b < batches; ++b) {
        u32x4 v[LOADS];
#pragma unroll
        for (int i = 0; i < LOADS; ++i) {
            const u32x4* p = reinterpret_cast<const u32x4*>(src + ((size_t)b * LOADS + i) * 4096 + t * 16);
            v[i] = NT ? __builtin_nontemporal_load(p) : *p;
        }
#pragma unroll
        for (int i = 0; i < LOADS; ++i) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <int LOADS, bool NT>
float run(const char* buf, size_t total, int grid, int nreg, unsigned* out, int iters) {
    const size_t per_wg = total / grid;
    const int batches = (int)(per_wg / ((size_t)LOADS * 4096));
    if (batches < 1 || per_wg % ((size_t)LOADS * 4096)) return -1.f;
    const size_t region = (total + (1 << 21)) & ~((size_t)(1 << 21) - 1);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((rd<LOADS, NT>), dim3(grid), dim3(256), 0, 0, buf, region, nreg, per_wg, batches, out, i);
    hipEventRecord(e0);
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL((rd<LOADS, NT>), dim3(grid), dim3(256), 0, 0, buf, region, nreg, per_wg, batches, out, i);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1000.f / iters;
}

int main() {
    const size_t cap = (size_t)2 << 30;
    char* buf;
    unsigned* out;
    if (hipMalloc(&buf, cap) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
    hipMemset(buf, 1, cap);
    hipDeviceSynchronize();
    const size_t sizes[] = {(size_t)32 << 20, (size_t)96 << 20, (size_t)172 << 20};
    for (size_t total : sizes) {
        const size_t region = (total + (1 << 21)) & ~((size_t)(1 << 21) - 1);
        const int nreg = (int)(cap / region);
        for (int grid : {256, 512, 1024, 2048, 4096}) {
            float a = run<8, true>(buf, total, grid, nreg, out, 50);
            float b = run<4, true>(buf, total, grid, nreg, out, 50);
            float c = run<8, false>(buf, total, grid, nreg, out, 50);
            float d = run<16, true>(buf, total, grid, nreg, out, 50);
            auto bw = [&](float us) { return us > 0 ? total / us / 1e3 : 0.0; };
            printf("{\"MB\": %zu, \"grid\": %d, \"per_wg_KB\": %zu, \"nt8_us\": %.2f, \"nt8_GBps\": %.0f, \"nt4_us\": %.2f, "
                   "\"nt4_GBps\": %.0f, \"plain8_us\": %.2f, \"plain8_GBps\": %.0f, \"nt16_us\": %.2f, \"nt16_GBps\": %.0f}\n",
                   total >> 20, grid, total / grid / 1024, a, bw(a), b, bw(b), c, bw(c), d, bw(d));
        }
    }
    return 0;
}
