// Probe: does a kernel launched with hipExtAnyOrderLaunch (AQL barrier bit clear)
// start before the previous kernel on the same stream has completed, and what
// gates its start? Every spin is a fixed wall-clock delay (nothing waits on
// another kernel), so a serialising runtime only makes the run slower.
//   hipcc --offload-arch=gfx950 -O2 anyorder.hip -o anyorder && ./anyorder
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

// slot[0] = first start, slot[1] = first end, slot[2] = last end; 100 MHz clock.
// Workgroup b spins base + (b == long_wg ? extra : 0) ticks.
__global__ void spin_kernel(unsigned long long* slot, int base, int long_wg, int extra) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long until = t0 + (unsigned long long)(base + ((int)blockIdx.x == long_wg ? extra : 0));
    while (__builtin_amdgcn_s_memrealtime() < until) __builtin_amdgcn_s_sleep(1);
    if (threadIdx.x == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        atomicMin(slot, t0);
        atomicMin(slot + 1, t1);
        atomicMax(slot + 2, t1);
    }
}

struct K { int grid; int base; int long_wg; int extra; int flags; };

static int run(hipStream_t s, unsigned long long* d, const K* ks, int n, const char* tag) {
    unsigned long long init[12];
    for (int i = 0; i < 4; ++i) { init[3 * i] = ~0ull; init[3 * i + 1] = ~0ull; init[3 * i + 2] = 0ull; }
    CK(hipMemcpy(d, init, sizeof(init), hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    for (int i = 0; i < n; ++i)
        hipExtLaunchKernelGGL(spin_kernel, dim3(ks[i].grid), dim3(256), 0, s, nullptr, nullptr, (unsigned)ks[i].flags,
                              d + 3 * i, ks[i].base, ks[i].long_wg, ks[i].extra);
    CK(hipGetLastError());
    CK(hipStreamSynchronize(s));
    unsigned long long h[12];
    CK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
    printf("{\"case\": \"%s\"", tag);
    for (int i = 0; i < n; ++i)
        printf(", \"k%d\": [%.2f, %.2f, %.2f]", i, ((long long)h[3 * i] - (long long)h[0]) / 100.0,
               ((long long)h[3 * i + 1] - (long long)h[0]) / 100.0, ((long long)h[3 * i + 2] - (long long)h[0]) / 100.0);
    printf("}\n");
    return 0;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned long long* d;
    CK(hipMalloc(&d, 256));
    const int AO = hipExtAnyOrderLaunch;
    for (int rep = 0; rep < 2; ++rep) {
        // [start, first end, last end] per kernel, us from k0's first start
        { K k[2] = {{1, 2000, -1, 0, 0}, {1, 500, -1, 0, AO}}; if (run(s, d, k, 2, "A 1wg 20us | B ao")) return 1; }
        { K k[2] = {{2, 2000, 1, 4000, 0}, {1, 500, -1, 0, AO}}; if (run(s, d, k, 2, "A 2wg 20/60us | B ao")) return 1; }
        { K k[2] = {{256, 4000, -1, 0, 0}, {1, 500, -1, 0, AO}}; if (run(s, d, k, 2, "A 256wg 40us | B ao")) return 1; }
        { K k[2] = {{1024, 6000, 5, -4000, 0}, {64, 500, -1, 0, AO}}; if (run(s, d, k, 2, "A 1024wg 60us (wg5 20us) | B ao")) return 1; }
        { K k[2] = {{1024, 2000, 5, 4000, 0}, {64, 500, -1, 0, AO}}; if (run(s, d, k, 2, "A 1024wg 20us (wg5 60us) | B ao")) return 1; }
        { K k[3] = {{1024, 2000, 5, 4000, 0}, {64, 500, -1, 0, AO}, {64, 500, -1, 0, AO}}; if (run(s, d, k, 3, "A 1024wg 20us (wg5 60us) | B ao | C ao")) return 1; }
        { K k[2] = {{1024, 2000, 5, 4000, 0}, {64, 500, -1, 0, 0}}; if (run(s, d, k, 2, "A 1024wg 20us (wg5 60us) | B barrier")) return 1; }
        { K k[2] = {{1, 2000, -1, 0, AO}, {1, 500, -1, 0, AO}}; if (run(s, d, k, 2, "A ao 1wg 20us | B ao")) return 1; }
    }
    CK(hipFree(d));
    return 0;
}
