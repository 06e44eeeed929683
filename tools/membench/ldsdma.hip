// LDS-DMA streaming microbenchmark (the ring layer's loader in isolation): one
// 256-thread workgroup per CU, LW loader waves stream a contiguous per-CU region
// into an LDS ring of NS slots of SB bytes with global_load_lds_dwordx4 (nt or
// default policy), keeping D slots in flight per wave (counted vmcnt); no consumer.
// Reports chip-wide GB/s. Launches cycle through a 2 GiB buffer (HBM, not MALL).
#include <hip/hip_runtime.h>
#include <cstdio>

template <bool NT>
__device__ __forceinline__ void glds16(const void* g, unsigned lds) {
    unsigned keep;
    if (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}

template <int SB, int D, int LW, bool NT, int PAIRS = 0>
__global__ __launch_bounds__(256, 1) void stream(const char* base, size_t region, int nreg, size_t per_cu, int iter) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave >= LW) return;
    constexpr int NI = SB / 1024;      // DMA instructions per slot
    constexpr int NS = 96 * 1024 / SB; // ring slots (96 KB)
    const char* src = base + (size_t)(iter % nreg) * region + (size_t)blockIdx.x * per_cu;
    const int nslots = (int)(per_cu / SB);
    const unsigned ring = (unsigned)(uintptr_t)smem;
    for (int s = wave; s < nslots; s += LW) {
        const unsigned dst = __builtin_amdgcn_readfirstlane(ring + ((s / LW) % (NS / LW) * LW + wave) * SB);
        // PAIRS: even slots stream region A, odd slots region B = A + 96 MB (gate / up rows)
        const char* ps = PAIRS ? src + (size_t)(s >> 1) * SB + (size_t)(s & 1) * ((size_t)96 << 20) : src + (size_t)s * SB;
#pragma unroll
        for (int j = 0; j < NI; ++j) glds16<NT>(ps + j * 1024 + lane * 16, dst + j * 1024);
        if (s / LW >= D - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(NI * (D - 1)) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int SB, int D, int LW, bool NT, int PAIRS = 0>
void run(const char* buf, size_t cap, int cus) {
    const size_t total = (size_t)300 << 20;
    const size_t per_cu = (total / cus) / SB * SB;
    const size_t region = ((per_cu * cus) + (1 << 21)) & ~((size_t)(1 << 21) - 1);
    const int nreg = (int)(cap / region);
    auto k = stream<SB, D, LW, NT, PAIRS>;
    hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 2; ++i) hipLaunchKernelGGL(k, dim3(cus), dim3(256), 96 * 1024, 0, buf, region, nreg, per_cu, i);
    hipEventRecord(e0);
    const int it = 20;
    for (int i = 0; i < it; ++i) hipLaunchKernelGGL(k, dim3(cus), dim3(256), 96 * 1024, 0, buf, region, nreg, per_cu, i);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1000.0 / it;
    printf("{\"slot_KB\": %d, \"depth\": %d, \"loader_waves\": %d, \"nt\": %d, \"pairs\": %d, \"MB\": %.1f, \"us\": %.2f, \"GBps\": %.0f}\n", SB / 1024, D,
           LW, NT ? 1 : 0, PAIRS, per_cu * cus / 1e6, us, per_cu * cus / us / 1e3);
}

int main() {
    const size_t cap = (size_t)2 << 30;
    char* buf;
    if (hipMalloc(&buf, cap) != hipSuccess) return 1;
    hipMemset(buf, 1, cap);
    hipDeviceSynchronize();
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    run<8192, 7, 1, true>(buf, cap, cus);
    run<8192, 7, 1, true, 1>(buf, cap, cus);
    run<8192, 4, 1, true, 1>(buf, cap, cus);
    run<8192, 5, 2, true, 1>(buf, cap, cus);
    run<8192, 7, 1, false>(buf, cap, cus);
    run<8192, 4, 1, true>(buf, cap, cus);
    run<16384, 3, 1, true>(buf, cap, cus);
    run<8192, 5, 2, true>(buf, cap, cus);
    run<8192, 6, 2, true>(buf, cap, cus);
    run<8192, 3, 4, true>(buf, cap, cus);
    run<4096, 6, 4, true>(buf, cap, cus);
    run<8192, 7, 1, true>(buf, cap, cus);
    return 0;
}
