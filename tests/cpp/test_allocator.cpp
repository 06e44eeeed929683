// Pool policy of HipCachingAllocator (include/llmi/allocator.h) = the reference's
// CudaAllocator (cuda_allocator.h), checked with a fake raw backend (distinct fake
// addresses, no memory touched) so it runs without a GPU. Prints "allocator ok".
#include <cassert>
#include <cstdint>
#include <cstdio>
#include <map>
#include <set>

#include "llmi/allocator.h"

static int g_allocs = 0, g_releases = 0, g_zeroed = 0;
static size_t g_budget = SIZE_MAX, g_live = 0;
static uintptr_t g_next = 0x100000;
static std::set<void*> g_released;
static std::map<void*, size_t> g_size;

static void* fake_alloc(size_t n) {
    if (g_live + n > g_budget) return nullptr;
    ++g_allocs;
    g_live += n;
    void* p = reinterpret_cast<void*>(g_next);
    g_size[p] = n;
    g_next += (n + 4095) / 4096 * 4096 + 4096;
    return p;
}
static void fake_release(void* p) {
    ++g_releases;
    g_released.insert(p);
    if (g_size.count(p)) g_live -= g_size[p];
}
static void fake_zero(void*, size_t) { ++g_zeroed; }

#define CHECK_(c)                                                  \
    do {                                                           \
        if (!(c)) {                                                \
            std::printf("FAILED line %d: %s\n", __LINE__, #c);     \
            return 1;                                              \
        }                                                          \
    } while (0)

int main() {
    RawDeviceBackend be;
    be.alloc = fake_alloc;
    be.release = fake_release;
    be.zero = fake_zero;
    {
        HipCachingAllocator a(be);
        // small: 32-B rounding, best-fit reuse, zeroed on first allocation only
        void* s1 = a.UnifyMalloc(nullptr, 100);
        CHECK_(a.total_allocated() == 128 && g_zeroed == 1);
        a.UnifyFree(s1, false);
        CHECK_(a.free_small_bytes() == 128);
        void* s2 = a.UnifyMalloc(nullptr, 64);
        CHECK_(s2 == s1 && g_allocs == 1 && g_zeroed == 1 && a.free_small_bytes() == 0);
        void* s3 = a.UnifyMalloc(nullptr, 64);  // s1 busy -> a new block
        CHECK_(s3 != s1 && g_allocs == 2);
        a.UnifyFree(s3, false);
        a.UnifyFree(s2, false);
        void* s4 = a.UnifyMalloc(nullptr, 60);  // best fit: the 64-B block, not the 128-B one
        CHECK_(s4 == s3);
        // big: reuse only when the slack is < 1 MiB
        void* b1 = a.UnifyMalloc(nullptr, 3u << 20);
        a.UnifyFree(b1, false);
        void* b2 = a.UnifyMalloc(nullptr, (5u << 20) / 2);  // 2.5 MiB: slack 0.5 MiB -> reuse
        CHECK_(b2 == b1);
        a.UnifyFree(b2, false);
        const int before = g_allocs;
        void* b3 = a.UnifyMalloc(nullptr, (3u << 20) / 2);  // 1.5 MiB: slack 1.5 MiB -> new block
        CHECK_(b3 != b1 && g_allocs == before + 1 && a.big_blocks() == 2);
        // allocation failure: free big blocks are released and the request retried
        g_budget = g_live + (2u << 20);
        void* b4 = a.UnifyMalloc(nullptr, 4u << 20);
        CHECK_(b4 != nullptr && g_released.count(b1) == 1 && a.big_blocks() == 2);
        g_budget = SIZE_MAX;
        // pointers the pools do not own are released directly
        void* foreign = reinterpret_cast<void*>(0xdead000);
        a.UnifyFree(foreign, false);
        CHECK_(g_released.count(foreign) == 1);
        // host requests are zeroed host memory
        int* h = static_cast<int*>(a.UnifyMalloc(nullptr, 64, true));
        CHECK_(h && h[0] == 0 && h[15] == 0);
        a.UnifyFree(h, true);
        // > 1 GiB of idle small blocks are returned at the next free
        std::vector<void*> many;
        for (int i = 0; i < 1024; ++i) many.push_back(a.UnifyMalloc(nullptr, 1u << 20));
        for (void* p : many) a.UnifyFree(p, false);
        CHECK_(a.free_small_bytes() > (1u << 30));
        const size_t nsmall = a.small_blocks();
        a.UnifyFree(s4, false);  // triggers the release of every idle small block
        CHECK_(a.small_blocks() == 1 && nsmall > 1000 && a.free_small_bytes() == 64);
        (void)b3;
        (void)b4;
    }
    CHECK_(g_releases > 1024);  // the destructor returns what is left
    std::printf("allocator ok\n");
    return 0;
}
