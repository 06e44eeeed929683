// HipCachingAllocator on the device (default C-ABI backend): new blocks read back as
// zeros, a freed block is handed out again, big/small pools both work. Prints "ok".
#include <cstdio>
#include <vector>

#include "llmi/allocator.h"

int main() {
    HipCachingAllocator a;
    float* s = a.Malloc(static_cast<float*>(nullptr), 1000 * sizeof(float), false);
    float* b = a.Malloc(static_cast<float*>(nullptr), (3u << 20), false);
    std::vector<float> h(1000, 1.f), big((3u << 20) / 4, 1.f);
    LLMI_CALL(llmi_memcpy(h.data(), s, h.size() * 4, 1));
    LLMI_CALL(llmi_memcpy(big.data(), b, big.size() * 4, 1));
    for (float v : h) if (v != 0.f) { std::printf("small block not zeroed\n"); return 1; }
    for (float v : big) if (v != 0.f) { std::printf("big block not zeroed\n"); return 1; }
    a.Free(s, false);
    a.Free(b, false);
    float* s2 = a.Malloc(static_cast<float*>(nullptr), 900 * sizeof(float), false);
    float* b2 = a.Malloc(static_cast<float*>(nullptr), (5u << 20) / 2, false);
    if (s2 != s || b2 != b) { std::printf("blocks not reused\n"); return 1; }
    a.Free(s2, false);
    a.Free(b2, false);
    std::printf("ok total=%zu\n", a.total_allocated());
    return 0;
}
