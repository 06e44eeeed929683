// Caching device allocator with the reference's pool policy: CudaAllocator
// (src/memory/allocator/cuda_allocator.h) behind BaseAllocator (base_allocator.h:7-31).
//   * host requests: zeroed malloc.
//   * big blocks (> 1 MiB): best fit among free blocks whose slack is < 1 MiB; otherwise a new
//     zeroed block of size rounded up to 32 B; if that fails, release the free big blocks and
//     retry once (TryReleaseBigBlocksAndRetry).
//   * small blocks: best fit among free blocks, otherwise a new zeroed 32-B-rounded block.
//   * free: the block is marked free; once more than 1 GiB of small blocks sit free they are
//     returned to the device; pointers the pools do not own are freed directly.
// One pool per allocator instance (create one per device; the engine itself allocates every
// buffer once and needs no pool). Thread-safe (recursive mutex, as the reference).
// The raw backend is pluggable so the policy is testable without a GPU; the default backend
// is the C ABI (llmi_device_alloc / llmi_device_free / llmi_device_memset).
#pragma once
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "layers.h"

struct RawDeviceBackend {
    // return nullptr on failure (no throw), like cudaMalloc's error path
    void* (*alloc)(size_t bytes) = [](size_t bytes) -> void* {
        void* p = nullptr;
        return llmi_device_alloc(&p, bytes) == LLMI_OK ? p : nullptr;
    };
    void (*release)(void* p) = [](void* p) { (void)llmi_device_free(p); };
    void (*zero)(void* p, size_t bytes) = [](void* p, size_t bytes) { LLMI_CALL(llmi_device_memset(p, 0, bytes)); };
};

class HipCachingAllocator : public BaseAllocator {
public:
    static constexpr size_t kBig = 1u << 20;          // cuda_allocator.h: size > 1024*1024
    static constexpr size_t kSmallRelease = 1u << 30;  // free small bytes before release

    struct Block {
        void* data;
        size_t size;
        bool is_allocated;
    };

    explicit HipCachingAllocator(RawDeviceBackend be = RawDeviceBackend()) : be_(be) {}
    ~HipCachingAllocator() override {
        std::lock_guard<std::recursive_mutex> lock(mu_);
        for (auto& b : small_) be_.release(b.data);
        for (auto& b : big_) be_.release(b.data);
    }

    void* UnifyMalloc(void* ptr, size_t size, bool is_host = false) override {
        (void)ptr;
        if (is_host) return std::calloc(1, size ? size : 1);
        std::lock_guard<std::recursive_mutex> lock(mu_);
        const size_t s32 = (size + 31) / 32 * 32;
        if (size > kBig) {
            Block* best = nullptr;
            for (auto& b : big_)
                if (!b.is_allocated && b.size >= size && b.size - size < kBig && (!best || b.size < best->size))
                    best = &b;
            if (best) {
                best->is_allocated = true;
                return best->data;
            }
            void* p = be_.alloc(s32);
            if (!p) {  // TryReleaseBigBlocksAndRetry
                std::vector<Block> keep;
                for (auto& b : big_) {
                    if (b.is_allocated) {
                        keep.push_back(b);
                    } else {
                        be_.release(b.data);
                        total_ -= b.size;
                    }
                }
                big_.swap(keep);
                p = be_.alloc(s32);
                LLM_CHECK_WITH_INFO(p != nullptr, "HipCachingAllocator: big allocation failed after releasing free blocks");
            }
            be_.zero(p, s32);
            total_ += s32;
            big_.push_back({p, s32, true});
            return p;
        }
        Block* best = nullptr;
        for (auto& b : small_)
            if (!b.is_allocated && b.size >= size && (!best || b.size < best->size)) best = &b;
        if (best) {
            best->is_allocated = true;
            free_small_ = free_small_ > best->size ? free_small_ - best->size : 0;
            return best->data;
        }
        void* p = be_.alloc(s32);
        LLM_CHECK_WITH_INFO(p != nullptr, "HipCachingAllocator: small allocation failed");
        be_.zero(p, s32);
        total_ += s32;
        small_.push_back({p, s32, true});
        return p;
    }

    void UnifyFree(void* ptr, bool is_host) override {
        if (!ptr) return;
        if (is_host) {
            std::free(ptr);
            return;
        }
        std::lock_guard<std::recursive_mutex> lock(mu_);
        if (free_small_ > kSmallRelease) {  // return idle small blocks to the device
            std::vector<Block> keep;
            for (auto& b : small_) {
                if (b.is_allocated) keep.push_back(b);
                else {
                    be_.release(b.data);
                    total_ -= b.size;
                }
            }
            small_.swap(keep);
            free_small_ = 0;
        }
        for (auto& b : small_)
            if (b.data == ptr) {
                b.is_allocated = false;
                free_small_ += b.size;
                return;
            }
        for (auto& b : big_)
            if (b.data == ptr) {
                b.is_allocated = false;
                return;
            }
        be_.release(ptr);
    }

    // introspection for tests and diagnostics
    size_t total_allocated() const { return total_; }
    size_t free_small_bytes() const { return free_small_; }
    size_t small_blocks() const { return small_.size(); }
    size_t big_blocks() const { return big_.size(); }

private:
    RawDeviceBackend be_;
    std::recursive_mutex mu_;
    std::vector<Block> small_, big_;
    size_t free_small_ = 0, total_ = 0;
};
