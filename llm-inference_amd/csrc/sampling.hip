// Stochastic top-K sampling: the reference's
// launchTopKforBeamSearch (src/kernels/topK.cu:24-191, topK.h:6-56) followed by
// launchSampling (src/kernels/sampling.cu:28-115), as Llama<T>::Sampling wires them
// (src/models/llama/llama.cpp:245-262). The engine's greedy path keeps its fused
// argmax epilogue (K = 1 reduces to it); these launches serve callers that sample.
//
// topk: one workgroup of 1024 lanes per row. Every lane keeps a sorted K-list of the
// values it strides over (coalesced, one HBM pass over the row), then K rounds of a
// workgroup argmax over the lanes' heads pop the row's top K in order. Order is
// value-descending with ties to the lower index -- the reference's heap is the same
// sort but its tie order depends on the CUB reduction tree, so equal logits are the
// one place the build is deterministic where the reference is not. Roofline: HBM,
// rows * vocab * sizeof(T) bytes read; at batch 1 the row is 128 KB and the launch is
// latency-bound (a few us), far below the 13 GB the token's GEMVs stream.
//
// sampling: one lane per row (K is small, the reference runs the whole loop on
// tid 0 too). Semantics follow SamplingKernel (sampling.cu:28-84) exactly:
// exp(v - v[0]) in place (stored as T), threshold = u * sum, first i whose running
// subtraction reaches <= 0, ids taken % vocab, seqlen / is_finished update, rows already
// finished untouched. u is the reference's own draw, curand_uniform of
// curand_init(step, row, 0) -- cuRAND's XORWOW restated in xorwow.h (row > 0 jumps the
// state by row * 2^67 steps through a GF(2) matrix table built here on the host); the
// oracle (oracle/sampling.py over oracle/xorwow.py) makes the same draw, so the
// selection is bit-exact against it.
#include <array>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "kernels.h"
#include "xorwow.h"

namespace llmi {
namespace {

constexpr int kTopkThreads = 1024;

template <typename T> __device__ __forceinline__ float ldv(const T* p) { return (float)*p; }
template <> __device__ __forceinline__ float ldv<__half>(const __half* p) { return __half2float(*p); }
template <typename T> __device__ __forceinline__ void stv(T* p, float v) { *p = v; }
template <> __device__ __forceinline__ void stv<__half>(__half* p, float v) { *p = __float2half(v); }

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off, kWave);
        v = o > v ? o : v;
    }
    return v;
}

template <typename T, int K>
__global__ __launch_bounds__(kTopkThreads) void topk_kernel(const T* __restrict__ logits, int vocab,
                                                            int32_t* __restrict__ out_ids, T* __restrict__ out_vals) {
    const T* row = logits + (size_t)blockIdx.x * vocab;
    // lane-local sorted list, descending by argmax key; key 0 = empty slot
    unsigned long long key[K];
#pragma unroll
    for (int j = 0; j < K; ++j) key[j] = 0ull;
    for (int i = threadIdx.x; i < vocab; i += kTopkThreads) {
        unsigned long long c = argmax_key(ldv(row + i), (uint32_t)i);
        if (c > key[K - 1]) {
            key[K - 1] = c;
#pragma unroll
            for (int j = K - 2; j >= 0; --j) {
                if (key[j + 1] > key[j]) {
                    const unsigned long long t = key[j];
                    key[j] = key[j + 1];
                    key[j + 1] = t;
                }
            }
        }
    }
    __shared__ unsigned long long wbest[kTopkThreads / kWave];
    const int lane = threadIdx.x % kWave, wid = threadIdx.x / kWave;
    for (int r = 0; r < K; ++r) {
        unsigned long long b = wave_max_u64(key[0]);
        if (lane == 0) wbest[wid] = b;
        __syncthreads();
        b = lane < kTopkThreads / kWave ? wbest[lane] : 0ull;
        b = wave_max_u64(b);
        if (key[0] == b && b != 0ull) {  // keys are unique per index: exactly one lane pops
#pragma unroll
            for (int j = 0; j < K - 1; ++j) key[j] = key[j + 1];
            key[K - 1] = 0ull;
        }
        if (threadIdx.x == 0) {
            const size_t o = (size_t)blockIdx.x * K + r;
            if (b == 0ull) {  // vocab < K: the reference's init() values (topK.h:15-20)
                out_ids[o] = -1;
                stv(out_vals + o, 1e-20f);
            } else {
                const uint32_t idx = argmax_key_index(b);
                out_ids[o] = (int32_t)idx;
                out_vals[o] = row[idx];  // the stored value itself, no float round trip
            }
        }
        __syncthreads();
    }
}

template <typename T>
__global__ void sampling_kernel(const int32_t* __restrict__ topk_ids, T* __restrict__ topk_vals, int rows, int K,
                                int32_t* __restrict__ output_id, int32_t* __restrict__ seqlen,
                                uint8_t* __restrict__ is_finished, int step, int end_id, int vocab,
                                const uint32_t* __restrict__ jumps) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= rows || is_finished[b]) return;
    T* v = topk_vals + (size_t)b * K;
    const int32_t* id = topk_ids + (size_t)b * K;
    const float mx = ldv(v);
    float sum = 0.f;
    for (int i = 0; i < K; ++i) {
        stv(v + i, expf(ldv(v + i) - mx));
        sum += ldv(v + i);
    }
    // curand_init((unsigned long long)step, b, 0); curand_uniform (sampling.cu:66-69)
    XorwowState rs = xorwow_init((uint64_t)(int64_t)step);
    if (b > 0) xorwow_jump(rs, (uint32_t)b, jumps);
    float thr = xorwow_uniform(xorwow_next(rs)) * sum;
    int out = id[0];
    for (int i = 0; i < K; ++i) {
        thr -= ldv(v + i);
        if (thr <= 0.f) {
            out = id[i] % vocab;
            break;
        }
    }
    output_id[b] = out;
    seqlen[b] += 1;
    is_finished[b] = out == end_id ? 1 : 0;
}

__global__ void sample_pick_kernel(const DecodeState* st, const int32_t* __restrict__ ids, float* __restrict__ v,
                                   int K, uint64_t seed, unsigned long long* __restrict__ partials, int np) {
    if (threadIdx.x == 0) {
        const float mx = v[0];
        float sum = 0.f;
        for (int i = 0; i < K; ++i) {
            v[i] = expf(v[i] - mx);
            sum += v[i];
        }
        // the reference's step = tokens so far (llama.cpp:405-423) = cur_pos + 1, offset by
        // the caller's seed (0: the reference's stream); batch row 0: no subsequence jump
        const uint64_t step = seed + (uint64_t)(st->cur_pos + 1);
        XorwowState rs = xorwow_init(step);
        float thr = xorwow_uniform(xorwow_next(rs)) * sum;
        int out = ids[0];
        for (int i = 0; i < K; ++i) {
            thr -= v[i];
            if (thr <= 0.f) {
                out = ids[i] % st->vocab;
                break;
            }
        }
        partials[0] = argmax_key(1.0f, (uint32_t)out);
    }
    for (int i = 1 + threadIdx.x; i < np; i += blockDim.x) partials[i] = 0ull;
}

template <typename T>
int topk_dispatch(const void* logits, int rows, int vocab, int k, int32_t* ids, void* vals, hipStream_t s) {
    const T* x = static_cast<const T*>(logits);
    T* y = static_cast<T*>(vals);
    switch (k) {
#define LLMI_TOPK_CASE(KK) \
    case KK: hipLaunchKernelGGL((topk_kernel<T, KK>), dim3(rows), dim3(kTopkThreads), 0, s, x, vocab, ids, y); break;
        LLMI_TOPK_CASE(1) LLMI_TOPK_CASE(2) LLMI_TOPK_CASE(3) LLMI_TOPK_CASE(4) LLMI_TOPK_CASE(5)
        LLMI_TOPK_CASE(6) LLMI_TOPK_CASE(7) LLMI_TOPK_CASE(8) LLMI_TOPK_CASE(9) LLMI_TOPK_CASE(10)
        LLMI_TOPK_CASE(11) LLMI_TOPK_CASE(12) LLMI_TOPK_CASE(13) LLMI_TOPK_CASE(14) LLMI_TOPK_CASE(15)
        LLMI_TOPK_CASE(16)
#undef LLMI_TOPK_CASE
        default: return LLMI_EINVAL;
    }
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

// columns of M^(2^67 * 2^i), i < kXorwowJumpBits, M the one-step map of the 160-bit v
std::vector<uint32_t> build_jump_table() {
    typedef std::array<uint32_t, 5> V;
    std::vector<V> cols(160), next(160);
    for (int c = 0; c < 160; ++c) {
        XorwowState s{};
        s.v[c >> 5] = 1u << (c & 31);
        (void)xorwow_next(s);
        for (int w = 0; w < 5; ++w) cols[c][w] = s.v[w];
    }
    auto square = [&]() {
        for (int c = 0; c < 160; ++c) {
            V r{};
            for (int j = 0; j < 160; ++j)
                if ((cols[c][j >> 5] >> (j & 31)) & 1u)
                    for (int w = 0; w < 5; ++w) r[w] ^= cols[j][w];
            next[c] = r;
        }
        cols.swap(next);
    };
    for (int i = 0; i < 67; ++i) square();
    std::vector<uint32_t> t((size_t)kXorwowJumpBits * 160 * 5);
    for (int i = 0; i < kXorwowJumpBits; ++i) {
        for (int c = 0; c < 160; ++c)
            for (int w = 0; w < 5; ++w) t[((size_t)i * 160 + c) * 5 + w] = cols[c][w];
        if (i + 1 < kXorwowJumpBits) square();
    }
    return t;
}

}  // namespace

const std::vector<uint32_t>& xorwow_host_table() {
    static const std::vector<uint32_t> host = build_jump_table();  // thread-safe static init
    return host;
}

const uint32_t* xorwow_jump_table() {
    static std::mutex mu;
    static std::unordered_map<int, uint32_t*> per_device;
    std::lock_guard<std::mutex> lock(mu);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    auto it = per_device.find(dev);
    if (it != per_device.end()) return it->second;
    const std::vector<uint32_t>& host = xorwow_host_table();
    uint32_t* d = nullptr;
    if (hipMalloc(&d, host.size() * 4) != hipSuccess) return nullptr;
    if (hipMemcpy(d, host.data(), host.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(d);
        return nullptr;
    }
    per_device[dev] = d;
    return d;
}

int sample_pick_launch(const DecodeState* st, const int32_t* ids, float* vals, int k, uint64_t seed,
                       unsigned long long* partials, int np, hipStream_t s) {
    LLMI_REQUIRE(st && ids && vals && partials && k >= 1 && k <= 16 && np >= 1, "sample_pick: bad arguments");
    hipLaunchKernelGGL(sample_pick_kernel, dim3(1), dim3(256), 0, s, st, ids, vals, k, seed, partials, np);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

int topk_launch(const void* logits, int dtype, int rows, int vocab, int k, int32_t* ids, void* vals, hipStream_t s) {
    LLMI_REQUIRE(logits && ids && vals && rows > 0 && vocab > 0, "topk: bad arguments");
    LLMI_REQUIRE(k >= 1 && k <= 16, "topk: k must be in [1, 16]");
    LLMI_REQUIRE(dtype == LLMI_F32 || dtype == LLMI_F16, "topk: dtype must be f32 or f16");
    return dtype == LLMI_F32 ? topk_dispatch<float>(logits, rows, vocab, k, ids, vals, s)
                           : topk_dispatch<__half>(logits, rows, vocab, k, ids, vals, s);
}

int sampling_launch(const int32_t* topk_ids, void* topk_vals, int dtype, int rows, int k, int32_t* output_id,
                    int32_t* seqlen, uint8_t* is_finished, int step, int end_id, int vocab, hipStream_t s) {
    LLMI_REQUIRE(topk_ids && topk_vals && output_id && seqlen && is_finished && rows > 0 && k >= 1 && vocab > 0,
                 "sampling: bad arguments");
    LLMI_REQUIRE(dtype == LLMI_F32 || dtype == LLMI_F16, "sampling: dtype must be f32 or f16");
    LLMI_REQUIRE(rows <= (1 << kXorwowJumpBits), "sampling: at most 65536 rows (curand subsequence jumps)");
    const uint32_t* jumps = nullptr;  // rows > 1 jump their curand state by row * 2^67
    if (rows > 1) {
        jumps = xorwow_jump_table();
        LLMI_REQUIRE(jumps != nullptr, "sampling: cannot place the XORWOW jump table on the device");
    }
    const int grid = (rows + kWave - 1) / kWave;
    if (dtype == LLMI_F32)
        hipLaunchKernelGGL(sampling_kernel<float>, dim3(grid), dim3(kWave), 0, s, topk_ids,
                           static_cast<float*>(topk_vals), rows, k, output_id, seqlen, is_finished, step, end_id,
                           vocab, jumps);
    else
        hipLaunchKernelGGL(sampling_kernel<__half>, dim3(grid), dim3(kWave), 0, s, topk_ids,
                           static_cast<__half*>(topk_vals), rows, k, output_id, seqlen, is_finished, step, end_id,
                           vocab, jumps);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

}  // namespace llmi

// host-side restatement check (no device work): the first curand_uniform of
// curand_init(seed, subsequence, 0), from the same xorwow.h code and jump table the
// sampling kernel uses
extern "C" int llmi_curand_uniform(uint64_t seed, uint32_t subsequence, float* out) {
    using namespace llmi;
    LLMI_REQUIRE(out, "curand_uniform: null output");
    LLMI_REQUIRE(subsequence < (1u << kXorwowJumpBits), "curand_uniform: subsequence must be < 65536");
    XorwowState s = xorwow_init(seed);
    if (subsequence) xorwow_jump(s, subsequence, xorwow_host_table().data());
    *out = xorwow_uniform(xorwow_next(s));
    return LLMI_OK;
}
