// One-shot peer-write exchange for tensor-parallel decode (config 4).
//
// What it replaces: the RCCL all-reduces of the decode step -- the int64 fixed-point
// residual after o_proj and after down (2 per layer) and the uint64 max of the
// vocab-parallel argmax keys (1 per token): the sum of the row-parallel partials of
// modeling_llama.py's `pretraining_tp` (modeling_llama.py:251-266, 443-446). Each is a
// 32 KB message, far too small to be bandwidth-bound on xGMI: RCCL's ring/tree steps
// make it latency-bound (2 L + 1 = 65 of them per 7B token).
//
// One launch per exchange instead, no collective library:
//   * every rank owns an INBOX in its own HBM (uncached, hipDeviceMallocUncached, so a
//     peer's write over xGMI is what a later load returns): data [2 phases][world][cap_n]
//     int64 and flags [2 phases][world][kXchgMaxSlices] uint64; every rank holds the
//     IPC-mapped inbox base of every peer (peers[q]);
//   * workgroup g owns slice g (kXchgSlice elements) of the vector: it writes its
//     rank's slice into slot [phase][rank] of EVERY rank's inbox (its own too), then
//     -- after a system-scope release -- stores the exchange's epoch into flag
//     [phase][rank][g] of every inbox;
//   * then it waits until flag [phase][q][g] of its own inbox holds the epoch for every
//     rank q, and reduces the W slots in rank order (int64 sum: exact, so the result
//     is bitwise the RCCL one and independent of arrival order; uint64 max) into buf.
// Epochs: a per-slice counter in the rank's own memory (e = count + 1); phase = e & 1.
// A rank can run at most one exchange ahead of the slowest peer (its next push needs
// every peer's flag of the current one), so two phases never alias.
// Liveness: every wait is bounded (kXchgTimeoutTicks of the 100 MHz clock); a timeout
// sets bit 8 of the decode state's error word -- tokens_out raises -- and later waits
// of the run are skipped, so a lost peer ends the run with an error instead of a hang.
#include "xchg_impl.h"

namespace llmi {
namespace {

constexpr int kXThreads = kXchgSlice / 2;          // two 8-B elements (one 16-B access) per thread

__global__ __launch_bounds__(kXThreads) void xchg_kernel(XchgArgs a) {
    const int g = blockIdx.x;
    const unsigned long long e = a.ep[g] + 1;
    if (a.mode & 1) xchg_detail::push_slice<false>(a, g, e);  // this rank's slice into every inbox
    if (a.mode & 2) xchg_detail::reduce_slice(a, g, e);       // every rank's slice, summed in rank order
}

}  // namespace

size_t xchg_inbox_bytes(int world, int cap_n) {
    return (size_t)2 * world * cap_n * 8 + (size_t)2 * world * kXchgMaxSlices * 8;
}

int xchg_launch(const XchgArgs& a, hipStream_t s) {
    LLMI_REQUIRE(a.buf && a.peers && a.ep && a.err, "xchg: null pointer");
    LLMI_REQUIRE(a.world >= 1 && a.world <= a.cap_w && a.world <= kXchgMaxWorld && a.rank >= 0 && a.rank < a.world,
                 "xchg: bad rank/world (at most 8 ranks)");
    LLMI_REQUIRE(a.n >= 0 && a.n <= a.cap_n && a.n <= kXchgSlice * kXchgMaxSlices, "xchg: n exceeds the inbox");
    LLMI_REQUIRE(a.cap_n % 2 == 0, "xchg: inbox slots must hold an even element count (16-B accesses)");
    LLMI_REQUIRE(a.op == 0 || a.op == 2, "xchg: op must be 0 (int64 sum) or 2 (uint64 max)");
    LLMI_REQUIRE(a.mode >= 1 && a.mode <= 3, "xchg: mode must be 1 (push), 2 (reduce) or 3 (both)");
    if (a.n == 0) return LLMI_OK;
    const int grid = (a.n + kXchgSlice - 1) / kXchgSlice;
    hipLaunchKernelGGL(xchg_kernel, dim3(grid), dim3(kXThreads), 0, s, a);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

}  // namespace llmi
