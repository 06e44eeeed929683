// Internal kernel launch interface (C++). The public C ABI (include/llmi.h)
// and the decode engine (engine.hip) are both built on these.
#pragma once
#include <cmath>

#include "common.h"

namespace llmi {

// ------------------------------------------------------------------ GEMV
enum GemvEpi : int {
    EPI_STORE = 0,     // y[r] = acc
    EPI_ADD = 1,       // y[r] = acc + resid_scale * resid[r]   (resid may alias y)
    EPI_SILU_MUL = 2,  // rows (g, g + pair_off): y[g] = silu(acc0) * acc1
    EPI_ARGMAX = 3,    // y[r] = acc; per-block argmax key -> partials[blockIdx]
    EPI_ATOMIC = 4,    // yacc[r] += fixed(acc) (int64 2^-32 units; exact, order-independent), split-K
    EPI_SLAB = 5,      // gemm2 split-K: partial [slice][m][ldy] stored; the next rows_split adds the slices in order
};

// one-shot peer exchange of a vector (xchg.hip / xchg_impl.h); also carried by the
// producer kernels (GemvArgs / OprojArgs::xt) for the producer-fused form (buf null = off)
struct XchgArgs {
    long long* buf = nullptr;         // this rank's contribution in, the reduction out (n 8-B elements)
    int n = 0;
    int op = 0;                       // 0: int64 sum, 2: uint64 max
    int rank = 0, world = 1;
    char* const* peers = nullptr;     // device array [world]: every rank's inbox (peers[rank] = own)
    unsigned long long* ep = nullptr; // [kXchgMaxSlices] epoch counters (this rank's memory)
    int* err = nullptr;               // DecodeState::error; bit 8 = a peer never arrived (timeout)
    int mode = 3;                     // 1: push only, 2: wait + reduce only, 3: both
    int cap_n = 0, cap_w = 0;         // inbox geometry: elements per slot, slots per phase
    // loopback (one-GPU pricing of a rank's exchange, llmi_engine_xchg_loopback): every peer is
    // this rank's own inbox; the push fills slot / flag [ph][q] for every q (this rank's vector
    // in its own slot, zeros in the others: the same W x n x 8 bytes of writes as a real push),
    // so the reduce finds all W arrivals and sums to this rank's own partial
    int loop = 0;
};

struct GemvArgs {
    unsigned long long* stamps = nullptr;  // debug timeline (WgStamp), null = off
    const void* w = nullptr;       // [n_rows, k] row-major, dtype w_dtype
    const __half* scales = nullptr;  // int8: per-row fp16 scale
    int w_dtype = LLMI_F16;
    int n_rows = 0;                // rows of W
    int k = 0;
    const float* x = nullptr;      // [k]
    const long long* x_fixed = nullptr;  // alternative x source: int64 fixed point (value * 2^32)
    float* x_out = nullptr;        // with x_fixed: workgroup 0 writes the fp32 x here
    // prologue: optional RMSNorm of x (gamma dtype g_dtype), x_add: x += x_add first
    const void* gamma = nullptr;
    int g_dtype = LLMI_F16;
    float eps = 1e-5f;
    // epilogue
    int epi = EPI_STORE;
    float* y = nullptr;
    const float* resid = nullptr;
    float resid_scale = 1.f;
    int pair_off = 0;              // EPI_SILU_MUL: row offset of the `up` row
    unsigned long long* partials = nullptr;  // EPI_ARGMAX: [grid]
    uint32_t idx_base = 0;         // EPI_ARGMAX: global index of row 0 (vocab shard)
    int grid = 0;                  // 0 = auto
    int ldw = 0;                   // row stride of W in elements (0: k)
    int ksplit = 1;                // EPI_ATOMIC: K split over ksplit workgroups (k % (ksplit * 16 B) == 0)
    long long* yacc = nullptr;     // EPI_ATOMIC target
    // EPI_ATOMIC with ksplit 1 and yacc_single set: every row has ONE producer, so the row is
    // written (write-through) as yacc_base[r] + fixed(acc) (yacc_base null: fixed(acc) alone)
    // instead of an atomic add into a seeded yacc -- the same integer, no seed pass, no atomic
    int yacc_single = 0;
    const long long* yacc_base = nullptr;
    long long* yacc_copy = nullptr;  // yacc_single: the same value also written here (next o_proj's seed)
    // residual hand-over: the workgroups copy seed_src[0..seed_n) (or zeros when !seed_keep)
    // to seed_dst, one slice each (the next fixed-point accumulator's starting value)
    const long long* seed_src = nullptr;
    long long* seed_dst = nullptr;
    int seed_n = 0;
    int seed_keep = 1;
    // producer-fused TP exchange of the vector this launch produces (yacc / partials):
    // xt.buf null = off; xt_cnt = the engine's arrival counter pair (xchg_impl.h xchg_tail)
    XchgArgs xt;
    unsigned* xt_cnt = nullptr;
    // K split INSIDE a workgroup (small shards, e.g. a TP-8 rank's q/k/v and gate_up, whose
    // 192 / 344 four-wave workgroups leave CUs idle or doubled): kpar waves (2 or 4) share one
    // row group, each streaming 1/kpar of K; their partial dots meet in LDS and the first
    // adds them in order. Grid = ceil(groups / (4 / kpar)), every wave exactly one group.
    // EPI_STORE / EPI_SILU_MUL only; 0 / 1 = off.
    int kpar = 0;
    // EPI_STORE inside the fused q/k/v + attention launch (qkv_attn.hip): row r is published as
    // the 8-byte granule {fp32 bits, tag} in y_tag[r] (one write-through store), tag =
    // *tag_epoch * 128 + tag_layer, so the attention workgroups of the same launch can tell a
    // finished row from the previous layer's without any flag or fence
    unsigned long long* y_tag = nullptr;
    const unsigned* tag_epoch = nullptr;
    unsigned tag_layer = 0;
    int tag_heads = 0;  // > 0 (= heads = kv_heads, head_dim 128): rows computed head-major (q, k, v of head 0 first)
};


int gemv_launch(const GemvArgs& a, hipStream_t s);
int gemv_grid(const GemvArgs& a);  // blocks gemv_launch will use

// ------------------------------------------------------ prefill GEMM (MFMA)
// Y[m, n] (op)= sum_k A[m, k] W[n, k] for M prompt rows; see gemm.hip.
struct GemmArgs {
    const float* a = nullptr;      // [m, lda] fp32 activations
    int lda = 0;
    const void* gamma = nullptr;   // non-null: RMSNorm of each A row folded in (gamma dtype g_dtype)
    int g_dtype = LLMI_F16;
    float eps = 1e-5f;
    const void* w = nullptr;       // [n, k] fp16 or int8
    int w_kblock = 0;              // > 0: W stored as [k / w_kblock][n][w_kblock] (head-major W_o)
    const __half* scales = nullptr;  // int8: per-row fp16 scale
    int w_dtype = LLMI_F16;
    int m = 0, n = 0, k = 0;
    int split = 2;                 // 2: fp32-faithful (hi + lo fp16 halves of A); 1: fp16 A
    int epi = EPI_STORE;           // EPI_STORE, EPI_ADD (y += ..), EPI_SILU_MUL (y[m, g] = silu(g) * up)
    int pair_off = 0;              // EPI_SILU_MUL: row offset of `up` in W (= n / 2)
    float* y = nullptr;            // [m, ldy]
    int ldy = 0;
    int n_tiles = 0;               // set by gemm_launch
};
bool gemm_supported(int w_dtype, int n, int k, int epi);
int gemm_bm(const GemmArgs& a);
int gemm_launch(GemmArgs a, hipStream_t s);

// LDS-DMA MFMA GEMM for fp16 weights (gemm2.hip): A arrives as `planes` fp16
// planes (hi[, lo]) written by rows_split_launch or the gate_up epilogue.
struct Gemm2Args {
    const _Float16* a[2] = {nullptr, nullptr};  // [m, lda] planes
    int planes = 2;
    int lda = 0;
    const void* w = nullptr;       // [n, k] fp16 (or head-major blocks, w_kblock)
    int w_kblock = 0;
    int m = 0, n = 0, k = 0;
    int epi = EPI_STORE;           // EPI_STORE, EPI_ADD, EPI_SILU_MUL
    int pair_off = 0;
    float* y = nullptr;            // [m, ldy] fp32
    _Float16* y_hi = nullptr;      // EPI_SILU_MUL: write the result as fp16 planes instead
    _Float16* y_lo = nullptr;
    int ldy = 0;
    int ksplit = 1;                // EPI_SLAB: K slices (K / ksplit a multiple of 64, and of w_kblock)
    float* slab = nullptr;         // EPI_SLAB: [ksplit][m][ldy] partial sums
    int n_tiles = 0;               // set by gemm2_launch
    // gemm3 only, planes = 2: the lo plane a[1] is e4m3 of lo * 2^kLo8Exp (common.h) in
    // the first lda bytes of each 2 lda-byte row, against w8 = e4m3(W * 2^w8_exp) (rows of
    // 2 k bytes, the first k used; w8_prepare) on the block-scaled fp8 MFMA; EPI_SILU_MUL
    // then writes y_lo in the same byte format (K a multiple of 128)
    int lo8 = 0;
    const void* w8 = nullptr;
    int w8_exp = 0;
    // gemm3 EPI_SILU_MUL with lo8 only: spread the fp8 lo pass over the CUs the tiles leave
    // idle (gemm3_silu_bal_kernel): bal_grid workgroups (the CU count), fp32 partial slots
    // [tiles][2][256 x 256] and their flags [tiles][2] (zeroed once; epochs never repeat)
    float* bal_slab = nullptr;
    unsigned* bal_flags = nullptr;
    int bal_grid = 0;
    unsigned bal_epoch = 0;        // set by gemm3_launch
    int bal_own = 0;               // set by gemm3_launch: lo tile pairs each owner keeps
    int* err = nullptr;                    // sticky error word (bit 16: a lo / stream-K partial never arrived)
    unsigned long long* stamps = nullptr;  // debug timeline of the balanced kernel (WgStamp), null = off
    // gemm3 stream-K (EPI_STORE / EPI_SILU_MUL with fewer 256 x 256 tiles than CUs; see
    // gemm3_sk_kernel): sk_grid workgroups (<= the CU count) share the tiles' K work evenly;
    // a tile's later pieces go to fp32 partial slots [tiles][sk_pmax][256 x 256] and raise flags
    // [tiles][sk_pmax] to the launch's epoch (zeroed once, never reset: a piece that publishes
    // after its owner gave up cannot satisfy a later launch's wait). sk_ctl: [0] the epoch of
    // the last completed launch, [32] the launch's finished-workgroup count (the last one
    // advances [0] and re-zeroes [32]), so graph replays get fresh epochs too.
    float* sk_slab = nullptr;
    unsigned* sk_flags = nullptr;
    unsigned* sk_ctl = nullptr;    // = sk_flags - kSkCtlWords (the kernel derives it from sk_flags)
    int sk_grid = 0;
    int sk_pmax = 0;               // set by gemm3_launch; bits 8+: fault injection (llmi_debug_stream_k:
                                   // 1 never publish, 2 publish 2.5 s late)
};
constexpr int kSkCtlWords = 64;    // stream-K control words ahead of the flags (256 B)
// the next `launches` stream-K launches run with sk_test = mode (llmi_debug_stream_k)
void gemm3_sk_debug(int mode, int launches);
void prefill_stamps_debug(unsigned long long* stamps);  // llmi_debug_prefill_stamps
// stream-K plan for gemm3 (m rows, n columns -- gate_up: 2 x inter --, k, planes / lo8 as in
// Gemm2Args) on g workgroups: slots per tile (0: stream-K does not apply), and the bytes of
// partial slots and of flags it needs
struct Gemm3SkPlan {
    int pmax = 0;
    size_t slab_bytes = 0, flag_bytes = 0;
};
Gemm3SkPlan gemm3_sk_plan(int m, int n, int k, int epi, int planes, int lo8, int g);
// attach the stream-K workspace (per device and stream, gemm2.hip) to a gemm3 launch of g's
// shape when the plan keeps <= 3 slots a tile; false: launch as before (LLMI_SK=0: never)
bool gemm3_sk_attach(Gemm2Args& g, hipStream_t s);
// reads and clears the sticky error bits that launches on s (this device) recorded when
// their caller passed no error word (16: a stream-K partial never arrived); syncs s
int stream_errors(hipStream_t s, int* flags);
// bytes of the balanced gate_up's partial slots for m rows, n = 2 x intermediate (0: not used)
size_t gemm3_bal_slab_bytes(int m, int n);
// e4m3(W * 2^exp) of an fp16 [rows, cols] weight (exp chosen so that max |W| * 2^exp <= 448),
// rows of 2 cols bytes with the first cols used (the fp16 row stride, gemm3.hip); synchronises s
int w8_prepare(const void* w16, int rows, int cols, void* w8, int* exp_out, hipStream_t s);
bool gemm2_supported(int n, int k, int epi);
// the context FFN (gate_up + SiLU*up + down) on the matrix cores, fp16 weights (gemm2.hip)
bool ffn_mfma_supported(int m, int hidden, int inter);
// residual epilogue of llmi_linear_residual / llmi_ffn_residual: resid += the projection
// (its K slices summed in slice order first), then out = gamma ? RMSNorm(resid) * gamma
// : resid (out null: the residual update alone); n <= 8192, a multiple of 4
struct ResidEpi {
    float* resid = nullptr;
    float* out = nullptr;
    const void* gamma = nullptr;
    int g_dtype = 0;
    float eps = 0.f;
};
int ffn_mfma_launch(const float* x, const void* w_gu, const void* w_down, float* y, int m, int hidden, int inter,
                    hipStream_t s, const ResidEpi* re = nullptr);
int gemm2_launch(Gemm2Args a, hipStream_t s);
// the same GEMM on 256 x 256 tiles with a ping-pong 8-wave schedule (gemm3.hip)
bool gemm3_supported(int n, int k, int epi, int ksplit);
int gemm3_launch(Gemm2Args a, hipStream_t s);
// llmi_linear for fp16 weights (the layer API's projections): fp32 x split into planes,
// then gemm3 / gemm2 (+ split-K slices summed in order); see gemm2.hip
bool linear_mfma_supported(int m, int n, int k);
// slab_out / ks_out: the ks K slices ([ks][m][n] fp32 in the stream's linear workspace,
// valid until the next llmi_linear-family call on s) instead of their sum
int linear_mfma_launch(const float* x, const void* w, float* y, int m, int n, int k, hipStream_t s,
                       const ResidEpi* re = nullptr, const float** slab_out = nullptr, int* ks_out = nullptr);
// rows of x (+= the ksplit slices of slab, in slice order, written back to x),
// then optional RMSNorm, then fp16 planes hi[, lo] (hi null: the combine alone)
int rows_split_launch(float* x, int ldx, int m, int k, const void* gamma, int g_dtype, float eps, _Float16* hi,
                      _Float16* lo, int ldh, hipStream_t s, const float* slab = nullptr, int ksplit = 0,
                      bool lo8 = false);  // lo8: e4m3 lo bytes in the first ldh bytes of each row (common.h lo8_pack4)

// ------------------------------------------------- prefill attention
// rope + KV-cache write of M rows, then causal attention over cache slots
// [0, p0 + m] per row; see prefill.hip.
struct PrefillAttnArgs {
    float* qkv = nullptr;          // [m, (heads + 2 kv) * D] fp32; q rotated in place
    const float* qkv2 = nullptr;   // optional second K slice of qkv (same layout), added first
    void* k_cache = nullptr;       // layer base [kv_heads, max_seq, D]
    void* v_cache = nullptr;
    int cache_dtype = LLMI_F16;
    int max_seq = 0;
    int m = 0, p0 = 0;
    int heads = 0, kv_heads = 0, head_dim = 128;
    const float* rope_tab = nullptr;  // [max_seq][D/2] (cos, sin)
    float* out = nullptr;          // [m, heads * D]
    // fp16 cache only: 1 or 2 = the MFMA kernel with that many fp16 planes of q and
    // p (2: fp32-faithful); out_hi (, out_lo) given: write the output as fp16 planes
    int mfma_planes = 0;
    _Float16* out_hi = nullptr;
    _Float16* out_lo = nullptr;
    int out_lo8 = 0;               // out_lo rows hold e4m3 bytes in their first half (common.h lo8_pack4)
    // MFMA form: scratch for the split-key partials (null: one workgroup per query block)
    float* split_ws = nullptr;
    size_t split_ws_floats = 0;
};
int prefill_attn_launch(const PrefillAttnArgs& a, hipStream_t s);
// after a prefill of prompt rows [p0, p0 + n): record them as tokens and
// advance the decode state (next_pos = p0 + n)
int prefill_finish_launch(struct DecodeState* st, const int32_t* prompt, int32_t* tokens, int p0, int n,
                          hipStream_t s);

// ------------------------------------------------------------- attention
struct AttnArgs {
    unsigned long long* stamps = nullptr;  // debug timeline (WgStamp), null = off
    const float* qkv = nullptr;    // [(heads + 2 kv_heads) * D]
    void* k_cache = nullptr;       // layer base: [kv_heads, max_seq, D]
    void* v_cache = nullptr;
    int cache_dtype = LLMI_F16;
    int max_seq = 0;
    const int* pos_dev = nullptr;  // device position (engine); else pos_host
    int pos_host = 0;
    int heads = 0, kv_heads = 0, head_dim = 128;
    int rope = 1;
    float rope_base = 10000.f;
    const float* rope_tab = nullptr;  // [max_seq][D/2] (cos, sin) pairs; else computed in-kernel
    float* out = nullptr;          // [heads * D]
    void* workspace = nullptr;
    // 1 (operator API): normalized output in `out` (merge kernel when > 1 split);
    // 0 (engine): split partials only, consumed by attn_oproj_launch
    int direct_out = 1;
    // engine: seed the fixed-point residual accumulator (see attn_oproj_launch) with
    // resid_fixed (int64 residual stream; or fixed(resid) when only fp32 is given) on the
    // rank that carries the residual (resid_scale != 0), zeros elsewhere
    long long* xacc = nullptr;
    const float* resid = nullptr;
    const long long* resid_fixed = nullptr;
    float resid_scale = 1.f;
    int hidden = 0;
    // > 0: the caller knows the position's split count, ceil((pos + 1) / 64) (the engine
    // tracks the position on the host): the grid is exactly the active splits and every
    // K/V load is issued before the device position arrives; 0: grid = max_seq / 64,
    // inactive splits exit after reading the position
    int nact = 0;
    // HOST_SIZED (nact > 0): the kernel checks nact against the device position; on a
    // mismatch it sets bit 4 here (DecodeState::error) and does no work
    int* err = nullptr;
    // fused q/k/v + attention launch (qkv_attn.hip): q, k, v come from the GEMV's granules
    // {fp32 bits, tag} of this launch (qkv_tag, polled until every tag is
    // *tag_epoch * 128 + tag_layer) instead of qkv; a wait past ~2 s sets error bit 64
    const unsigned long long* qkv_tag = nullptr;
    const unsigned* tag_epoch = nullptr;
    unsigned tag_layer = 0;
    int tag_poll_all = 0;  // 1: poll every granule from the first look (no single-granule phase)
    // 1 (the fused launch with its o_proj part): partials stored write-through, then one arrival
    // per workgroup on the head's counter (workspace counters word 0) for the o_proj blocks
    int publish = 0;
};

// Merge of the split partials fused into the o_proj, split by head: workgroup
// (h, row chunk) merges head h's partials and adds W_o[rows, h*d:(h+1)*d] . o_h into
// xacc[rows] with int64 fixed-point atomics (exact, so the sum is independent of
// arrival order: deterministic). xacc was seeded by the attention kernel.
struct OprojArgs {
    unsigned long long* stamps = nullptr;  // debug timeline (WgStamp), null = off
    const void* w = nullptr;        // W_o (rank shard): [n_rows, ldw] row-major, or head-major
    const __half* scales = nullptr; // int8 per-row scales
    int head_major = 0;             // 1: w is [heads][n_rows][head_dim] (each head's slice contiguous)
    int w_dtype = LLMI_F16;
    int n_rows = 0, ldw = 0;
    int heads = 0, head_dim = 128;
    int max_seq = 0;
    const int* pos_dev = nullptr;
    int pos_host = 0;
    const void* workspace = nullptr;  // attention partials
    long long* xacc = nullptr;
    int nact = 0;  // > 0: active split count known on the host (no position read); see AttnArgs
    XchgArgs xt;              // producer-fused TP exchange of xacc (xt.buf null = off)
    unsigned* xt_cnt = nullptr;
    int* err = nullptr;       // the fused launch's o_proj part: bit 64 when its heads never arrive
};
int attn_oproj_launch(const OprojArgs& a, hipStream_t s);

// Persistent ring layer (ring.hip): after layer l's attention, ONE launch runs
//   o_proj (merge fused, by head) -> RMSNorm + gate_up + SiLU*up -> down (K split by CU)
//   -> [RMSNorm + next layer's q/k/v]
// on one workgroup per CU whose loader waves stream every weight the CU needs into an
// LDS ring, running ahead across the two in-launch hand-offs (the o_proj and down sums,
// int64 fixed-point atomics + a sharded arrival counter). fp16 weights, hidden 4096.
constexpr int kRingShards = 8, kRingShardWords = 32;           // one 128-B line per shard
constexpr int kRingCntWords = 2 * kRingShards * kRingShardWords;  // a layer's two fan-in counters
struct RingArgs {
    const void* w_o = nullptr;      // [hidden][heads * 128] fp16
    const void* w_gu = nullptr;     // [2 inter][hidden] fp16 (gate rows, then up rows)
    const void* w_dt = nullptr;     // [inter][hidden] fp16: W_down transposed
    const void* w_qkv = nullptr;    // next layer's [n_qkv][hidden] fp16; null: no q/k/v phase
    const void* g_ffn = nullptr;    // this layer's post-attention RMSNorm gamma (fp16)
    const void* g_attn = nullptr;   // next layer's input RMSNorm gamma (fp16)
    const void* attn_ws = nullptr;  // this layer's split-KV attention partials (attn_impl.h Ws)
    long long* acc_x = nullptr;     // x_l (fixed point, read)
    long long* acc_mid = nullptr;   // x_l + o_proj (atomics; zero at launch)
    long long* acc_out = nullptr;   // x_{l+1} = mid + down (atomics; zero at launch)
    long long* zero0 = nullptr;     // accumulators of the next launches, zeroed here (may be null)
    long long* zero1 = nullptr;
    unsigned* cnt = nullptr;        // this layer's counters [2][kRingShards][kRingShardWords] (zero at launch)
    unsigned* cnt_zero = nullptr;   // the next ring launch's counters, zeroed here
    float* qkv_out = nullptr;       // next layer's q/k/v rows (fp32)
    int hidden = 0, heads = 0, inter = 0, n_qkv = 0, max_seq = 0, nact = 0;
    float eps = 1e-5f;
    int* err = nullptr;             // DecodeState::error: bit 32 = a hand-off wait timed out
    unsigned long long* stamps = nullptr;  // per-CU timeline [8] (null = off)
};
bool ring_supported(int hidden, int heads, int head_dim, int inter, int n_qkv, int n_cu);
int ring_layer_launch(const RingArgs& a, int grid, hipStream_t s);
int ring_residency(int* per_cu);  // workgroups of the ring kernel one CU admits (must be >= 1)
// W_down [rows][cols] fp16 -> its transpose [cols][rows] (the ring's K split by CU)
int transpose_f16_launch(const void* src, void* dst, int rows, int cols, hipStream_t s);

// fixed-point residual accumulator: value = int64 * 2^-32
__host__ __device__ __forceinline__ long long to_fixed(float v) {
#ifdef __HIP_DEVICE_COMPILE__
    return __float2ll_rn(v * 4294967296.0f);
#else
    return (long long)std::llrintf(v * 4294967296.0f);
#endif
}
__host__ __device__ __forceinline__ float from_fixed(long long v) {
    return (float)v * 2.3283064365386963e-10f;  // (float) rounds once; * 2^-32 is exact
}
#ifndef LLMI_ATTN_CH
#define LLMI_ATTN_CH 64
#endif
constexpr int kAttnChunk = LLMI_ATTN_CH;  // cached positions per workgroup (split-KV)
size_t attn_workspace_bytes(int heads, int head_dim, int max_seq);
int attn_decode_launch(const AttnArgs& a, hipStream_t s);
// the q/k/v GEMV (g: EPI_STORE, rmsnorm, fixed-point x) and the attention (at: host-sized)
// of one decode layer as ONE launch, q/k/v handed over as tagged granules (qkv_attn.hip)
bool qkv_attn_supported(const GemvArgs& g, const AttnArgs& at);
int qkv_attn_launch(const GemvArgs& g, const AttnArgs& at, hipStream_t s);
// ... and the layer's o_proj in the same launch (o non-null: fp16 weights, MHA, xacc seeded before
// the launch -- the attention part seeds nothing -- and no fused exchange)
bool qkv_attn_o_supported(const GemvArgs& g, const AttnArgs& at, const OprojArgs& o);
int qkv_attn_o_launch(const GemvArgs& g, const AttnArgs& at, const OprojArgs* o, hipStream_t s);
void qkv_attn_set_grid(int cap);  // A/B: cap the GEMV part of the fused grid (0: all resident slots)
void qkv_attn_set_order(int head_major);  // A/B: 1 head-major rows + attention blocks (default), 0 natural
void qkv_attn_set_poll(int all);          // A/B: 1 poll every granule from the start, 0 one granule first (default)

// ------------------------------------------------------ decode-loop state
struct DecodeState {
    int next_pos;     // position the next forward will process
    int cur_pos;      // position of the forward in flight
    int prompt_len;
    int vocab;
    int error;        // sticky error flags (1: token id out of range, 2: position overflow,
                      // 4: host-sized attention grid != device position's split count,
                      // 8: a tensor-parallel peer never arrived (one-shot exchange timeout, xchg.hip),
                      // 16: a prefill gate_up lo partial never arrived, gemm3_silu_bal_kernel,
                      // 32: a ring-layer hand-off or ring-slot wait timed out, ring.hip,
                      // 64: a fused q/k/v + attention workgroup's wait for its rows timed out)
    unsigned epoch;   // forwards stepped since the engine was created (step_start; never reset
                      // by set_prompt): tags the fused q/k/v launch's granules
    int pad[2];
};

// step start: pick the token for position next_pos (prompt id or argmax of
// the previous forward's partials), record it, gather its embedding row.
// Also seeds the int64 residual stream xres = fixed(x) (may be null) and zeroes the
// dataflow layer counters (cnt, cnt_words u32; may be null).
int step_start_launch(DecodeState* st, const int32_t* prompt, const unsigned long long* partials,
                      int n_partials, int32_t* tokens, const void* table, int table_dtype, int hidden,
                      float* x, long long* xres, int max_seq, unsigned* cnt, int cnt_words, hipStream_t s,
                      long long* xres2 = nullptr);  // xres2: a second copy of fixed(x) (layer 0's o_proj seed)
// after the last forward: tokens[next_pos] = argmax(partials) (no state change)
int finalize_launch(DecodeState* st, const unsigned long long* partials, int n_partials,
                    int32_t* tokens, int max_seq, hipStream_t s);

// ------------------------------------------------------- elementwise ops
int embedding_launch(const int32_t* ids, int n, const void* table, int t_dtype, int vocab, int hidden,
                     float* out, hipStream_t s);
int rmsnorm_launch(const float* x, float* out, float* resid_out, const void* gamma, int g_dtype,
                   int n, int hidden, float eps, hipStream_t s);
int add_resid_rmsnorm_launch(float* resid, float* out, const void* bias, int b_dtype,
                             const void* gamma, int g_dtype, int n, int hidden, float eps,
                             hipStream_t s);
int add_resid_launch(const float* resid, float* out, int n, int hidden, hipStream_t s);
int silu_mul_launch(const float* gu, float* out, int n, int inter, hipStream_t s);
// context-phase operators (context_ops.hip)
int causal_mask_launch(void* mask, int dtype, const int* q_lens, const int* k_lens, int batch, int max_q, int max_k,
                       hipStream_t s);
int masked_softmax_launch(const void* qk, const void* mask, void* score, int dtype, int batch, int heads, int q_len,
                          int k_len, float scale, hipStream_t s);
// fused ragged-batch context attention over the layer's cache (context_ops.hip)
int context_attention_launch(const float* q, const void* k_cache, const void* v_cache, int cache_dtype, int layer,
                             const int* history_length, const int* input_length, int batch, int heads, int kv_heads,
                             int max_q, int max_seq, int head_dim, float scale, float* out, hipStream_t s);
// + RoPE and the cache append in front (the layer's whole middle from the q/k/v rows)
int context_attention_qkv_launch(const float* qkv, const int* padding_offset, const int* history_length,
                                 const int* input_length, int num_tokens, int batch, int max_q, int heads,
                                 int kv_heads, int head_dim, float rope_base, void* k_cache, void* v_cache,
                                 int cache_dtype, int layer, int max_seq, float scale, float* q_scratch, float* out,
                                 hipStream_t s, int ks = 1, size_t ks_stride = 0);  // qkv as ks summed K slices
int kv_append_launch(const void* k_src, const void* v_src, int dtype, int layer, const int* cur_q, const int* hist,
                     int batch, int kv_heads, int max_q, int d, int max_seq, void* k_cache, void* v_cache,
                     hipStream_t s);
int transpose_remove_pad_launch(const void* src, const int* po, void* dst, int dtype, int num_tokens, int batch,
                                int seq_len, int heads, int d, hipStream_t s);
int batched_matmul_launch(const void* a, const void* b, void* c, int dtype, int batch, int m, int n, int k,
                          int trans_a, int trans_b, hipStream_t s);
int padding_offset_launch(int* po, int* cum, const int* lens, int batch, int max_q, hipStream_t s);
int rope_qkv_prefill_launch(const void* qkv, void* q, void* k, void* v, int dtype, const int* po, const int* hist,
                            int num_tokens, int batch, int seq_len, int heads, int kv_heads, int d, float base,
                            hipStream_t s);
int rope_decode_launch(float* qkv, int pos, int heads, int kv_heads, int head_dim, float base,
                       hipStream_t s);
int argmax_launch(const float* logits, int n, int32_t* out_id, unsigned long long* scratch,
                  hipStream_t s);
// engine sampling: u from llmi-prng-v1 with step = seed + (cur_pos + 1) (the position the
// token is chosen for), sampling.cu's rule over the top-K, result written as the only
// non-zero argmax partial so step_start / finalize pick it.
int sample_pick_launch(const struct DecodeState* st, const int32_t* ids, float* vals, int k, uint64_t seed,
                       unsigned long long* partials, int np, hipStream_t s);
int topk_launch(const void* logits, int dtype, int rows, int vocab, int k, int32_t* ids, void* vals, hipStream_t s);
int sampling_launch(const int32_t* topk_ids, void* topk_vals, int dtype, int rows, int k, int32_t* output_id,
                    int32_t* seqlen, uint8_t* is_finished, int step, int end_id, int vocab, hipStream_t s);
int repeat_kv_launch(const void* k_cache, const void* v_cache, int dtype, int layer, const int* ctx_len, int batch,
                     int kv_heads, int max_seq, int heads, int max_k_len, int d, void* k_dst, void* v_dst,
                     hipStream_t s);

// --------------------------------------------- one-shot TP exchange (xchg.hip)
constexpr int kXchgSlice = 256;     // vector elements per workgroup
constexpr int kXchgMaxSlices = 64;  // n <= 16384 elements
constexpr int kXchgMaxWorld = 8;    // ranks of one exchange (one node's GPUs)
size_t xchg_inbox_bytes(int world, int cap_n);
int xchg_launch(const XchgArgs& a, hipStream_t s);

// ---------------------------------------------------------- synthetic
// in-place reduction over W rank buffers (device array of pointers); op 0 i64 sum, 1 f32 sum, 2 u64 max
int convert_launch(const void* src, int src_dtype, void* dst, int dst_dtype, size_t n, hipStream_t s);
// measured HBM read peak (llmi_hbm_read_bench, include/llmi.h)
int hbm_read_bench(size_t bytes, int iters, float* us, float* gbps, size_t* bytes_read);
// src [rows][cols] -> dst [cols][rows] for 2- or 4-byte elements (raw bits)
int transpose_launch(const void* src, void* dst, int rows, int cols, int elem_bytes, hipStream_t s);
int group_reduce_launch(void* const* dev_bufs, int W, int n, int op, hipStream_t s);
int synth_fill_launch(void* out, int out_dtype, int kind, uint64_t seed, uint32_t tid, int rows,
                      int cols, int row0, int col0, int ld, hipStream_t s);
int synth_fill_host(void* out, int out_dtype, int kind, uint64_t seed, uint32_t tid, int rows,
                    int cols, int row0, int col0, int ld);

}  // namespace llmi
