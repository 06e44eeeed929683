// One launch for a decode layer's q/k/v GEMV and its split-KV attention (round 6).
//
// Replaces the pair gemv_launch(q/k/v) -> attn_decode_launch of the engine's layer (the
// reference's launchLinearGemm(qkv) + launchRoPE + launchDecoderMaskedMHA,
// src/layers/attention/masked_self_attention.cpp:54-92) with one grid:
//   * blocks [0, G): the q/k/v GEMV (gemv_body, rmsnorm fused), each output row published as
//     an 8-byte {fp32 bits, tag} granule with one write-through store (tag = the forward's
//     epoch * 128 + layer, so a row of the previous layer or forward never passes);
//   * blocks [G, G + heads * nact): the attention workgroups (attn_body, TAGGED). They issue
//     their K/V cache rows at once -- that stream does not depend on this token -- and wave 0
//     polls the head's granules; the position's RoPE, scores, softmax and P V follow as in the
//     separate kernel, and the split partials go to the o_proj launch as before.
// What it removes: the launch boundary between the two kernels and the attention's K/V burst
// and prologue after it -- the K/V rows (16.8 MB a layer at ctx 1024) stream while the GEMV's
// last row groups finish, instead of after the boundary.
//
// Deadlock freedom: only the attention blocks wait, and only on GEMV blocks, which wait on
// nothing; the GEMV blocks come first in the grid (dispatched in order, observed -- HIP does
// not promise it, so every wait is bounded: 2 s of s_memrealtime, then error bit 64 and no
// partials). The hand-off is the microarch guide's granule form (R2): one 8-byte sc1 store per
// row, sc1 loads on the reader, no flag, no fence.
//
// Results are bitwise those of the two launches: the GEMV and attention bodies are the same
// code (gemv_body with TAG, attn_body with TAGGED), only the q/k/v transport differs.
#include "attn_impl.h"
#include "gemv_launch.h"

// waves per SIMD the kernel is built for (= workgroups per CU): 4, as the q/k/v GEMV alone, where
// that fits 128 VGPRs without spills (fp16 / fp32 weights at U = 4: 125 / 110), else 3 (int8 and
// U = 5 spilled 6-11 VGPRs at 4)
#ifndef LLMI_QA_MINW_SPILL
#define LLMI_QA_MINW_SPILL 3  // waves per SIMD for the shapes that spill at 4 (A/B builds: 4)
#endif
template <typename WT, int U> constexpr int qa_minw() {
    return (sizeof(WT) >= 2 && U == 4) || sizeof(WT) == 4 ? 4 : LLMI_QA_MINW_SPILL;
}

namespace llmi {
namespace {

// A/B switches (engine options qa_grid / qa_order / qa_poll): process-wide, read at launch (graph
// capture) time, so an engine's already captured graphs keep the values they were captured with
int qa_grid_cap = 0;  // cap on the GEMV part of the grid (0 = every resident slot); qkv_attn_set_grid
int qa_order = 1;     // 1: GEMV rows and attention blocks head-major (MHA); 0: natural order
int qa_poll_all = 0;  // 1: attention polls every granule from the start

// WITH_O: blocks past the attention's run the o_proj (oproj_body2, FUSED: two heads per block,
// W_o slices issued at once, then a wait on the pair's arrival counters), pair-major so the
// heads the GEMV finishes first are projected first
template <typename WT, typename GT, int XPT, int U, typename KT, bool WITH_O>
__global__ __launch_bounds__(256, (qa_minw<WT, U>())) void qkv_attn_kernel(GemvArgs g, AttnArgs at, OprojArgs o,
                                                                            int g_grid, int ns) {
    extern __shared__ __attribute__((aligned(16))) float4 xs[];
    WgStamp ts(g.stamps);
    if constexpr (WITH_O) {
        const int ob = (int)blockIdx.x - g_grid - at.heads * at.nact;
        if (ob >= 0) {
            const int n_chunks = (o.n_rows + 63) / 64;
            attn_detail::oproj_body2<WT, 8, PlainIO, true>(o, ob / n_chunks, ob % n_chunks, ns,
                                                           reinterpret_cast<float*>(xs));
            return;
        }
    }
    if ((int)blockIdx.x < g_grid) {
        gemv_detail::gemv_body<WT, gemv_detail::kRows, EPI_STORE, true, GT, XPT, U, true, PlainIO, 1, true>(
            g, blockIdx.x, g_grid, xs);
    } else {
        // head-major block order with head-major rows (g.tag_heads): a head's splits dispatch
        // together, in the order the GEMV finishes the heads
        const int b = (int)blockIdx.x - g_grid;
        const int h = g.tag_heads > 0 ? b / at.nact : b % at.heads;
        const int sp = g.tag_heads > 0 ? b - h * at.nact : b / at.heads;
        attn_detail::attn_body<KT, PlainIO, true, true>(at, h, sp, ns, reinterpret_cast<float*>(xs), &ts);
    }
}

template <typename WT, typename GT, int XPT, int U, typename KT, bool WITH_O>
int launch_k(const GemvArgs& g, const AttnArgs& at, const OprojArgs* o, hipStream_t s) {
    auto kern = qkv_attn_kernel<WT, GT, XPT, U, KT, WITH_O>;
    size_t lds = std::max(gemv_detail::gemv_lds_bytes(g.k), attn_detail::kAttnLds);
    if (WITH_O) lds = std::max(lds, attn_detail::oproj2_lds<8>());
    int G = gemv_grid(g);
    // resident blocks of this kernel: the GEMV takes at most all of them (a looping grid), the
    // attention blocks fill the slots GEMV blocks leave
    static size_t occ_lds = ~(size_t)0;
    static int occ_blocks = 0;
    if (lds != occ_lds) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(kern), 256, lds) != hipSuccess)
            n = 0;
        occ_blocks = n * gemv_detail::device_cus();
        occ_lds = lds;
    }
    if (occ_blocks > 0 && G > occ_blocks) G = occ_blocks;
    if (qa_grid_cap > 0 && qa_grid_cap < G) G = qa_grid_cap;
    const int ns = (at.max_seq + attn_detail::CH - 1) / attn_detail::CH;
    int grid = G + at.heads * at.nact;
    GemvArgs gg = g;
    AttnArgs aa = at;
    OprojArgs oo;
    gg.tag_heads = (qa_order && at.heads == at.kv_heads && g.n_rows == 3 * at.heads * attn_detail::D) ? at.heads : 0;
    aa.tag_poll_all = qa_poll_all;
    if (WITH_O) {
        oo = *o;
        aa.publish = 1;
        grid += (at.heads / 2) * ((o->n_rows + 63) / 64);
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, s, gg, aa, oo, G, ns);
    LLMI_HIP(hipGetLastError());
    return LLMI_OK;
}

template <typename WT, typename GT, int XPT, int U>
int launch_kt(const GemvArgs& g, const AttnArgs& at, const OprojArgs* o, hipStream_t s) {
    if constexpr (sizeof(WT) == 2 && XPT == 4 && U == 4) {  // the o_proj part: fp16 7B-width shapes
        if (o)
            return at.cache_dtype == LLMI_F16 ? launch_k<WT, GT, XPT, U, __half, true>(g, at, o, s)
                                              : launch_k<WT, GT, XPT, U, float, true>(g, at, o, s);
    }
    return at.cache_dtype == LLMI_F16 ? launch_k<WT, GT, XPT, U, __half, false>(g, at, nullptr, s)
                                      : launch_k<WT, GT, XPT, U, float, false>(g, at, nullptr, s);
}

template <typename WT, typename GT>
int launch_w(const GemvArgs& g, const AttnArgs& at, const OprojArgs* o, int xpt, int u, hipStream_t s) {
    if (xpt == 4) return u == 4 ? launch_kt<WT, GT, 4, 4>(g, at, o, s) : launch_kt<WT, GT, 4, 5>(g, at, o, s);
    return u == 4 ? launch_kt<WT, GT, 5, 4>(g, at, o, s) : launch_kt<WT, GT, 5, 5>(g, at, o, s);
}


int epl_of(int dt) { return dt == LLMI_F16 ? 8 : dt == LLMI_F32 ? 4 : dt == LLMI_I8 ? 16 : 0; }

// the GEMV part's unroll: 4 or 5 whenever that covers a row in whole batches (a TP rank's
// few row groups would otherwise pick 8, which this kernel does not instantiate), else the
// standalone GEMV's choice
int pick_u(const GemvArgs& g) {
    const int nc = g.k / epl_of(g.w_dtype);
    if (nc % (64 * 4) == 0) return 4;
    if (nc % (64 * 5) == 0) return 5;
    const int groups = (g.n_rows + gemv_detail::kRows - 1) / gemv_detail::kRows;
    switch (g.w_dtype) {
        case LLMI_F16: return gemv_detail::pick_unroll<__half, EPI_STORE>(g, groups);
        case LLMI_F32: return gemv_detail::pick_unroll<float, EPI_STORE>(g, groups);
        case LLMI_I8: return gemv_detail::pick_unroll<int8_t, EPI_STORE>(g, groups);
    }
    return 0;
}

}  // namespace

bool qkv_attn_supported(const GemvArgs& g, const AttnArgs& at) {
    const int epl = epl_of(g.w_dtype);
    if (epl == 0 || g.k <= 0 || g.k % epl != 0 || g.k > 5 * 4 * 256) return false;
    if (g.epi != EPI_STORE || !g.x_fixed || !g.gamma || g.kpar > 1 || g.grid != 0 || g.ldw != 0) return false;
    // instantiated pairs: fp16 / int8 weights with fp16 gammas (the engine's fp16 models),
    // fp32 weights with fp32 gammas (the parity models)
    if (g.g_dtype != (g.w_dtype == LLMI_F32 ? LLMI_F32 : LLMI_F16)) return false;
    if (g.w_dtype == LLMI_I8 && !g.scales) return false;
    const int u = pick_u(g);
    if (u != 4 && u != 5) return false;
    // where the standalone GEMV would stream a row group in one unroll-8 batch and its grid fills
    // every CU at least twice (a TP-2 rank's q/k/v: 768 workgroups), the fused form's unroll 4
    // costs more than the boundary it saves (TP 2 1,961 -> 1,982 us a token, r07s); with fewer
    // workgroups than that (TP 4: 384, TP 8: 192) it wins (-1.8 % / -4.1 %, r07e)
    {
        const int groups = (g.n_rows + gemv_detail::kRows - 1) / gemv_detail::kRows;
        int su = 0;
        switch (g.w_dtype) {
            case LLMI_F16: su = gemv_detail::pick_unroll<__half, EPI_STORE>(g, groups); break;
            case LLMI_F32: su = gemv_detail::pick_unroll<float, EPI_STORE>(g, groups); break;
            case LLMI_I8: su = gemv_detail::pick_unroll<int8_t, EPI_STORE>(g, groups); break;
        }
        const int cus = gemv_detail::device_cus() > 0 ? gemv_detail::device_cus() : 256;
        if (su != u && gemv_grid(g) >= 2 * cus) return false;
    }
    if (at.head_dim != attn_detail::D || at.nact <= 0 || !at.pos_dev || at.direct_out) return false;
    if (at.cache_dtype != LLMI_F16 && at.cache_dtype != LLMI_F32) return false;
    if (at.heads <= 0 || at.kv_heads <= 0 || at.heads % at.kv_heads != 0) return false;
    return g.n_rows == (at.heads + 2 * at.kv_heads) * attn_detail::D;
}

void qkv_attn_set_grid(int cap) { qa_grid_cap = cap > 0 ? cap : 0; }
void qkv_attn_set_order(int head_major) { qa_order = head_major != 0; }
void qkv_attn_set_poll(int all) { qa_poll_all = all != 0; }

bool qkv_attn_o_supported(const GemvArgs& g, const AttnArgs& at, const OprojArgs& o) {
    if (!qkv_attn_supported(g, at) || g.w_dtype != LLMI_F16 || g.k / 4 > 4 * 256 || pick_u(g) != 4) return false;
    if (at.xacc != nullptr || at.heads % 2 != 0 || at.heads != at.kv_heads) return false;
    return o.w_dtype == LLMI_F16 && !o.head_major && o.heads == at.heads && o.nact == at.nact && o.xacc &&
           o.workspace == at.workspace && o.n_rows % 64 == 0 && o.ldw >= o.heads * attn_detail::D &&
           (long)o.heads * o.n_rows / (1024 * 16) >= 8 && !o.xt.buf;  // oproj_npl 8, no fused exchange
}

int qkv_attn_launch(const GemvArgs& g, const AttnArgs& at, hipStream_t s) { return qkv_attn_o_launch(g, at, nullptr, s); }

int qkv_attn_o_launch(const GemvArgs& g, const AttnArgs& at, const OprojArgs* o, hipStream_t s) {
    LLMI_REQUIRE(!o || qkv_attn_o_supported(g, at, *o), "qkv_attn_o: unsupported shape (qkv_attn_o_supported)");
    LLMI_REQUIRE(qkv_attn_supported(g, at), "qkv_attn: unsupported shape (qkv_attn_supported)");
    LLMI_REQUIRE(g.w && g.x_fixed && g.y_tag && g.tag_epoch && at.qkv_tag == g.y_tag && at.tag_epoch == g.tag_epoch &&
                     at.tag_layer == g.tag_layer && g.tag_layer < 128,
                 "qkv_attn: the GEMV and the attention must share the granule buffer and tag (layer < 128)");
    LLMI_REQUIRE(at.k_cache && at.v_cache && at.workspace && at.max_seq > 0, "qkv_attn: null pointer");
    const int ns = (at.max_seq + attn_detail::CH - 1) / attn_detail::CH;
    LLMI_REQUIRE(ns <= attn_detail::kMaxSplits && at.nact <= ns, "qkv_attn: nact / max_seq out of range");
    LLMI_REQUIRE(!at.xacc || at.resid || at.resid_fixed, "qkv_attn: xacc seeding needs resid");
    const int xpt = g.k / 4 <= 4 * 256 ? 4 : 5;
    const int u = pick_u(g);
    switch (g.w_dtype) {
        case LLMI_F16: return launch_w<__half, __half>(g, at, o, xpt, u, s);
        case LLMI_F32: return launch_w<float, float>(g, at, nullptr, xpt, u, s);
        case LLMI_I8: return launch_w<int8_t, __half>(g, at, nullptr, xpt, u, s);
    }
    return LLMI_EINVAL;
}

}  // namespace llmi
