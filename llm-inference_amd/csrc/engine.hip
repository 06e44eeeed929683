// DecodeEngine: the Llama<T> single-stream greedy decode loop on one GPU (or
// one tensor-parallel rank), as one hipGraph per token.
//
// Reference call stack replaced:
//   Llama<T>::Response / continueTokenGen       src/models/llama/llama.cpp:318-349, 362-457
//   LlamaSelfDecoder<T>::forward                src/layers/decoder/self_decoder.cpp:23-89
//   LLaMASelfAttentionLayer<T>::Forward         src/layers/attention/masked_self_attention.cpp:54-92
//   LLaMAFFNLayer<T>::forward                   src/layers/ffn/ffn.cpp:52-93
//   LMHeadAndTopKSample                         src/models/llama/llama.cpp:214-269
// The reference issues ~326 launches per token, each followed by
// cudaDeviceSynchronize, plus a D2H and an H2D copy per token. Here one token is
//   step_start (token pick + embedding)
//   L x [ rmsnorm+QKV gemv | rope+kv-write+split-KV attention | O gemv+residual
//         (| allreduce) | rmsnorm+gate_up gemv+silu*mul | down gemv+residual (| allreduce) ]
//   final rmsnorm + lm_head gemv + argmax partials (| allreduce max)
// = 5L + 2 kernels, captured once into a hipGraph; positions, token ids and the
// argmax hand-off live in device memory, so tokens are produced with no host sync.
//
// HBM layout (one allocation each): all weights contiguous per layer in
// forward order (qkv, o, gate_up, down, norms), then lm_head, final norm,
// embedding; KV cache [layers, kv_heads, max_seq, head_dim] per K and V
// (concat_past_kv.cu:122 layout, batch 1); fp32 activations (16-44 KB) and
// the decode state in a small scratch block.
//
// Tensor parallel: Megatron column/row split over tp_world
// ranks, one process per GPU; q/k/v and gate/up rows split by heads / inter
// columns, o and down split on their input columns. Rank 0 adds the residual
// in the o/down epilogue, every other rank stores its bare partial, and an RCCL
// all-reduce(sum) over xGMI yields residual + sum of partials in place: 2 per
// layer. The vocab-parallel lm_head produces per-workgroup argmax keys with
// global row ids; an all-reduce(max) of the keys gives every rank the same
// next token. Weights are generated shard-by-shard from the same global PRNG
// indices, so every TP degree computes the same model.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include <string>

#include "kernels.h"
#include "xchg_impl.h"
#include "prng.h"

namespace llmi {

namespace {
size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
}  // namespace

#ifndef LLMI_F16_DOWN_KSPLIT
#define LLMI_F16_DOWN_KSPLIT 1  // fp16 down K slices (int64 atomics: exact in any order)
#endif
#ifndef LLMI_I8_DOWN_KSPLIT
#define LLMI_I8_DOWN_KSPLIT 4  // int8 down K slices: 13B down 18.2 -> 16.5 us, 8-layer loop 682 -> 665 us (A/B)
#endif

// The token graphs, one per active split count nact = pos / 64 + 1: the attention
// and o_proj grids are sized on the host (AttnArgs::nact), so one captured step is
// valid for 64 consecutive positions. Built lazily, before a decode run's launches.
struct StepGraphs {
    std::vector<hipGraph_t> g;
    std::vector<hipGraphExec_t> x;
    void clear() {
        for (auto e : x)
            if (e) (void)hipGraphExecDestroy(e);
        for (auto h : g)
            if (h) (void)hipGraphDestroy(h);
        x.clear();
        g.clear();
    }
    ~StepGraphs() { clear(); }
    bool empty() const { return x.empty(); }
    // capture record() (which records one step for nact) on s unless cached
    template <typename F>
    int build(int nact, hipStream_t s, F&& record) {
        if ((int)x.size() <= nact) {
            x.resize(nact + 1, nullptr);
            g.resize(nact + 1, nullptr);
        }
        if (x[nact]) return LLMI_OK;
        LLMI_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        int rc = record();
        hipGraph_t h = nullptr;
        hipError_t e = hipStreamEndCapture(s, &h);
        if (rc != LLMI_OK) {
            if (h) (void)hipGraphDestroy(h);
            return rc;
        }
        LLMI_HIP(e);
        g[nact] = h;
        LLMI_HIP(hipGraphInstantiate(&x[nact], h, nullptr, nullptr, 0));
        return LLMI_OK;
    }
};

#ifndef LLMI_GU_XOUT
#define LLMI_GU_XOUT 0
#endif
#ifndef LLMI_SEED_FROM_DOWN
#define LLMI_SEED_FROM_DOWN 1  // single rank: down seeds the next o_proj sum; the attention writes no seed (0: A/B)
#endif
#ifndef LLMI_QKV_ATTN
#define LLMI_QKV_ATTN 1  // one q/k/v GEMV + attention launch (qkv_attn.hip); engine option "qkv_attn"
#endif
#ifndef LLMI_QKV_ATTN_O
#define LLMI_QKV_ATTN_O 0  // the fused launch also runs the o_proj (fp16 MHA, single rank); option "qa_o"
#endif
#ifndef LLMI_DOWN_STORE
#define LLMI_DOWN_STORE 1  // unsplit down: rows written as xmid + fixed(y), not seeded + atomically added (0: A/B)
#endif

struct Engine {
    llmi_config c{};
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = true;  // false inside an in-process group (the group's stream)
    bool grouped = false;    // rank of an in-process TP group: reductions are the group's
    // local (per-rank) dims
    int hl = 0, kvl = 0, ql = 0, kvrows = 0, il = 0, vl = 0;
    int wdt = LLMI_F16;      // linear weight dtype
    int edt = LLMI_F16;      // embedding / lm_head / norm dtype
    size_t wsz = 2, esz = 2;

    struct Layer {
        void *qkv = nullptr, *o = nullptr, *gu = nullptr, *down = nullptr;
        __half *qkv_s = nullptr, *o_s = nullptr, *gu_s = nullptr, *down_s = nullptr;
        void *attn_norm = nullptr, *ffn_norm = nullptr;
    };
    std::vector<Layer> layers;
    void *embed = nullptr, *lm_head = nullptr, *final_norm = nullptr;
    char* wblob = nullptr;
    size_t wbytes = 0;
    uint64_t stream_bytes = 0;  // weight bytes one forward reads

    void *kcache = nullptr, *vcache = nullptr;
    size_t kv_layer_elems = 0;

    char* scratch = nullptr;
    float *x = nullptr, *qkv_buf = nullptr, *attn_out = nullptr, *act = nullptr, *logits = nullptr;
    // Residual stream in int64 fixed point (value * 2^32): res[l % 2] is layer l's input,
    // xacc the mid-layer accumulator (residual + o_proj), res[(l + 1) % 2] the output
    // (mid + down). Every residual add is an exact integer add, so sums are
    // independent of workgroup order and of the TP reduction order.
    long long* xacc = nullptr;
    long long* res[2] = {nullptr, nullptr};
    unsigned long long* partials = nullptr;
    int lm_grid = 0;
    void* attn_ws = nullptr;
    float* rope_tab = nullptr;  // [max_seq][head_dim/2] (cos, sin): modeling_llama.py:130-146 cache
    DecodeState* st = nullptr;
    int32_t *prompt = nullptr, *tokens = nullptr;

    StepGraphs graphs;
    int rec_nact = 0;  // active split count the next recorded step's attention is sized for
    // fused q/k/v + attention launch (qkv_attn.hip) where the shapes allow it; option "qkv_attn",
    // default LLMI_QKV_ATTN (A/B); qtag: its granule buffer [(heads + 2 kv) * d]
    bool qa_fuse = LLMI_QKV_ATTN != 0;
    bool qa_o = LLMI_QKV_ATTN_O != 0;  // ... with the o_proj in the same launch (option "qa_o")
    unsigned long long* qtag = nullptr;
    ncclComm_t comm = nullptr;
    // one-shot peer exchange (xchg.hip): this rank's inbox (uncached HBM), every rank's
    // inbox base (IPC-mapped for peers) in device memory, per-slice epoch counters.
    // xchg_mode 1 replaces the RCCL all-reduces of the token graph (RCCL stays selectable);
    // xchg_mode 2 moves the exchange into the producing launches (o_proj, down, lm_head
    // finish with xchg_tail: push + wait + reduce, no exchange launch). tail_mode: what
    // those launches do (0 nothing, 1 push only -- the in-process group, 3 push + reduce);
    // xt_cnt their arrival counters (xchg_impl.h: sharded, zeroed here, re-zeroed by every
    // fused launch's finishers).
    int xchg_mode = 0;
    int tail_mode = 0;
    unsigned* xt_cnt = nullptr;
    char* inbox = nullptr;
    char** peers_dev = nullptr;
    unsigned long long* xchg_ep = nullptr;
    std::vector<void*> peers_opened;  // IPC mappings to close
    int xchg_cap_n = 0;
    // prefill scratch (allocated on first use): rows of one prefill chunk
    char* pf = nullptr;
    int pf_rows = 0;
    float *pf_x = nullptr, *pf_qkv = nullptr, *pf_o = nullptr, *pf_act = nullptr;
    _Float16 *pf_ah = nullptr, *pf_al = nullptr;  // fp16 activation planes (gemm2 path)
    float* pf_slab = nullptr;      // split-K partial slabs of the o_proj / down GEMMs [kPfSlabs][R][H]
    float* pf_split = nullptr;     // split-key prefill attention partials
    size_t pf_split_floats = 0;
    int pf_pending = 0;            // slices in pf_slab not yet added into pf_x
    static constexpr int kPfSplit = 2;   // o_proj (gemm2) K slices
    static constexpr int kPfDown = 8;    // down (gemm3) K slices
    static constexpr int kPfSlabs = 8;
    // split mode 3: e4m3 copies of the prefill GEMM weights (W * 2^exp, gemm3.hip), made on first use
    struct W8Layer {
        void *qkv = nullptr, *o = nullptr, *gu = nullptr, *down = nullptr;
        int qkv_e = 0, o_e = 0, gu_e = 0, down_e = 0;
    };
    std::vector<W8Layer> w8l;
    char* w8blob = nullptr;
    // split mode 3's gate_up on every CU (gemm3_silu_bal_kernel): lo partial slots + flags
    float* pf_bal = nullptr;
    unsigned* pf_bal_flags = nullptr;
    int n_cu = 0;
    // decode mode 1: the persistent ring layer (ring.hip) -- per token step_start, q/k/v(0),
    // L x [attention, ring], lm_head. rl_acc holds the int64 residual accumulators in
    // five slots [A0][A1][B0][A2][B1] (A: layer inputs x_l, slot l % 3; B: mid-layer sums,
    // slot l % 2), A1 + B0 adjacent so step_start zeroes both; rl_cnt the per-layer fan-in
    // counters; wdt the transposed W_down copies the ring's K split reads.
    int decode_mode = 0;
    long long* rl_acc = nullptr;
    unsigned* rl_cnt = nullptr;
    char* wdt_blob = nullptr;
    bool wdt_valid = false;
    long long* acc_a(int l) const { static const int s[3] = {0, 1, 3}; return rl_acc + (size_t)s[l % 3] * c.hidden; }
    long long* acc_b(int l) const { return rl_acc + (size_t)(l % 2 ? 4 : 2) * c.hidden; }
    void* wdt_of(int l) const { return wdt_blob + (size_t)l * il * c.hidden * 2; }
    int host_next_pos = 0, prompt_len = 0;
    unsigned long long* dbg_stamps = nullptr;  // llmi_engine_debug_stamps: per-workgroup timeline
    // llmi_engine_debug_timeline: every stamped launch of a recorded step gets its own
    // region of dbg_stride workgroups (slot = launch order), dbg_slots regions in all
    int dbg_stride = 0, dbg_slots = 0;
    mutable int dbg_slot = 0;
    unsigned long long* stamp_ptr() const {
        if (!dbg_stamps || dbg_stride == 0) return dbg_stamps;
        const int s = dbg_slot++;
        return s < dbg_slots ? dbg_stamps + (size_t)s * dbg_stride * 8 : nullptr;
    }
    uint64_t seed = 0;
    // stochastic sampling (Llama<T>::Sampling, llama.cpp:245-262): 0 = greedy argmax
    int sample_k = 0;
    uint64_t sample_seed = 0;
    int32_t* samp_ids = nullptr;
    float* samp_vals = nullptr;

    ~Engine() {  // teardown errors are not actionable; ignore them explicitly
        if (samp_ids) (void)hipFree(samp_ids);
        if (samp_vals) (void)hipFree(samp_vals);
        graphs.clear();
        if (comm) (void)ncclCommDestroy(comm);
        for (void* p : peers_opened) (void)hipIpcCloseMemHandle(p);
        if (inbox) (void)hipFree(inbox);
        if (peers_dev) (void)hipFree(peers_dev);
        if (xchg_ep) (void)hipFree(xchg_ep);
        if (xt_cnt) (void)hipFree(xt_cnt);
        if (wblob) (void)hipFree(wblob);
        if (kcache) (void)hipFree(kcache);
        if (vcache) (void)hipFree(vcache);
        if (scratch) (void)hipFree(scratch);
        if (pf) (void)hipFree(pf);
        if (w8blob) (void)hipFree(w8blob);
        if (pf_bal) (void)hipFree(pf_bal);
        if (pf_bal_flags) (void)hipFree(pf_bal_flags);
        if (rl_acc) (void)hipFree(rl_acc);
        if (rl_cnt) (void)hipFree(rl_cnt);
        if (wdt_blob) (void)hipFree(wdt_blob);
        if (stream && own_stream) (void)hipStreamDestroy(stream);
    }

    // ---------------------------------------------------------------- setup
    // ext_stream != nullptr: rank of an in-process group (no RCCL communicator)
    int init(const llmi_config& cfg, int dev, const void* tp_id, hipStream_t ext_stream = nullptr) {
        c = cfg;
        device = dev;
        const int W = c.tp_world;
        LLMI_REQUIRE(W >= 1 && c.tp_rank >= 0 && c.tp_rank < W, "engine: bad tp rank/world");
        LLMI_REQUIRE(c.head_dim == 128, "engine: head_dim must be 128");
        LLMI_REQUIRE(c.heads * c.head_dim == c.hidden, "engine: hidden != heads * head_dim");
        LLMI_REQUIRE(c.heads % c.kv_heads == 0, "engine: heads % kv_heads != 0");
        LLMI_REQUIRE(c.heads % W == 0 && c.kv_heads % W == 0 && c.inter % W == 0 && c.vocab % W == 0,
                     "engine: heads, kv_heads, inter and vocab must divide by tp_world");
        LLMI_REQUIRE(c.max_seq > 0 && c.layers > 0 && c.vocab > 0, "engine: bad dims");
        LLMI_REQUIRE(c.kv_dtype == LLMI_F16 || c.kv_dtype == LLMI_F32, "engine: kv dtype must be f16/f32");
        wdt = c.weight_dtype;
        LLMI_REQUIRE(wdt == LLMI_F16 || wdt == LLMI_F32 || wdt == LLMI_I8, "engine: bad weight dtype");
        edt = (wdt == LLMI_F32) ? LLMI_F32 : LLMI_F16;
        wsz = dtype_size(wdt);
        esz = dtype_size(edt);
        hl = c.heads / W;
        kvl = c.kv_heads / W;
        ql = hl * c.head_dim;
        kvrows = kvl * c.head_dim;
        il = c.inter / W;
        vl = c.vocab / W;
        const int epl = 16 / (int)wsz;
        LLMI_REQUIRE(c.hidden % epl == 0 && ql % epl == 0 && il % epl == 0,
                     "engine: hidden, q rows per rank and inter per rank must be multiples of 16 bytes");

        LLMI_HIP(hipSetDevice(device));
        LLMI_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device));
        if (ext_stream) {
            stream = ext_stream;
            own_stream = false;
            grouped = true;
        } else {
            LLMI_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        }
        // a communicator whenever an id is given -- also at tp_world 1, where the
        // all-reduces are identities but still run (captured in the token graph)
        // tp_world > 1 without an id: no RCCL; the ranks must open the one-shot peer
        // exchange (llmi_engine_xchg_open) before they decode
        if (!grouped && tp_id != nullptr) {
            ncclUniqueId id;
            std::memcpy(&id, tp_id, sizeof(id));
            ncclResult_t r = ncclCommInitRank(&comm, W, id, c.tp_rank);
            LLMI_REQUIRE(r == ncclSuccess, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        }
        LLMI_TRY(alloc_weights());
        LLMI_TRY(alloc_state());
        return LLMI_OK;
    }

    int alloc_weights() {
        const size_t H = c.hidden, A = 256;
        size_t off = 0;
        auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + bytes, A); return o; };
        struct Off { size_t qkv, o, gu, down, qs, os, gs, ds, an, fn; };
        std::vector<Off> lo(c.layers);
        const size_t qkv_rows = ql + 2 * kvrows;
        for (int l = 0; l < c.layers; ++l) {
            Off& t = lo[l];
            t.qkv = take(qkv_rows * H * wsz);
            t.o = take(H * ql * wsz);
            t.gu = take(2 * il * H * wsz);
            t.down = take(H * il * wsz);
            if (wdt == LLMI_I8) {
                t.qs = take(qkv_rows * 2);
                t.os = take(H * 2);
                t.gs = take(2 * il * 2);
                t.ds = take(H * 2);
            }
            t.an = take(H * esz);
            t.fn = take(H * esz);
        }
        const size_t lm = take((size_t)vl * H * esz), fnorm = take(H * esz), emb = take((size_t)c.vocab * H * esz);
        wbytes = off;
        LLMI_HIP(hipMalloc(&wblob, wbytes));
        layers.resize(c.layers);
        for (int l = 0; l < c.layers; ++l) {
            Layer& L = layers[l];
            L.qkv = wblob + lo[l].qkv;
            L.o = wblob + lo[l].o;
            L.gu = wblob + lo[l].gu;
            L.down = wblob + lo[l].down;
            if (wdt == LLMI_I8) {
                L.qkv_s = (__half*)(wblob + lo[l].qs);
                L.o_s = (__half*)(wblob + lo[l].os);
                L.gu_s = (__half*)(wblob + lo[l].gs);
                L.down_s = (__half*)(wblob + lo[l].ds);
            }
            L.attn_norm = wblob + lo[l].an;
            L.ffn_norm = wblob + lo[l].fn;
        }
        lm_head = wblob + lm;
        final_norm = wblob + fnorm;
        embed = wblob + emb;
        // bytes streamed per forward: every linear weight (+scales), norms, lm_head, one embedding row
        uint64_t per_layer = (qkv_rows * H + H * ql + 2 * il * H + H * il) * wsz + 2 * H * esz;
        if (wdt == LLMI_I8) per_layer += (qkv_rows + H + 2 * il + H) * 2;
        stream_bytes = per_layer * c.layers + (uint64_t)vl * H * esz + H * esz + H * esz;
        return LLMI_OK;
    }

    int alloc_state() {
        const size_t H = c.hidden;
        kv_layer_elems = (size_t)kvl * c.max_seq * c.head_dim;
        const size_t kvb = (size_t)c.layers * kv_layer_elems * dtype_size(c.kv_dtype);
        LLMI_HIP(hipMalloc(&kcache, kvb));
        LLMI_HIP(hipMalloc(&vcache, kvb));
        LLMI_HIP(hipMemsetAsync(kcache, 0, kvb, stream));
        LLMI_HIP(hipMemsetAsync(vcache, 0, kvb, stream));

        GemvArgs lmargs = lm_args();
        lm_grid = gemv_grid(lmargs);
        const size_t A = 256;
        size_t off = 0;
        auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + bytes, A); return o; };
        const size_t o_ws = take(attn_workspace_bytes(hl, c.head_dim, c.max_seq));  // counters first
        const size_t o_st = take(sizeof(DecodeState));
        const size_t o_x = take(H * 4), o_qkv = take((ql + 2 * kvrows) * 4), o_att = take(ql * 4);
        const size_t o_xacc = take(H * 8), o_res0 = take(H * 8), o_res1 = take(H * 8);
        const size_t o_act = take((size_t)il * 4), o_log = take((size_t)vl * 4);
        const size_t o_par = take((size_t)lm_grid * 8);
        const size_t o_pr = take((size_t)c.max_seq * 4), o_tok = take((size_t)(c.max_seq + 1) * 4);
        const size_t o_rope = take((size_t)c.max_seq * c.head_dim * 4);
        const size_t o_qtag = take((size_t)(ql + 2 * kvrows) * 8);
            LLMI_HIP(hipMalloc(&scratch, off));
        LLMI_HIP(hipMemsetAsync(scratch, 0, off, stream));
        attn_ws = scratch + o_ws;
        st = (DecodeState*)(scratch + o_st);
        x = (float*)(scratch + o_x);
        xacc = (long long*)(scratch + o_xacc);
        res[0] = (long long*)(scratch + o_res0);
        res[1] = (long long*)(scratch + o_res1);
        qkv_buf = (float*)(scratch + o_qkv);
        attn_out = (float*)(scratch + o_att);
        act = (float*)(scratch + o_act);
        logits = (float*)(scratch + o_log);
        partials = (unsigned long long*)(scratch + o_par);
        prompt = (int32_t*)(scratch + o_pr);
        tokens = (int32_t*)(scratch + o_tok);
        rope_tab = (float*)(scratch + o_rope);
        qtag = (unsigned long long*)(scratch + o_qtag);  // zeroed: tag 0 never matches (epochs start at 1)
        // cos/sin cache with HF's fp32 arithmetic (LlamaRotaryEmbedding._set_cos_sin_cache):
        // inv_freq = 1 / fp32(base ** (2i/d)) (torch's fp32 pow is correctly rounded),
        // angle = fp32(pos * inv_freq), cos/sin correctly rounded to fp32
        std::vector<float> tab((size_t)c.max_seq * c.head_dim);
        const int half = c.head_dim / 2;
        for (int i = 0; i < half; ++i) {
            const float p = (float)std::pow((double)c.rope_base, (double)(2 * i) / (double)c.head_dim);
            volatile float inv = 1.0f / p;
            for (int pos = 0; pos < c.max_seq; ++pos) {
                volatile float ang = (float)pos * inv;
                tab[((size_t)pos * half + i) * 2 + 0] = (float)std::cos((double)ang);
                tab[((size_t)pos * half + i) * 2 + 1] = (float)std::sin((double)ang);
            }
        }
        LLMI_HIP(hipMemcpyAsync(rope_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice, stream));
        LLMI_HIP(hipStreamSynchronize(stream));
        return LLMI_OK;
    }

    // ----------------------------------------------------------- weights
    // Every copy derived from the weights (the split-3 prefill's e4m3 copies) is dropped
    // before any weight is written; it is rebuilt from the new weights on next use.
    int weights_changed() {
        wdt_valid = false;  // the ring's W_down^T copies are rebuilt before the next ring decode
        if (w8blob) {
            LLMI_HIP(hipStreamSynchronize(stream));  // a prefill may still read them
            LLMI_HIP(hipFree(w8blob));
            w8blob = nullptr;
            w8l.clear();
        }
        return LLMI_OK;
    }

    int load_synthetic(uint64_t sd) {
        LLMI_TRY(weights_changed());
        seed = sd;
        const int H = c.hidden, r = c.tp_rank;
        const int lin = (wdt == LLMI_I8) ? LLMI_SYN_INT8 : LLMI_SYN_LINEAR;
        auto fill = [&](void* dst, size_t row_off, int kind, int dt, uint32_t tid, int rows, int cols, int row0,
                        int col0, int ld) -> int {
            char* p = (char*)dst + row_off * (size_t)cols * dtype_size(dt);
            return synth_fill_launch(p, dt, kind, seed, tid, rows, cols, row0, col0, ld, stream);
        };
        for (int l = 0; l < c.layers; ++l) {
            Layer& L = layers[l];
            auto t = [&](uint32_t k) { return prng::layer_tid(l, k); };
            // fused [q; k; v] rows of this rank's heads (layer_weights.cc:25 order)
            LLMI_TRY(fill(L.qkv, 0, lin, wdt, t(prng::Q), ql, H, r * ql, 0, H));
            LLMI_TRY(fill(L.qkv, ql, lin, wdt, t(prng::K), kvrows, H, r * kvrows, 0, H));
            LLMI_TRY(fill(L.qkv, ql + kvrows, lin, wdt, t(prng::V), kvrows, H, r * kvrows, 0, H));
            // W_o row-major [H, ql] (a head-major layout measured no faster for the
            // split-by-head o_proj)
            LLMI_TRY(fill(L.o, 0, lin, wdt, t(prng::O), H, ql, 0, r * ql, c.heads * c.head_dim));
            // fused [gate; up] rows (layer_weights.cc:40 order)
            LLMI_TRY(fill(L.gu, 0, lin, wdt, t(prng::GATE), il, H, r * il, 0, H));
            LLMI_TRY(fill(L.gu, il, lin, wdt, t(prng::UP), il, H, r * il, 0, H));
            LLMI_TRY(fill(L.down, 0, lin, wdt, t(prng::DOWN), H, il, 0, r * il, c.inter));
            if (wdt == LLMI_I8) {
                const int S = LLMI_SYN_INT8_SCALE;
                LLMI_TRY(fill(L.qkv_s, 0, S, LLMI_F16, t(prng::Q), ql, 1, r * ql, 0, 1));
                LLMI_TRY(fill(L.qkv_s, ql, S, LLMI_F16, t(prng::K), kvrows, 1, r * kvrows, 0, 1));
                LLMI_TRY(fill(L.qkv_s, ql + kvrows, S, LLMI_F16, t(prng::V), kvrows, 1, r * kvrows, 0, 1));
                LLMI_TRY(fill(L.o_s, 0, S, LLMI_F16, t(prng::O), H, 1, 0, 0, 1));
                LLMI_TRY(fill(L.gu_s, 0, S, LLMI_F16, t(prng::GATE), il, 1, r * il, 0, 1));
                LLMI_TRY(fill(L.gu_s, il, S, LLMI_F16, t(prng::UP), il, 1, r * il, 0, 1));
                LLMI_TRY(fill(L.down_s, 0, S, LLMI_F16, t(prng::DOWN), H, 1, 0, 0, 1));
            }
            LLMI_TRY(fill(L.attn_norm, 0, LLMI_SYN_GAMMA, edt, t(prng::ATTN_NORM), 1, H, 0, 0, H));
            LLMI_TRY(fill(L.ffn_norm, 0, LLMI_SYN_GAMMA, edt, t(prng::FFN_NORM), 1, H, 0, 0, H));
        }
        LLMI_TRY(fill(lm_head, 0, LLMI_SYN_LINEAR, edt, prng::LM_HEAD, vl, H, r * vl, 0, H));
        LLMI_TRY(fill(final_norm, 0, LLMI_SYN_GAMMA, edt, prng::FINAL_NORM, 1, H, 0, 0, H));
        LLMI_TRY(fill(embed, 0, LLMI_SYN_EMBED, edt, prng::EMBED, c.vocab, H, 0, 0, H));
        LLMI_HIP(hipStreamSynchronize(stream));
        return LLMI_OK;
    }

    // ------------------------------------------------ weights from the reference's files
    // LlamaWeight<T>::loadWeights / LlamaLayerWeight<T>::loadWeights (llama_weights.cc:41-53,
    // layer_weights.cc:48-66) with loadWeightFromBin<T, float> (weight_utils.cu:90-187): one
    // raw fp32 file per (unsharded) tensor, fused qkv [(heads + 2 kv) * d, H] and gate_up
    // [2 I, H]. The host converts to the engine's dtype (RNE, like the reference's
    // fp32 -> half cast) and copies this rank's slice: q/k/v and gate/up rows, o/down
    // columns, lm_head rows (the layout load_synthetic fills).
    static int put_host(void* dst, int dt, const float* src, size_t src_ld, int rows, int cols, size_t row0,
                        size_t col0, hipStream_t s) {
        const size_t n = (size_t)rows * cols, es = dtype_size(dt);
        std::vector<uint8_t> h(n * es);
        for (int r = 0; r < rows; ++r) {
            const float* a = src + (row0 + r) * src_ld + col0;
            if (dt == LLMI_F32) {
                std::memcpy(h.data() + (size_t)r * cols * 4, a, (size_t)cols * 4);
            } else {
                _Float16* o = reinterpret_cast<_Float16*>(h.data()) + (size_t)r * cols;
                for (int c2 = 0; c2 < cols; ++c2) o[c2] = (_Float16)a[c2];
            }
        }
        LLMI_HIP(hipMemcpyAsync(dst, h.data(), h.size(), hipMemcpyHostToDevice, s));
        LLMI_HIP(hipStreamSynchronize(s));  // h is released on return
        return LLMI_OK;
    }

    // name: the reference's file stem without ".bin" (e.g. "model.layers.3.self_attn.qkv.weight")
    int load_tensor(const char* name, const float* src, size_t count) {
        LLMI_REQUIRE(name && src, "load_tensor: null argument");
        LLMI_TRY(weights_changed());
        const std::string nm(name);
        const size_t H = c.hidden, D = c.head_dim, QR = (size_t)c.heads * D, KR = (size_t)c.kv_heads * D;
        const size_t I = c.inter, r = c.tp_rank;
        auto need = [&](size_t n) -> int {
            if (count != n) {
                set_last_error("[llmi][ERROR] load_tensor: " + nm + " has " + std::to_string(count) + " values, expected " +
                          std::to_string(n));
                return LLMI_EINVAL;
            }
            return LLMI_OK;
        };
        auto lin_ok = [&]() -> int {
            LLMI_REQUIRE(wdt != LLMI_I8, "load_tensor: int8 engines take synthetic weights only "
                                         "(the reference's .bin format is fp32; W8A16 is build-defined)");
            return LLMI_OK;
        };
        if (nm == "model.embed_tokens.weight") {
            LLMI_TRY(need((size_t)c.vocab * H));
            return put_host(embed, edt, src, H, c.vocab, (int)H, 0, 0, stream);
        }
        if (nm == "lm_head.weight") {
            LLMI_TRY(need((size_t)c.vocab * H));
            return put_host(lm_head, edt, src, H, vl, (int)H, r * vl, 0, stream);
        }
        if (nm == "model.norm.weight") {
            LLMI_TRY(need(H));
            return put_host(final_norm, edt, src, H, 1, (int)H, 0, 0, stream);
        }
        const std::string pre = "model.layers.";
        LLMI_REQUIRE(nm.compare(0, pre.size(), pre) == 0, ("load_tensor: unknown tensor " + nm).c_str());
        size_t dot = nm.find('.', pre.size());
        LLMI_REQUIRE(dot != std::string::npos, ("load_tensor: unknown tensor " + nm).c_str());
        const int l = std::atoi(nm.substr(pre.size(), dot - pre.size()).c_str());
        LLMI_REQUIRE(l >= 0 && l < c.layers, ("load_tensor: layer out of range in " + nm).c_str());
        const std::string leaf = nm.substr(dot + 1);
        Layer& L = layers[l];
        const size_t ws = dtype_size(wdt);
        if (leaf == "input_layernorm.weight" || leaf == "post_attention_layernorm.weight") {
            LLMI_TRY(need(H));
            return put_host(leaf[0] == 'i' ? L.attn_norm : L.ffn_norm, edt, src, H, 1, (int)H, 0, 0, stream);
        }
        if (leaf == "self_attn.qkv.weight") {
            LLMI_TRY(lin_ok());
            LLMI_TRY(need((QR + 2 * KR) * H));
            char* d = (char*)L.qkv;
            LLMI_TRY(put_host(d, wdt, src, H, ql, (int)H, r * ql, 0, stream));
            LLMI_TRY(put_host(d + (size_t)ql * H * ws, wdt, src, H, kvrows, (int)H, QR + r * kvrows, 0, stream));
            return put_host(d + (size_t)(ql + kvrows) * H * ws, wdt, src, H, kvrows, (int)H, QR + KR + r * kvrows,
                            0, stream);
        }
        if (leaf == "self_attn.o_proj.weight") {
            LLMI_TRY(lin_ok());
            LLMI_TRY(need(H * QR));
            return put_host(L.o, wdt, src, QR, (int)H, ql, 0, r * ql, stream);
        }
        if (leaf == "mlp.gate_up_proj.weight") {
            LLMI_TRY(lin_ok());
            LLMI_TRY(need(2 * I * H));
            LLMI_TRY(put_host(L.gu, wdt, src, H, il, (int)H, r * il, 0, stream));
            return put_host((char*)L.gu + (size_t)il * H * ws, wdt, src, H, il, (int)H, I + r * il, 0, stream);
        }
        if (leaf == "mlp.down_proj.weight") {
            LLMI_TRY(lin_ok());
            LLMI_TRY(need(H * I));
            return put_host(L.down, wdt, src, I, (int)H, il, 0, r * il, stream);
        }
        set_last_error("[llmi][ERROR] load_tensor: unknown tensor " + nm);
        return LLMI_EINVAL;
    }

    // Llama<T>::loadWeights(weight_path): weight_path + "<name>.bin" for every tensor.
    int load_bin(const char* weight_path) {
        LLMI_REQUIRE(weight_path, "load_bin: null path");
        std::vector<std::string> names = {"model.norm.weight", "lm_head.weight", "model.embed_tokens.weight"};
        for (int l = 0; l < c.layers; ++l)
            for (const char* leaf : {"input_layernorm.weight", "post_attention_layernorm.weight",
                                     "self_attn.qkv.weight", "self_attn.o_proj.weight", "mlp.gate_up_proj.weight",
                                     "mlp.down_proj.weight"})
                names.push_back("model.layers." + std::to_string(l) + "." + leaf);
        std::vector<float> buf;
        for (const std::string& nm : names) {
            const std::string path = std::string(weight_path) + nm + ".bin";
            FILE* f = std::fopen(path.c_str(), "rb");
            if (!f) {
                set_last_error("[llmi][ERROR] load_bin: cannot open " + path);
                return LLMI_EINVAL;
            }
            std::fseek(f, 0, SEEK_END);
            const long bytes = std::ftell(f);
            std::fseek(f, 0, SEEK_SET);
            if (bytes < 0 || bytes % 4 != 0) {
                std::fclose(f);
                set_last_error("[llmi][ERROR] load_bin: " + path + " is not an fp32 file");
                return LLMI_EINVAL;
            }
            buf.resize((size_t)bytes / 4);
            const size_t got = std::fread(buf.data(), 4, buf.size(), f);
            std::fclose(f);
            if (got != buf.size()) {
                set_last_error("[llmi][ERROR] load_bin: short read on " + path);
                return LLMI_EINVAL;
            }
            LLMI_TRY(load_tensor(nm.c_str(), buf.data(), buf.size()));
        }
        return LLMI_OK;
    }

    // ---------------------------------------------------------- one token
    GemvArgs lm_args(bool from_x = false) const {
        GemvArgs a;
        a.stamps = stamp_ptr();
        a.w = lm_head;
        a.w_dtype = edt;
        a.n_rows = vl;
        a.k = c.hidden;
        if (from_x) {
            a.x = x;
        } else {
            a.x_fixed = res[c.layers % 2];  // final residual; fp32 copy to x by workgroup 0
            a.x_out = x;
        }
        a.gamma = final_norm;
        a.g_dtype = edt;
        a.eps = c.rms_eps;
        a.epi = EPI_ARGMAX;
        a.y = logits;
        a.partials = partials;
        a.idx_base = (uint32_t)(c.tp_rank * vl);
        return a;
    }

    // K split inside the workgroup for row-group counts that leave CUs idle or doubled with
    // one group per wave (a TP rank's q/k/v and gate_up): 4 waves per group below one
    // workgroup per CU, 2 below two; TP 1 shapes never qualify (tp_world 1 keeps kpar off so
    // its sums stay bitwise those of the fixtures' runs)
    int kpar_of(int groups) const {
        if (c.tp_world == 1 || kpar_off) return 0;
        // the K-parted kernel stages x for k <= 5120 and splits a row's 16-B chunks evenly
        // (a wider model must fall back to kpar 0, not fail the launch)
        const int epl = wdt == LLMI_I8 ? 16 : wdt == LLMI_F16 ? 8 : 4;
        if (c.hidden > 5120 || c.hidden % epl != 0) return 0;
        const int cus = n_cu > 0 ? n_cu : 256;
        const int blocks = (groups + 3) / 4;
        const int kp = blocks < cus ? 4 : blocks < 2 * cus ? 2 : 0;
        return kp > 0 && (c.hidden / epl) % kp == 0 ? kp : 0;
    }
    bool kpar_off = false;

    GemvArgs qkv_args(int l) const {
        const Layer& L = layers[l];
        GemvArgs a;
        a.stamps = stamp_ptr();
        a.w = L.qkv; a.scales = L.qkv_s; a.w_dtype = wdt;
        a.n_rows = ql + 2 * kvrows; a.k = c.hidden;
        a.x_fixed = res[l % 2]; a.gamma = L.attn_norm; a.g_dtype = edt; a.eps = c.rms_eps;
        a.epi = EPI_STORE; a.y = qkv_buf;
        a.kpar = kpar_of((a.n_rows + 1) / 2);
        return a;
    }
    AttnArgs attn_args(int l) const {
        AttnArgs a;
        a.stamps = stamp_ptr();
        const size_t eb = dtype_size(c.kv_dtype);
        a.qkv = qkv_buf;
        a.k_cache = (char*)kcache + (size_t)l * kv_layer_elems * eb;
        a.v_cache = (char*)vcache + (size_t)l * kv_layer_elems * eb;
        a.cache_dtype = c.kv_dtype;
        a.max_seq = c.max_seq;
        a.pos_dev = &st->cur_pos;
        a.heads = hl; a.kv_heads = kvl; a.head_dim = c.head_dim;
        a.rope = 1; a.rope_base = c.rope_base; a.rope_tab = rope_tab;
        a.direct_out = 0;  // partials -> attn_oproj
        a.xacc = xacc;
        a.resid_fixed = res[l % 2];
        a.resid_scale = (c.tp_rank == 0) ? 1.f : 0.f;  // rank 0 carries the residual into the all-reduce
        a.hidden = c.hidden;
        a.out = attn_out; a.workspace = attn_ws;
        a.nact = rec_nact;
        a.err = &st->error;
        if (seed_from_down()) a.xacc = nullptr;  // layer l - 1's down (layer 0: step_start) seeded xacc already
        return a;
    }
    OprojArgs o_args(int l) const {
        const Layer& L = layers[l];
        OprojArgs a;
        a.stamps = stamp_ptr();
        a.w = L.o; a.scales = L.o_s; a.w_dtype = wdt;
        a.head_major = 0;
        a.n_rows = c.hidden; a.ldw = ql;
        a.heads = hl; a.head_dim = c.head_dim; a.max_seq = c.max_seq;
        a.pos_dev = &st->cur_pos;
        a.workspace = attn_ws; a.xacc = xacc;
        a.nact = rec_nact;
        a.err = &st->error;
        return a;
    }
    GemvArgs gu_args(int l) const {
        const Layer& L = layers[l];
        GemvArgs a;
        a.stamps = stamp_ptr();
        a.w = L.gu; a.scales = L.gu_s; a.w_dtype = wdt;
        a.n_rows = 2 * il; a.k = c.hidden;
        a.x_fixed = xacc;  // residual after attention (fixed point)
        // (no fp32 copy into x here: the lm_head launch writes the final hidden state there, and
        // nothing reads a mid-layer copy -- it was 16 KB of stores on workgroup 0 every layer;
        // LLMI_GU_XOUT=1 restores it for A/B)
        if (LLMI_GU_XOUT) a.x_out = x;
        // hand the mid-layer residual to the layer output accumulator (rank 0 carries it) --
        // unless the down GEMV writes each output row itself (down_single)
        if (!down_single()) {
            a.seed_src = xacc; a.seed_dst = res[(l + 1) % 2]; a.seed_n = c.hidden;
            a.seed_keep = c.tp_rank == 0 ? 1 : 0;
        }
        a.gamma = L.ffn_norm; a.g_dtype = edt; a.eps = c.rms_eps;
        a.epi = EPI_SILU_MUL; a.pair_off = il; a.y = act;
        a.kpar = kpar_of(il);
        return a;
    }
    GemvArgs down_args(int l) const {
        const Layer& L = layers[l];
        GemvArgs a;
        a.stamps = stamp_ptr();
        a.w = L.down; a.scales = L.down_s; a.w_dtype = wdt;
        a.n_rows = c.hidden; a.k = il; a.x = act;
        a.epi = EPI_ATOMIC; a.yacc = res[(l + 1) % 2];
        // int8 rows are half the bytes of fp16 ones: K slices keep the loads per row in
        // flight and the x image per workgroup small (exact: int64 atomics)
        a.ksplit = down_ksplit();
        if (down_single()) {  // one producer per row: x_{l+1}[r] = xmid[r] + fixed(down_r), no seed, no atomic
            a.yacc_single = 1;
            a.yacc_base = c.tp_rank == 0 ? xacc : nullptr;  // the other TP ranks carry no residual
            // single rank: the same row also seeds the next layer's o_proj sum (xacc), so that
            // layer's attention writes no seed (seed_from_down)
            if (seed_from_down()) a.yacc_copy = xacc;
        }
        return a;
    }
    int down_ksplit() const {
        return (wdt == LLMI_I8 && il % (16 * LLMI_I8_DOWN_KSPLIT) == 0) ? LLMI_I8_DOWN_KSPLIT
               : (wdt == LLMI_F16 && il % (8 * LLMI_F16_DOWN_KSPLIT) == 0) ? LLMI_F16_DOWN_KSPLIT
                                                                           : 1;
    }
    // the down GEMV writes its rows itself (LLMI_DOWN_STORE; round 6) when K is not split
    bool down_single() const { return LLMI_DOWN_STORE && down_ksplit() == 1; }
    // ... and on a single rank also the next layer's o_proj seed (with TP the seed must be the
    // all-reduced residual, which only exists after the exchange)
    bool seed_from_down() const { return LLMI_SEED_FROM_DOWN && down_single() && c.tp_world == 1 && !grouped; }


    // One token = start, L x (attention phase | reduce xacc, ffn phase | reduce x),
    // head | reduce partials. The phases are separate so that an in-process
    // group (struct Group) can interleave its ranks between the reductions.
    int rec_start() {
        return step_start_launch(st, prompt, partials, lm_grid, tokens, embed, edt, c.hidden, x, res[0], c.max_seq,
                                 nullptr, 0, stream, seed_from_down() ? xacc : nullptr);
    }
    int rec_attn(int l) {
        GemvArgs q = qkv_args(l);
        AttnArgs at = attn_args(l);
        if (qa_fuse && qtag && l < 128) {
            GemvArgs qf = q;
            qf.kpar = 0;  // the fused GEMV part streams a row group per wave (kpar: +0.3 % alone at TP 8)
            qf.y_tag = qtag; qf.tag_epoch = &st->epoch; qf.tag_layer = (unsigned)l;
            AttnArgs af = at;
            af.qkv_tag = qtag; af.tag_epoch = &st->epoch; af.tag_layer = (unsigned)l;
            OprojArgs o = o_args(l);
            if (qa_o && !tail_mode && qkv_attn_o_supported(qf, af, o))  // q/k/v, attention and o_proj: one launch
                return qkv_attn_o_launch(qf, af, &o, stream);
            if (qkv_attn_supported(qf, af)) return rec_oproj(qkv_attn_launch(qf, af, stream), o);  // one launch
            return rec_oproj(gemv_launch(q, stream), o, &at);
        }
        LLMI_TRY(gemv_launch(q, stream));
        return rec_oproj(LLMI_OK, o_args(l), &at);
    }
    // the layer's o_proj launch (after the attention launch when `at` is given)
    int rec_oproj(int prev, OprojArgs o, const AttnArgs* at = nullptr) {
        LLMI_TRY(prev);
        if (at) LLMI_TRY(attn_decode_launch(*at, stream));
        if (tail_mode) {  // the o_proj launch pushes (and reduces) xacc itself
            o.xt = xchg_args(xacc, c.hidden, 0, tail_mode);
            o.xt_cnt = xt_cnt;
        }
        return attn_oproj_launch(o, stream);
    }
    int rec_ffn(int l) {
        LLMI_TRY(gemv_launch(gu_args(l), stream));
        GemvArgs d = down_args(l);
        if (tail_mode) {  // the down launch pushes (and reduces) the layer output itself
            d.xt = xchg_args(res[(l + 1) % 2], c.hidden, 0, tail_mode);
            d.xt_cnt = xt_cnt;
        }
        return gemv_launch(d, stream);
    }
    int rec_head(bool from_x = false) {
        GemvArgs h = lm_args(from_x);
        if (tail_mode) {  // the lm_head launch max-reduces the argmax keys itself
            h.xt = xchg_args(partials, lm_grid, 2, tail_mode);
            h.xt_cnt = xt_cnt;
        }
        LLMI_TRY(gemv_launch(h, stream));
        if (sample_k == 0) return LLMI_OK;
        // top-K of this token's logits, then the sampled id replaces the argmax partials
        LLMI_TRY(topk_launch(logits, LLMI_F32, 1, c.vocab, sample_k, samp_ids, samp_vals, stream));
        return sample_pick_launch(st, samp_ids, samp_vals, sample_k, sample_seed, partials, lm_grid, stream);
    }

    // ------------------------------------------------- TP exchange (config 4)
    // The per-token collectives: int64 sum of the residual partials (op 0) or uint64 max of
    // the argmax keys (op 2), over RCCL or the one-shot peer exchange.
    int alloc_xchg() {
        if (inbox) return LLMI_OK;
        const int W = c.tp_world;
        LLMI_REQUIRE(W <= kXchgMaxWorld, "xchg: the one-shot exchange takes at most 8 ranks");
        xchg_cap_n = std::max(c.hidden, lm_grid);
        xchg_cap_n += xchg_cap_n & 1;
        LLMI_REQUIRE(xchg_cap_n <= kXchgSlice * kXchgMaxSlices, "xchg: hidden / lm_head partials exceed the inbox");
        const size_t bytes = xchg_inbox_bytes(W, xchg_cap_n);
        LLMI_HIP(hipExtMallocWithFlags(reinterpret_cast<void**>(&inbox), bytes, hipDeviceMallocUncached));
        LLMI_HIP(hipMemset(inbox, 0, bytes));
        LLMI_HIP(hipMalloc(&xchg_ep, kXchgMaxSlices * sizeof(unsigned long long)));
        LLMI_HIP(hipMemset(xchg_ep, 0, kXchgMaxSlices * sizeof(unsigned long long)));
        LLMI_HIP(hipMalloc(&peers_dev, (size_t)W * sizeof(char*)));
        LLMI_HIP(hipMalloc(&xt_cnt, xchg_detail::kTailWords * sizeof(unsigned)));
        LLMI_HIP(hipMemset(xt_cnt, 0, xchg_detail::kTailWords * sizeof(unsigned)));
        return LLMI_OK;
    }
    // every rank's inbox base, in rank order (peers[rank] must be this rank's own inbox)
    int set_peers(const std::vector<char*>& p) {
        LLMI_REQUIRE((int)p.size() == c.tp_world && p[c.tp_rank] == inbox, "xchg: bad peer table");
        LLMI_HIP(hipMemcpy(peers_dev, p.data(), p.size() * sizeof(char*), hipMemcpyHostToDevice));
        return LLMI_OK;
    }
    XchgArgs xchg_args(void* buf, int n, int op, int mode) const {
        XchgArgs a;
        a.buf = static_cast<long long*>(buf);
        a.n = n;
        a.op = op;
        a.rank = c.tp_rank;
        a.world = c.tp_world;
        a.peers = peers_dev;
        a.ep = xchg_ep;
        a.err = &st->error;
        a.mode = mode;
        a.cap_n = xchg_cap_n;
        a.cap_w = c.tp_world;
        a.loop = xchg_loop;
        return a;
    }
    int exchange(void* buf, int n, int op) {
        if (xchg_mode == 1) return xchg_launch(xchg_args(buf, n, op, 3), stream);
        if (xchg_mode == 2) return LLMI_OK;  // the producing launch's tail did it
        if (!comm) return LLMI_OK;
        const ncclResult_t r = op == 0 ? ncclAllReduce(buf, buf, n, ncclInt64, ncclSum, comm, stream)
                                       : ncclAllReduce(buf, buf, n, ncclUint64, ncclMax, comm, stream);
        LLMI_REQUIRE(r == ncclSuccess, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
        return LLMI_OK;
    }
    int set_exchange(int mode) {
        LLMI_REQUIRE(mode >= 0 && mode <= 2,
                     "set_exchange: mode must be 0 (RCCL), 1 (one-shot peer exchange) or 2 (fused into the producers)");
        LLMI_REQUIRE(!grouped, "set_exchange: a group rank's exchange is its group's");
        LLMI_REQUIRE(mode == 0 || (inbox && peers_ready), "set_exchange: open the peer exchange first (xchg_open)");
        LLMI_HIP(hipStreamSynchronize(stream));
        graphs.clear();  // the captured steps change
        xchg_mode = mode;
        tail_mode = mode == 2 ? 3 : 0;
        return LLMI_OK;
    }
    int set_option(const std::string& name, int value) {
        LLMI_HIP(hipStreamSynchronize(stream));
        if (name == "kpar") {
            LLMI_REQUIRE(value == 0 || value == 1, "set_option kpar: 1 on (default), 0 off");
            kpar_off = value == 0;
        } else if (name == "qkv_attn") {
            LLMI_REQUIRE(value == 0 || value == 1, "set_option qkv_attn: 1 one q/k/v + attention launch, 0 two");
            qa_fuse = value == 1;
        } else if (name == "qa_grid") {
            LLMI_REQUIRE(value >= 0, "set_option qa_grid: workgroups of the fused launch's GEMV part (0 = all resident)");
            qkv_attn_set_grid(value);
        } else if (name == "qa_o") {
            qa_o = value != 0;
        } else if (name == "qa_order") {
            qkv_attn_set_order(value);
        } else if (name == "qa_poll") {
            qkv_attn_set_poll(value);
        } else {
            LLMI_REQUIRE(false, "set_option: unknown option (kpar, qkv_attn, qa_o, qa_grid, qa_order, qa_poll)");
        }
        graphs.clear();  // the captured steps change
        return LLMI_OK;
    }
    bool peers_ready = false;
    int xchg_loop = 0;  // llmi_engine_xchg_loopback: one rank alone, every peer its own inbox

    int set_sampling(int k, uint64_t sd) {
        LLMI_REQUIRE(k >= 0 && k <= 16, "set_sampling: k must be in [0, 16] (0 = greedy)");
        LLMI_REQUIRE(k == 0 || (c.tp_world == 1 && !grouped), "set_sampling: sampling needs the full logits (tp_world 1)");
        if (k > 0 && !samp_ids) {
            LLMI_HIP(hipMalloc(&samp_ids, 16 * sizeof(int32_t)));
            LLMI_HIP(hipMalloc(&samp_vals, 16 * sizeof(float)));
        }
        if (!graphs.empty()) {  // the captured step changes: re-capture on the next graph decode
            LLMI_HIP(hipStreamSynchronize(stream));  // a replay may still be in flight
            graphs.clear();
        }
        sample_k = k;
        sample_seed = sd;
        return LLMI_OK;
    }

    // ------------------------------------------------ persistent ring layer (mode 1)
    bool ring_ok() const {
        // layers >= 2: a launch zeroes the NEXT launch's counter block ((l + 1) % L), which for
        // one layer would be its own, while its workgroups arrive on it
        return wdt == LLMI_F16 && edt == LLMI_F16 && c.tp_world == 1 && !grouped && c.layers >= 2 &&
               ring_supported(c.hidden, hl, c.head_dim, il, ql + 2 * kvrows, n_cu);
    }
    int set_decode_mode(int mode) {
        LLMI_REQUIRE(mode == 0 || mode == 1, "set_decode_mode: mode must be 0 (launches) or 1 (ring layer)");
        LLMI_HIP(hipStreamSynchronize(stream));
        if (mode == 1) {
            if (n_cu == 0) LLMI_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device));
            if (!ring_ok()) {
                set_last_error("[llmi][ERROR] set_decode_mode: the ring layer needs fp16 weights, hidden 4096, "
                               "head_dim 128, heads dividing the CU count, tp_world 1, >= 2 layers");
                return LLMI_EUNSUPPORTED;
            }
            int per_cu = 0;
            LLMI_TRY(ring_residency(&per_cu));
            LLMI_REQUIRE(per_cu >= 1, "set_decode_mode: the ring layer's workgroup does not fit a CU");
            if (!rl_acc) {
                LLMI_HIP(hipMalloc(&rl_acc, (size_t)5 * c.hidden * 8));
                LLMI_HIP(hipMalloc(&rl_cnt, (size_t)c.layers * kRingCntWords * 4));
                LLMI_HIP(hipMalloc(&wdt_blob, (size_t)c.layers * il * c.hidden * 2));
            }
            LLMI_HIP(hipMemset(rl_acc, 0, (size_t)5 * c.hidden * 8));
            LLMI_HIP(hipMemset(rl_cnt, 0, (size_t)c.layers * kRingCntWords * 4));
        }
        graphs.clear();  // the captured steps change
        decode_mode = mode;
        return LLMI_OK;
    }
    int prepare_ring() {  // W_down^T of every layer, from the current weights
        if (wdt_valid) return LLMI_OK;
        for (int l = 0; l < c.layers; ++l) LLMI_TRY(transpose_f16_launch(layers[l].down, wdt_of(l), c.hidden, il, stream));
        LLMI_HIP(hipStreamSynchronize(stream));
        wdt_valid = true;
        return LLMI_OK;
    }
    // ring launch of layer l; wrap: the timing loop's cyclic form (every launch has a
    // q/k/v phase and prepares layer (l + 1) % L's state)
    RingArgs ring_args(int l, bool wrap = false) const {
        const int L = c.layers;
        const bool next = l + 1 < L || wrap;
        const Layer& Lw = layers[l];
        RingArgs r;
        r.w_o = Lw.o; r.w_gu = Lw.gu; r.w_dt = wdt_of(l); r.g_ffn = Lw.ffn_norm;
        if (next) {
            r.w_qkv = layers[(l + 1) % L].qkv;
            r.g_attn = layers[(l + 1) % L].attn_norm;
            r.qkv_out = qkv_buf;
        }
        r.attn_ws = attn_ws;
        r.acc_x = acc_a(l); r.acc_mid = acc_b(l); r.acc_out = acc_a(l + 1);
        r.zero0 = next ? acc_b(l + 1) : nullptr;
        r.zero1 = (l + 2 <= L || wrap) ? acc_a(l + 2) : nullptr;
        r.cnt = rl_cnt + (size_t)l * kRingCntWords;
        r.cnt_zero = rl_cnt + (size_t)((l + 1) % L) * kRingCntWords;
        r.hidden = c.hidden; r.heads = hl; r.inter = il; r.n_qkv = ql + 2 * kvrows; r.max_seq = c.max_seq;
        r.nact = rec_nact; r.eps = c.rms_eps; r.err = &st->error;
        r.stamps = stamp_ptr();
        return r;
    }
    int record_step_ring() {
        dbg_slot = 0;
        // step_start: x_0 into slot A0, zero A1 + B0 (adjacent) for layer 0's sums
        LLMI_TRY(step_start_launch(st, prompt, partials, lm_grid, tokens, embed, edt, c.hidden, x, acc_a(0), c.max_seq,
                                   reinterpret_cast<unsigned*>(acc_a(1)), 4 * c.hidden, stream));
        GemvArgs q = qkv_args(0);
        q.x_fixed = acc_a(0);
        LLMI_TRY(gemv_launch(q, stream));
        for (int l = 0; l < c.layers; ++l) {
            AttnArgs at = attn_args(l);
            at.xacc = nullptr;  // the ring seeds the o_proj sum itself
            LLMI_TRY(attn_decode_launch(at, stream));
            LLMI_TRY(ring_layer_launch(ring_args(l), n_cu, stream));
        }
        GemvArgs h = lm_args();
        h.x_fixed = acc_a(c.layers);
        LLMI_TRY(gemv_launch(h, stream));
        if (sample_k == 0) return LLMI_OK;
        LLMI_TRY(topk_launch(logits, LLMI_F32, 1, c.vocab, sample_k, samp_ids, samp_vals, stream));
        return sample_pick_launch(st, samp_ids, samp_vals, sample_k, sample_seed, partials, lm_grid, stream);
    }

    int record_step() {
        LLMI_REQUIRE(!grouped, "engine: a group rank is stepped by its group");
        if (decode_mode == 1) return record_step_ring();
        dbg_slot = 0;
        LLMI_TRY(rec_start());
        for (int l = 0; l < c.layers; ++l) {
            LLMI_TRY(rec_attn(l));
            LLMI_TRY(exchange(xacc, c.hidden, 0));  // exact int64 sum of the fixed-point residual partials
            LLMI_TRY(rec_ffn(l));
            LLMI_TRY(exchange(res[(l + 1) % 2], c.hidden, 0));  // layer output (rank 0 carried the residual)
        }
        LLMI_TRY(rec_head());
        return exchange(partials, lm_grid, 2);  // max of the vocab-parallel argmax keys
    }

    static int nact_of(int pos) { return pos / kAttnChunk + 1; }
    int build_graph(int nact) {
        rec_nact = nact;
        return graphs.build(nact, stream, [&]() { return record_step(); });
    }

    // ------------------------------------------------------------- driving
    int set_prompt(const int32_t* ids, int n) {
        LLMI_REQUIRE(ids && n >= 1 && n <= c.max_seq, "set_prompt: need 1 <= n <= max_seq ids");
        for (int i = 0; i < n; ++i)
            LLMI_REQUIRE(ids[i] >= 0 && ids[i] < c.vocab, "set_prompt: token id out of range");
        DecodeState h{};
        h.next_pos = 0;
        h.cur_pos = 0;
        h.prompt_len = n;
        h.vocab = c.vocab;
        h.error = 0;
        LLMI_HIP(hipMemcpyAsync(prompt, ids, (size_t)n * 4, hipMemcpyHostToDevice, stream));
        // (the epoch and what follows it are left alone: the fused q/k/v launch's granule tags
        // must never repeat the tag its buffer already holds, across prompts too)
        LLMI_HIP(hipMemcpyAsync(st, &h, offsetof(DecodeState, epoch), hipMemcpyHostToDevice, stream));
        LLMI_HIP(hipStreamSynchronize(stream));
        host_next_pos = 0;
        prompt_len = n;
        return LLMI_OK;
    }

    int decode(int n, int use_graph) {
        LLMI_REQUIRE(prompt_len > 0, "decode: set_prompt first");
        LLMI_REQUIRE(c.tp_world == 1 || comm || xchg_mode >= 1 || xchg_loop,
                     "decode: tp_world > 1 needs an RCCL id at create or the one-shot exchange (xchg_open + set_exchange)");
        LLMI_REQUIRE(n >= 0 && host_next_pos + n <= c.max_seq, "decode: would run past max_seq");
        if (decode_mode == 1 && n > 0) LLMI_TRY(prepare_ring());
        if (use_graph && n > 0)  // every graph this run replays, captured before the first launch
            for (int k = nact_of(host_next_pos); k <= nact_of(host_next_pos + n - 1); ++k) LLMI_TRY(build_graph(k));
        for (int i = 0; i < n; ++i) {
            const int k = nact_of(host_next_pos + i);
            if (use_graph) {
                LLMI_HIP(hipGraphLaunch(graphs.x[k], stream));
            } else {
                rec_nact = k;
                LLMI_TRY(record_step());
            }
        }
        host_next_pos += n;
        return LLMI_OK;
    }

    // ------------------------------------------------------------ prefill
    // Llama<T>::firstTokenGen (llama.cpp:273-316) / LlamaContextDecoder::forward
    // (context_decoder.cpp:47-143): prompt rows [p0, p0 + n) in chunks of up to
    // kPrefillRows through the MFMA GEMMs and the causal prefill attention, KV
    // slots written; then the last row's final norm + lm_head + argmax, leaving
    // the decode state exactly where n decode steps would have left it.
    static constexpr int kPrefillRows = 512;

    int alloc_prefill() {
        if (pf) return LLMI_OK;
        pf_rows = std::min(kPrefillRows, c.max_seq);
        const size_t R = pf_rows, A = 256;
        size_t off = 0;
        auto take = [&](size_t bytes) { size_t o = off; off = align_up(off + bytes, A); return o; };
        // qkv: two K slices of the gemm3 GEMM, summed by the rope kernel into slice 0
        const size_t ox = take(R * c.hidden * 4), oq = take(2 * R * (ql + 2 * kvrows) * 4), oo = take(R * ql * 4),
                     oa = take(R * il * 4);
        const size_t wide = std::max<size_t>(std::max<size_t>(c.hidden, ql), il);
        const size_t oh = take(R * wide * 2), ol = take(R * wide * 2), os = take(kPfSlabs * R * c.hidden * 4);
        // split-key attention partials: [heads][R / 64][8 chunks][64 x 128 + 128] fp32
        pf_split_floats = (size_t)hl * ((R + 63) / 64) * 8 * (64 * 128 + 128);
        const size_t osp = take(pf_split_floats * 4);
        LLMI_HIP(hipMalloc(&pf, off));
        pf_slab = (float*)(pf + os);
        pf_split = (float*)(pf + osp);
        pf_ah = (_Float16*)(pf + oh);
        pf_al = (_Float16*)(pf + ol);
        pf_x = (float*)(pf + ox);
        pf_qkv = (float*)(pf + oq);
        pf_o = (float*)(pf + oo);
        pf_act = (float*)(pf + oa);
        LLMI_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device));
        return LLMI_OK;
    }
    // split mode 3's gate_up on every CU (gemm3_silu_bal_kernel): lo partial slots + flags,
    // allocated on the first split-3 prefill (~88 MB at 7B; the other modes never read them)
    int alloc_bal() {
        if (pf_bal) return LLMI_OK;
        const size_t sb = gemm3_bal_slab_bytes(pf_rows, 2 * il);
        if (sb > 0) {
            const size_t nflags = sb / ((size_t)256 * 256 * 4);  // two slots per tile, one flag each
            LLMI_HIP(hipMalloc(&pf_bal, sb));
            LLMI_HIP(hipMalloc(&pf_bal_flags, nflags * sizeof(unsigned)));
            LLMI_HIP(hipMemset(pf_bal_flags, 0, nflags * sizeof(unsigned)));
        }
        return LLMI_OK;
    }

    // split mode 3 needs the fp8 lo pass of gemm3 on all four GEMMs (K multiples of 128)
    bool lo8_supported() const {
        return wdt == LLMI_F16 && c.kv_dtype == LLMI_F16 && gemm3_supported(ql + 2 * kvrows, c.hidden, EPI_SLAB, 2) &&
               gemm3_supported(c.hidden, ql, EPI_SLAB, kPfDown) && gemm3_supported(2 * il, c.hidden, EPI_SILU_MUL, 1) &&
               gemm3_supported(c.hidden, il, EPI_SLAB, kPfDown) && c.hidden % 128 == 0 && ql % 128 == 0 &&
               il % 128 == 0 && ql / 128 >= kPfDown && il / 128 >= kPfDown;
    }
    int alloc_w8() {
        if (w8blob) return LLMI_OK;
        // e4m3 rows keep the fp16 row stride (2 K bytes, the first K used: gemm3.hip)
        const int H = c.hidden;
        const size_t nq = (size_t)(ql + 2 * kvrows) * H * 2, no = (size_t)H * ql * 2, ng = (size_t)2 * il * H * 2,
                     nd = (size_t)H * il * 2;
        auto al = [](size_t b) { return align_up(b, 256); };
        const size_t per = al(nq) + al(no) + al(ng) + al(nd);
        LLMI_HIP(hipMalloc(&w8blob, per * layers.size()));
        w8l.assign(layers.size(), W8Layer{});
        for (size_t l = 0; l < layers.size(); ++l) {
            char* p = w8blob + l * per;
            W8Layer& w = w8l[l];
            w.qkv = p; p += al(nq);
            w.o = p; p += al(no);
            w.gu = p; p += al(ng);
            w.down = p;
            LLMI_TRY(w8_prepare(layers[l].qkv, ql + 2 * kvrows, H, w.qkv, &w.qkv_e, stream));
            LLMI_TRY(w8_prepare(layers[l].o, H, ql, w.o, &w.o_e, stream));
            LLMI_TRY(w8_prepare(layers[l].gu, 2 * il, H, w.gu, &w.gu_e, stream));
            LLMI_TRY(w8_prepare(layers[l].down, H, il, w.down, &w.down_e, stream));
        }
        LLMI_HIP(hipStreamSynchronize(stream));
        return LLMI_OK;
    }

    // One prefill layer on the LDS-DMA GEMM (gemm2.hip): RMSNorm + split into fp16
    // planes, q/k/v GEMM, rope + KV write + causal attention, split, o_proj (+residual),
    // RMSNorm + split, gate_up GEMM writing silu(g) * u as planes, down (+residual).
    int prefill_layer_gemm2(int l, int m, int p0, int split) {
        const Layer& L = layers[l];
        const int H = c.hidden;
        const size_t eb = dtype_size(c.kv_dtype);
        // split 3: the lo planes are e4m3 bytes against the e4m3 weight copies (gemm3.hip)
        const bool f8 = split == 3;
        const W8Layer* W8 = f8 ? &w8l[l] : nullptr;
        _Float16* lo = split >= 2 ? pf_al : nullptr;
        Gemm2Args g;
        g.a[0] = pf_ah; g.a[1] = lo; g.planes = split >= 2 ? 2 : 1; g.m = m; g.lo8 = f8 ? 1 : 0;
        // (previous down slices into x) + rmsnorm + qkv
        LLMI_TRY(rows_split_launch(pf_x, H, m, H, L.attn_norm, edt, c.rms_eps, pf_ah, lo, H, stream,
                                   pf_pending ? pf_slab : nullptr, pf_pending, f8));
        pf_pending = 0;
        g.lda = H; g.w = L.qkv; g.n = ql + 2 * kvrows; g.k = H;
        g.ldy = g.n;
        if (f8) { g.w8 = W8->qkv; g.w8_exp = W8->qkv_e; }
        const bool qkv3 = gemm3_supported(g.n, H, EPI_SLAB, 2);
        if (qkv3) {  // two K slices (96 tiles alone would leave most CUs idle)
            g.epi = EPI_SLAB; g.ksplit = 2; g.slab = pf_qkv;
            LLMI_TRY(gemm3_launch(g, stream));
        } else {
            g.epi = EPI_STORE; g.y = pf_qkv;
            LLMI_TRY(gemm2_launch(g, stream));
        }
        // rope (+ the second qkv slice) + kv write + causal attention
        PrefillAttnArgs pa;
        pa.qkv = pf_qkv;
        pa.qkv2 = qkv3 ? pf_qkv + (size_t)m * g.n : nullptr;
        pa.k_cache = (char*)kcache + (size_t)l * kv_layer_elems * eb;
        pa.v_cache = (char*)vcache + (size_t)l * kv_layer_elems * eb;
        pa.cache_dtype = c.kv_dtype; pa.max_seq = c.max_seq; pa.m = m; pa.p0 = p0;
        pa.heads = hl; pa.kv_heads = kvl; pa.head_dim = c.head_dim; pa.rope_tab = rope_tab; pa.out = pf_o;
        if (c.kv_dtype == LLMI_F16) {  // MFMA attention writes the o_proj input planes itself
            pa.mfma_planes = split >= 2 ? 2 : 1; pa.out_hi = pf_ah; pa.out_lo = lo; pa.out_lo8 = f8 ? 1 : 0;
            pa.split_ws = pf_split; pa.split_ws_floats = pf_split_floats;
        }
        LLMI_TRY(prefill_attn_launch(pa, stream));
        // o_proj + residual
        if (c.kv_dtype != LLMI_F16)
            LLMI_TRY(rows_split_launch(pf_o, ql, m, ql, nullptr, edt, 0.f, pf_ah, lo, ql, stream, nullptr, 0, f8));
        // split-K into slabs (128 tiles alone would leave half the CUs idle); the next
        // rows_split adds the slices into x in slice order (deterministic). The fp8 lo
        // pass is gemm3's: 8 slices of 256 x 256 tiles (256 workgroups)
        int so = (ql % (kPfSplit * 64)) == 0 ? kPfSplit : 1;
        g.lda = ql; g.w = L.o; g.w_kblock = 0; g.n = H; g.k = ql;
        g.epi = EPI_SLAB; g.ksplit = so; g.slab = pf_slab; g.y = pf_x; g.ldy = H;
        static const bool o3 = [] {  // A/B: LLMI_PF_O3=1 puts the fp16 o_proj on gemm3 (8 K slices) too; measured
                                     // 0.1 ms slower a 7B prefill than gemm2's 2 slices (r07l), so gemm2 stays
            const char* e = std::getenv("LLMI_PF_O3");
            return e && std::string(e) == "1";
        }();
        if (f8) {
            so = kPfDown; g.ksplit = so; g.w8 = W8->o; g.w8_exp = W8->o_e;
            LLMI_TRY(gemm3_launch(g, stream));
        } else if (o3 && gemm3_supported(H, ql, EPI_SLAB, kPfDown)) {
            so = kPfDown; g.ksplit = so;
            LLMI_TRY(gemm3_launch(g, stream));
        } else {
            LLMI_TRY(gemm2_launch(g, stream));
        }
        g.w_kblock = 0;
        // (o slices into x) + rmsnorm + gate_up + silu * up -> planes of the down GEMM's input
        LLMI_TRY(rows_split_launch(pf_x, H, m, H, L.ffn_norm, edt, c.rms_eps, pf_ah, lo, H, stream, pf_slab, so, f8));
        g.lda = H; g.w = L.gu; g.n = 2 * il; g.k = H;
        static const bool sk_f8 = [] {  // fp8-lo gate_up: stream-K (LLMI_SK_F8=0: the lo-pass balance)
            const char* e = std::getenv("LLMI_SK_F8");
            return !(e && std::string(e) == "0");
        }();
        if (f8) {  // + the fp8 lo pass spread over the CUs its 256 x 256 tiles leave idle (the
                   // fp16 lo pass balanced the same way measured 231 vs 225 us: not used)
            g.w8 = W8->gu; g.w8_exp = W8->gu_e;
            if (!sk_f8) { g.bal_slab = pf_bal; g.bal_flags = pf_bal_flags; g.bal_grid = n_cu; }
            g.err = &st->error;
        }
        g.epi = EPI_SILU_MUL; g.pair_off = il; g.y = nullptr; g.y_hi = pf_act_h(); g.y_lo = split >= 2 ? pf_act_l() : nullptr;
        g.ldy = il;
        g.sk_slab = nullptr; g.sk_flags = nullptr; g.sk_grid = 0;
        // the whole K work of gate_up's 172 tiles spread evenly over every CU (gemm3 stream-K)
        if (gemm3_supported(g.n, H, EPI_SILU_MUL, 1) && (!f8 || sk_f8)) {
            g.err = &st->error;
            (void)gemm3_sk_attach(g, stream);
        }
        LLMI_TRY(gemm3_supported(g.n, H, EPI_SILU_MUL, 1) ? gemm3_launch(g, stream) : gemm2_launch(g, stream));
        // down + residual: K slices into slabs (gemm3: 8 uneven slices, 256 workgroups)
        g.bal_slab = nullptr; g.bal_flags = nullptr;
        g.sk_slab = nullptr; g.sk_flags = nullptr; g.sk_grid = 0;
        g.a[0] = pf_act_h(); g.a[1] = split >= 2 ? pf_act_l() : nullptr;
        g.lda = il; g.w = L.down; g.n = H; g.k = il;
        if (f8) { g.w8 = W8->down; g.w8_exp = W8->down_e; }
        g.epi = EPI_SLAB; g.pair_off = 0; g.y = pf_x; g.y_hi = g.y_lo = nullptr; g.ldy = H; g.slab = pf_slab;
        int sd;
        if (gemm3_supported(H, il, EPI_SLAB, kPfDown)) {
            sd = kPfDown; g.ksplit = sd;
            LLMI_TRY(gemm3_launch(g, stream));
        } else {
            sd = (il % (kPfSplit * 64)) == 0 ? kPfSplit : 1; g.ksplit = sd;
            LLMI_TRY(gemm2_launch(g, stream));
        }
        pf_pending = sd;  // added by the next layer's rows_split (or prefill_flush)
        return LLMI_OK;
    }
    int prefill_flush(int m) {  // pending down slices into x (after the last layer)
        if (!pf_pending) return LLMI_OK;
        LLMI_TRY(rows_split_launch(pf_x, c.hidden, m, c.hidden, nullptr, edt, 0.f, nullptr, nullptr, c.hidden, stream,
                                   pf_slab, pf_pending));
        pf_pending = 0;
        return LLMI_OK;
    }
    // the SiLU output planes reuse pf_act's bytes (fp32 [R, il] = two fp16 planes)
    _Float16* pf_act_h() { return reinterpret_cast<_Float16*>(pf_act); }
    _Float16* pf_act_l() { return reinterpret_cast<_Float16*>(pf_act) + (size_t)pf_rows * il; }

    int prefill(int n, int split) {
        LLMI_REQUIRE(!grouped && c.tp_world == 1, "prefill: tensor-parallel prefill is not supported");
        LLMI_REQUIRE(prompt_len > 0, "prefill: set_prompt first");
        LLMI_REQUIRE(n >= 1 && host_next_pos + n <= prompt_len, "prefill: rows must lie inside the prompt");
        LLMI_REQUIRE(split >= 1 && split <= 3,
                     "prefill: split must be 1 (fp16 A), 2 (fp32-faithful) or 3 (fp16 hi + fp8 lo planes)");
        if (!gemm_supported(wdt, ql + 2 * kvrows, c.hidden, EPI_STORE) || !gemm_supported(wdt, c.hidden, ql, EPI_ADD) ||
            !gemm_supported(wdt, 2 * il, c.hidden, EPI_SILU_MUL) || !gemm_supported(wdt, c.hidden, il, EPI_ADD))
            return decode(n, 1);  // fp32 weights / odd shapes: the decode kernels, one row at a time
        LLMI_TRY(alloc_prefill());
        const bool use_gemm2 = wdt == LLMI_F16 && gemm2_supported(ql + 2 * kvrows, c.hidden, EPI_STORE) &&
                               gemm2_supported(c.hidden, ql, EPI_ADD) && gemm2_supported(2 * il, c.hidden, EPI_SILU_MUL) &&
                               gemm2_supported(c.hidden, il, EPI_ADD) && c.head_dim % 64 == 0;
        if (split == 3 && !(use_gemm2 && lo8_supported())) split = 2;  // shapes without the fp8 lo pass: exact planes
        if (split == 3) {
            LLMI_TRY(alloc_w8());
            LLMI_TRY(alloc_bal());
        }
        const int H = c.hidden, p_begin = host_next_pos;
        const size_t eb = dtype_size(c.kv_dtype);
        for (int p0 = p_begin; p0 < p_begin + n; p0 += pf_rows) {
            const int m = std::min(pf_rows, p_begin + n - p0);
            LLMI_TRY(embedding_launch(prompt + p0, m, embed, edt, c.vocab, H, pf_x, stream));
            for (int l = 0; l < c.layers; ++l) {
                const Layer& L = layers[l];
                if (use_gemm2) {
                    LLMI_TRY(prefill_layer_gemm2(l, m, p0, split));
                    continue;
                }
                GemmArgs g;
                g.split = split == 3 ? 2 : split;
                g.w_dtype = wdt;
                g.m = m;
                // rmsnorm + qkv
                g.a = pf_x; g.lda = H; g.gamma = L.attn_norm; g.g_dtype = edt; g.eps = c.rms_eps;
                g.w = L.qkv; g.scales = L.qkv_s; g.n = ql + 2 * kvrows; g.k = H;
                g.epi = EPI_STORE; g.y = pf_qkv; g.ldy = g.n;
                LLMI_TRY(gemm_launch(g, stream));
                // rope + kv write + causal attention
                PrefillAttnArgs pa;
                pa.qkv = pf_qkv;
                pa.k_cache = (char*)kcache + (size_t)l * kv_layer_elems * eb;
                pa.v_cache = (char*)vcache + (size_t)l * kv_layer_elems * eb;
                pa.cache_dtype = c.kv_dtype; pa.max_seq = c.max_seq; pa.m = m; pa.p0 = p0;
                pa.heads = hl; pa.kv_heads = kvl; pa.head_dim = c.head_dim; pa.rope_tab = rope_tab; pa.out = pf_o;
                LLMI_TRY(prefill_attn_launch(pa, stream));
                // o_proj + residual
                g.a = pf_o; g.lda = ql; g.gamma = nullptr;
                g.w = L.o; g.scales = L.o_s; g.n = H; g.k = ql;
                g.epi = EPI_ADD; g.y = pf_x; g.ldy = H;
                LLMI_TRY(gemm_launch(g, stream));
                g.w_kblock = 0;
                // rmsnorm + gate_up + silu * up
                g.a = pf_x; g.lda = H; g.gamma = L.ffn_norm;
                g.w = L.gu; g.scales = L.gu_s; g.n = 2 * il; g.k = H;
                g.epi = EPI_SILU_MUL; g.pair_off = il; g.y = pf_act; g.ldy = il;
                LLMI_TRY(gemm_launch(g, stream));
                // down + residual
                g.a = pf_act; g.lda = il; g.gamma = nullptr;
                g.w = L.down; g.scales = L.down_s; g.n = H; g.k = il;
                g.epi = EPI_ADD; g.pair_off = 0; g.y = pf_x; g.ldy = H;
                LLMI_TRY(gemm_launch(g, stream));
            }
            LLMI_TRY(prefill_flush(m));
            if (p0 + m == p_begin + n)  // last row -> x for the final norm + lm_head
                LLMI_HIP(hipMemcpyAsync(x, pf_x + (size_t)(m - 1) * H, (size_t)H * 4, hipMemcpyDeviceToDevice, stream));
        }
        // the decode state first (cur_pos = last prompt row), then the head exactly as a
        // decode step runs it -- lm_head + argmax keys, and the top-K draw at step
        // seed + cur_pos + 1 when sampling (Llama<T>::firstTokenGen samples its token too)
        LLMI_TRY(prefill_finish_launch(st, prompt, tokens, p_begin, n, stream));
        LLMI_TRY(rec_head(true));
        host_next_pos += n;
        return LLMI_OK;
    }

    int tokens_out(int32_t* out, int n, int* n_valid) {
        int valid = host_next_pos;
        if (host_next_pos >= prompt_len && host_next_pos <= c.max_seq) {
            LLMI_TRY(finalize_launch(st, partials, lm_grid, tokens, c.max_seq, stream));
            valid = host_next_pos + 1;
        }
        LLMI_HIP(hipStreamSynchronize(stream));
        DecodeState h;
        LLMI_HIP(hipMemcpy(&h, st, sizeof(h), hipMemcpyDeviceToHost));
        LLMI_REQUIRE(h.error == 0, "decode: device error flag " + std::to_string(h.error) +
                                       " (1: token id out of range, 2: position overflow, 4: attention split count != device position, "
                                       "8: a tensor-parallel peer never arrived (one-shot exchange timeout), "
                                       "16: a prefill gate_up lo partial never arrived, 32: a ring-layer hand-off timed out, "
                                       "64: a fused q/k/v + attention wait timed out)");
        const int m = n < valid ? n : valid;
        if (m > 0) LLMI_HIP(hipMemcpy(out, tokens, (size_t)m * 4, hipMemcpyDeviceToHost));
        if (n_valid) *n_valid = valid;
        return LLMI_OK;
    }
};

// In-process tensor-parallel group: W rank engines (tp_rank 0..W-1) on ONE
// device and ONE stream, stepped phase by phase with group_reduce_kernel in
// place of the RCCL all-reduces. RCCL refuses two ranks on one device, so this
// is how the sharded path (per-rank weights, rank-0 residual, vocab-parallel
// argmax keys) is parity-tested on a single GPU; numerically it differs from
// the RCCL path only in the fp32 summation order of the down-proj partials.
struct Group {
    std::vector<std::unique_ptr<Engine>> r;
    hipStream_t stream = nullptr;
    void** ptrs = nullptr;  // device [4][W]: xacc, res[0], res[1], partials of every rank
    StepGraphs graphs;
    // 0: group_reduce_kernel; 1: the one-shot peer exchange's kernels (xchg.hip) -- every
    // rank's push, then every rank's reduce (one stream: the waits find their flags set);
    // 2: the producer-fused form -- every rank's o_proj / down / lm_head launch pushes from
    // its tail (tail_mode 1), then every rank's reduce kernel
    int xchg_mode = 0;

    ~Group() {
        graphs.clear();
        r.clear();
        if (ptrs) (void)hipFree(ptrs);
        if (stream) (void)hipStreamDestroy(stream);
    }

    int init(const llmi_config& cfg, int world, int dev) {
        LLMI_REQUIRE(world >= 1 && world <= 64, "group: world must be 1..64");
        LLMI_HIP(hipSetDevice(dev));
        LLMI_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        for (int i = 0; i < world; ++i) {
            llmi_config c = cfg;
            c.tp_rank = i;
            c.tp_world = world;
            r.emplace_back(new Engine());
            LLMI_TRY(r.back()->init(c, dev, nullptr, stream));
        }
        std::vector<void*> h(4 * world);
        for (int i = 0; i < world; ++i) {
            h[i] = r[i]->xacc;
            h[world + i] = r[i]->res[0];
            h[2 * world + i] = r[i]->res[1];
            h[3 * world + i] = r[i]->partials;
        }
        LLMI_HIP(hipMalloc(&ptrs, h.size() * sizeof(void*)));
        LLMI_HIP(hipMemcpy(ptrs, h.data(), h.size() * sizeof(void*), hipMemcpyHostToDevice));
        return LLMI_OK;
    }

    int set_exchange(int mode) {
        LLMI_REQUIRE(mode >= 0 && mode <= 2,
                     "group set_exchange: mode must be 0 (reduce kernel), 1 (one-shot) or 2 (push fused into the producers)");
        if (mode >= 1) {
            std::vector<char*> inboxes;
            for (auto& e : r) {
                LLMI_TRY(e->alloc_xchg());
                inboxes.push_back(e->inbox);
            }
            for (auto& e : r) LLMI_TRY(e->set_peers(inboxes));  // same device: the inboxes themselves
        }
        LLMI_HIP(hipStreamSynchronize(stream));
        graphs.clear();
        xchg_mode = mode;
        for (auto& e : r) e->tail_mode = mode == 2 ? 1 : 0;
        return LLMI_OK;
    }
    // slot: 0 xacc, 1 res[0], 2 res[1], 3 argmax partials
    int reduce(int slot, int n, int op) {
        const int W = (int)r.size();
        if (W == 1) return LLMI_OK;
        if (xchg_mode == 0) return group_reduce_launch(ptrs + slot * W, W, n, op, stream);
        auto buf = [&](Engine& e) -> void* {
            return slot == 0 ? (void*)e.xacc : slot == 3 ? (void*)e.partials : (void*)e.res[slot - 1];
        };
        if (xchg_mode == 1)  // (mode 2: the producers pushed already)
            for (auto& e : r) LLMI_TRY(xchg_launch(e->xchg_args(buf(*e), n, op, 1), stream));
        for (auto& e : r) LLMI_TRY(xchg_launch(e->xchg_args(buf(*e), n, op, 2), stream));
        return LLMI_OK;
    }

    int record_step(int nact) {
        const int H = r[0]->c.hidden;
        for (auto& e : r) e->rec_nact = nact;
        for (auto& e : r) LLMI_TRY(e->rec_start());
        for (int l = 0; l < r[0]->c.layers; ++l) {
            for (auto& e : r) LLMI_TRY(e->rec_attn(l));
            LLMI_TRY(reduce(0, H, 0));
            for (auto& e : r) LLMI_TRY(e->rec_ffn(l));
            LLMI_TRY(reduce(1 + (l + 1) % 2, H, 0));
        }
        for (auto& e : r) LLMI_TRY(e->rec_head());
        return reduce(3, r[0]->lm_grid, 2);
    }

    int decode(int n, int use_graph) {
        Engine& e0 = *r[0];
        LLMI_REQUIRE(e0.prompt_len > 0, "group decode: set_prompt first");
        LLMI_REQUIRE(n >= 0 && e0.host_next_pos + n <= e0.c.max_seq, "group decode: would run past max_seq");
        if (use_graph && n > 0)
            for (int k = Engine::nact_of(e0.host_next_pos); k <= Engine::nact_of(e0.host_next_pos + n - 1); ++k)
                LLMI_TRY(graphs.build(k, stream, [&]() { return record_step(k); }));
        for (int i = 0; i < n; ++i) {
            const int k = Engine::nact_of(e0.host_next_pos + i);
            if (use_graph)
                LLMI_HIP(hipGraphLaunch(graphs.x[k], stream));
            else
                LLMI_TRY(record_step(k));
        }
        for (auto& e : r) e->host_next_pos += n;
        return LLMI_OK;
    }
};

}  // namespace llmi

// ============================================================== C ABI (engine)
using llmi::Engine;
struct llmi_tp_comm {
    ncclComm_t c = nullptr;
};

struct llmi_engine {
    Engine e;
};
struct llmi_group {
    llmi::Group g;
};

namespace {
float h2f(uint16_t h) {
    __half v;
    std::memcpy(&v, &h, 2);
    return __half2float(v);
}
}  // namespace

extern "C" {

int llmi_config_preset(const char* name, llmi_config* cfg) {
    LLMI_REQUIRE(name && cfg, "preset: null argument");
    llmi_config c{};
    c.hidden = 4096; c.heads = 32; c.kv_heads = 32; c.head_dim = 128; c.inter = 11008;
    c.layers = 32; c.vocab = 32000; c.max_seq = 2048; c.rms_eps = 1e-5f; c.rope_base = 10000.f;
    c.weight_dtype = LLMI_F16; c.kv_dtype = LLMI_F16; c.tp_rank = 0; c.tp_world = 1;
    const std::string n(name);
    if (n == "llama2-7b") {
    } else if (n == "llama2-13b") {
        c.hidden = 5120; c.heads = 40; c.kv_heads = 40; c.inter = 13824; c.layers = 40;
    } else if (n == "tiny") {
        c.hidden = 512; c.heads = 4; c.kv_heads = 4; c.inter = 1024; c.layers = 2; c.max_seq = 64;
    } else {
        LLMI_REQUIRE(false, "preset: unknown name " + n);
    }
    *cfg = c;
    return LLMI_OK;
}

int llmi_tp_unique_id(void* out128) {
    LLMI_REQUIRE(out128, "tp_unique_id: null");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    LLMI_REQUIRE(r == ncclSuccess, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    static_assert(sizeof(id) == 128, "ncclUniqueId must be 128 bytes");
    std::memcpy(out128, &id, sizeof(id));
    return LLMI_OK;
}

int llmi_tp_comm_create(const void* tp_id, int world, int rank, int device, llmi_tp_comm** out) {
    LLMI_REQUIRE(tp_id && out && world >= 1 && rank >= 0 && rank < world, "tp_comm_create: bad arguments");
    *out = nullptr;
    LLMI_HIP(hipSetDevice(device));
    ncclUniqueId id;
    std::memcpy(&id, tp_id, sizeof(id));
    auto h = std::make_unique<llmi_tp_comm>();
    ncclResult_t r = ncclCommInitRank(&h->c, world, id, rank);
    LLMI_REQUIRE(r == ncclSuccess, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    *out = h.release();
    return LLMI_OK;
}

int llmi_tp_allreduce(llmi_tp_comm* comm, void* buf, size_t count, int dtype, llmi_stream_t stream) {
    LLMI_REQUIRE(comm && comm->c && (buf || count == 0), "tp_allreduce: bad arguments");
    ncclDataType_t t;
    switch (dtype) {
        case LLMI_F32: t = ncclFloat32; break;
        case LLMI_F16: t = ncclFloat16; break;
        case LLMI_I32: t = ncclInt32; break;
        case LLMI_I64: t = ncclInt64; break;
        default: LLMI_REQUIRE(false, "tp_allreduce: dtype must be f32, f16, i32 or i64");
    }
    if (count == 0) return LLMI_OK;
    ncclResult_t r = ncclAllReduce(buf, buf, count, t, ncclSum, comm->c, reinterpret_cast<hipStream_t>(stream));
    LLMI_REQUIRE(r == ncclSuccess, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    return LLMI_OK;
}

int llmi_tp_comm_destroy(llmi_tp_comm* comm) {
    if (!comm) return LLMI_OK;
    ncclResult_t r = comm->c ? ncclCommDestroy(comm->c) : ncclSuccess;
    delete comm;
    LLMI_REQUIRE(r == ncclSuccess, std::string("ncclCommDestroy: ") + ncclGetErrorString(r));
    return LLMI_OK;
}

int llmi_engine_create(const llmi_config* cfg, int device, const void* tp_id, llmi_engine** out) {
    LLMI_REQUIRE(cfg && out, "engine_create: null argument");
    *out = nullptr;
    auto h = std::make_unique<llmi_engine>();
    int rc = h->e.init(*cfg, device, tp_id);
    if (rc != LLMI_OK) return rc;
    *out = h.release();
    return LLMI_OK;
}

int llmi_engine_destroy(llmi_engine* e) {
    if (e) {
        (void)hipSetDevice(e->e.device);
        (void)hipStreamSynchronize(e->e.stream);
        delete e;
    }
    return LLMI_OK;
}

int llmi_engine_load_synthetic(llmi_engine* e, uint64_t seed) {
    LLMI_REQUIRE(e, "null engine");
    LLMI_HIP(hipSetDevice(e->e.device));
    return e->e.load_synthetic(seed);
}

int llmi_engine_load_tensor(llmi_engine* e, const char* name, const float* host, size_t count) {
    LLMI_REQUIRE(e, "null engine");
    LLMI_HIP(hipSetDevice(e->e.device));
    return e->e.load_tensor(name, host, count);
}

int llmi_engine_set_sampling(llmi_engine* e, int k, uint64_t seed) {
    LLMI_REQUIRE(e, "null engine");
    LLMI_HIP(hipSetDevice(e->e.device));
    return e->e.set_sampling(k, seed);
}

int llmi_engine_load_bin(llmi_engine* e, const char* weight_path) {
    LLMI_REQUIRE(e, "null engine");
    LLMI_HIP(hipSetDevice(e->e.device));
    return e->e.load_bin(weight_path);
}

int llmi_engine_set_prompt(llmi_engine* e, const int32_t* ids, int n) {
    LLMI_REQUIRE(e, "null engine");
    LLMI_HIP(hipSetDevice(e->e.device));
    return e->e.set_prompt(ids, n);
}

int llmi_engine_decode(llmi_engine* e, int n_steps, int use_graph) {
    LLMI_REQUIRE(e, "null engine");
    LLMI_HIP(hipSetDevice(e->e.device));
    return e->e.decode(n_steps, use_graph);
}

int llmi_engine_prefill(llmi_engine* e, int n_tokens, int exact) {
    LLMI_REQUIRE(e, "null engine");
    LLMI_REQUIRE(exact >= 0 && exact <= 2, "prefill: exact must be 0 (fp16 A), 1 (fp32-faithful) or 2 (fp8 lo planes)");
    LLMI_HIP(hipSetDevice(e->e.device));
    return e->e.prefill(n_tokens, exact == 2 ? 3 : exact ? 2 : 1);
}

int llmi_engine_sync(llmi_engine* e) {
    LLMI_REQUIRE(e, "null engine");
    LLMI_HIP(hipStreamSynchronize(e->e.stream));
    return LLMI_OK;
}

int llmi_engine_tokens(llmi_engine* e, int32_t* out, int n, int* n_valid) {
    LLMI_REQUIRE(e && (out || n == 0), "null argument");
    LLMI_HIP(hipSetDevice(e->e.device));
    return e->e.tokens_out(out, n, n_valid);
}

int llmi_engine_logits(llmi_engine* e, float* out, int n) {
    LLMI_REQUIRE(e && out && n <= e->e.vl, "engine_logits: bad arguments");
    LLMI_HIP(hipStreamSynchronize(e->e.stream));
    LLMI_HIP(hipMemcpy(out, e->e.logits, (size_t)n * 4, hipMemcpyDeviceToHost));
    return LLMI_OK;
}

int llmi_engine_hidden(llmi_engine* e, float* out, int n) {
    LLMI_REQUIRE(e && out && n <= e->e.c.hidden, "engine_hidden: bad arguments");
    LLMI_HIP(hipStreamSynchronize(e->e.stream));
    LLMI_HIP(hipMemcpy(out, e->e.x, (size_t)n * 4, hipMemcpyDeviceToHost));
    return LLMI_OK;
}

int llmi_engine_kv_slot(llmi_engine* e, int layer, int pos, int which_v, float* out) {
    LLMI_REQUIRE(e && out, "kv_slot: null argument");
    Engine& g = e->e;
    LLMI_REQUIRE(layer >= 0 && layer < g.c.layers && pos >= 0 && pos < g.c.max_seq, "kv_slot: out of range");
    LLMI_HIP(hipStreamSynchronize(g.stream));
    const size_t eb = llmi::dtype_size(g.c.kv_dtype), D = g.c.head_dim;
    const char* base = (const char*)(which_v ? g.vcache : g.kcache) + (size_t)layer * g.kv_layer_elems * eb;
    std::vector<char> tmp(D * eb);
    for (int h = 0; h < g.kvl; ++h) {
        LLMI_HIP(hipMemcpy(tmp.data(), base + ((size_t)h * g.c.max_seq + pos) * D * eb, D * eb,
                           hipMemcpyDeviceToHost));
        for (size_t d = 0; d < D; ++d) {
            if (g.c.kv_dtype == LLMI_F32)
                std::memcpy(out + h * D + d, tmp.data() + d * 4, 4);
            else
                out[h * D + d] = h2f(*reinterpret_cast<uint16_t*>(tmp.data() + d * 2));
        }
    }
    return LLMI_OK;
}

int llmi_engine_bytes(llmi_engine* e, uint64_t* weight_bytes, uint64_t* kv_bytes_per_pos) {
    LLMI_REQUIRE(e, "null engine");
    const Engine& g = e->e;
    if (weight_bytes) *weight_bytes = g.stream_bytes;
    if (kv_bytes_per_pos)
        *kv_bytes_per_pos = (uint64_t)g.c.layers * g.kvl * g.c.head_dim * 2 * llmi::dtype_size(g.c.kv_dtype);
    return LLMI_OK;
}

llmi_stream_t llmi_engine_stream(llmi_engine* e) { return e ? (llmi_stream_t)e->e.stream : nullptr; }

int llmi_engine_xchg_handle(llmi_engine* e, void* out64) {
    LLMI_REQUIRE(e && out64, "xchg_handle: null argument");
    Engine& g = e->e;
    LLMI_REQUIRE(!g.grouped, "xchg_handle: not on a group rank");
    LLMI_HIP(hipSetDevice(g.device));
    LLMI_TRY(g.alloc_xchg());
    static_assert(sizeof(hipIpcMemHandle_t) == 64, "IPC handle must be 64 bytes");
    hipIpcMemHandle_t h;
    LLMI_HIP(hipIpcGetMemHandle(&h, g.inbox));
    std::memcpy(out64, &h, sizeof(h));
    return LLMI_OK;
}

int llmi_engine_xchg_open(llmi_engine* e, const void* handles) {
    LLMI_REQUIRE(e && handles, "xchg_open: null argument");
    Engine& g = e->e;
    LLMI_REQUIRE(!g.grouped && g.inbox, "xchg_open: call llmi_engine_xchg_handle first");
    LLMI_REQUIRE(!g.peers_ready, "xchg_open: already open");
    LLMI_HIP(hipSetDevice(g.device));
    const int W = g.c.tp_world;
    std::vector<char*> p(W, nullptr);
    for (int q = 0; q < W; ++q) {
        if (q == g.c.tp_rank) {
            p[q] = g.inbox;
            continue;
        }
        hipIpcMemHandle_t h;
        std::memcpy(&h, static_cast<const char*>(handles) + (size_t)q * 64, 64);
        void* ptr = nullptr;
        LLMI_HIP(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess));
        g.peers_opened.push_back(ptr);
        p[q] = static_cast<char*>(ptr);
    }
    LLMI_TRY(g.set_peers(p));
    g.peers_ready = true;
    return LLMI_OK;
}

int llmi_engine_set_option(llmi_engine* e, const char* name, int value) {
    LLMI_REQUIRE(e && name, "set_option: null argument");
    LLMI_HIP(hipSetDevice(e->e.device));
    return e->e.set_option(name, value);
}

int llmi_engine_xchg_loopback(llmi_engine* e) {
    LLMI_REQUIRE(e, "xchg_loopback: null engine");
    Engine& g = e->e;
    LLMI_REQUIRE(!g.grouped && !g.comm, "xchg_loopback: not on a group rank or an engine with an RCCL communicator");
    LLMI_REQUIRE(!g.peers_ready, "xchg_loopback: the peer exchange is already open");
    LLMI_HIP(hipSetDevice(g.device));
    LLMI_TRY(g.alloc_xchg());
    LLMI_TRY(g.set_peers(std::vector<char*>(g.c.tp_world, g.inbox)));
    g.peers_ready = true;
    g.xchg_loop = 1;
    return LLMI_OK;
}

int llmi_engine_set_decode_mode(llmi_engine* e, int mode) {
    LLMI_REQUIRE(e, "set_decode_mode: null engine");
    LLMI_HIP(hipSetDevice(e->e.device));
    return e->e.set_decode_mode(mode);
}

int llmi_engine_set_exchange(llmi_engine* e, int mode) {
    LLMI_REQUIRE(e, "set_exchange: null engine");
    LLMI_HIP(hipSetDevice(e->e.device));
    return e->e.set_exchange(mode);
}

int llmi_group_set_exchange(llmi_group* g, int mode) {
    LLMI_REQUIRE(g, "group_set_exchange: null group");
    return g->g.set_exchange(mode);
}

int llmi_engine_debug_set_next_pos(llmi_engine* e, int next_pos) {
    LLMI_REQUIRE(e, "debug_set_next_pos: null engine");
    Engine& g = e->e;
    LLMI_HIP(hipSetDevice(g.device));
    LLMI_HIP(hipStreamSynchronize(g.stream));
    LLMI_HIP(hipMemcpy(&g.st->next_pos, &next_pos, sizeof(int), hipMemcpyHostToDevice));
    return LLMI_OK;
}

int llmi_engine_debug_stamps(llmi_engine* e, void* dev_buf) {
    LLMI_REQUIRE(e, "debug_stamps: null engine");
    e->e.dbg_stamps = static_cast<unsigned long long*>(dev_buf);
    return LLMI_OK;
}

int llmi_engine_debug_timeline(llmi_engine* e, void* dev_buf, size_t bytes, int slot_wgs) {
    LLMI_REQUIRE(e, "debug_timeline: null engine");
    Engine& g = e->e;
    LLMI_HIP(hipSetDevice(g.device));
    LLMI_HIP(hipStreamSynchronize(g.stream));
    g.graphs.clear();  // the captured steps carry the stamp pointers: re-capture
    if (!dev_buf) {
        g.dbg_stamps = nullptr;
        g.dbg_stride = g.dbg_slots = 0;
        return LLMI_OK;
    }
    // every decode launch's grid must fit its region: GEMVs <= 1024 workgroups, attention
    // heads x splits, o_proj heads x (hidden / 16 rows) at most
    const int ns = (g.c.max_seq + llmi::kAttnChunk - 1) / llmi::kAttnChunk;
    const int need = std::max(std::max(1024, g.hl * ns), g.hl * ((g.c.hidden + 15) / 16));
    LLMI_REQUIRE(slot_wgs >= need, "debug_timeline: slot_wgs must be >= " + std::to_string(need));
    g.dbg_stamps = static_cast<unsigned long long*>(dev_buf);
    g.dbg_stride = slot_wgs;
    g.dbg_slots = (int)std::min<size_t>(bytes / ((size_t)slot_wgs * 64), 1 << 20);
    LLMI_REQUIRE(g.dbg_slots > 0, "debug_timeline: buffer smaller than one slot");
    return LLMI_OK;
}

int llmi_engine_time_kernel(llmi_engine* e, int which, int iters, float* avg_us, uint64_t* bytes) {
    LLMI_REQUIRE(e && avg_us && iters > 0, "time_kernel: bad arguments");
    Engine& g = e->e;
    LLMI_HIP(hipSetDevice(g.device));
    LLMI_REQUIRE(g.prompt_len > 0 && g.host_next_pos > 0, "time_kernel: decode at least one step first");
    g.rec_nact = Engine::nact_of(g.host_next_pos - 1);  // attention sized for the current position
    const size_t H = g.c.hidden;
    uint64_t b = 0;
    // launch i uses layer i % layers: every launch streams weights (and KV) the
    // previous launches did not touch, as in the decode loop -- replaying one layer
    // would serve its weights from the 256 MiB Infinity Cache and read high
    int li = 0;
    auto launch = [&]() -> int {
        const int l = li++ % g.c.layers;
        switch (which) {
            case 0: return llmi::gemv_launch(g.qkv_args(l), g.stream);
            case 1: return llmi::attn_decode_launch(g.attn_args(l), g.stream);
            case 2: return llmi::attn_oproj_launch(g.o_args(l), g.stream);
            case 3: return llmi::gemv_launch(g.gu_args(l), g.stream);
            case 4: return llmi::gemv_launch(g.down_args(l), g.stream);
            case 5: return llmi::gemv_launch(g.lm_args(), g.stream);
            case 6:
            case 7: {  // the per-token TP exchange: one residual all-reduce (int64, hidden)
                ncclResult_t r = ncclAllReduce(g.xacc, g.xacc, H, ncclInt64, ncclSum, g.comm, g.stream);
                LLMI_REQUIRE(r == ncclSuccess, std::string("ncclAllReduce(int64): ") + ncclGetErrorString(r));
                return LLMI_OK;
            }
            case 8:
            case 9:  // the same exchange over the one-shot peer path
                return llmi::xchg_launch(g.xchg_args(g.xacc, (int)H, 0, 3), g.stream);
            case 10:  // the persistent ring layer (o_proj, gate_up, down, next q/k/v)
                return llmi::ring_layer_launch(g.ring_args(l, true), g.n_cu, g.stream);
            case 11: {  // the fused q/k/v + attention launch (the decode default; consecutive launches
                        // cycle layers, so each finds the previous layer's tags in the granule buffer)
                llmi::GemvArgs q = g.qkv_args(l);
                llmi::AttnArgs at = g.attn_args(l);
                q.kpar = 0;
                q.y_tag = g.qtag; q.tag_epoch = &g.st->epoch; q.tag_layer = (unsigned)l;
                at.qkv_tag = g.qtag; at.tag_epoch = &g.st->epoch; at.tag_layer = (unsigned)l;
                at.xacc = nullptr;  // (timing only: no residual seed)
                return llmi::qkv_attn_launch(q, at, g.stream);
            }
        }
        LLMI_REQUIRE(false, "time_kernel: which must be 0..11");
    };
    LLMI_REQUIRE(which < 6 || which > 7 || g.comm != nullptr,
                 "time_kernel: the all-reduce needs an RCCL communicator (tp_id)");
    LLMI_REQUIRE(which < 8 || which > 9 || g.peers_ready, "time_kernel: the one-shot exchange needs xchg_open");
    LLMI_REQUIRE(which != 10 || (g.decode_mode == 1 && g.wdt_valid), "time_kernel: the ring layer needs decode mode 1");
    const uint64_t ws = g.wsz, sc = (g.wdt == LLMI_I8) ? 2 : 0;
    switch (which) {
        case 0: b = (uint64_t)(g.ql + 2 * g.kvrows) * H * ws + (g.ql + 2 * g.kvrows) * sc; break;
        case 1: {
            llmi::DecodeState hs;
            LLMI_HIP(hipMemcpy(&hs, g.st, sizeof(hs), hipMemcpyDeviceToHost));
            const uint64_t eb = llmi::dtype_size(g.c.kv_dtype);
            b = (uint64_t)2 * (hs.cur_pos + 1) * g.kvl * g.c.head_dim * eb + 2ull * g.kvl * g.c.head_dim * eb;
            break;
        }
        case 2: b = (uint64_t)H * g.ql * ws + H * sc; break;
        case 3: b = (uint64_t)2 * g.il * H * ws + 2 * g.il * sc; break;
        case 4: b = (uint64_t)H * g.il * ws + H * sc; break;
        case 5: b = (uint64_t)g.vl * H * g.esz; break;
        case 6:
        case 7:
        case 8:
        case 9: b = (uint64_t)H * 8; break;
        case 10: b = ((uint64_t)H * g.ql + 3ull * g.il * H + (uint64_t)(g.ql + 2 * g.kvrows) * H) * ws; break;
        case 11: {
            llmi::DecodeState hs;
            LLMI_HIP(hipMemcpy(&hs, g.st, sizeof(hs), hipMemcpyDeviceToHost));
            const uint64_t eb = llmi::dtype_size(g.c.kv_dtype);
            b = (uint64_t)(g.ql + 2 * g.kvrows) * H * ws + (g.ql + 2 * g.kvrows) * sc +
                (uint64_t)2 * (hs.cur_pos + 1) * g.kvl * g.c.head_dim * eb + 2ull * g.kvl * g.c.head_dim * eb;
            break;
        }
    }
    // timing launches modify the residual stream (o/down epilogues add into x),
    // so save and restore the small activation state around them
    std::vector<char> save(H * 4), save_fx(3 * H * 8);
    LLMI_HIP(hipMemcpyAsync(save.data(), g.x, H * 4, hipMemcpyDeviceToHost, g.stream));
    long long* fx[3] = {g.xacc, g.res[0], g.res[1]};
    for (int i = 0; i < 3; ++i)
        LLMI_HIP(hipMemcpyAsync(save_fx.data() + i * H * 8, fx[i], H * 8, hipMemcpyDeviceToHost, g.stream));
    // the attention launches write the current position's K/V row into every layer they
    // cycle through (from the last layer's q/k/v): keep each layer's row at cur_pos
    llmi::DecodeState hst{};
    std::vector<char> save_kv;
    const size_t kv_eb = llmi::dtype_size(g.c.kv_dtype), kv_row = (size_t)g.c.head_dim * kv_eb;
    const size_t kv_pitch = (size_t)g.c.max_seq * kv_row;
    auto kv_rows = [&](int l, int v) {
        return (char*)(v ? g.vcache : g.kcache) + (size_t)l * g.kv_layer_elems * kv_eb + (size_t)hst.cur_pos * kv_row;
    };
    LLMI_REQUIRE(which != 11 || (g.layers.size() >= 2 && g.c.layers < 128),
                 "time_kernel: the fused q/k/v + attention launch cycles >= 2 layers (its tags must change)");
    if (which == 1 || which == 11) {
        LLMI_HIP(hipMemcpyAsync(&hst, g.st, sizeof(hst), hipMemcpyDeviceToHost, g.stream));
        LLMI_HIP(hipStreamSynchronize(g.stream));
        save_kv.resize((size_t)g.c.layers * 2 * g.kvl * kv_row);
        for (int l = 0; l < g.c.layers; ++l)
            for (int v = 0; v < 2; ++v)
                LLMI_HIP(hipMemcpy2D(save_kv.data() + ((size_t)l * 2 + v) * g.kvl * kv_row, kv_row, kv_rows(l, v),
                                     kv_pitch, kv_row, g.kvl, hipMemcpyDeviceToHost));
    }
    std::vector<char> save_rl;
    if (which == 10) {
        save_rl.resize((size_t)5 * H * 8);
        LLMI_HIP(hipMemcpyAsync(save_rl.data(), g.rl_acc, save_rl.size(), hipMemcpyDeviceToHost, g.stream));
    }
    LLMI_TRY(launch());  // warm
    hipGraph_t cg = nullptr;
    hipGraphExec_t ce = nullptr;
    if (which == 7 || which == 9) {  // the exchanges captured into one graph, as the decode step replays them
        LLMI_HIP(hipStreamBeginCapture(g.stream, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < iters; ++i) LLMI_TRY(launch());
        LLMI_HIP(hipStreamEndCapture(g.stream, &cg));
        LLMI_HIP(hipGraphInstantiate(&ce, cg, nullptr, nullptr, 0));
        LLMI_HIP(hipGraphLaunch(ce, g.stream));  // warm
    }
    hipEvent_t t0, t1;
    LLMI_HIP(hipEventCreate(&t0));
    LLMI_HIP(hipEventCreate(&t1));
    LLMI_HIP(hipEventRecord(t0, g.stream));
    if (ce) {
        LLMI_HIP(hipGraphLaunch(ce, g.stream));
    } else {
        for (int i = 0; i < iters; ++i) LLMI_TRY(launch());
    }
    LLMI_HIP(hipEventRecord(t1, g.stream));
    LLMI_HIP(hipEventSynchronize(t1));
    float ms = 0.f;
    LLMI_HIP(hipEventElapsedTime(&ms, t0, t1));
    (void)hipEventDestroy(t0);
    (void)hipEventDestroy(t1);
    if (ce) (void)hipGraphExecDestroy(ce);
    if (cg) (void)hipGraphDestroy(cg);
    LLMI_HIP(hipMemcpy(g.x, save.data(), H * 4, hipMemcpyHostToDevice));
    for (int i = 0; i < 3; ++i) LLMI_HIP(hipMemcpy(fx[i], save_fx.data() + i * H * 8, H * 8, hipMemcpyHostToDevice));
    if (which == 1 || which == 11)
        for (int l = 0; l < g.c.layers; ++l)
            for (int v = 0; v < 2; ++v)
                LLMI_HIP(hipMemcpy2D(kv_rows(l, v), kv_pitch, save_kv.data() + ((size_t)l * 2 + v) * g.kvl * kv_row,
                                     kv_row, kv_row, g.kvl, hipMemcpyHostToDevice));
    if (which == 10) {  // accumulators back, every layer's counters zero again
        LLMI_HIP(hipMemcpy(g.rl_acc, save_rl.data(), save_rl.size(), hipMemcpyHostToDevice));
        LLMI_HIP(hipMemset(g.rl_cnt, 0, (size_t)g.c.layers * llmi::kRingCntWords * 4));
    }
    *avg_us = ms * 1000.f / iters;
    if (bytes) *bytes = b;
    return LLMI_OK;
}

// ---- in-process TP group (single-device parity harness for the sharded path)
int llmi_group_create(const llmi_config* cfg, int world, int device, llmi_group** out) {
    LLMI_REQUIRE(cfg && out, "group_create: null argument");
    *out = nullptr;
    auto h = std::make_unique<llmi_group>();
    int rc = h->g.init(*cfg, world, device);
    if (rc != LLMI_OK) return rc;
    *out = h.release();
    return LLMI_OK;
}

int llmi_group_destroy(llmi_group* g) {
    if (g) {
        (void)hipSetDevice(g->g.r.empty() ? 0 : g->g.r[0]->device);
        (void)hipStreamSynchronize(g->g.stream);
        delete g;
    }
    return LLMI_OK;
}

int llmi_group_load_synthetic(llmi_group* g, uint64_t seed) {
    LLMI_REQUIRE(g, "null group");
    for (auto& e : g->g.r) LLMI_TRY(e->load_synthetic(seed));
    return LLMI_OK;
}

int llmi_group_load_bin(llmi_group* g, const char* weight_path) {
    LLMI_REQUIRE(g, "null group");
    for (auto& e : g->g.r) {
        LLMI_HIP(hipSetDevice(e->device));
        LLMI_TRY(e->load_bin(weight_path));
    }
    return LLMI_OK;
}

int llmi_group_set_prompt(llmi_group* g, const int32_t* ids, int n) {
    LLMI_REQUIRE(g, "null group");
    for (auto& e : g->g.r) LLMI_TRY(e->set_prompt(ids, n));
    return LLMI_OK;
}

int llmi_group_decode(llmi_group* g, int n_steps, int use_graph) {
    LLMI_REQUIRE(g, "null group");
    return g->g.decode(n_steps, use_graph);
}

int llmi_group_tokens(llmi_group* g, int rank, int32_t* out, int n, int* n_valid) {
    LLMI_REQUIRE(g && (out || n == 0) && rank >= 0 && rank < (int)g->g.r.size(), "group_tokens: bad arguments");
    return g->g.r[rank]->tokens_out(out, n, n_valid);
}

int llmi_group_logits(llmi_group* g, float* out, int n) {
    LLMI_REQUIRE(g && out, "group_logits: null argument");
    LLMI_HIP(hipStreamSynchronize(g->g.stream));
    int off = 0;
    for (auto& e : g->g.r) {  // vocab-parallel slices in rank order = the full vocab
        const int m = std::min(e->vl, n - off);
        if (m <= 0) break;
        LLMI_HIP(hipMemcpy(out + off, e->logits, (size_t)m * 4, hipMemcpyDeviceToHost));
        off += m;
    }
    return LLMI_OK;
}

int llmi_group_hidden(llmi_group* g, int rank, float* out, int n) {
    LLMI_REQUIRE(g && out && rank >= 0 && rank < (int)g->g.r.size() && n <= g->g.r[0]->c.hidden,
                 "group_hidden: bad arguments");
    LLMI_HIP(hipStreamSynchronize(g->g.stream));
    LLMI_HIP(hipMemcpy(out, g->g.r[rank]->x, (size_t)n * 4, hipMemcpyDeviceToHost));
    return LLMI_OK;
}

}  // extern "C"
