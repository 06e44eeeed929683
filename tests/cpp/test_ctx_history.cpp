// LlamaContextDecoder<half> (context_decoder.cpp:47-143) on a ragged batch WITH history:
// the cache already holds history_length[b] positions of sequence b (uploaded from the
// reference's own run, tests/golden/f8_*.npz) and the batch's chunk rows are appended
// after them (rope at history + t, KV concat at slot history + t, causal mask over
// history + chunk). Inputs from <dir>/*.bin, outputs to <dir>/out_*.bin for the pytest
// driver (tests/test_gpu_ctx_history.py):
//   test_ctx_history <dir> <heads> <kv_heads> <head> <inter> <layers> <vocab> <max_seq> <seed> <bs> [f16|f32] [unfused]
// With "f16" the caches are TensorWrapper<half> (LLaMAContextAttentionLayer<half>,
// context_attention.cpp:177): uploaded rounded to fp16, written back widened to fp32.
// "unfused": the reference's attention chain (repeat, QK^T, mask + softmax, PV,
// transpose) instead of the fused llmi_context_attention core.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "llmi/layers.h"

static HipAllocator g_alloc;

template <typename T> struct Dev {
    T* p = nullptr;
    size_t n = 0;
    explicit Dev(size_t n) : n(n) { p = g_alloc.Malloc(p, n * sizeof(T), false); }
    ~Dev() { g_alloc.Free(p, false); }
    void put(const std::vector<T>& h) { LLMI_CALL(llmi_memcpy(p, h.data(), n * sizeof(T), 0)); }
    std::vector<T> get() const {
        std::vector<T> h(n);
        LLMI_CALL(llmi_memcpy(h.data(), p, n * sizeof(T), 1));
        return h;
    }
};

template <typename T> static std::vector<T> load(const std::string& path, size_t n) {
    std::vector<T> v(n);
    FILE* f = std::fopen(path.c_str(), "rb");
    LLM_CHECK_WITH_INFO(f && std::fread(v.data(), sizeof(T), n, f) == n, "cannot read " + path);
    std::fclose(f);
    return v;
}
template <typename T> static void save(const std::string& path, const std::vector<T>& v) {
    FILE* f = std::fopen(path.c_str(), "wb");
    LLM_CHECK_WITH_INFO(f && std::fwrite(v.data(), sizeof(T), v.size(), f) == v.size(), "cannot write " + path);
    std::fclose(f);
}

int main(int argc, char** argv) {
    if (argc < 11) return 2;
    try {
        const std::string dir = argv[1];
        const int heads = std::atoi(argv[2]), kv = std::atoi(argv[3]), hd = std::atoi(argv[4]), I = std::atoi(argv[5]);
        const int L = std::atoi(argv[6]), V = std::atoi(argv[7]), S = std::atoi(argv[8]);
        const uint64_t seed = std::strtoull(argv[9], nullptr, 10);
        const int bs = std::atoi(argv[10]);
        const bool f16 = argc > 11 && std::string(argv[11]) == "f16";
        const bool unfused = argc > 12 && std::string(argv[12]) == "unfused";
        const int H = heads * hd;
        const std::vector<int> hist = load<int>(dir + "/hist.bin", bs), lens = load<int>(dir + "/lens.bin", bs);
        int tokens = 0, maxq = 0, maxk = 0;
        std::vector<int> ctx(bs);
        for (int b = 0; b < bs; ++b) {
            tokens += lens[b];
            ctx[b] = hist[b] + lens[b];
            maxq = std::max(maxq, lens[b]);
            maxk = std::max(maxk, ctx[b]);
        }
        const std::vector<int> ids = load<int>(dir + "/ids.bin", tokens);
        const size_t cache_n = (size_t)L * bs * kv * S * hd;

        LLaMAAttentionStaticParams sp;
        std::vector<LlamaLayerWeight<half_t>*> lw;
        for (int l = 0; l < L; ++l) {
            lw.push_back(new LlamaLayerWeight<half_t>(heads, kv, hd, I, WeightType::FP16_W, false, &g_alloc, l));
            lw.back()->loadWeights(seed);
        }
        Dev<half_t> emb((size_t)V * H), lm((size_t)V * H), fnorm(H);
        LLMI_CALL(llmi_synth_fill(emb.p, LLMI_F16, LLMI_SYN_EMBED, seed, 1, V, H, 0, 0, H, nullptr));
        LLMI_CALL(llmi_synth_fill(lm.p, LLMI_F16, LLMI_SYN_LINEAR, seed, 2, V, H, 0, 0, H, nullptr));
        LLMI_CALL(llmi_synth_fill(fnorm.p, LLMI_F16, LLMI_SYN_GAMMA, seed, 3, 1, H, 0, 0, H, nullptr));
        EmbeddingWeight<half_t> E;
        E.shape = {V, H};
        E.data = emb.p;
        BaseWeight<half_t> LM;
        LM.shape = {V, H};
        LM.data = lm.p;
        LayerNormWeight<half_t> FN{fnorm.p};

        Dev<int> did(tokens), dhist(bs), dlens(bs), dctx(bs);
        did.put(ids);
        dhist.put(hist);
        dlens.put(lens);
        dctx.put(ctx);
        Dev<float> x((size_t)tokens * H), y((size_t)tokens * H), kc(cache_n), vc(cache_n), un(H), logits(V);
        kc.put(load<float>(dir + "/kcache.bin", cache_n));
        vc.put(load<float>(dir + "/vcache.bin", cache_n));
        Dev<half_t> kh(f16 ? cache_n : 1), vh(f16 ? cache_n : 1);
        if (f16) {
            LLMI_CALL(llmi_convert(kc.p, LLMI_F32, kh.p, LLMI_F16, cache_n, nullptr));
            LLMI_CALL(llmi_convert(vc.p, LLMI_F32, vh.p, LLMI_F16, cache_n, nullptr));
        }
        TensorWrapper<int> id_t(GPU, INT32, {tokens}, did.p), hist_t(GPU, INT32, {bs}, dhist.p),
            q_t(GPU, INT32, {bs}, dlens.p), k_t(GPU, INT32, {bs}, dctx.p);
        TensorWrapper<float> in(GPU, FP32, {tokens, H}, x.p), out(GPU, FP32, {tokens, H}, y.p);
        TensorWrapper<float> kcache(GPU, FP32, {L, bs, kv, S, hd}, kc.p), vcache(GPU, FP32, {L, bs, kv, S, hd}, vc.p);
        TensorWrapper<half_t> kcache16(GPU, FP16, {L, bs, kv, S, hd}, kh.p), vcache16(GPU, FP16, {L, bs, kv, S, hd}, vh.p);
        TensorWrapper<float> unused(GPU, FP32, {1, H}, un.p), probs(GPU, FP32, {1, V}, logits.p);
        int layer0 = 0;
        TensorWrapper<int> layer_t(CPU, INT32, {1}, &layer0);
        launchInputEmbedding(&id_t, &in, &E);
        LlamaContextDecoder<half_t> dec(heads, kv, hd, I, L, sp, 1e-5f, nullptr, nullptr, &g_alloc);
        dec.setFusedAttentionCore(!unfused);
        LLaMAAttentionDynParams p;
        p.batch_size = bs;
        p.num_tokens = tokens;
        p.max_q_len = maxq;
        p.max_k_len = maxk;
        p.num_layers = L;
        TensorMap cin{{"decoder_input", &in}, {"history_length", &hist_t}, {"input_length", &q_t},
                      {"context_length", &k_t}, {"layer_id", &layer_t}};
        TensorMap cout{{"decoder_output", &out}, {"all_k_cache", &kcache}, {"all_v_cache", &vcache}};
        if (f16) {
            cout.insert("all_k_cache", &kcache16);
            cout.insert("all_v_cache", &vcache16);
        }
        dec.forward(cin, lw, cout, p);
        std::vector<float> all_logits;
        int row = 0;
        for (int b = 0; b < bs; ++b) {  // the last row of each sequence -> final norm -> lm_head
            row += lens[b];
            TensorWrapper<float> last(GPU, FP32, {1, H}, y.p + (size_t)(row - 1) * H);
            launchRMSNorm(&last, &unused, FN, 1e-5f, true);
            launchLinearGemm(&last, LM, &probs, nullptr, false, true);
            const std::vector<float> lg = logits.get();
            all_logits.insert(all_logits.end(), lg.begin(), lg.end());
        }
        save(dir + "/out_logits.bin", all_logits);
        if (f16) {  // widened back for the comparison
            LLMI_CALL(llmi_convert(kh.p, LLMI_F16, kc.p, LLMI_F32, cache_n, nullptr));
            LLMI_CALL(llmi_convert(vh.p, LLMI_F16, vc.p, LLMI_F32, cache_n, nullptr));
        }
        save(dir + "/out_k.bin", kc.get());
        save(dir + "/out_v.bin", vc.get());
        for (auto* w : lw) delete w;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    std::printf("ok\n");
    return 0;
}
