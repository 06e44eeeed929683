// Decode speed of the reference's layer API: LlamaSelfDecoder<half>::forward
// (self_decoder.cpp:23-89) + final RMSNorm + lm_head + top-1, one token per call with
// the reference's per-token D2H of the id (llama.cpp:266), at Llama-2-7B width, fp16
// KV cache, random-init weights (llmi-prng). Each sublayer is its own launch sequence
// (GEMVs, RoPE, masked MHA, norms, residual adds) -- the per-op path a reference caller
// of the layer classes gets; the fused graph-replayed engine (llmi_engine_*) is bench.py.
//   self_decoder_bench <layers> <ctx_from> <tokens>     (decode positions ctx_from .. +tokens)
// Prints one JSON line: ms per token and tokens/s.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "llmi/allocator.h"

static HipCachingAllocator g_alloc;

template <typename T> struct Dev {
    T* p = nullptr;
    explicit Dev(size_t n) { p = g_alloc.Malloc(p, n * sizeof(T), false); }
    ~Dev() { g_alloc.Free(p, false); }
};

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    try {
        const int heads = 32, kv = 32, hd = 128, H = heads * hd, I = 11008, V = 32000;
        const int L = std::atoi(argv[1]), from = std::atoi(argv[2]), n = std::atoi(argv[3]);
        const int S = from + n + 1;
        LLaMAAttentionStaticParams sp;
        std::vector<LlamaLayerWeight<half_t>*> lw;
        for (int l = 0; l < L; ++l) {
            lw.push_back(new LlamaLayerWeight<half_t>(heads, kv, hd, I, WeightType::FP16_W, false, &g_alloc, l));
            lw.back()->loadWeights(1);
        }
        Dev<half_t> emb((size_t)V * H), lm((size_t)V * H), fnorm(H);
        LLMI_CALL(llmi_synth_fill(emb.p, LLMI_F16, LLMI_SYN_EMBED, 1, 1, V, H, 0, 0, H, nullptr));
        LLMI_CALL(llmi_synth_fill(lm.p, LLMI_F16, LLMI_SYN_LINEAR, 1, 2, V, H, 0, 0, H, nullptr));
        LLMI_CALL(llmi_synth_fill(fnorm.p, LLMI_F16, LLMI_SYN_GAMMA, 1, 3, 1, H, 0, 0, H, nullptr));
        EmbeddingWeight<half_t> E;
        E.shape = {V, H};
        E.data = emb.p;
        BaseWeight<half_t> LM;
        LM.shape = {V, H};
        LM.data = lm.p;
        LayerNormWeight<half_t> FN{fnorm.p};

        const size_t cache_n = (size_t)L * kv * S * hd;
        Dev<half_t> kc(cache_n), vc(cache_n);  // history positions: zero-filled keys/values
        Dev<float> x(H), y(H), unused(H), logits(V);
        Dev<int> ids(1), next(1);
        TensorWrapper<float> dec_in(GPU, FP32, {1, H}, x.p), dec_out(GPU, FP32, {1, H}, y.p), un(GPU, FP32, {1, H}, unused.p);
        TensorWrapper<half_t> kcache(GPU, FP16, {L, 1, kv, S, hd}, kc.p), vcache(GPU, FP16, {L, 1, kv, S, hd}, vc.p);
        TensorWrapper<float> probs(GPU, FP32, {1, V}, logits.p);
        TensorWrapper<int> id_t(GPU, INT32, {1}, ids.p), next_t(GPU, INT32, {1}, next.p);
        int step = 0;
        bool fin = false;
        TensorWrapper<int> step_t(CPU, INT32, {1}, &step);
        TensorWrapper<bool> fin_t(CPU, BOOL, {1}, &fin);
        LlamaSelfDecoder<half_t> dec(heads, kv, hd, I, L, sp, 1e-5f, nullptr, nullptr, &g_alloc);
        LLaMAAttentionDynParams dp;
        dp.num_layers = L;
        TensorMap in{{"decoder_input", &dec_in}, {"step", &step_t}, {"finished", &fin_t}};
        TensorMap out{{"decoder_output", &dec_out}, {"all_k_cache", &kcache}, {"all_v_cache", &vcache}};
        int tok = 1;
        auto one = [&](int pos) {
            LLMI_CALL(llmi_memcpy(ids.p, &tok, 4, 0));
            launchInputEmbedding(&id_t, &dec_in, &E);
            step = pos + 1;
            dec.forward(in, lw, out, dp);
            launchRMSNorm(&dec_out, &un, FN, 1e-5f, true);
            launchLinearGemm(&dec_out, LM, &probs, nullptr, false, true);
            launchTopKforBeamSearch(&probs, &next_t);
            LLMI_CALL(llmi_memcpy(&tok, next.p, 4, 1));
        };
        one(from);  // warm-up (first-use allocations)
        LLMI_CALL(llmi_device_sync());
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < n; ++i) one(from + 1 + i);
        LLMI_CALL(llmi_device_sync());
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / n;
        std::printf("{\"api\": \"LlamaSelfDecoder<half>::forward + norm + lm_head + top-1\", \"layers\": %d, "
                    "\"ctx\": [%d, %d], \"kv_cache\": \"f16\", \"ms_per_token\": %.3f, \"tokens_per_s\": %.1f}\n",
                    L, from + 1, from + n, ms, 1e3 / ms);
        for (auto* w : lw) delete w;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
