// Throughput of the reference's context-decoder API (LlamaContextDecoder<half>::forward,
// context_decoder.cpp:47-143) on a ragged batch at Llama-2-7B width: every projection on
// the MFMA GEMM (llmi_linear, fp32-faithful split), QK^T / PV on the MFMA batched matmul,
// mask/softmax/transpose as their own launches. Random-init weights (llmi-prng), 32 layers.
//   ctx_decoder_bench <layers> <reps> <len0> [len1 ...]      (history 0, max_seq = max len)
// LLMI_CTX_UNFUSED=1: the reference's unfused attention chain instead of the fused core.
// (per-forward scratch through HipCachingAllocator, as the reference's CudaAllocator).
// Prints one JSON line: ms per forward over the batch, rows/s.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "llmi/allocator.h"

// the reference pairs its layers with the pooled CudaAllocator; its restatement here
static HipCachingAllocator g_alloc;

template <typename T> struct Dev {
    T* p = nullptr;
    explicit Dev(size_t n) { p = g_alloc.Malloc(p, n * sizeof(T), false); }
    ~Dev() { g_alloc.Free(p, false); }
};

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    try {
        const int heads = 32, kv = 32, hd = 128, I = 11008, V = 32000, H = heads * hd;
        const int L = std::atoi(argv[1]), reps = std::atoi(argv[2]);
        std::vector<int> lens;
        for (int i = 3; i < argc; ++i) lens.push_back(std::atoi(argv[i]));
        const int bs = (int)lens.size();
        int tokens = 0, S = 0;
        for (int l : lens) tokens += l, S = std::max(S, l);
        std::vector<int> hist(bs, 0), ids(tokens);
        for (int i = 0; i < tokens; ++i) ids[i] = (i * 7919 + 13) % V;

        LLaMAAttentionStaticParams sp;
        std::vector<LlamaLayerWeight<half_t>*> lw;
        for (int l = 0; l < L; ++l) {
            lw.push_back(new LlamaLayerWeight<half_t>(heads, kv, hd, I, WeightType::FP16_W, false, &g_alloc, l));
            lw.back()->loadWeights(1);
        }
        Dev<half_t> emb((size_t)V * H);
        LLMI_CALL(llmi_synth_fill(emb.p, LLMI_F16, LLMI_SYN_EMBED, 1, 1, V, H, 0, 0, H, nullptr));
        EmbeddingWeight<half_t> E;
        E.shape = {V, H};
        E.data = emb.p;

        const size_t cache_n = (size_t)L * bs * kv * S * hd;
        Dev<int> did(tokens), dhist(bs), dlens(bs), dctx(bs);
        LLMI_CALL(llmi_memcpy(did.p, ids.data(), tokens * sizeof(int), 0));
        LLMI_CALL(llmi_memcpy(dhist.p, hist.data(), bs * sizeof(int), 0));
        LLMI_CALL(llmi_memcpy(dlens.p, lens.data(), bs * sizeof(int), 0));
        LLMI_CALL(llmi_memcpy(dctx.p, lens.data(), bs * sizeof(int), 0));
        Dev<float> x((size_t)tokens * H), y((size_t)tokens * H), kc(cache_n), vc(cache_n);
        TensorWrapper<int> id_t(GPU, INT32, {tokens}, did.p), hist_t(GPU, INT32, {bs}, dhist.p),
            q_t(GPU, INT32, {bs}, dlens.p), k_t(GPU, INT32, {bs}, dctx.p);
        TensorWrapper<float> in(GPU, FP32, {tokens, H}, x.p), out(GPU, FP32, {tokens, H}, y.p);
        TensorWrapper<float> kcache(GPU, FP32, {L, bs, kv, S, hd}, kc.p), vcache(GPU, FP32, {L, bs, kv, S, hd}, vc.p);
        int layer0 = 0;
        TensorWrapper<int> layer_t(CPU, INT32, {1}, &layer0);
        LlamaContextDecoder<half_t> dec(heads, kv, hd, I, L, sp, 1e-5f, nullptr, nullptr, &g_alloc);
        const char* uf = std::getenv("LLMI_CTX_UNFUSED");
        const bool unfused = uf && std::string(uf) == "1";
        dec.setFusedAttentionCore(!unfused);
        LLaMAAttentionDynParams p;
        p.batch_size = bs;
        p.num_tokens = tokens;
        p.max_q_len = S;
        p.max_k_len = S;
        p.num_layers = L;
        TensorMap cin{{"decoder_input", &in}, {"history_length", &hist_t}, {"input_length", &q_t},
                      {"context_length", &k_t}, {"layer_id", &layer_t}};
        TensorMap cout{{"decoder_output", &out}, {"all_k_cache", &kcache}, {"all_v_cache", &vcache}};
        double best = 1e30, sum = 0;
        for (int r = 0; r <= reps; ++r) {  // r = 0: warm-up
            launchInputEmbedding(&id_t, &in, &E);
            LLMI_CALL(llmi_device_sync());
            const auto t0 = std::chrono::steady_clock::now();
            dec.forward(cin, lw, cout, p);
            LLMI_CALL(llmi_device_sync());
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            if (r) best = std::min(best, ms), sum += ms;
        }
        std::string ls;
        for (int l : lens) ls += (ls.empty() ? "" : ",") + std::to_string(l);
        std::printf("{\"api\": \"LlamaContextDecoder<half>::forward\", \"layers\": %d, \"lens\": [%s], \"rows\": %d, "
                    "\"ms_best\": %.3f, \"ms_mean\": %.3f, \"rows_per_s\": %.1f, \"attention_core\": \"%s\"}\n",
                    L, ls.c_str(), tokens, best, sum / reps, tokens / (best * 1e-3), unfused ? "unfused" : "fused");
        for (auto* w : lw) delete w;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
