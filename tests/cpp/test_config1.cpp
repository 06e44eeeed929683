// BASELINE config 1 on the HIP path: one Llama-2 decoder layer (hidden 4096, seq 8) through
// the reference's layer API, LlamaContextDecoder<float>::forward (context_decoder.cpp:47-143;
// modeling_llama.py:764-823 is what F2 recorded), fp32 activations, fp32 weights and cache,
// given x (tests/golden/f2_layer.npz: x, PRNG weights of seed 12).
//   test_config1 <dir> <seed>     reads <dir>/x.bin [8, 4096] fp32, writes <dir>/y.bin
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "llmi/layers.h"

static HipAllocator g_alloc;

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    try {
        const std::string dir = argv[1];
        const uint64_t seed = std::strtoull(argv[2], nullptr, 10);
        const int heads = 32, kv = 32, hd = 128, I = 11008, L = 1, S = 16, T = 8, H = heads * hd;
        std::vector<float> x((size_t)T * H);
        FILE* f = std::fopen((dir + "/x.bin").c_str(), "rb");
        LLM_CHECK_WITH_INFO(f && std::fread(x.data(), 4, x.size(), f) == x.size(), "cannot read x.bin");
        std::fclose(f);

        LlamaLayerWeight<float> w(heads, kv, hd, I, WeightType::FP32_W, false, &g_alloc, 0);
        w.loadWeights(seed);
        std::vector<LlamaLayerWeight<float>*> lw{&w};
        const size_t cache_n = (size_t)L * 1 * kv * S * hd;
        float *dx = nullptr, *dy = nullptr, *kc = nullptr, *vc = nullptr;
        int *dhist = nullptr, *dlen = nullptr, *dctx = nullptr;
        dx = g_alloc.Malloc(dx, x.size() * 4, false);
        dy = g_alloc.Malloc(dy, x.size() * 4, false);
        kc = g_alloc.Malloc(kc, cache_n * 4, false);
        vc = g_alloc.Malloc(vc, cache_n * 4, false);
        dhist = g_alloc.Malloc(dhist, 4, false);
        dlen = g_alloc.Malloc(dlen, 4, false);
        dctx = g_alloc.Malloc(dctx, 4, false);
        const int zero = 0, len = T;
        LLMI_CALL(llmi_memcpy(dx, x.data(), x.size() * 4, 0));
        LLMI_CALL(llmi_memcpy(dhist, &zero, 4, 0));
        LLMI_CALL(llmi_memcpy(dlen, &len, 4, 0));
        LLMI_CALL(llmi_memcpy(dctx, &len, 4, 0));
        LLMI_CALL(llmi_device_memset(kc, 0, cache_n * 4));
        LLMI_CALL(llmi_device_memset(vc, 0, cache_n * 4));
        TensorWrapper<float> in(GPU, FP32, {T, H}, dx), out(GPU, FP32, {T, H}, dy);
        TensorWrapper<float> kcache(GPU, FP32, {L, 1, kv, S, hd}, kc), vcache(GPU, FP32, {L, 1, kv, S, hd}, vc);
        TensorWrapper<int> hist_t(GPU, INT32, {1}, dhist), q_t(GPU, INT32, {1}, dlen), k_t(GPU, INT32, {1}, dctx);
        int layer0 = 0;
        TensorWrapper<int> layer_t(CPU, INT32, {1}, &layer0);
        LLaMAAttentionStaticParams sp;
        LlamaContextDecoder<float> dec(heads, kv, hd, I, L, sp, 1e-5f, nullptr, nullptr, &g_alloc);
        LLaMAAttentionDynParams p;
        p.batch_size = 1;
        p.num_tokens = T;
        p.max_q_len = T;
        p.max_k_len = T;
        p.num_layers = L;
        TensorMap cin{{"decoder_input", &in}, {"history_length", &hist_t}, {"input_length", &q_t},
                      {"context_length", &k_t}, {"layer_id", &layer_t}};
        TensorMap cout{{"decoder_output", &out}, {"all_k_cache", &kcache}, {"all_v_cache", &vcache}};
        dec.forward(cin, lw, cout, p);
        std::vector<float> y(x.size());
        LLMI_CALL(llmi_memcpy(y.data(), dy, y.size() * 4, 1));
        f = std::fopen((dir + "/y.bin").c_str(), "wb");
        LLM_CHECK_WITH_INFO(f && std::fwrite(y.data(), 4, y.size(), f) == y.size(), "cannot write y.bin");
        std::fclose(f);
        for (void* q : {(void*)dx, (void*)dy, (void*)kc, (void*)vc, (void*)dhist, (void*)dlen, (void*)dctx})
            g_alloc.UnifyFree(q, false);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    std::printf("ok\n");
    return 0;
}
