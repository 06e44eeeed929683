// Model-level API: the reference's Llama<T> decode loop (src/models/llama/llama.h,
// llama.cpp:318-349 continueTokenGen, :362-457 Response) and
// llm::CreateDummyLLMModel (src/utils/model_utils.h:63-70), backed by the fused,
// graph-captured engine (llmi_engine_*). Token ids in and out: the SentencePiece
// tokenizer and string prompts are out of scope, so
// MakeInput/MakeHistory are not provided.
#pragma once
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "tensor.h"

namespace llm {

// basemodel.h CallBack: index 0 = first generated token, -1 = end of the answer
using TokenCallBack = std::function<void(int index, int token)>;

class LlamaModel {
public:
    // preset: "llama2-7b", "llama2-13b", "tiny"; weight_dtype LLMI_F16 / LLMI_F32 / LLMI_I8
    LlamaModel(const std::string& preset, int weight_dtype = LLMI_F16, int kv_dtype = LLMI_F16, int max_seq = 0,
               int device = 0) {
        LLMI_CALL(llmi_config_preset(preset.c_str(), &cfg));
        cfg.weight_dtype = weight_dtype;
        cfg.kv_dtype = kv_dtype;
        if (max_seq > 0) cfg.max_seq = max_seq;
        LLMI_CALL(llmi_engine_create(&cfg, device, nullptr, &eng));
    }
    ~LlamaModel() { llmi_engine_destroy(eng); }
    LlamaModel(const LlamaModel&) = delete;
    LlamaModel& operator=(const LlamaModel&) = delete;

    void loadWeightsFromDummy(uint64_t seed = 0) { LLMI_CALL(llmi_engine_load_synthetic(eng, seed)); }
    // Llama<T>::loadWeights(weight_path) (llama_weights.cc:41-53): weight_path + "<name>.bin", raw fp32
    void loadWeights(const std::string& weight_path) { LLMI_CALL(llmi_engine_load_bin(eng, weight_path.c_str())); }
    // Llama<T>::Sampling's top-k (llama.cpp:245-262) in the decode step; k = 0 (default) is greedy
    void setSampling(int k, uint64_t seed = 0) { LLMI_CALL(llmi_engine_set_sampling(eng, k, seed)); }

    // Greedy generation (the reference's K = 1 top-k + sampling). tokens_per_sync
    // forwards run back to back (graph replays) between host reads, so the host
    // round trip the reference paid per token (llama.cpp:266,443) is amortised.
    std::vector<int> Response(const std::vector<int>& prompt, int output_token_limit, const TokenCallBack& cb = nullptr,
                              int eos_token_id = 2, int tokens_per_sync = 16) {
        LLM_CHECK_WITH_INFO(!prompt.empty(), "empty prompt");
        LLMI_CALL(llmi_engine_set_prompt(eng, prompt.data(), (int)prompt.size()));
        std::vector<int> out;
        std::vector<int> all(cfg.max_seq + 1);
        int done = 0, emitted = 0;
        const int total = std::min<int>((int)prompt.size() - 1 + output_token_limit, cfg.max_seq);
        while (done < total) {
            const int n = std::min(tokens_per_sync, total - done);
            LLMI_CALL(llmi_engine_decode(eng, n, 1));
            done += n;
            int valid = 0;
            LLMI_CALL(llmi_engine_tokens(eng, all.data(), (int)all.size(), &valid));
            for (int p = (int)prompt.size() + emitted; p < valid && emitted < output_token_limit; ++p, ++emitted) {
                out.push_back(all[p]);
                if (cb) cb(emitted, all[p]);
                if (all[p] == eos_token_id) {
                    if (cb) cb(-1, -1);
                    return out;
                }
            }
        }
        if (cb) cb(-1, -1);
        return out;
    }
    std::vector<float> lastLogits() {
        std::vector<float> l(cfg.vocab);
        LLMI_CALL(llmi_engine_logits(eng, l.data(), cfg.vocab));
        return l;
    }
    const llmi_config& config() const { return cfg; }

private:
    llmi_config cfg{};
    llmi_engine* eng = nullptr;
};

// model_utils.h:73-82 (CreateRealLLMModel): weights from the reference's .bin files (token ids in
// and out: the tokenizer stays with the caller)
inline std::unique_ptr<LlamaModel> CreateRealLLMModel(const std::string& weight_path,
                                                      const std::string& preset = "llama2-7b",
                                                      int weight_dtype = LLMI_F16) {
    auto m = std::make_unique<LlamaModel>(preset, weight_dtype);
    m->loadWeights(weight_path);
    return m;
}

// model_utils.h:63-70
inline std::unique_ptr<LlamaModel> CreateDummyLLMModel(const std::string& preset = "llama2-7b",
                                                       int weight_dtype = LLMI_F16, uint64_t seed = 0) {
    auto m = std::make_unique<LlamaModel>(preset, weight_dtype);
    m->loadWeightsFromDummy(seed);
    return m;
}

}  // namespace llm
