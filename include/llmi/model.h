// Model-level API.
//  * BaseModel / Llama<T> / llm::CreateModelWithName / CreateDummyLLMModel /
//    CreateRealLLMModel: the reference's string-in, string-out interface
//    (src/models/basemodel.h:14-42, src/models/llama/llama.h, llama.cpp:149-162
//    MakeInput/MakeHistory, :362-457 Response, src/utils/model_utils.h:17-82), so
//    user_entry.cpp compiles against this header with only its includes changed
//    (examples/user_entry.cpp). Response tokenizes the context (tokenizer.h), runs
//    the prompt as ONE batched prefill (firstTokenGen, llama.cpp:273-316) and then
//    the graph-replayed decode loop (continueTokenGen, :318-349) of the engine.
//  * LlamaModel: the same loop with token ids in and out.
#pragma once
#include <algorithm>
#include <functional>
#include <memory>
#include <string>
#include <type_traits>
#include <vector>

#include "layers.h"
#include "tensor.h"
#include "tokenizer.h"

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

// token-id variants of model_utils.h:63-82 (preset name instead of the template type)
inline std::unique_ptr<LlamaModel> CreateRealLLMModel(const std::string& weight_path,
                                                      const std::string& preset = "llama2-7b",
                                                      int weight_dtype = LLMI_F16) {
    auto m = std::make_unique<LlamaModel>(preset, weight_dtype);
    m->loadWeights(weight_path);
    return m;
}

inline std::unique_ptr<LlamaModel> CreateDummyLLMModel(const std::string& preset = "llama2-7b",
                                                       int weight_dtype = LLMI_F16, uint64_t seed = 0) {
    auto m = std::make_unique<LlamaModel>(preset, weight_dtype);
    m->loadWeightsFromDummy(seed);
    return m;
}

}  // namespace llm

// ------------------------------------------------------------------ BaseModel
// basemodel.h:10 -- index 0 = first generated piece, > 0 the next ones, -1 = end
// (content = the whole answer)
using CallBack = std::function<void(int index, const char* GenerateContent)>;

// basemodel.h:14-42. The stream / blas handle / device properties are carried for
// source compatibility; the engine owns its own HIP stream.
class BaseModel {
public:
    std::string model_name;
    void* stream;
    cublasWrapper* cublas_wrapper;
    BaseAllocator* allocator;
    void* cuda_device_prop;
    BaseModel(void* stream, cublasWrapper* cublas_wrapper, BaseAllocator* allocator, void* cuda_device_prop = nullptr)
        : stream(stream), cublas_wrapper(cublas_wrapper), allocator(allocator), cuda_device_prop(cuda_device_prop) {}
    virtual ~BaseModel() = default;
    virtual void loadTokenizer(std::string file) = 0;
    virtual void loadWeights(std::string file) = 0;
    virtual void loadWeightsFromDummy() = 0;
    virtual std::vector<std::string> MakeInput(const std::string& history, int round, const std::string& input) = 0;
    virtual std::string MakeHistory(const std::string& history, int round, const std::string& input,
                                    const std::string& output) = 0;
    virtual std::string Response(const std::vector<std::string>& input, CallBack PrintRes) = 0;
};

// llama.h: Llama<T> with T = float (the reference's working instantiation: fp32
// weights, fp32 KV cache) or half_t (fp16 weights and KV cache: the throughput
// engine). Same constructor arguments as llama.h:88-101.
template <typename T>
class Llama : public BaseModel {
    static_assert(std::is_same<T, float>::value || std::is_same<T, half_t>::value, "Llama<T>: T = float or half_t");

public:
    Llama(int head_num, int kv_head_num, int head_size, int inter_size, int num_layers, int vocab_size,
          const LLaMAAttentionStaticParams& attn_static_params, int max_seq_len, void* stream,
          cublasWrapper* cublas_wrapper, BaseAllocator* allocator, void* cuda_device_prop = nullptr, int device = 0)
        : BaseModel(stream, cublas_wrapper, allocator, cuda_device_prop) {
        model_name = "llama";
        cfg.hidden = head_num * head_size;
        cfg.heads = head_num;
        cfg.kv_heads = kv_head_num;
        cfg.head_dim = head_size;
        cfg.inter = inter_size;
        cfg.layers = num_layers;
        cfg.vocab = vocab_size;
        cfg.max_seq = max_seq_len;
        cfg.rms_eps = rmsnorm_eps;
        cfg.rope_base = attn_static_params.rotary_embedding_base;
        cfg.weight_dtype = std::is_same<T, float>::value ? LLMI_F32 : LLMI_F16;
        cfg.kv_dtype = cfg.weight_dtype;
        cfg.tp_rank = 0;
        cfg.tp_world = 1;
        LLMI_CALL(llmi_engine_create(&cfg, device, nullptr, &eng));
    }
    ~Llama() override { llmi_engine_destroy(eng); }
    Llama(const Llama&) = delete;
    Llama& operator=(const Llama&) = delete;

    void loadTokenizer(std::string file) override { tokenizer.Initialize(file); }
    // llama_weights.cc:41-53: weight_path + "<name>.bin", raw fp32 per tensor
    void loadWeights(std::string file) override { LLMI_CALL(llmi_engine_load_bin(eng, file.c_str())); }
    // layer_weights.cc dummy path -> llmi-prng-v1 synthetic weights
    void loadWeightsFromDummy() override { LLMI_CALL(llmi_engine_load_synthetic(eng, dummy_seed)); }

    // llama.cpp:149-156: {history + input (round > 0), history, input}
    std::vector<std::string> MakeInput(const std::string& history, int round, const std::string& input) override {
        return {(round == 0 ? "" : history) + input, history, input};
    }
    // llama.cpp:159-162
    std::string MakeHistory(const std::string& history, int round, const std::string& input,
                            const std::string& output) override {
        return (round == 0 ? prompt : history) + input + output;
    }

    // llama.cpp:362-457. input[0] (history + query) is tokenized with BOS first (the
    // ids the reference hard-codes at llama.cpp:371,382 are exactly that), prefilled in
    // one batched pass, then decoded until EOS, output_token_limit or max_seq. Every
    // generated piece goes to PrintRes(index, piece); PrintRes(-1, answer) at the end.
    std::string Response(const std::vector<std::string>& input, CallBack PrintRes) override {
        LLM_CHECK_WITH_INFO(!input.empty(), "Response: empty input (use MakeInput)");
        std::vector<int> ids = {bos_token_id};
        const std::vector<int> body = tokenizer.Encode(input[0]);
        ids.insert(ids.end(), body.begin(), body.end());
        // a history longer than the context window keeps BOS and its most recent half
        // (the reference has no policy: its fixed buffers overflow)
        if ((int)ids.size() >= cfg.max_seq) {
            const int keep = cfg.max_seq / 2;
            ids.erase(ids.begin() + 1, ids.end() - (keep - 1));
        }
        LLMI_CALL(llmi_engine_set_prompt(eng, ids.data(), (int)ids.size()));
        LLMI_CALL(llmi_engine_prefill(eng, (int)ids.size(), 1));  // firstTokenGen
        std::string res;
        std::vector<int> all(cfg.max_seq + 1);
        const int limit = std::min(output_token_limit, cfg.max_seq - (int)ids.size() + 1);
        int produced = 0, valid = 0;
        bool done = false;
        while (!done) {
            LLMI_CALL(llmi_engine_tokens(eng, all.data(), (int)all.size(), &valid));
            for (int p = (int)ids.size() + produced; p < valid && !done; ++p) {
                const int tok = all[p];
                if (produced > 0 && tok == eos_token_id) {  // llama.cpp:420-422
                    done = true;
                    break;
                }
                const std::string piece = tokenizer.Decode({tok});
                res += piece;
                if (PrintRes) PrintRes(produced, piece.c_str());
                if (++produced >= limit) done = true;
            }
            if (done) break;
            // continueTokenGen: graph replays, several tokens per host read
            const int n = std::min(tokens_per_sync, limit - produced);
            LLMI_CALL(llmi_engine_decode(eng, n, 1));
        }
        if (PrintRes) PrintRes(-1, res.c_str());
        return res;
    }

    // the generated ids of the last Response (for tests and callers that keep ids)
    std::vector<int> lastTokens() {
        std::vector<int> all(cfg.max_seq + 1);
        int valid = 0;
        LLMI_CALL(llmi_engine_tokens(eng, all.data(), (int)all.size(), &valid));
        all.resize(valid);
        return all;
    }
    const llmi_config& config() const { return cfg; }
    Tokenizer& getTokenizer() { return tokenizer; }

    int output_token_limit = 256;  // llama.h:29
    int bos_token_id = 1, eos_token_id = 2;
    int tokens_per_sync = 16;
    uint64_t dummy_seed = 0;
    std::string prompt = "";  // llama.h:42 built-in prompt for round 0 of MakeHistory

private:
    float rmsnorm_eps = 1e-5f;  // llama.h:22
    llmi_config cfg{};
    llmi_engine* eng = nullptr;
    Tokenizer tokenizer;
};

namespace llm {

// model_utils.h:17-61 -- the reference's dummy geometry: Llama-2-7B widths, 3 layers,
// max_seq_len 64 (its debugging configuration), rope base 10000.
template <typename T>
BaseModel* CreateModelWithName(const std::string& model_name) {
    LLM_CHECK_WITH_INFO(model_name == "llama", "dont support other models except llama yet!");
    const int head_num = 32, kv_head_num = 32, head_size = 128, inter_size = 11008, num_layers = 3;
    const int max_seq_len = 64, vocab_size = 32000;
    LLaMAAttentionStaticParams attn_static_params;
    attn_static_params.rotary_embedding_dim = 128;
    attn_static_params.rotary_embedding_base = 10000;
    attn_static_params.max_position_embeddings = 4096;
    attn_static_params.use_dynamic_ntk = false;
    static HipAllocator allocator;
    return new Llama<T>(head_num, kv_head_num, head_size, inter_size, num_layers, vocab_size, attn_static_params,
                        max_seq_len, nullptr, nullptr, &allocator);
}

// model_utils.h:63-70
template <typename T>
std::unique_ptr<BaseModel> CreateDummyLLMModel(std::string tokenizer_file) {
    BaseModel* model = CreateModelWithName<T>("llama");
    std::unique_ptr<BaseModel> owned(model);
    model->loadTokenizer(tokenizer_file);
    model->loadWeightsFromDummy();
    return owned;
}

// model_utils.h:73-82
template <typename T>
std::unique_ptr<BaseModel> CreateRealLLMModel(std::string model_dir, std::string tokenizer_file) {
    BaseModel* model = CreateModelWithName<T>("llama");
    std::unique_ptr<BaseModel> owned(model);
    model->loadTokenizer(tokenizer_file);
    model->loadWeights(model_dir);
    return owned;
}

}  // namespace llm
