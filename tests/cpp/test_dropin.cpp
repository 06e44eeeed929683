// Drop-in checks for the reference's layer / model API (include/llmi/*.h):
//  * compile-time: the reference's call syntax -- selfAttn->Forward(...) and
//    self_decoder->forward(...) as self_decoder.cpp:64 / llama.cpp:339 write them,
//    ctxAttn->forward(..., static_params) and context_decoder->forward(...) as
//    context_decoder.cpp:108 / llama.cpp:300, BaseModel* from Llama<T> -- with no
//    template arguments at the call sites;
//  * on the GPU (argv[1] = tokenizer file): Llama<half_t>::Response (tokenize ->
//    batched prefill -> decode) against the id-level decode-only loop on the same
//    weights; prints one JSON line.
#include <cstdio>
#include <string>
#include <vector>

#include "llmi/model.h"

// the reference's member-pointer call sites, verbatim in shape
template <typename T>
struct ReferenceCallSites {
    LLaMASelfAttentionLayer<T>* selfAttn;
    LlamaSelfDecoder<T>* self_decoder;
    LLaMAContextAttentionLayer<T>* ctxAttn;
    LlamaContextDecoder<T>* context_decoder;
    LLaMAFFNLayer<T>* ffn;
    void decode_layer(TensorMap& self_attn_inputs, TensorMap& self_attn_outputs, LlamaLayerWeight<T>* w,
                      LLaMAAttentionDynParams& dyn_params, TensorMap& ffn_inputs, TensorMap& ffn_outputs) {
        selfAttn->Forward(self_attn_inputs, self_attn_outputs, w->self_attn_weight, dyn_params);  // self_decoder.cpp:64
        ffn->forward(ffn_inputs, ffn_outputs, w->ffn_weight, dyn_params);                        // self_decoder.cpp:79
    }
    void decode(TensorMap& decoder_inputs, std::vector<LlamaLayerWeight<T>*>& layers, TensorMap& decoder_outputs,
                LLaMAAttentionDynParams& attn_dyn_params) {
        self_decoder->forward(decoder_inputs, layers, decoder_outputs, attn_dyn_params);  // llama.cpp:339
    }
    void context(TensorMap& ctx_attn_inputs, TensorMap& ctx_attn_output, LlamaLayerWeight<T>* w,
                 LLaMAAttentionDynParams& dyn_params, TensorMap& decoder_inputs, std::vector<LlamaLayerWeight<T>*>& layers,
                 TensorMap& decoder_outputs) {
        ctxAttn->forward(ctx_attn_inputs, ctx_attn_output, w->self_attn_weight, dyn_params,
                         ctxAttn->GetAttnStaticParams());                                    // context_decoder.cpp:108
        context_decoder->forward(decoder_inputs, layers, decoder_outputs, dyn_params);      // llama.cpp:300
    }
};
template struct ReferenceCallSites<float>;
template struct ReferenceCallSites<half_t>;

static void print_ids(const char* key, const std::vector<int>& v) {
    std::printf("\"%s\": [", key);
    for (size_t i = 0; i < v.size(); ++i) std::printf("%s%d", i ? ", " : "", v[i]);
    std::printf("]");
}

int main(int argc, char** argv) {
    if (argc < 2) return 0;  // compile / link check only
    try {
        const std::string query = "Hey, are you conscious? Can you talk to me?";
        static HipAllocator alloc;
        LLaMAAttentionStaticParams sp;
        // the tiny preset's geometry (4 heads x 128, inter 1024, 2 layers, 64 positions)
        Llama<half_t> model(4, 4, 128, 1024, 2, 32000, sp, 64, nullptr, nullptr, &alloc);
        BaseModel* base = &model;
        base->loadTokenizer(argv[1]);
        base->loadWeightsFromDummy();
        model.output_token_limit = 24;
        model.eos_token_id = -1;  // synthetic weights: generate the full budget
        std::vector<std::string> pieces;
        const std::string answer = base->Response(base->MakeInput("", 0, query), [&](int index, const char* s) {
            if (index >= 0) pieces.emplace_back(s);
        });
        std::vector<int> all = model.lastTokens();
        const int n_prompt = 1 + (int)model.getTokenizer().Encode(query).size();
        std::vector<int> prompt(all.begin(), all.begin() + n_prompt);
        std::vector<int> gen(all.begin() + n_prompt, all.end());
        // the same request through the decode-only loop (every prompt row a decode step)
        llm::LlamaModel ids_model("tiny", LLMI_F16, LLMI_F16);
        ids_model.loadWeightsFromDummy(0);
        std::vector<int> dec = ids_model.Response(prompt, (int)gen.size(), nullptr, /*eos*/ -1);
        std::printf("{");
        print_ids("prompt", prompt);
        std::printf(", ");
        print_ids("prefill_tokens", gen);
        std::printf(", ");
        print_ids("decode_tokens", dec);
        std::string joined;
        for (auto& p : pieces) joined += p;
        std::printf(", \"pieces\": %zu, \"answer_matches_pieces\": %s, \"answer_matches_decode\": %s}\n", pieces.size(),
                    joined == answer ? "true" : "false",
                    answer == model.getTokenizer().Decode(gen) ? "true" : "false");
    } catch (const std::exception& e) {
        std::printf("{\"exception\": \"%s\"}\n", e.what());
        return 2;
    }
    return 0;
}
