// Weight and parameter structs with the reference's names and fields:
//   WeightType / BaseWeight<T>                    src/weights/base_weights.h:7-38
//   LayerNormWeight<T>                            src/weights/llama/norm_weights.h
//   EmbeddingWeight<T>                            src/weights/llama/embedding_weights.h
//   LLaMAattentionWeights<T> / LLaMAFFNWeights<T> src/weights/llama/{attention,ffn}_weights.h
//   LLaMAAttentionStaticParams / DynParams        src/models/llama/llama_params.h:3-37
// T is the weight element type: float, half_t (fp16 bits) or int8_t (W8A16; then
// `scale` points at one fp16 scale per output row -- a field the reference's
// INT8_W enum never got, base_weights.h:7-30, linear.h:15 TODO).
#pragma once
#include <type_traits>
#include <vector>

#include "tensor.h"

enum class WeightType { FP32_W, FP16_W, INT8_W, UNSUPPORTED_W };

template <typename T> inline WeightType getWeightType() {
    if (std::is_same<T, float>::value) return WeightType::FP32_W;
    if (std::is_same<T, half_t>::value) return WeightType::FP16_W;
    if (std::is_same<T, int8_t>::value) return WeightType::INT8_W;
    return WeightType::UNSUPPORTED_W;
}
inline int llmiWeightDtype(WeightType t) {
    return t == WeightType::FP32_W ? LLMI_F32 : t == WeightType::FP16_W ? LLMI_F16 : t == WeightType::INT8_W ? LLMI_I8 : -1;
}

template <typename T>
struct BaseWeight {
    std::vector<int> shape;  // [out_features, in_features] (nn.Linear layout)
    WeightType type = getWeightType<T>();
    T* data = nullptr;       // device, row-major
    T* bias = nullptr;       // unused by Llama-2 (no biases); accepted and ignored where the reference ignored it
    const half_t* scale = nullptr;  // int8 only: per-output-row fp16 scales
};

template <typename T> struct LayerNormWeight { T* gamma = nullptr; };
template <typename T> struct EmbeddingWeight : public BaseWeight<T> {};

template <typename T>
struct LLaMAattentionWeights {
    BaseWeight<T> q, k, v;   // split projections (unused: the fused qkv is used, as in the reference)
    BaseWeight<T> qkv;       // [(heads + 2 kv_heads) * head_dim, hidden], rows q;k;v
    BaseWeight<T> output;    // [hidden, heads * head_dim]
};

template <typename T>
struct LLaMAFFNWeights {
    BaseWeight<T> gate, up;  // split (unused)
    BaseWeight<T> down;      // [hidden, inter]
    BaseWeight<T> gateAndup; // [2 * inter, hidden], gate rows then up rows
};

struct LLaMAAttentionStaticParams {
    int rotary_embedding_dim = 128;
    float rotary_embedding_base = 10000.f;
    int max_position_embeddings = 4096;
    bool use_dynamic_ntk = false;  // accepted, unused (as in the reference)
};

struct LLaMAAttentionDynParams {
    int batch_size = 1;
    int num_tokens = 1;
    int max_q_len = 1;
    int max_k_len = 1;
    int num_layers = 0;
    bool is_ctx = false;
};
