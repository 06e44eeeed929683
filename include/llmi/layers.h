// The reference's layer API over the llmi operator launchers:
//   BaseAllocator / allocator            src/memory/allocator/base_allocator.h:7-31
//   LlamaLayerWeight<T>                  src/weights/llama/layer_weights.h:8-44
//   LLaMASelfAttentionLayer<T>::Forward  src/layers/attention/masked_self_attention.h:53
//   LLaMAFFNLayer<T>::forward            src/layers/ffn/ffn.h:50
//   LlamaSelfDecoder<T>::forward         src/layers/decoder/self_decoder.h:65
//   LLaMAContextAttentionLayer<T>::forward src/layers/attention/context_attention.h:60
//   LlamaContextDecoder<T>::forward      src/layers/decoder/context_decoder.h:74
// Same TensorMap keys ("attention_input", "attention_output", "all_k_cache",
// "all_v_cache", "step", "layer_id", "finished", "ffn_input", "ffn_output",
// "decoder_input", "decoder_output") and the same per-layer dataflow
// (RMSNorm -> attention -> fused residual+RMSNorm -> FFN -> residual,
// self_decoder.cpp:53-86), launched op by op. The decode step with every op
// fused and graph-captured is the engine (llmi_engine_*, include/llmi/model.h).
// Fixes carried relative to the reference: the FFN keys match
// (#13), layer_id is a valid host tensor per layer (#14), decode FFN scratch is
// one token (#15), the down weight is [H, I] (#21).
#pragma once
#include <cmath>
#include <cstdlib>
#include <memory>
#include <vector>

#include "kernels.h"

class BaseAllocator {
public:
    virtual ~BaseAllocator() = default;
    template <typename T> T* Malloc(T* ptr, size_t size, bool is_host) {
        return static_cast<T*>(UnifyMalloc(static_cast<void*>(ptr), size, is_host));
    }
    virtual void* UnifyMalloc(void* ptr, size_t size, bool is_host = false) = 0;
    template <typename T> void Free(T* ptr, bool is_host) { UnifyFree(static_cast<void*>(ptr), is_host); }
    virtual void UnifyFree(void* ptr, bool is_host) = 0;
};

// Plain device/host allocations; the reference's pooled CudaAllocator policy is
// HipCachingAllocator (include/llmi/allocator.h). The engine allocates every buffer once.
class HipAllocator : public BaseAllocator {
public:
    void* UnifyMalloc(void* ptr, size_t size, bool is_host = false) override {
        (void)ptr;
        if (is_host) return std::calloc(1, size);
        void* p = nullptr;
        LLMI_CALL(llmi_device_alloc(&p, size));
        return p;
    }
    void UnifyFree(void* ptr, bool is_host) override {
        if (!ptr) return;
        if (is_host) std::free(ptr);
        else LLMI_CALL(llmi_device_free(ptr));
    }
};

namespace llmi_detail {
// The layers compute in fp32 (fp32 activations keep the logits within 1e-3 of the
// reference). An activation of the reference's fp16 instantiation
// (TensorWrapper<half>, self_decoder.cpp:59-81 with T = half) is staged: converted into
// an fp32 buffer on entry (load) and rounded back to fp16 by store(); an FP32 tensor is
// used in place; any other dtype is an error.
class ActF32 {
public:
    ActF32(Tensor* t, BaseAllocator* alloc, void* stream, bool load, const char* what)
        : t_(t), alloc_(alloc), stream_(stream) {
        LLM_CHECK_WITH_INFO(t && (t->dtype == FP32 || t->dtype == FP16),
                            std::string(what) + ": activations must be FP32 or FP16 tensors");
        if (t->dtype == FP32) {
            view_ = t->as<float>();
            return;
        }
        const size_t n = (size_t)t->size();
        buf_ = alloc->Malloc(buf_, n * sizeof(float), false);
        own_ = std::make_unique<TensorWrapper<float>>(t->location, FP32, t->shape, buf_);
        view_ = own_.get();
        if (load) LLMI_CALL(llmi_convert(t->as<half_t>()->data, LLMI_F16, buf_, LLMI_F32, n, stream));
    }
    ActF32(const ActF32&) = delete;
    ActF32& operator=(const ActF32&) = delete;
    ~ActF32() {
        if (buf_) alloc_->Free(buf_, false);
    }
    TensorWrapper<float>* get() const { return view_; }
    void store() {  // fp16 output: the fp32 result rounded back (RNE)
        if (own_) LLMI_CALL(llmi_convert(buf_, LLMI_F32, t_->as<half_t>()->data, LLMI_F16, (size_t)t_->size(), stream_));
    }

private:
    Tensor* t_;
    BaseAllocator* alloc_;
    void* stream_;
    float* buf_ = nullptr;
    std::unique_ptr<TensorWrapper<float>> own_;
    TensorWrapper<float>* view_ = nullptr;
};
}  // namespace llmi_detail

// --------------------------------------------------------------- weights
template <typename T>
class LlamaLayerWeight {
    static_assert(!std::is_same<T, int8_t>::value,
                  "the layer-by-layer API mirrors Llama<float/half>; W8A16 runs in the engine (llmi_engine_*)");

public:
    LlamaLayerWeight(int head_num, int kv_head_num, int head_size, int inter_size, WeightType weight_type, bool attn_bias,
                     BaseAllocator* alloc, int layer_id = 0)
        : head_num(head_num), kv_head_num(kv_head_num), head_size(head_size), inter_size(inter_size),
          hidden(head_num * head_size), layer_id(layer_id), alloc(alloc) {
        (void)attn_bias;
        LLM_CHECK_WITH_INFO(weight_type == getWeightType<T>(), "weight type does not match T");
        const int qkv_rows = (head_num + 2 * kv_head_num) * head_size;
        self_attn_weight.qkv = make({qkv_rows, hidden});
        self_attn_weight.output = make({hidden, head_num * head_size});
        ffn_weight.gateAndup = make({2 * inter_size, hidden});
        ffn_weight.down = make({hidden, inter_size});
        attn_norm_weight.gamma = static_cast<T*>(alloc->UnifyMalloc(nullptr, sizeof(T) * hidden));
        ffn_norm_weight.gamma = static_cast<T*>(alloc->UnifyMalloc(nullptr, sizeof(T) * hidden));
        owned = {attn_norm_weight.gamma, ffn_norm_weight.gamma};
    }
    ~LlamaLayerWeight() {
        for (void* p : owned) alloc->UnifyFree(p, false);
        for (void* p : owned_w) alloc->UnifyFree(p, false);
    }
    // layer_weights.cc:69-146 dummy path -> llmi-prng-v1 synthetic weights (the same
    // values the engine and the oracle generate for (seed, layer)).
    void loadWeights(uint64_t seed = 0) {
        const int H = hidden, q = head_num * head_size, kv = kv_head_num * head_size, I = inter_size;
        const int dt = llmiWeightDtype(getWeightType<T>());
        const int kind = LLMI_SYN_LINEAR;
        auto tid = [&](uint32_t k) { return ((uint32_t)(layer_id + 1) << 8) | k; };
        auto fill = [&](BaseWeight<T>& w, size_t row_off, uint32_t k, int rows, int cols, int ld) {
            LLMI_CALL(llmi_synth_fill(w.data + row_off * cols, dt, kind, seed, tid(k), rows, cols, 0, 0, ld, nullptr));
        };
        fill(self_attn_weight.qkv, 0, 0, q, H, H);
        fill(self_attn_weight.qkv, q, 1, kv, H, H);
        fill(self_attn_weight.qkv, q + kv, 2, kv, H, H);
        fill(self_attn_weight.output, 0, 3, H, q, q);
        fill(ffn_weight.gateAndup, 0, 4, I, H, H);
        fill(ffn_weight.gateAndup, I, 5, I, H, H);
        fill(ffn_weight.down, 0, 6, H, I, I);
        LLMI_CALL(llmi_synth_fill(attn_norm_weight.gamma, dt, LLMI_SYN_GAMMA, seed, tid(7), 1, H, 0, 0, H, nullptr));
        LLMI_CALL(llmi_synth_fill(ffn_norm_weight.gamma, dt, LLMI_SYN_GAMMA, seed, tid(8), 1, H, 0, 0, H, nullptr));
    }
    LayerNormWeight<T> attn_norm_weight, ffn_norm_weight;
    LLaMAattentionWeights<T> self_attn_weight;
    LLaMAFFNWeights<T> ffn_weight;

private:
    BaseWeight<T> make(std::vector<int> shape) {
        BaseWeight<T> w;
        w.shape = shape;
        const size_t n = (size_t)shape[0] * shape[1];
        w.data = static_cast<T*>(alloc->UnifyMalloc(nullptr, n * sizeof(T)));
        owned_w.push_back(w.data);
        return w;
    }
    int head_num, kv_head_num, head_size, inter_size, hidden, layer_id;
    BaseAllocator* alloc;
    std::vector<void*> owned, owned_w;
};

// ------------------------------------------------------------ attention
template <typename T>
class LLaMASelfAttentionLayer {
public:
    LLaMASelfAttentionLayer(int head_num, int kv_head_num, int head_size, LLaMAAttentionStaticParams attn_params,
                            void* stream, cublasWrapper* cublas_wrapper, BaseAllocator* allocator)
        : head_num(head_num), kv_head_num(kv_head_num), head_size(head_size), hidden(head_num * head_size),
          attn_static_params(attn_params), stream(stream), cublas_wrapper(cublas_wrapper), allocator(allocator) {}
    ~LLaMASelfAttentionLayer() { freeBuf(); }
    LLaMAAttentionStaticParams& GetAttnStaticParams() { return attn_static_params; }

    void allocForForward(LLaMAAttentionDynParams& params) {
        if (qkv_buf) return;
        const int qkv_heads = head_num + 2 * kv_head_num;
        qkv_ptr = allocator->Malloc(qkv_ptr, sizeof(float) * params.batch_size * qkv_heads * head_size, false);
        mha_ptr = allocator->Malloc(mha_ptr, sizeof(float) * params.batch_size * hidden, false);
        qkv_buf = std::make_unique<TensorWrapper<float>>(GPU, FP32, std::vector<int>{params.batch_size, qkv_heads, head_size}, qkv_ptr);
        mha_output = std::make_unique<TensorWrapper<float>>(GPU, FP32, std::vector<int>{params.batch_size, head_num, head_size}, mha_ptr);
    }
    void freeBuf() {
        if (qkv_ptr) allocator->Free(qkv_ptr, false);
        if (mha_ptr) allocator->Free(mha_ptr, false);
        qkv_ptr = mha_ptr = nullptr;
        qkv_buf.reset();
        mha_output.reset();
    }

    // masked_self_attention.cpp:54-92: qkv GEMV -> RoPE -> fused KV write + MHA -> o_proj.
    // The reference's call (self_decoder.cpp:64): the cache element type comes from the
    // "all_k_cache" tensor's dtype at run time (FP32 for parity, FP16 for throughput).
    void Forward(TensorMap& inputs, TensorMap& outputs, LLaMAattentionWeights<T>& weights,
                 LLaMAAttentionDynParams& params) {
        const DataType cdt = outputs["all_k_cache"]->dtype;
        LLM_CHECK_WITH_INFO(outputs["all_v_cache"]->dtype == cdt, "k and v caches must have the same dtype");
        if (cdt == FP32)
            ForwardCache<float>(inputs, outputs, weights, params);
        else if (cdt == FP16)
            ForwardCache<half_t>(inputs, outputs, weights, params);
        else
            LLM_CHECK_WITH_INFO(false, "kv cache dtype must be FP32 or FP16");
    }

private:
    template <typename CT>
    void ForwardCache(TensorMap& inputs, TensorMap& outputs, LLaMAattentionWeights<T>& weights,
                      LLaMAAttentionDynParams& params) {
        allocForForward(params);
        llmi_detail::ActF32 in(inputs["attention_input"], allocator, stream, true, "LLaMASelfAttentionLayer");
        llmi_detail::ActF32 out(outputs["attention_output"], allocator, stream, false, "LLaMASelfAttentionLayer");
        TensorWrapper<float>* attention_input = in.get();
        TensorWrapper<float>* attention_output = out.get();
        TensorWrapper<CT>* key_cache = outputs["all_k_cache"]->as<CT>();
        TensorWrapper<CT>* value_cache = outputs["all_v_cache"]->as<CT>();
        TensorWrapper<bool>* finished = inputs["finished"]->as<bool>();
        TensorWrapper<int>* step = inputs["step"]->as<int>();
        TensorWrapper<int>* layer_id = inputs["layer_id"]->as<int>();
        cublasWrapper cw{stream};
        launchLinearGemm(attention_input, weights.qkv, qkv_buf.get(), cublas_wrapper ? cublas_wrapper : &cw, false, true);
        launchRoPE(qkv_buf.get(), step, attn_static_params, kv_head_num, stream);
        launchDecoderMaskedMHA(qkv_buf.get(), weights.qkv, layer_id, key_cache, value_cache, finished, step,
                               mha_output.get(), attn_static_params, stream);
        launchLinearGemm(mha_output.get(), weights.output, attention_output, cublas_wrapper ? cublas_wrapper : &cw,
                         false, true);
        out.store();
    }

    int head_num, kv_head_num, head_size, hidden;
    LLaMAAttentionStaticParams attn_static_params;
    void* stream;
    cublasWrapper* cublas_wrapper;
    BaseAllocator* allocator;
    float *qkv_ptr = nullptr, *mha_ptr = nullptr;
    std::unique_ptr<TensorWrapper<float>> qkv_buf, mha_output;
};

// ------------------------------------------------------------------ FFN
template <typename T>
class LLaMAFFNLayer {
public:
    LLaMAFFNLayer(int head_num, int head_size, int inter_size, void* stream, cublasWrapper* cublas_wrapper,
                  BaseAllocator* allocator)
        : inter_size(inter_size), hidden(head_num * head_size), stream(stream), cublas_wrapper(cublas_wrapper),
          allocator(allocator) {}
    ~LLaMAFFNLayer() { freeBuf(); }
    // rows: batch_size in decode, num_tokens in the context phase (ffn.cpp:55-60)
    void allocForForward(int rows) {
        if (rows > cap) {
            freeBuf();
            gu_ptr = allocator->Malloc(gu_ptr, sizeof(float) * rows * 2 * inter_size, false);
            act_ptr = allocator->Malloc(act_ptr, sizeof(float) * rows * inter_size, false);
            cap = rows;
        }
        SwiGLU_input = std::make_unique<TensorWrapper<float>>(GPU, FP32, std::vector<int>{rows, 2, inter_size}, gu_ptr);
        down_proj_input = std::make_unique<TensorWrapper<float>>(GPU, FP32, std::vector<int>{rows, inter_size}, act_ptr);
    }
    void freeBuf() {
        if (gu_ptr) allocator->Free(gu_ptr, false);
        if (act_ptr) allocator->Free(act_ptr, false);
        gu_ptr = act_ptr = nullptr;
        cap = 0;
        SwiGLU_input.reset();
        down_proj_input.reset();
    }
    // ffn.cpp:52-93: gate_up GEMV -> SiLU*mul -> down GEMV
    void forward(TensorMap& inputs, TensorMap& outputs, LLaMAFFNWeights<T>& weights, LLaMAAttentionDynParams& params) {
        allocForForward(params.is_ctx ? params.num_tokens : params.batch_size);
        llmi_detail::ActF32 in(inputs["ffn_input"], allocator, stream, true, "LLaMAFFNLayer");
        llmi_detail::ActF32 out(outputs["ffn_output"], allocator, stream, false, "LLaMAFFNLayer");
        cublasWrapper cw{stream};
        cublasWrapper* c = cublas_wrapper ? cublas_wrapper : &cw;
        const int rows = params.is_ctx ? params.num_tokens : params.batch_size;
        // context rows with fp16 weights: gate_up + SiLU*up + down in one fused call
        // (llmi_ffn; same products as the three launches below, the SiLU*up rows handed to
        // the down GEMM as its fp16 input planes instead of an fp32 buffer)
        const int rc = (params.is_ctx && rows >= 16 && getTensorType<T>() == FP16 &&
                        weights.gateAndup.type == WeightType::FP16_W && weights.down.type == WeightType::FP16_W)
                           ? llmi_ffn(in.get()->data, weights.gateAndup.data, weights.down.data, LLMI_F16,
                                      out.get()->data, rows, hidden, inter_size, stream)
                           : LLMI_EUNSUPPORTED;
        if (rc == LLMI_OK) {
            out.store();
            if (check_errors) llmi_detail::checkStreamErrors(stream, "LLaMAFFNLayer::forward");
            return;
        }
        if (rc != LLMI_EUNSUPPORTED) LLMI_CALL(rc);
        launchLinearGemm(in.get(), weights.gateAndup, SwiGLU_input.get(), c, false, true);
        launchAct(SwiGLU_input.get(), down_proj_input.get(), stream);
        launchLinearGemm(down_proj_input.get(), weights.down, out.get(), c, false, true);
        out.store();
        if (check_errors) llmi_detail::checkStreamErrors(stream, "LLaMAFFNLayer::forward");
    }
    // false: the caller (a decoder running many layers) checks once per forward instead
    bool check_errors = true;

private:
    int inter_size, hidden;
    void* stream;
    cublasWrapper* cublas_wrapper;
    BaseAllocator* allocator;
    float *gu_ptr = nullptr, *act_ptr = nullptr;
    int cap = 0;
    std::unique_ptr<TensorWrapper<float>> SwiGLU_input, down_proj_input;
};

// -------------------------------------------------------------- decoder
template <typename T>
class LlamaSelfDecoder {
public:
    LlamaSelfDecoder(int head_num, int kv_head_num, int head_size, int inter_size, int num_layer,
                     const LLaMAAttentionStaticParams& attn_params, float rmsnorm_eps, void* stream,
                     cublasWrapper* cublas_wrapper, BaseAllocator* allocator)
        : hidden(head_num * head_size), num_layer(num_layer), rmsnorm_eps(rmsnorm_eps), stream(stream),
          allocator(allocator),
          selfAttn(head_num, kv_head_num, head_size, attn_params, stream, cublas_wrapper, allocator),
          ffn(head_num, head_size, inter_size, stream, cublas_wrapper, allocator) {}
    ~LlamaSelfDecoder() {
        if (resid_ptr) allocator->Free(resid_ptr, false);
        for (float* p : fbuf)
            if (p) allocator->Free(p, false);
    }

    // self_decoder.cpp:23-89 for one token; inputs "decoder_input" [1, H], "step" and
    // "layer_id" (host int), "finished"; outputs "decoder_output", "all_k_cache", "all_v_cache"
    // (FP32 or FP16 caches, chosen by their dtype).
    // A batch-1 token runs five launches per layer instead of the reference's ten (same math,
    // fp32 activations): RMSNorm folded into the q/k/v GEMV, RoPE into the attention (which
    // writes the KV slot), the residual adds into the o_proj / down GEMV epilogues, RMSNorm +
    // SiLU * up into the gate_up GEMV (llmi_linear_fused). Other batch sizes go op by op.
    void forward(TensorMap& input_tensors, const std::vector<LlamaLayerWeight<T>*>& layerWeights,
                 TensorMap& output_tensors, LLaMAAttentionDynParams& dyn_params) {
        if (dyn_params.batch_size == 1 && fused_ok(input_tensors, output_tensors)) {
            llmi_detail::ActF32 din(input_tensors["decoder_input"], allocator, stream, true, "LlamaSelfDecoder");
            llmi_detail::ActF32 dout(output_tensors["decoder_output"], allocator, stream, false, "LlamaSelfDecoder");
            forward_fused(din.get(), dout.get(), input_tensors, output_tensors, layerWeights);
            dout.store();
            return;
        }
        if (!resid_ptr) {
            resid_ptr = allocator->Malloc(resid_ptr, sizeof(float) * dyn_params.batch_size * hidden, false);
            decoder_residual = std::make_unique<TensorWrapper<float>>(GPU, FP32, std::vector<int>{dyn_params.batch_size, hidden}, resid_ptr);
        }
        dyn_params.is_ctx = false;  // one token: FFN scratch is batch_size rows
        // fp16 activations (Llama<half>) are staged once here; the sublayers then run fp32
        llmi_detail::ActF32 din(input_tensors["decoder_input"], allocator, stream, true, "LlamaSelfDecoder");
        llmi_detail::ActF32 dout(output_tensors["decoder_output"], allocator, stream, false, "LlamaSelfDecoder");
        TensorWrapper<float>* decoder_input = din.get();
        TensorWrapper<float>* decoder_output = dout.get();
        int layer = 0;
        TensorWrapper<int> layer_id(CPU, INT32, {1}, &layer);
        TensorMap attn_in{{"attention_input", decoder_input}, {"finished", input_tensors["finished"]},
                          {"step", input_tensors["step"]}, {"layer_id", &layer_id}};
        TensorMap attn_out{{"attention_output", decoder_output}, {"all_k_cache", output_tensors["all_k_cache"]},
                           {"all_v_cache", output_tensors["all_v_cache"]}};
        TensorMap ffn_in{{"ffn_input", decoder_output}}, ffn_out{{"ffn_output", decoder_output}};
        for (layer = 0; layer < num_layer; ++layer) {
            LlamaLayerWeight<T>* w = layerWeights[layer];
            // decoder_input <- RMSNorm(x), residual <- x
            launchRMSNorm(decoder_input, decoder_residual.get(), w->attn_norm_weight, rmsnorm_eps, false, stream);
            selfAttn.Forward(attn_in, attn_out, w->self_attn_weight, dyn_params);
            // residual += attention_out; decoder_output <- RMSNorm(residual)
            BaseWeight<T> no_bias;
            launchFusedAddBiasResidualRMSNorm(decoder_residual.get(), decoder_output, no_bias, w->ffn_norm_weight.gamma,
                                              rmsnorm_eps, stream);
            ffn.forward(ffn_in, ffn_out, w->ffn_weight, dyn_params);
            launchAddResidual(decoder_residual.get(), decoder_output, false, stream);  // x = residual + ffn_out
            decoder_input = decoder_output;
            attn_in.insert("attention_input", decoder_output);
        }
        dout.store();
    }

private:
    bool fused_ok(TensorMap& in, TensorMap& out) {
        Tensor* x = in["decoder_input"];
        Tensor* k = out["all_k_cache"];
        Tensor* v = out["all_v_cache"];
        return x->size() == hidden && k->shape.size() == 5 && k->shape[1] == 1 && v->dtype == k->dtype &&
               (k->dtype == FP32 || k->dtype == FP16);
    }
    float* scratch(int slot, size_t n) {
        if (n > fcap[slot]) {
            if (fbuf[slot]) allocator->Free(fbuf[slot], false);
            fbuf[slot] = allocator->Malloc(fbuf[slot], n * sizeof(float), false);
            fcap[slot] = n;
        }
        return fbuf[slot];
    }
    void forward_fused(TensorWrapper<float>* xin, TensorWrapper<float>* xout, TensorMap& in, TensorMap& out,
                       const std::vector<LlamaLayerWeight<T>*>& lw) {
        Tensor* kc = out["all_k_cache"];
        Tensor* vc = out["all_v_cache"];
        const int kv = kc->shape[2], max_seq = kc->shape[3], hd = kc->shape[4];
        const int step = in["step"]->as<int>()->getVal();
        LLM_CHECK_WITH_INFO(step >= 1 && step <= max_seq, "LlamaSelfDecoder: step out of the cache range");
        LLM_CHECK_WITH_INFO((int)lw.size() >= num_layer, "LlamaSelfDecoder: fewer layer weights than layers");
        const int wdt = llmiWeightDtype(getWeightType<T>());
        const int cdt = kc->dtype == FP16 ? LLMI_F16 : LLMI_F32;
        const float base = selfAttn.GetAttnStaticParams().rotary_embedding_base;
        auto raw = [](Tensor* t) -> void* {
            return t->dtype == FP16 ? (void*)t->as<half_t>()->data : (void*)t->as<float>()->data;
        };
        void* kd = raw(kc);
        void* vd = raw(vc);
        float* x = xin->data;
        float* y = xout->data;
        for (int l = 0; l < num_layer; ++l) {
            LlamaLayerWeight<T>* w = lw[l];
            const int qkv_rows = w->self_attn_weight.qkv.shape[0], inter = w->ffn_weight.down.shape[1];
            const int heads = qkv_rows / hd - 2 * kv;
            float* qkv = scratch(0, qkv_rows);
            float* mha = scratch(1, (size_t)heads * hd);
            float* r = scratch(2, hidden);
            float* act = scratch(3, inter);
            void* ws = llmi_detail::attn_workspace(heads, hd, max_seq);
            // RMSNorm(x) . Wqkv^T; rope + KV slot step - 1 + masked MHA; r = x + o . Wo^T
            LLMI_CALL(llmi_linear_fused(x, w->self_attn_weight.qkv.data, wdt, nullptr, qkv, qkv_rows, hidden,
                                        w->attn_norm_weight.gamma, wdt, rmsnorm_eps, 0, nullptr, stream));
            LLMI_CALL(llmi_attn_decode(qkv, kd, vd, cdt, l, max_seq, step - 1, heads, kv, hd, 1, base, mha,
                                       ws, stream));
            LLMI_CALL(llmi_linear_fused(mha, w->self_attn_weight.output.data, wdt, nullptr, r, hidden, heads * hd,
                                        nullptr, wdt, 0.f, 1, x, stream));
            // silu(RMSNorm(r) . Wg^T) * (RMSNorm(r) . Wu^T); out = r + act . Wd^T
            LLMI_CALL(llmi_linear_fused(r, w->ffn_weight.gateAndup.data, wdt, nullptr, act, 2 * inter, hidden,
                                        w->ffn_norm_weight.gamma, wdt, rmsnorm_eps, 2, nullptr, stream));
            LLMI_CALL(llmi_linear_fused(act, w->ffn_weight.down.data, wdt, nullptr, y, hidden, inter, nullptr, wdt, 0.f,
                                        1, r, stream));
            x = y;
        }
    }

    int hidden, num_layer;
    float rmsnorm_eps;
    void* stream;
    BaseAllocator* allocator;
    LLaMASelfAttentionLayer<T> selfAttn;
    LLaMAFFNLayer<T> ffn;
    float* resid_ptr = nullptr;
    std::unique_ptr<TensorWrapper<float>> decoder_residual;
    float* fbuf[4] = {nullptr, nullptr, nullptr, nullptr};
    size_t fcap[4] = {0, 0, 0, 0};
};

// ------------------------------------------------------ context phase
// LLaMAContextAttentionLayer<T>::forward (context_attention.cpp:85-174) over the
// context launchers: qkv GEMM -> RoPE + transpose (with history offsets) -> KV
// concat -> repeat_kv -> QK^T -> scale + causal mask + softmax -> PV -> transpose +
// remove padding -> o_proj. Activations and caches fp32 (the reference's working
// Llama<float>); the engine's fused MFMA prefill (llmi_engine_prefill) is the fast
// path. Fixed relative to the reference: the qkv buffer holds all
// (heads + 2 kv) heads and QK^T uses the repeated cache (history included), not the
// current query's un-repeated k.
template <typename T>
class LLaMAContextAttentionLayer {
public:
    LLaMAContextAttentionLayer(int head_num, int kv_head_num, int head_size, LLaMAAttentionStaticParams attn_params,
                               void* stream, cublasWrapper* cublas_wrapper, BaseAllocator* allocator)
        : head_num(head_num), kv_head_num(kv_head_num), head_size(head_size), hidden_units(head_num * head_size),
          q_head_per_kv(head_num / kv_head_num), scale(1.0f / std::sqrt((float)head_size)),
          attn_static_params(attn_params), stream(stream), cublas_wrapper(cublas_wrapper), allocator(allocator) {}
    ~LLaMAContextAttentionLayer() { freeBuf(); }
    LLaMAAttentionStaticParams& GetAttnStaticParams() { return attn_static_params; }

    // context_attention.cpp:26-74: buffers sized by batch_size, num_tokens, max_q_len, max_k_len
    // (with the fused attention core -- head_size 128 -- the repeated caches, the score
    // matrix and the padded output are never materialised, so they are not allocated)
    void allocForForward(LLaMAAttentionDynParams& p) {
        freeBuf();
        const int qkv_heads = head_num + 2 * kv_head_num, b = p.batch_size, q = p.max_q_len, k = p.max_k_len;
        qkv_buf_wo_pad = make({p.num_tokens, qkv_heads, head_size});
        q_buf_w_pad = make({b, head_num, q, head_size});
        if (!fused()) {
            k_buf_w_pad = make({b, kv_head_num, q, head_size});
            v_buf_w_pad = make({b, kv_head_num, q, head_size});
            k_cache_buf = make({b, head_num, k, head_size});
            v_cache_buf = make({b, head_num, k, head_size});
            qk_buf = make({b, head_num, q, k});
            qkv_buf_w_pad = make({b, head_num, q, head_size});
        }
        qkv_buf_wo_pad_1 = make({p.num_tokens, head_num, head_size});
    }
    // llmi_context_attention's shape: the whole repeat -> QK^T -> mask + softmax -> PV ->
    // transpose chain as one launch (context_ops.hip). It applies llmi_causal_mask's mask
    // (what LlamaContextDecoder builds, context_decoder.cpp:68-71) and ignores the
    // "attention_mask" input; a caller with another mask calls setFusedCore(false).
    bool fused() const { return fused_core && head_size == 128 && head_num % kv_head_num == 0; }
    void setFusedCore(bool on) { fused_core = on; }
    void freeBuf() {
        for (auto& t : bufs) allocator->Free(t->data, false);
        bufs.clear();
        for (auto& t : hbufs) allocator->Free(t->data, false);
        hbufs.clear();
    }

    // inputs: "attention_input" [num_tokens, H], "padding_offset", "history_length",
    // "input_length", "context_length" (device int), "layer_id" (host int),
    // "attention_mask" [bs, max_q_len, max_k_len]; outputs: "attention_output"
    // [num_tokens, H], "all_k_cache" / "all_v_cache" [layers, bs, kv_heads, max_seq, head]
    void forward(TensorMap& inputs, TensorMap& outputs, LLaMAattentionWeights<T>& weights,
                 LLaMAAttentionDynParams& params, LLaMAAttentionStaticParams& static_params) {
        const DataType cdt = outputs["all_k_cache"]->dtype;
        LLM_CHECK_WITH_INFO((cdt == FP32 || cdt == FP16) && outputs["all_v_cache"]->dtype == cdt,
                            "the context attention layer's k/v caches must both be FP32 or both FP16");
        allocForForward(params);
        cublasWrapper cw{stream};
        cublasWrapper* c = cublas_wrapper ? cublas_wrapper : &cw;
        TensorWrapper<int>* padding_offset = inputs["padding_offset"]->as<int>();
        TensorWrapper<int>* history_length = inputs["history_length"]->as<int>();
        TensorWrapper<int>* input_length = inputs["input_length"]->as<int>();
        TensorWrapper<int>* context_length = inputs["context_length"]->as<int>();
        TensorWrapper<int>* layer_id = inputs["layer_id"]->as<int>();
        llmi_detail::ActF32 in(inputs["attention_input"], allocator, stream, true, "LLaMAContextAttentionLayer");
        llmi_detail::ActF32 out(outputs["attention_output"], allocator, stream, false, "LLaMAContextAttentionLayer");
        if (fused()) {
            launchLinearGemm(forwardCore(in.get(), inputs, outputs, weights, params, static_params), weights.output,
                             out.get(), c, false, true);
            out.store();
            freeBuf();
            if (check_errors) llmi_detail::checkStreamErrors(stream, "LLaMAContextAttentionLayer::forward");
            return;
        }
        // 1. qkv linear
        launchLinearGemm(in.get(), weights.qkv, qkv_buf_wo_pad, c, false, true);
        // 2. RoPE (position history + s) and [num_tokens, ...] -> [bs, heads, max_q_len, head]
        launchAddFusedQKVBiasTransposeAndRoPE(q_buf_w_pad, k_buf_w_pad, v_buf_w_pad, qkv_buf_wo_pad, weights.qkv,
                                              padding_offset, history_length, input_length, static_params, stream);
        // positions past a sequence's context are never written by the repeat: zero them,
        // so the masked columns of QK^T / PV multiply finite values
        LLMI_CALL(llmi_device_memset_async(k_cache_buf->data, 0, k_cache_buf->size() * sizeof(float), stream));
        LLMI_CALL(llmi_device_memset_async(v_cache_buf->data, 0, v_cache_buf->size() * sizeof(float), stream));
        if (cdt == FP32) {
            TensorWrapper<float>* all_k_cache = outputs["all_k_cache"]->as<float>();
            TensorWrapper<float>* all_v_cache = outputs["all_v_cache"]->as<float>();
            // 3. append this prompt's k, v to the layer's cache after the history
            launchConcatKVCache(k_buf_w_pad, v_buf_w_pad, layer_id, input_length, history_length, all_k_cache,
                                all_v_cache, stream);
            // 4. history + prompt, kv heads repeated to the query heads
            launchRepeatKVCache(all_k_cache, all_v_cache, context_length, layer_id, k_cache_buf, v_cache_buf, stream);
        } else {
            // LLaMAContextAttentionLayer<half> (context_attention.cpp:177): the caches hold fp16.
            // The new k/v rows are rounded to fp16 as they enter the cache (what the reference's
            // half instantiation stores) and the repeated cache is widened back to fp32.
            TensorWrapper<half_t>* all_k_cache = outputs["all_k_cache"]->as<half_t>();
            TensorWrapper<half_t>* all_v_cache = outputs["all_v_cache"]->as<half_t>();
            TensorWrapper<half_t>* kh = make_half(k_buf_w_pad->shape);
            TensorWrapper<half_t>* vh = make_half(v_buf_w_pad->shape);
            LLMI_CALL(llmi_convert(k_buf_w_pad->data, LLMI_F32, kh->data, LLMI_F16, kh->size(), stream));
            LLMI_CALL(llmi_convert(v_buf_w_pad->data, LLMI_F32, vh->data, LLMI_F16, vh->size(), stream));
            launchConcatKVCache(kh, vh, layer_id, input_length, history_length, all_k_cache, all_v_cache, stream);
            TensorWrapper<half_t>* kr = make_half(k_cache_buf->shape);
            TensorWrapper<half_t>* vr = make_half(v_cache_buf->shape);
            LLMI_CALL(llmi_device_memset_async(kr->data, 0, kr->size() * sizeof(half_t), stream));
            LLMI_CALL(llmi_device_memset_async(vr->data, 0, vr->size() * sizeof(half_t), stream));
            launchRepeatKVCache(all_k_cache, all_v_cache, context_length, layer_id, kr, vr, stream);
            LLMI_CALL(llmi_convert(kr->data, LLMI_F16, k_cache_buf->data, LLMI_F32, kr->size(), stream));
            LLMI_CALL(llmi_convert(vr->data, LLMI_F16, v_cache_buf->data, LLMI_F32, vr->size(), stream));
        }
        launchLinearStridedBatchGemm(q_buf_w_pad, k_cache_buf, qk_buf, c, false, true);
        launchScaleMaskAndSoftmax(qk_buf, inputs["attention_mask"]->as<float>(), qk_buf, scale, stream);
        launchLinearStridedBatchGemm(qk_buf, v_cache_buf, qkv_buf_w_pad, c, false, false);
        // 5. [bs, heads, max_q_len, head] -> [num_tokens, H], then o_proj
        launchTransposeOutRemovePadding(qkv_buf_w_pad, padding_offset, qkv_buf_wo_pad_1, stream);
        launchLinearGemm(qkv_buf_wo_pad_1, weights.output, out.get(), c, false, true);
        out.store();
        freeBuf();
        if (check_errors) llmi_detail::checkStreamErrors(stream, "LLaMAContextAttentionLayer::forward");
    }
    // false: the caller (LlamaContextDecoder) checks once per forward instead
    bool check_errors = true;

    // forward's steps 1-5 without o_proj, fused core only (fused(), after allocForForward):
    // qkv projection of x (fp32 [num_tokens, H]; for fp16 weights inside
    // llmi_context_attention_proj, its K slices summed by the RoPE kernel), then RoPE with the k / v rows stored
    // straight into the cache after the history, then the attention core over the cache (one
    // launch each; fp16 caches are read as they are: the unfused chain widens exactly these
    // values to fp32). Returns the [num_tokens, H] attention rows, valid until freeBuf().
    TensorWrapper<float>* forwardCore(TensorWrapper<float>* x, TensorMap& inputs, TensorMap& outputs,
                                      LLaMAattentionWeights<T>& weights, LLaMAAttentionDynParams& params,
                                      LLaMAAttentionStaticParams& static_params) {
        LLM_CHECK_WITH_INFO(fused() && qkv_buf_wo_pad_1, "forwardCore: fused core after allocForForward only");
        const DataType cdt = outputs["all_k_cache"]->dtype;
        void* kcache = cdt == FP32 ? (void*)outputs["all_k_cache"]->as<float>()->data
                                   : (void*)outputs["all_k_cache"]->as<half_t>()->data;
        void* vcache = cdt == FP32 ? (void*)outputs["all_v_cache"]->as<float>()->data
                                   : (void*)outputs["all_v_cache"]->as<half_t>()->data;
        const int* po = inputs["padding_offset"]->as<int>()->data;
        const int* hist = inputs["history_length"]->as<int>()->data;
        const int* ql = inputs["input_length"]->as<int>()->data;
        const int cd = cdt == FP32 ? LLMI_F32 : LLMI_F16, layer = inputs["layer_id"]->as<int>()->getVal();
        const int max_seq = outputs["all_k_cache"]->shape[3];
        const float base = static_params.rotary_embedding_base;
        // fp16 weights: the projection's K slices go straight into the RoPE kernel
        int rc = llmi_context_attention_proj(x->data, weights.qkv.data, llmiWeightDtype(getWeightType<T>()),
                                             weights.qkv.shape[1], po, hist, ql, params.num_tokens, params.batch_size,
                                             params.max_q_len, head_num, kv_head_num, head_size, base, kcache, vcache,
                                             cd, layer, max_seq, scale, q_buf_w_pad->data, qkv_buf_wo_pad_1->data,
                                             stream);
        if (rc == LLMI_EUNSUPPORTED) {
            cublasWrapper cw{stream};
            launchLinearGemm(x, weights.qkv, qkv_buf_wo_pad, cublas_wrapper ? cublas_wrapper : &cw, false, true);
            rc = llmi_context_attention_qkv(qkv_buf_wo_pad->data, po, hist, ql, params.num_tokens, params.batch_size,
                                            params.max_q_len, head_num, kv_head_num, head_size, base, kcache, vcache,
                                            cd, layer, max_seq, scale, q_buf_w_pad->data, qkv_buf_wo_pad_1->data,
                                            stream);
        }
        LLMI_CALL(rc);
        return qkv_buf_wo_pad_1;
    }

private:
    TensorWrapper<float>* make(std::vector<int> shape) {
        size_t n = 1;
        for (int d : shape) n *= (size_t)d;
        float* p = nullptr;
        p = allocator->Malloc(p, sizeof(float) * n, false);
        bufs.push_back(std::make_unique<TensorWrapper<float>>(GPU, FP32, shape, p));
        return bufs.back().get();
    }
    TensorWrapper<half_t>* make_half(std::vector<int> shape) {  // fp16-cache staging
        size_t n = 1;
        for (int d : shape) n *= (size_t)d;
        half_t* p = nullptr;
        p = allocator->Malloc(p, sizeof(half_t) * n, false);
        hbufs.push_back(std::make_unique<TensorWrapper<half_t>>(GPU, FP16, shape, p));
        return hbufs.back().get();
    }
    std::vector<std::unique_ptr<TensorWrapper<half_t>>> hbufs;
    bool fused_core = true;
    int head_num, kv_head_num, head_size, hidden_units, q_head_per_kv;
    float scale;
    LLaMAAttentionStaticParams attn_static_params;
    void* stream;
    cublasWrapper* cublas_wrapper;
    BaseAllocator* allocator;
    std::vector<std::unique_ptr<TensorWrapper<float>>> bufs;
    TensorWrapper<float> *qkv_buf_wo_pad = nullptr, *q_buf_w_pad = nullptr, *k_buf_w_pad = nullptr,
                         *v_buf_w_pad = nullptr, *k_cache_buf = nullptr, *v_cache_buf = nullptr, *qk_buf = nullptr,
                         *qkv_buf_w_pad = nullptr, *qkv_buf_wo_pad_1 = nullptr;
};

// LlamaContextDecoder<T>::forward (context_decoder.cpp:47-143): padding offsets and
// the causal mask once, then per layer RMSNorm -> context attention -> fused
// residual + RMSNorm -> FFN (num_tokens rows) -> residual.
// inputs: "decoder_input" [num_tokens, H] (embedded prompt rows, overwritten),
// "history_length", "input_length", "context_length" (device int [bs]),
// "layer_id" (host int); outputs: "decoder_output" [num_tokens, H], "all_k_cache",
// "all_v_cache" (fp32). dyn_params: batch_size, num_tokens, max_q_len, max_k_len.
template <typename T>
class LlamaContextDecoder {
public:
    LlamaContextDecoder(int head_num, int kv_head_num, int head_size, int inter_size, int num_layer,
                        const LLaMAAttentionStaticParams& attn_params, float rmsnorm_eps, void* stream,
                        cublasWrapper* cublas_wrapper, BaseAllocator* allocator)
        : hidden_units(head_num * head_size), num_layer(num_layer), rmsnorm_eps(rmsnorm_eps), stream(stream),
          allocator(allocator),
          ctxAttn(head_num, kv_head_num, head_size, attn_params, stream, cublas_wrapper, allocator),
          ffn(head_num, head_size, inter_size, stream, cublas_wrapper, allocator) {
        ctxAttn.check_errors = ffn.check_errors = false;  // checked once at the end of forward
    }
    ~LlamaContextDecoder() { freeBuf(); }
    // the attention core as one fused launch (default) or the reference's unfused chain
    void setFusedAttentionCore(bool on) { ctxAttn.setFusedCore(on); }

    void allocForForward(LLaMAAttentionDynParams& p) {
        freeBuf();
        mask_ptr = allocator->Malloc(mask_ptr, sizeof(float) * p.batch_size * p.max_q_len * p.max_k_len, false);
        po_ptr = allocator->Malloc(po_ptr, sizeof(int) * p.batch_size * p.max_q_len, false);
        cum_ptr = allocator->Malloc(cum_ptr, sizeof(int) * (p.batch_size + 1), false);
        resid_ptr = allocator->Malloc(resid_ptr, sizeof(float) * p.num_tokens * hidden_units, false);
        attention_mask = std::make_unique<TensorWrapper<float>>(GPU, FP32, std::vector<int>{p.batch_size, p.max_q_len, p.max_k_len}, mask_ptr);
        padding_offset = std::make_unique<TensorWrapper<int>>(GPU, INT32, std::vector<int>{p.batch_size, p.max_q_len}, po_ptr);
        cum_seqlens = std::make_unique<TensorWrapper<int>>(GPU, INT32, std::vector<int>{p.batch_size + 1}, cum_ptr);
        decoder_residual = std::make_unique<TensorWrapper<float>>(GPU, FP32, std::vector<int>{p.num_tokens, hidden_units}, resid_ptr);
    }
    void freeBuf() {
        for (void* p : {(void*)mask_ptr, (void*)po_ptr, (void*)cum_ptr, (void*)resid_ptr})
            if (p) allocator->UnifyFree(p, false);
        mask_ptr = resid_ptr = nullptr;
        po_ptr = cum_ptr = nullptr;
    }

    void forward(TensorMap& input_tensors, const std::vector<LlamaLayerWeight<T>*>& layerWeights,
                 TensorMap& output_tensors, LLaMAAttentionDynParams& dyn_params) {
        allocForForward(dyn_params);
        Tensor* seq_lens = input_tensors["input_length"];
        launchCalPaddingoffset(padding_offset.get(), cum_seqlens.get(), seq_lens->as<int>(), stream);
        launchBuildCausalMasks(attention_mask.get(), seq_lens->as<int>(), input_tensors["context_length"]->as<int>(),
                               stream);
        llmi_detail::ActF32 din(input_tensors["decoder_input"], allocator, stream, true, "LlamaContextDecoder");
        llmi_detail::ActF32 dout(output_tensors["decoder_output"], allocator, stream, false, "LlamaContextDecoder");
        TensorWrapper<float>* decoder_output = dout.get();
        int layer = 0;
        TensorWrapper<int> layer_id(CPU, INT32, {1}, &layer);
        TensorMap ctx_attn_inputs{{"attention_input", din.get()},
                                  {"padding_offset", padding_offset.get()},
                                  {"history_length", input_tensors["history_length"]},
                                  {"input_length", seq_lens},
                                  {"layer_id", &layer_id},
                                  {"context_length", input_tensors["context_length"]},
                                  {"attention_mask", attention_mask.get()}};
        TensorMap ctx_attn_output{{"attention_output", decoder_output},
                                  {"all_k_cache", output_tensors["all_k_cache"]},
                                  {"all_v_cache", output_tensors["all_v_cache"]}};
        TensorMap ffn_inputs{{"ffn_input", decoder_output}}, ffn_outputs{{"ffn_output", decoder_output}};
        dyn_params.is_ctx = true;  // FFN scratch of num_tokens rows
        LLM_CHECK_WITH_INFO((int)layerWeights.size() >= num_layer, "LlamaContextDecoder: fewer layer weights than layers");
        const bool fast = ctxAttn.fused();
        if (fast) launchRMSNorm(din.get(), decoder_residual.get(), layerWeights[0]->attn_norm_weight, rmsnorm_eps, false,
                                stream);
        fuse_o = fuse_f = true;
        for (layer = 0; layer < num_layer; ++layer) {
            LlamaLayerWeight<T>* w = layerWeights[layer];
            TensorWrapper<float>* decoder_input = ctx_attn_inputs["attention_input"]->as<float>();
            if (fast) {
                fast_layer(decoder_input, decoder_output, ctx_attn_inputs, ctx_attn_output, w,
                           layer + 1 < num_layer ? layerWeights[layer + 1] : nullptr, dyn_params);
                ctx_attn_inputs.insert("attention_input", decoder_output);
                continue;
            }
            launchRMSNorm(decoder_input, decoder_residual.get(), w->attn_norm_weight, rmsnorm_eps, false, stream);
            ctxAttn.forward(ctx_attn_inputs, ctx_attn_output, w->self_attn_weight, dyn_params,
                            ctxAttn.GetAttnStaticParams());
            BaseWeight<T> no_bias;  // Llama has no o_proj bias (the reference passed the weight itself)
            launchFusedAddBiasResidualRMSNorm(decoder_residual.get(), decoder_output, no_bias, w->ffn_norm_weight.gamma,
                                              rmsnorm_eps, stream);
            ffn.forward(ffn_inputs, ffn_outputs, w->ffn_weight, dyn_params);
            launchAddResidual(decoder_residual.get(), decoder_output, false, stream);
            ctx_attn_inputs.insert("attention_input", decoder_output);
        }
        dout.store();
        freeBuf();
        // one check per forward, where the reference would have thrown at its next
        // DeviceSyncAndCheckCudaError (context_attention.cpp:71-172)
        llmi_detail::checkStreamErrors(stream, "LlamaContextDecoder::forward");
    }

private:
    // One layer with the fused attention core and each projection + residual pair as one call
    // (llmi_linear_residual: o_proj + launchFusedAddBiasResidualRMSNorm; llmi_ffn_residual: the
    // FFN + launchAddResidual + the next layer's launchRMSNorm). Each falls back to those
    // separate launches when it returns LLMI_EUNSUPPORTED (fp32 weights, small batches).
    // Invariant entering a layer: residual = x_l, xn = RMSNorm(x_l) * attn_norm_l; leaving it,
    // the same for l + 1 in y (the last layer: y = x_L, the reference's decoder output).
    void fast_layer(TensorWrapper<float>* xn, TensorWrapper<float>* y, TensorMap& ain, TensorMap& aout,
                    LlamaLayerWeight<T>* w, LlamaLayerWeight<T>* next, LLaMAAttentionDynParams& p) {
        const int wdt = llmiWeightDtype(getWeightType<T>());
        const int rows = p.num_tokens, H = hidden_units, inter = w->ffn_weight.down.shape[1];
        float* r = decoder_residual->data;
        ctxAttn.allocForForward(p);
        TensorWrapper<float>* a = ctxAttn.forwardCore(xn, ain, aout, w->self_attn_weight, p,
                                                      ctxAttn.GetAttnStaticParams());
        // r += a . Wo^T; y = RMSNorm(r) * ffn_norm
        int rc = fuse_o ? llmi_linear_residual(a->data, w->self_attn_weight.output.data, wdt, rows, H, H, r, y->data,
                                               w->ffn_norm_weight.gamma, wdt, rmsnorm_eps, stream)
                        : LLMI_EUNSUPPORTED;
        if (rc == LLMI_EUNSUPPORTED) {
            fuse_o = false;
            cublasWrapper cw{stream};
            launchLinearGemm(a, w->self_attn_weight.output, y, &cw, false, true);
            BaseWeight<T> no_bias;
            launchFusedAddBiasResidualRMSNorm(decoder_residual.get(), y, no_bias, w->ffn_norm_weight.gamma, rmsnorm_eps,
                                              stream);
        } else {
            LLMI_CALL(rc);
        }
        ctxAttn.freeBuf();
        // r += FFN(y); y = RMSNorm(r) * the next layer's attn_norm (after the last layer: y = r)
        rc = fuse_f ? llmi_ffn_residual(y->data, w->ffn_weight.gateAndup.data, w->ffn_weight.down.data, wdt, rows, H,
                                        inter, r, y->data, next ? next->attn_norm_weight.gamma : nullptr, wdt,
                                        rmsnorm_eps, stream)
                    : LLMI_EUNSUPPORTED;
        if (rc == LLMI_EUNSUPPORTED) {
            fuse_f = false;
            TensorMap fi{{"ffn_input", y}}, fo{{"ffn_output", y}};
            ffn.forward(fi, fo, w->ffn_weight, p);
            launchAddResidual(decoder_residual.get(), y, false, stream);
            if (next) launchRMSNorm(y, decoder_residual.get(), next->attn_norm_weight, rmsnorm_eps, false, stream);
        } else {
            LLMI_CALL(rc);
        }
    }

    int hidden_units, num_layer;
    float rmsnorm_eps;
    void* stream;
    BaseAllocator* allocator;
    LLaMAContextAttentionLayer<T> ctxAttn;
    LLaMAFFNLayer<T> ffn;
    bool fuse_o = true, fuse_f = true;
    float *mask_ptr = nullptr, *resid_ptr = nullptr;
    int *po_ptr = nullptr, *cum_ptr = nullptr;
    std::unique_ptr<TensorWrapper<float>> attention_mask, decoder_residual;
    std::unique_ptr<TensorWrapper<int>> padding_offset, cum_seqlens;
};
