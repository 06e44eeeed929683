// The reference's own unit-test patterns (tests/unittests/*.cu, SURVEY.md §8c
// known answers) restated against the C++ mirror of its launcher / layer API,
// running the MI355X kernels through libllmi.so. Prints one JSON line per check;
// the layer-by-layer greedy decode prints its tokens for the pytest driver
// (tests/test_gpu_cpp_api.py) to compare with the reference fixture.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "llmi/layers.h"
#include "llmi/model.h"

static HipAllocator g_alloc;

template <typename T> struct Dev {
    T* p = nullptr;
    size_t n = 0;
    explicit Dev(size_t n) : n(n) { p = g_alloc.Malloc(p, n * sizeof(T), false); }
    Dev(const std::vector<T>& h) : Dev(h.size()) { put(h); }
    ~Dev() { g_alloc.Free(p, false); }
    void put(const std::vector<T>& h) { LLMI_CALL(llmi_memcpy(p, h.data(), n * sizeof(T), 0)); }
    std::vector<T> get() const {
        std::vector<T> h(n);
        LLMI_CALL(llmi_memcpy(h.data(), p, n * sizeof(T), 1));
        return h;
    }
};

static int fails = 0;
static void report(const char* name, double err, double tol) {
    const bool ok = err <= tol;
    fails += !ok;
    std::printf("{\"check\": \"%s\", \"max_err\": %.3e, \"tol\": %.1e, \"ok\": %s}\n", name, err, tol, ok ? "true" : "false");
}

// test_rmsnorm.cu:139-160 -- x = gamma = i%2+1, eps 1e-6, [64, 4096] -> x*gamma/sqrt(2.5+1e-6)
static void kat_rmsnorm() {
    const int n = 64, h = 4096;
    std::vector<float> x(n * h), g(h);
    for (int i = 0; i < n * h; ++i) x[i] = (float)(i % 2 + 1);
    for (int i = 0; i < h; ++i) g[i] = (float)(i % 2 + 1);
    Dev<float> dx(x), dr(n * h), dg(g);
    TensorWrapper<float> out(GPU, FP32, {n, h}, dx.p), resid(GPU, FP32, {n, h}, dr.p);
    LayerNormWeight<float> w{dg.p};
    launchRMSNorm(&out, &resid, w, 1e-6f);
    auto y = dx.get(), r = dr.get();
    double err = 0;
    for (int i = 0; i < n * h; ++i) {
        err = std::max(err, (double)std::fabs(y[i] - x[i] * g[i % h] / std::sqrt(2.5f + 1e-6f)));
        err = std::max(err, (double)std::fabs(r[i] - x[i]));
    }
    report("rmsnorm_kat", err, 1e-6);
}

// test_fused_addresidual_norm.cu:69-104 -- r = 0, out = 1, gamma = 1 -> 1/sqrt(1+eps)
static void kat_fused_add_norm() {
    const int n = 16, h = 4096;
    Dev<float> dr(std::vector<float>(n * h, 0.f)), dout(std::vector<float>(n * h, 1.f)), dg(std::vector<float>(h, 1.f));
    TensorWrapper<float> r(GPU, FP32, {n, h}, dr.p), o(GPU, FP32, {n, h}, dout.p);
    BaseWeight<float> nobias;
    launchFusedAddBiasResidualRMSNorm(&r, &o, nobias, dg.p, 1e-6f);
    auto y = dout.get(), rr = dr.get();
    double err = 0;
    for (int i = 0; i < n * h; ++i)
        err = std::max({err, (double)std::fabs(y[i] - 1.f / std::sqrt(1.f + 1e-6f)), (double)std::fabs(rr[i] - 1.f)});
    report("fused_addresidual_norm_kat", err, 1e-6);
}

// test_act.cu:44-50 -- all-ones [n, 2, inter] -> silu(1) = 0.7310586
static void kat_act() {
    const int n = 8, inter = 11008;
    Dev<float> din(std::vector<float>(n * 2 * inter, 1.f)), dout(n * inter);
    TensorWrapper<float> in(GPU, FP32, {n, 2, inter}, din.p), out(GPU, FP32, {n, inter}, dout.p);
    launchAct(&in, &out);
    double err = 0;
    for (float v : dout.get()) err = std::max(err, (double)std::fabs(v - 0.7310586f));
    report("silu_mul_kat", err, 1e-6);
}

// test_linear.cu:38-94 -- in = w = i%3, [13, 4096] x [4096, 4096]^T: exact integers
static void kat_linear() {
    const int m = 13, k = 4096, nout = 4096;
    std::vector<float> x(m * k), w((size_t)nout * k);
    for (int i = 0; i < m * k; ++i) x[i] = (float)(i % 3);
    for (size_t i = 0; i < w.size(); ++i) w[i] = (float)(i % 3);
    Dev<float> dx(x), dw(w), dy(m * nout);
    TensorWrapper<float> in(GPU, FP32, {m, k}, dx.p), out(GPU, FP32, {m, nout}, dy.p);
    BaseWeight<float> W;
    W.shape = {nout, k};
    W.data = dw.p;
    launchLinearGemm(&in, W, &out, nullptr, false, true);
    auto y = dy.get();
    double err = 0;
    for (int r = 0; r < m; ++r)
        for (int c = 0; c < nout; ++c) {
            double ref = 0;
            for (int j = 0; j < k; ++j) ref += (double)x[r * k + j] * w[(size_t)c * k + j];
            err = std::max(err, std::fabs(y[r * nout + c] - ref));
        }
    report("linear_kat_exact", err, 0.0);
}

// LlamaSelfDecoder<half> op by op (the reference's layer API) on the tiny preset:
// greedy tokens from a prompt, printed for comparison with the fixture + engine.
static void layer_decode(const std::vector<int>& prompt, int n_new, uint64_t seed) {
    const int heads = 4, kv = 4, hd = 128, H = heads * hd, I = 1024, L = 2, V = 32000, S = 64;
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

    Dev<float> kc((size_t)L * kv * S * hd), vc((size_t)L * kv * S * hd), x(H), y(H), unused(H), logits(V);
    Dev<int> ids(1), next(1);
    TensorWrapper<float> dec_in(GPU, FP32, {1, H}, x.p), dec_out(GPU, FP32, {1, H}, y.p), un(GPU, FP32, {1, H}, unused.p);
    TensorWrapper<float> kcache(GPU, FP32, {L, 1, kv, S, hd}, kc.p), vcache(GPU, FP32, {L, 1, kv, S, hd}, vc.p);
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
    std::vector<int> gen;
    int tok = prompt[0];
    for (int pos = 0; pos < (int)prompt.size() + n_new - 1; ++pos) {
        if (pos < (int)prompt.size()) tok = prompt[pos];
        LLMI_CALL(llmi_memcpy(ids.p, &tok, 4, 0));
        launchInputEmbedding(&id_t, &dec_in, &E);
        step = pos + 1;  // llama.cpp: step = total length including this token
        dec.forward(in, lw, out, dp);
        launchRMSNorm(&dec_out, &un, FN, 1e-5f, true);
        launchLinearGemm(&dec_out, LM, &probs, nullptr, false, true);
        launchTopKforBeamSearch(&probs, &next_t);
        LLMI_CALL(llmi_memcpy(&tok, next.p, 4, 1));  // the reference's per-token D2H (llama.cpp:266)
        if (pos >= (int)prompt.size() - 1) gen.push_back(tok);
    }
    std::printf("{\"layer_api_tokens\": [");
    for (size_t i = 0; i < gen.size(); ++i) std::printf("%s%d", i ? ", " : "", gen[i]);
    std::printf("]}\n");

    // ---- the same decode with the reference's fp16 activations (Llama<half>:
    // TensorWrapper<half> decoder_input / decoder_output, self_decoder.cpp:59-81); the
    // layers stage them through fp32, so the tokens must equal the fp32 run's
    {
        Dev<half_t> x16(H), y16(H);
        Dev<float> kc16((size_t)L * kv * S * hd), vc16((size_t)L * kv * S * hd);
        TensorWrapper<half_t> in16(GPU, FP16, {1, H}, x16.p), out16(GPU, FP16, {1, H}, y16.p);
        TensorWrapper<float> kcache16(GPU, FP32, {L, 1, kv, S, hd}, kc16.p), vcache16(GPU, FP32, {L, 1, kv, S, hd}, vc16.p);
        TensorMap hin{{"decoder_input", &in16}, {"step", &step_t}, {"finished", &fin_t}};
        TensorMap hout{{"decoder_output", &out16}, {"all_k_cache", &kcache16}, {"all_v_cache", &vcache16}};
        std::vector<int> gen16;
        tok = prompt[0];
        for (int pos = 0; pos < (int)prompt.size() + n_new - 1; ++pos) {
            if (pos < (int)prompt.size()) tok = prompt[pos];
            LLMI_CALL(llmi_memcpy(ids.p, &tok, 4, 0));
            launchInputEmbedding(&id_t, &in16, &E);
            step = pos + 1;
            dec.forward(hin, lw, hout, dp);
            LLMI_CALL(llmi_convert(y16.p, LLMI_F16, y.p, LLMI_F32, H, nullptr));  // head in fp32, as above
            launchRMSNorm(&dec_out, &un, FN, 1e-5f, true);
            launchLinearGemm(&dec_out, LM, &probs, nullptr, false, true);
            launchTopKforBeamSearch(&probs, &next_t);
            LLMI_CALL(llmi_memcpy(&tok, next.p, 4, 1));
            if (pos >= (int)prompt.size() - 1) gen16.push_back(tok);
        }
        std::printf("{\"layer_api_tokens_half\": [");
        for (size_t i = 0; i < gen16.size(); ++i) std::printf("%s%d", i ? ", " : "", gen16[i]);
        std::printf("]}\n");
        // an activation of another dtype is an error (the reference's as<T>() read it silently)
        Dev<int> bad(H);
        TensorWrapper<int> bad_t(GPU, INT32, {1, H}, bad.p);
        TensorMap bin{{"decoder_input", &bad_t}, {"step", &step_t}, {"finished", &fin_t}};
        bool threw = false;
        try {
            dec.forward(bin, lw, hout, dp);
        } catch (const std::runtime_error&) {
            threw = true;
        }
        report("layer_rejects_int32_activations", threw ? 0.0 : 1.0, 0.0);
    }

    // ---- the same request with the prompt through LlamaContextDecoder in ONE batched
    // pass (context_decoder.cpp:47-143, the reference's firstTokenGen path), then the
    // self decoder from position n on (fresh fp32 caches)
    const int n = (int)prompt.size();
    Dev<float> kc2((size_t)L * kv * S * hd), vc2((size_t)L * kv * S * hd), xs((size_t)n * H), ys((size_t)n * H);
    Dev<int> pids(prompt), hist(std::vector<int>{0}), qlen(std::vector<int>{n}), klen(std::vector<int>{n});
    TensorWrapper<int> pid_t(GPU, INT32, {n}, pids.p), hist_t(GPU, INT32, {1}, hist.p), qlen_t(GPU, INT32, {1}, qlen.p),
        klen_t(GPU, INT32, {1}, klen.p);
    TensorWrapper<float> ctx_in(GPU, FP32, {n, H}, xs.p), ctx_out(GPU, FP32, {n, H}, ys.p);
    TensorWrapper<float> kcache2(GPU, FP32, {L, 1, kv, S, hd}, kc2.p), vcache2(GPU, FP32, {L, 1, kv, S, hd}, vc2.p);
    int layer0 = 0;
    TensorWrapper<int> layer_t(CPU, INT32, {1}, &layer0);
    launchInputEmbedding(&pid_t, &ctx_in, &E);
    LlamaContextDecoder<half_t> ctx(heads, kv, hd, I, L, sp, 1e-5f, nullptr, nullptr, &g_alloc);
    LLaMAAttentionDynParams cp;
    cp.batch_size = 1;
    cp.num_tokens = n;
    cp.max_q_len = n;
    cp.max_k_len = n;
    cp.num_layers = L;
    TensorMap cin{{"decoder_input", &ctx_in}, {"history_length", &hist_t}, {"input_length", &qlen_t},
                  {"context_length", &klen_t}, {"layer_id", &layer_t}};
    TensorMap cout{{"decoder_output", &ctx_out}, {"all_k_cache", &kcache2}, {"all_v_cache", &vcache2}};
    ctx.forward(cin, lw, cout, cp);
    TensorWrapper<float> last(GPU, FP32, {1, H}, ys.p + (size_t)(n - 1) * H);
    launchRMSNorm(&last, &un, FN, 1e-5f, true);
    launchLinearGemm(&last, LM, &probs, nullptr, false, true);
    launchTopKforBeamSearch(&probs, &next_t);
    LLMI_CALL(llmi_memcpy(&tok, next.p, 4, 1));
    std::vector<int> gen2{tok};
    TensorMap out2{{"decoder_output", &dec_out}, {"all_k_cache", &kcache2}, {"all_v_cache", &vcache2}};
    for (int pos = n; pos < n + n_new - 1; ++pos) {
        LLMI_CALL(llmi_memcpy(ids.p, &tok, 4, 0));
        launchInputEmbedding(&id_t, &dec_in, &E);
        step = pos + 1;
        dec.forward(in, lw, out2, dp);
        launchRMSNorm(&dec_out, &un, FN, 1e-5f, true);
        launchLinearGemm(&dec_out, LM, &probs, nullptr, false, true);
        launchTopKforBeamSearch(&probs, &next_t);
        LLMI_CALL(llmi_memcpy(&tok, next.p, 4, 1));
        gen2.push_back(tok);
    }
    std::printf("{\"context_layer_tokens\": [");
    for (size_t i = 0; i < gen2.size(); ++i) std::printf("%s%d", i ? ", " : "", gen2[i]);
    std::printf("]}\n");

    // ---- a ragged batch through LlamaContextDecoder (context_decoder.cpp:47-143 with bs > 1):
    // three prefixes of the prompt (lengths n, n - 3, 4; no history) packed row after row,
    // padding offsets and per-sequence causal masks from the launchers; the last row of each
    // sequence -> final norm -> lm_head. The pytest driver compares every sequence with the
    // oracle's prefill of that prefix alone.
    {
        const std::vector<int> lens = {n, n - 3, 4};
        const int bs = (int)lens.size();
        int tokens = 0, maxq = 0;
        std::vector<int> rids;
        for (int b = 0; b < bs; ++b) {
            tokens += lens[b];
            maxq = std::max(maxq, lens[b]);
            for (int i = 0; i < lens[b]; ++i) rids.push_back(prompt[i]);
        }
        Dev<int> rid(rids), rhist(std::vector<int>(bs, 0)), rq(lens), rk(lens);
        Dev<float> rx((size_t)tokens * H), ry((size_t)tokens * H), rkc((size_t)L * bs * kv * S * hd),
            rvc((size_t)L * bs * kv * S * hd);
        TensorWrapper<int> rid_t(GPU, INT32, {tokens}, rid.p), rhist_t(GPU, INT32, {bs}, rhist.p),
            rq_t(GPU, INT32, {bs}, rq.p), rk_t(GPU, INT32, {bs}, rk.p);
        TensorWrapper<float> rin(GPU, FP32, {tokens, H}, rx.p), rout(GPU, FP32, {tokens, H}, ry.p);
        TensorWrapper<float> rkcache(GPU, FP32, {L, bs, kv, S, hd}, rkc.p), rvcache(GPU, FP32, {L, bs, kv, S, hd}, rvc.p);
        launchInputEmbedding(&rid_t, &rin, &E);
        LLaMAAttentionDynParams rp;
        rp.batch_size = bs;
        rp.num_tokens = tokens;
        rp.max_q_len = maxq;
        rp.max_k_len = maxq;
        rp.num_layers = L;
        TensorMap rcin{{"decoder_input", &rin}, {"history_length", &rhist_t}, {"input_length", &rq_t},
                       {"context_length", &rk_t}, {"layer_id", &layer_t}};
        TensorMap rcout{{"decoder_output", &rout}, {"all_k_cache", &rkcache}, {"all_v_cache", &rvcache}};
        ctx.forward(rcin, lw, rcout, rp);
        std::printf("{\"ragged_lens\": [%d, %d, %d], \"ragged_logits\": [", lens[0], lens[1], lens[2]);
        int row = 0;
        for (int b = 0; b < bs; ++b) {
            row += lens[b];
            TensorWrapper<float> lastb(GPU, FP32, {1, H}, ry.p + (size_t)(row - 1) * H);
            launchRMSNorm(&lastb, &un, FN, 1e-5f, true);
            launchLinearGemm(&lastb, LM, &probs, nullptr, false, true);
            const std::vector<float> lg = logits.get();
            std::printf("%s[", b ? ", " : "");
            for (int i = 0; i < V; ++i) std::printf("%s%.7g", i ? "," : "", lg[i]);
            std::printf("]");
        }
        std::printf("]}\n");
    }
    for (auto* w : lw) delete w;
}

int main(int argc, char** argv) {
    try {
        kat_rmsnorm();
        kat_fused_add_norm();
        kat_act();
        kat_linear();
        if (argc > 2) {  // seed n_new prompt ids...
            const uint64_t seed = std::strtoull(argv[1], nullptr, 10);
            const int n_new = std::atoi(argv[2]);
            std::vector<int> prompt;
            for (int i = 3; i < argc; ++i) prompt.push_back(std::atoi(argv[i]));
            layer_decode(prompt, n_new, seed);
            // the same request through the fused engine (model-level API)
            llm::LlamaModel m("tiny", LLMI_F16, LLMI_F32);
            m.loadWeightsFromDummy(seed);
            auto toks = m.Response(prompt, n_new, nullptr, /*eos*/ -1);
            std::printf("{\"engine_tokens\": [");
            for (size_t i = 0; i < toks.size(); ++i) std::printf("%s%d", i ? ", " : "", toks[i]);
            std::printf("]}\n");
        }
    } catch (const std::exception& e) {
        std::printf("{\"exception\": \"%s\"}\n", e.what());
        return 2;
    }
    return fails ? 1 : 0;
}
