// The reference's fp16 instantiation of the decode-path launchers (T = half: activations
// TensorWrapper<half>, weights half) through the C++ mirror: the known answers of the
// reference's unit tests (test_rmsnorm.cu, test_fused_addresidual_norm.cu, test_act.cu,
// test_linear.cu) in fp16, and RoPE / masked MHA / embedding / argmax against the fp32
// activations path on the same inputs. One JSON line per check.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "llmi/kernels.h"

static uint16_t f2h(float f) {  // round to nearest even
    uint32_t x;
    std::memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const int e = (int)((x >> 23) & 0xff) - 127 + 15;
    uint32_t m = x & 0x7fffffu;
    if (e >= 31) return (uint16_t)(sign | 0x7c00u);
    if (e <= 0) {
        if (e < -10) return (uint16_t)sign;
        m |= 0x800000u;
        const int sh = 14 - e;
        uint32_t h = m >> sh, rem = m & ((1u << sh) - 1), half = 1u << (sh - 1);
        if (rem > half || (rem == half && (h & 1))) ++h;
        return (uint16_t)(sign | h);
    }
    uint32_t h = ((uint32_t)e << 10) | (m >> 13);
    const uint32_t rem = m & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1))) ++h;
    return (uint16_t)(sign | h);
}
static float h2f(uint16_t h) {
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    int e = (h >> 10) & 0x1f;
    uint32_t m = h & 0x3ffu, x;
    if (e == 0) {
        if (m == 0) {
            x = sign;
        } else {
            e = 1;
            while (!(m & 0x400u)) { m <<= 1; --e; }
            m &= 0x3ffu;
            x = sign | ((uint32_t)(e - 15 + 127) << 23) | (m << 13);
        }
    } else if (e == 31) {
        x = sign | 0x7f800000u | (m << 13);
    } else {
        x = sign | ((uint32_t)(e - 15 + 127) << 23) | (m << 13);
    }
    float f;
    std::memcpy(&f, &x, 4);
    return f;
}

template <typename T> struct Dev {
    T* p = nullptr;
    size_t n = 0;
    explicit Dev(size_t n) : n(n) { LLMI_CALL(llmi_device_alloc(reinterpret_cast<void**>(&p), n * sizeof(T))); }
    explicit Dev(const std::vector<T>& h) : Dev(h.size()) { put(h); }
    ~Dev() { (void)llmi_device_free(p); }
    void put(const std::vector<T>& h) { LLMI_CALL(llmi_memcpy(p, h.data(), n * sizeof(T), 0)); }
    std::vector<T> get() const {
        std::vector<T> h(n);
        LLMI_CALL(llmi_memcpy(h.data(), p, n * sizeof(T), 1));
        return h;
    }
};
static std::vector<uint16_t> H(const std::vector<float>& v) {
    std::vector<uint16_t> o(v.size());
    for (size_t i = 0; i < v.size(); ++i) o[i] = f2h(v[i]);
    return o;
}

static int fails = 0;
static void report(const char* name, double err, double tol) {
    const bool ok = err <= tol;
    fails += !ok;
    std::printf("{\"check\": \"%s\", \"max_err\": %.3e, \"tol\": %.1e, \"ok\": %s}\n", name, err, tol, ok ? "true" : "false");
}

// test_rmsnorm.cu (fp16): x = gamma = i%2+1 -> x*gamma/sqrt(2.5+eps), residual = x
static void rmsnorm_half() {
    const int n = 64, h = 4096;
    std::vector<float> x(n * h), g(h);
    for (int i = 0; i < n * h; ++i) x[i] = (float)(i % 2 + 1);
    for (int i = 0; i < h; ++i) g[i] = (float)(i % 2 + 1);
    Dev<uint16_t> dx(H(x)), dr(n * h), dg(H(g));
    TensorWrapper<half_t> out(GPU, FP16, {n, h}, dx.p), resid(GPU, FP16, {n, h}, dr.p);
    LayerNormWeight<half_t> w{dg.p};
    launchRMSNorm(&out, &resid, w, 1e-6f);  // rmsnorm_kernel.h call syntax, T = half
    auto y = dx.get(), r = dr.get();
    double err = 0;
    for (int i = 0; i < n * h; ++i) {
        const float ref = x[i] * g[i % h] / std::sqrt(2.5f + 1e-6f);
        err = std::max(err, (double)std::fabs(h2f(y[i]) - ref) / ref);
        err = std::max(err, (double)std::fabs(h2f(r[i]) - x[i]));
    }
    report("rmsnorm_half_kat", err, 1e-3);
}

// test_fused_addresidual_norm.cu (fp16): r = 0, out = 1, gamma = 1 -> 1/sqrt(1+eps), r = 1
static void fused_add_norm_half() {
    const int n = 16, h = 4096;
    Dev<uint16_t> dr(H(std::vector<float>(n * h, 0.f))), dout(H(std::vector<float>(n * h, 1.f))),
        dg(H(std::vector<float>(h, 1.f)));
    TensorWrapper<half_t> r(GPU, FP16, {n, h}, dr.p), o(GPU, FP16, {n, h}, dout.p);
    BaseWeight<half_t> nobias;
    launchFusedAddBiasResidualRMSNorm(&r, &o, nobias, dg.p, 1e-6f);
    auto y = dout.get(), rr = dr.get();
    double err = 0;
    for (int i = 0; i < n * h; ++i)
        err = std::max({err, (double)std::fabs(h2f(y[i]) - 1.f / std::sqrt(1.f + 1e-6f)), (double)std::fabs(h2f(rr[i]) - 1.f)});
    report("fused_addresidual_norm_half_kat", err, 1e-3);
}

// test_act.cu (fp16): all ones -> silu(1) = 0.7310586; launchAddResidual: 1 + 0.731
static void act_and_add_half() {
    const int n = 8, inter = 11008;
    Dev<uint16_t> din(H(std::vector<float>(n * 2 * inter, 1.f))), dout(n * inter),
        dres(H(std::vector<float>(n * inter, 1.f)));
    TensorWrapper<half_t> in(GPU, FP16, {n, 2, inter}, din.p), out(GPU, FP16, {n, inter}, dout.p),
        res(GPU, FP16, {n, inter}, dres.p);
    launchAct(&in, &out);
    double err = 0;
    for (uint16_t v : dout.get()) err = std::max(err, (double)std::fabs(h2f(v) - 0.7310586f));
    report("silu_mul_half_kat", err, 1e-3);
    launchAddResidual(&res, &out);
    err = 0;
    for (uint16_t v : dout.get()) err = std::max(err, (double)std::fabs(h2f(v) - 1.7310586f));
    report("add_residual_half", err, 2e-3);
}

// test_linear.cu (fp16): in = w = i%3, [13, 256] x [512, 256]^T -> integers <= 1024 (exact in fp16)
static void linear_half() {
    const int m = 13, k = 256, nout = 512;
    std::vector<float> x(m * k), w((size_t)nout * k);
    for (int i = 0; i < m * k; ++i) x[i] = (float)(i % 3);
    for (size_t i = 0; i < w.size(); ++i) w[i] = (float)(i % 3);
    Dev<uint16_t> dx(H(x)), dw(H(w)), dy(m * nout);
    TensorWrapper<half_t> in(GPU, FP16, {m, k}, dx.p), out(GPU, FP16, {m, nout}, dy.p);
    BaseWeight<half_t> W;
    W.shape = {nout, k};
    W.data = dw.p;
    launchLinearGemm(&in, W, &out, nullptr, false, true);
    auto y = dy.get();
    double err = 0;
    for (int r = 0; r < m; ++r)
        for (int c = 0; c < nout; ++c) {
            double ref = 0;
            for (int j = 0; j < k; ++j) ref += (double)x[r * k + j] * w[(size_t)c * k + j];
            err = std::max(err, std::fabs(h2f(y[r * nout + c]) - ref));
        }
    report("linear_half_kat_exact", err, 0.0);
}

// RoPE + masked MHA + embedding + argmax: fp16 activations vs fp32 activations on the
// same fp16-representable inputs (fp16 caches)
static void decode_ops_half_vs_f32() {
    const int heads = 4, kv = 4, hd = 128, qh = heads + 2 * kv, S = 64, L = 2, pos = 9, V = 1000;
    int layer = 1;
    std::mt19937 rng(7);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<float> qkv(qh * hd), cache((size_t)L * kv * S * hd);
    for (auto& v : qkv) v = h2f(f2h(nd(rng)));
    for (auto& v : cache) v = nd(rng);
    const auto cache_h = H(cache);
    LLaMAAttentionStaticParams sp;
    int step = pos + 1;
    TensorWrapper<int> step_t(CPU, INT32, {1}, &step), layer_t(CPU, INT32, {1}, &layer);
    bool fin = false;
    TensorWrapper<bool> fin_t(CPU, BOOL, {1}, &fin);
    BaseWeight<half_t> qkv_w;
    // fp32 activations
    Dev<float> q32(qkv), o32(heads * hd);
    Dev<uint16_t> k32(cache_h), v32(cache_h);
    TensorWrapper<float> tq32(GPU, FP32, {1, qh, hd}, q32.p), to32(GPU, FP32, {1, heads * hd}, o32.p);
    TensorWrapper<half_t> tk32(GPU, FP16, {L, 1, kv, S, hd}, k32.p), tv32(GPU, FP16, {L, 1, kv, S, hd}, v32.p);
    launchRoPE(&tq32, &step_t, sp, kv);
    launchDecoderMaskedMHA(&tq32, qkv_w, &layer_t, &tk32, &tv32, &fin_t, &step_t, &to32, sp);
    // fp16 activations (the reference's T = half call syntax)
    Dev<uint16_t> q16(H(qkv)), o16(heads * hd), k16(cache_h), v16(cache_h);
    TensorWrapper<half_t> tq16(GPU, FP16, {1, qh, hd}, q16.p), to16(GPU, FP16, {1, heads * hd}, o16.p);
    TensorWrapper<half_t> tk16(GPU, FP16, {L, 1, kv, S, hd}, k16.p), tv16(GPU, FP16, {L, 1, kv, S, hd}, v16.p);
    launchRoPE(&tq16, &step_t, sp, kv);
    launchDecoderMaskedMHA(&tq16, qkv_w, &layer_t, &tk16, &tv16, &fin_t, &step_t, &to16, sp);
    double err = 0;
    {
        auto a = q32.get();
        auto b = q16.get();
        for (size_t i = 0; i < a.size(); ++i) err = std::max(err, (double)std::fabs(h2f(b[i]) - a[i]));
        report("rope_half_vs_f32", err, 4e-3);
    }
    {
        auto a = o32.get();
        auto b = o16.get();
        err = 0;
        for (size_t i = 0; i < a.size(); ++i) err = std::max(err, (double)std::fabs(h2f(b[i]) - a[i]));
        report("masked_mha_half_vs_f32", err, 4e-3);
        auto ka = k32.get(), kb = k16.get();
        size_t diff = 0;
        for (size_t i = 0; i < ka.size(); ++i) diff += ka[i] != kb[i];
        report("kv_slot_write_half_vs_f32", (double)diff, 0.0);
    }
    // embedding (exact: fp16 table -> fp16 activations) and argmax of fp16 probs
    std::vector<float> table((size_t)V * hd);
    for (auto& v : table) v = nd(rng);
    Dev<uint16_t> dt(H(table)), de(3 * hd);
    std::vector<int> ids = {5, 999, 0};
    Dev<int> did(ids), dbest(1);
    EmbeddingWeight<half_t> E;
    E.shape = {V, hd};
    E.data = dt.p;
    TensorWrapper<int> tid(GPU, INT32, {3}, did.p), tbest(GPU, INT32, {1}, dbest.p);
    TensorWrapper<half_t> te(GPU, FP16, {3, hd}, de.p);
    launchInputEmbedding(&tid, &te, &E);
    auto e = de.get();
    const auto th = H(table);
    size_t diff = 0;
    for (int t = 0; t < 3; ++t)
        for (int d = 0; d < hd; ++d) diff += e[t * hd + d] != th[(size_t)ids[t] * hd + d];
    report("embedding_half_exact", (double)diff, 0.0);
    std::vector<float> probs(V);
    for (int i = 0; i < V; ++i) probs[i] = (float)((i * 37) % 101) / 100.f;
    probs[613] = 2.f;
    Dev<uint16_t> dp(H(probs));
    TensorWrapper<half_t> tp(GPU, FP16, {1, V}, dp.p);
    launchTopKforBeamSearch(&tp, &tbest);
    report("argmax_half", (double)std::abs(dbest.get()[0] - 613), 0.0);
}

int main(int argc, char** argv) {
    if (argc < 2) return 0;  // compile / link check only
    try {
        rmsnorm_half();
        fused_add_norm_half();
        act_and_add_half();
        linear_half();
        decode_ops_half_vs_f32();
    } catch (const std::exception& e) {
        std::printf("{\"exception\": \"%s\"}\n", e.what());
        return 2;
    }
    return fails ? 1 : 0;
}
