// launchLinearGemm in all four forms of the reference (linear.h:16-22, linear.cu:38-99) and
// the layer API's stream-K failure path, through the C++ mirror (include/llmi/layers.h).
//   1. the reference's own call form, launchLinearGemm(in, weight, out, cublas_wrapper)
//      (tests/unittests/test_linear.cu:86: defaults trans_a = trans_b = false, weight
//      [in, out]), with its i%3 data: exact integers;
//   2. the same call with a NON-symmetric [4096, 4096] weight and with non-square weights,
//      fp32 and fp16, every (trans_a, trans_b) pair: rel-L2 vs float64 <= 1e-6;
//   3. LLaMAFFNLayer<half>::forward (context rows, the stream-K gate_up) with a stream-K
//      piece that never publishes (llmi_debug_stream_k mode 1) and one that publishes after
//      its owner gave up (mode 2): the forward throws "[oneLLM][ERROR] ...", and the next
//      forward is bitwise the clean result.
// Prints one JSON line per check; tests/test_cpp_api.py runs it on the GPU.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "llmi/layers.h"

static HipAllocator g_alloc;
static int fails = 0;

template <typename T> struct Dev {
    T* p = nullptr;
    size_t n = 0;
    explicit Dev(size_t n) : n(n) { p = g_alloc.Malloc(p, n * sizeof(T), false); }
    Dev(const std::vector<T>& h) : Dev(h.size()) { put(h); }
    ~Dev() { g_alloc.Free(p, false); }
    void put(const std::vector<T>& h) { LLMI_CALL(llmi_memcpy(p, h.data(), n * sizeof(T), 0)); }
    std::vector<T> get() const {
        std::vector<T> h(n);
        LLMI_CALL(llmi_device_sync());
        LLMI_CALL(llmi_memcpy(h.data(), p, n * sizeof(T), 1));
        return h;
    }
};

static void report(const std::string& name, double err, double tol) {
    const bool ok = err <= tol;
    fails += !ok;
    std::printf("{\"check\": \"%s\", \"err\": %.3e, \"tol\": %.1e, \"ok\": %s}\n", name.c_str(), err, tol,
                ok ? "true" : "false");
    std::fflush(stdout);
}

// deterministic, non-symmetric values in [-1, 1)
static std::vector<float> lcg(size_t n, uint64_t seed) {
    std::vector<float> v(n);
    uint64_t s = seed * 6364136223846793005ull + 1442695040888963407ull;
    for (size_t i = 0; i < n; ++i) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        v[i] = (float)((double)(s >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0);
    }
    return v;
}

// CPUlinear of test_linear.cu:13-22 generalised to the four forms, in float64:
// y[i][j] = sum_l op_a(x)[i][l] * op_b(w)[l][j]
static std::vector<double> ref_linear(const std::vector<float>& x, const std::vector<float>& w, int m, int k, int n,
                                      bool ta, bool tb) {
    std::vector<double> y((size_t)m * n, 0.0);
    for (int i = 0; i < m; ++i)
        for (int l = 0; l < k; ++l) {
            const double a = ta ? x[(size_t)l * m + i] : x[(size_t)i * k + l];
            for (int j = 0; j < n; ++j) y[(size_t)i * n + j] += a * (tb ? w[(size_t)j * k + l] : w[(size_t)l * n + j]);
        }
    return y;
}

static double rel_l2(const std::vector<float>& got, const std::vector<double>& want) {
    double num = 0, den = 0;
    for (size_t i = 0; i < want.size(); ++i) {
        num += (got[i] - want[i]) * (got[i] - want[i]);
        den += want[i] * want[i];
    }
    return std::sqrt(num / (den > 0 ? den : 1e-300));
}

// test_linear.cu:38-94 verbatim in shape and data: in = w = i%3, [13, 4096] x [4096, 4096]
static void kat_reference_call_form() {
    const int m = 13, h = 4096;
    std::vector<float> x((size_t)m * h), w((size_t)h * h);
    for (size_t i = 0; i < x.size(); ++i) x[i] = (float)(i % 3);
    for (size_t i = 0; i < w.size(); ++i) w[i] = (float)(i % 3);
    Dev<float> dx(x), dw(w), dy((size_t)m * h);
    TensorWrapper<float> in(GPU, FP32, {m, h}, dx.p), out(GPU, FP32, {m, h}, dy.p);
    BaseWeight<float> weight;
    weight.shape = {h, h};
    weight.data = dw.p;
    cublasWrapper cw;
    launchLinearGemm(&in, weight, &out, &cw);  // the reference's call, defaults and all
    const auto y = dy.get();
    const auto want = ref_linear(x, w, m, h, h, false, false);
    double err = 0;
    for (size_t i = 0; i < want.size(); ++i) err = std::max(err, std::fabs(y[i] - want[i]));
    report("linear_reference_call_form_i%3_exact", err, 0.0);
}

// every form with random non-symmetric data; T = float or half_t weights (fp16 rounding of
// the weights is part of the reference values: they are read back from the device)
template <typename T>
static void linear_case(int m, int k, int n, bool ta, bool tb, uint64_t seed) {
    const std::vector<float> x = lcg((size_t)m * k, seed), w32 = lcg((size_t)k * n, seed + 1);
    Dev<float> dx(x), dw32(w32), dy((size_t)m * n);
    Dev<T> dw((size_t)k * n);
    std::vector<float> w = w32;
    if (std::is_same<T, half_t>::value) {
        LLMI_CALL(llmi_convert(dw32.p, LLMI_F32, dw.p, LLMI_F16, w.size(), nullptr));
        LLMI_CALL(llmi_convert(dw.p, LLMI_F16, dw32.p, LLMI_F32, w.size(), nullptr));
        w = dw32.get();  // the fp16-rounded weights the kernel multiplies
    } else {
        LLMI_CALL(llmi_memcpy(dw.p, w32.data(), w32.size() * sizeof(float), 0));
    }
    TensorWrapper<float> in(GPU, FP32, ta ? std::vector<int>{k, m} : std::vector<int>{m, k}, dx.p);
    TensorWrapper<float> out(GPU, FP32, {m, n}, dy.p);
    BaseWeight<T> weight;
    weight.shape = tb ? std::vector<int>{n, k} : std::vector<int>{k, n};
    weight.data = dw.p;
    cublasWrapper cw;
    launchLinearGemm(&in, weight, &out, &cw, ta, tb);
    const double e = rel_l2(dy.get(), ref_linear(x, w, m, k, n, ta, tb));
    char name[160];
    std::snprintf(name, sizeof name, "linear_%s_m%d_k%d_n%d_ta%d_tb%d", std::is_same<T, half_t>::value ? "f16" : "f32",
                  m, k, n, (int)ta, (int)tb);
    report(name, e, 1e-6);
}

// a mismatched shape is the reference's own LLM_CHECK message, not a wrong answer
static void linear_shape_check() {
    Dev<float> dx(13 * 64), dw(64 * 32), dy(13 * 32);
    TensorWrapper<float> in(GPU, FP32, {13, 64}, dx.p), out(GPU, FP32, {13, 32}, dy.p);
    BaseWeight<float> weight;
    weight.shape = {32, 64};  // [out, in]: needs trans_b = true
    weight.data = dw.p;
    bool threw = false;
    try {
        launchLinearGemm(&in, weight, &out);
    } catch (const std::runtime_error& e) {
        threw = std::string(e.what()).find("[oneLLM][ERROR] 2nd dim of input MUST = 1st dim of weight") == 0;
    }
    report("linear_shape_mismatch_throws", threw ? 0.0 : 1.0, 0.0);
}

// LLaMAFFNLayer<half>::forward at a stream-K shape (512 rows, hidden 1024, inter 6144: the
// gate_up's 96 tiles run on every CU) with an injected stream-K fault
static void ffn_stream_k_fault(int mode) {
    const int m = 512, hidden = 1024, inter = 6144;
    Dev<half_t> wgu((size_t)2 * inter * hidden), wd((size_t)hidden * inter);
    LLMI_CALL(llmi_synth_fill(wgu.p, LLMI_F16, LLMI_SYN_LINEAR, 7, 100, 2 * inter, hidden, 0, 0, hidden, nullptr));
    LLMI_CALL(llmi_synth_fill(wd.p, LLMI_F16, LLMI_SYN_LINEAR, 7, 101, hidden, inter, 0, 0, inter, nullptr));
    Dev<float> dx(lcg((size_t)m * hidden, 11)), dy((size_t)m * hidden);
    LLaMAFFNWeights<half_t> w;
    w.gateAndup.shape = {2 * inter, hidden};
    w.gateAndup.data = wgu.p;
    w.down.shape = {hidden, inter};
    w.down.data = wd.p;
    LLaMAFFNLayer<half_t> ffn(hidden / 128, 128, inter, nullptr, nullptr, &g_alloc);
    TensorWrapper<float> x(GPU, FP32, {m, hidden}, dx.p), y(GPU, FP32, {m, hidden}, dy.p);
    TensorMap in{{"ffn_input", &x}}, out{{"ffn_output", &y}};
    LLaMAAttentionDynParams p;
    p.is_ctx = true;
    p.num_tokens = m;
    p.batch_size = 1;
    ffn.forward(in, out, w, p);
    const auto clean = dy.get();
    LLMI_CALL(llmi_debug_stream_k(mode, 1));
    std::string what;
    try {
        ffn.forward(in, out, w, p);
    } catch (const std::runtime_error& e) {
        what = e.what();
    }
    LLMI_CALL(llmi_debug_stream_k(0, 0));
    const bool threw = what.rfind("[oneLLM][ERROR] LLaMAFFNLayer::forward", 0) == 0 &&
                       what.find("stream-K partial never arrived") != std::string::npos;
    report("ffn_stream_k_fault_mode" + std::to_string(mode) + "_throws", threw ? 0.0 : 1.0, 0.0);
    ffn.forward(in, out, w, p);  // the next forward: no error, the clean result bit for bit
    const auto again = dy.get();
    report("ffn_stream_k_fault_mode" + std::to_string(mode) + "_next_forward_bitwise",
           std::memcmp(again.data(), clean.data(), clean.size() * sizeof(float)) == 0 ? 0.0 : 1.0, 0.0);
}

int main() {
    kat_reference_call_form();
    for (int tb = 0; tb < 2; ++tb)
        for (int ta = 0; ta < 2; ++ta) {
            linear_case<float>(13, 4096, 4096, ta, tb, 100 + 2 * tb + ta);  // square, non-symmetric
            linear_case<float>(13, 4096, 1000, ta, tb, 200 + 2 * tb + ta);  // non-square
            linear_case<half_t>(32, 1024, 1536, ta, tb, 300 + 2 * tb + ta);  // fp16, matrix-core rows
            linear_case<half_t>(3, 4096, 1000, ta, tb, 400 + 2 * tb + ta);   // fp16, decode rows
        }
    linear_shape_check();
    ffn_stream_k_fault(1);
    ffn_stream_k_fault(2);
    std::printf("{\"fails\": %d}\n", fails);
    return fails ? 1 : 0;
}
