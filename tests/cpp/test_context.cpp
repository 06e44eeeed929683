// The reference's context-attention launchers (context_attention.cpp:108-161 call
// order) through the C++ mirror (include/llmi/kernels.h), on a ragged batch read
// from <dir>/in_*.bin; every output is written to <dir>/out_*.bin for the pytest
// driver (tests/test_cpp_api.py) to compare with oracle/context_ops.py.
//   test_context <dir> <heads> <kv_heads> <head> <max_seq> <len_0> <hist_0> [<len_1> <hist_1> ...]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "llmi/layers.h"

static HipAllocator g_alloc;

template <typename T> struct Dev {
    T* p = nullptr;
    size_t n = 0;
    explicit Dev(size_t n) : n(n) { p = g_alloc.Malloc(p, n * sizeof(T), false); }
    ~Dev() { g_alloc.Free(p, false); }
    void put(const std::vector<T>& h) { LLMI_CALL(llmi_memcpy(p, h.data(), n * sizeof(T), 0)); }
    std::vector<T> get() const {
        std::vector<T> h(n);
        LLMI_CALL(llmi_memcpy(h.data(), p, n * sizeof(T), 1));
        return h;
    }
};

static std::vector<float> load(const std::string& path, size_t n) {
    std::vector<float> v(n);
    FILE* f = std::fopen(path.c_str(), "rb");
    LLM_CHECK_WITH_INFO(f && std::fread(v.data(), 4, n, f) == n, "cannot read " + path);
    std::fclose(f);
    return v;
}
static void save(const std::string& path, const std::vector<float>& v) {
    FILE* f = std::fopen(path.c_str(), "wb");
    LLM_CHECK_WITH_INFO(f && std::fwrite(v.data(), 4, v.size(), f) == v.size(), "cannot write " + path);
    std::fclose(f);
}

int main(int argc, char** argv) {
    LLM_CHECK_WITH_INFO(argc >= 8 && argc % 2 == 0, "usage: test_context dir heads kv head max_seq (len hist)+");
    const std::string dir = argv[1];
    const int heads = std::atoi(argv[2]), kv = std::atoi(argv[3]), hd = std::atoi(argv[4]), S = std::atoi(argv[5]);
    std::vector<int> lens, hist, klens;
    for (int i = 6; i < argc; i += 2) {
        lens.push_back(std::atoi(argv[i]));
        hist.push_back(std::atoi(argv[i + 1]));
        klens.push_back(lens.back() + hist.back());
    }
    const int bs = (int)lens.size();
    int mq = 0, mk = 0, tokens = 0;
    for (int b = 0; b < bs; ++b) {
        mq = std::max(mq, lens[b]);
        mk = std::max(mk, klens[b]);
        tokens += lens[b];
    }

    const size_t nqkv = (size_t)tokens * (heads + 2 * kv) * hd;
    Dev<float> qkv(nqkv), q((size_t)bs * heads * mq * hd), k((size_t)bs * kv * mq * hd), v((size_t)bs * kv * mq * hd);
    Dev<float> kc((size_t)bs * kv * S * hd), vc((size_t)bs * kv * S * hd), mask((size_t)bs * mq * mk);
    Dev<float> qk((size_t)bs * heads * mq * mk), score((size_t)bs * heads * mq * mk), tout((size_t)tokens * heads * hd);
    Dev<int> d_po((size_t)bs * mq), d_cum(bs + 1), d_hist(bs), d_lens(bs), d_klens(bs);
    qkv.put(load(dir + "/in_qkv.bin", nqkv));
    qk.put(load(dir + "/in_qk.bin", qk.n));
    kc.put(std::vector<float>(kc.n, 0.f));
    vc.put(std::vector<float>(vc.n, 0.f));
    q.put(std::vector<float>(q.n, 0.f));
    k.put(std::vector<float>(k.n, 0.f));
    v.put(std::vector<float>(v.n, 0.f));
    d_hist.put(hist);
    d_lens.put(lens);
    d_klens.put(klens);

    TensorWrapper<float> Q(GPU, FP32, {bs, heads, mq, hd}, q.p), K(GPU, FP32, {bs, kv, mq, hd}, k.p),
        V(GPU, FP32, {bs, kv, mq, hd}, v.p), QKV(GPU, FP32, {tokens, heads + 2 * kv, hd}, qkv.p);
    TensorWrapper<float> KC(GPU, FP32, {1, bs, kv, S, hd}, kc.p), VC(GPU, FP32, {1, bs, kv, S, hd}, vc.p);
    TensorWrapper<float> M(GPU, FP32, {bs, mq, mk}, mask.p), QK(GPU, FP32, {bs, heads, mq, mk}, qk.p),
        SC(GPU, FP32, {bs, heads, mq, mk}, score.p), TO(GPU, FP32, {tokens, heads, hd}, tout.p);
    TensorWrapper<int> PO(GPU, INT32, {tokens}, d_po.p), HIST(GPU, INT32, {bs}, d_hist.p),
        LENS(GPU, INT32, {bs}, d_lens.p), KLENS(GPU, INT32, {bs}, d_klens.p);
    int layer = 0;
    TensorWrapper<int> LAYER(CPU, INT32, {1}, &layer);
    BaseWeight<float> no_bias;
    LLaMAAttentionStaticParams params;
    params.rotary_embedding_dim = hd;
    params.rotary_embedding_base = 10000.f;

    TensorWrapper<int> PO_FULL(GPU, INT32, {bs, mq}, d_po.p), CUM(GPU, INT32, {bs + 1}, d_cum.p);
    launchCalPaddingoffset(&PO_FULL, &CUM, &LENS);
    launchAddFusedQKVBiasTransposeAndRoPE(&Q, &K, &V, &QKV, no_bias, &PO, &HIST, &LENS, params);
    launchConcatKVCache(&K, &V, &LAYER, &LENS, &HIST, &KC, &VC);
    Dev<float> kr((size_t)bs * heads * mk * hd), vr((size_t)bs * heads * mk * hd);
    kr.put(std::vector<float>(kr.n, 0.f));
    vr.put(std::vector<float>(vr.n, 0.f));
    TensorWrapper<float> KR(GPU, FP32, {bs, heads, mk, hd}, kr.p), VR(GPU, FP32, {bs, heads, mk, hd}, vr.p);
    launchRepeatKVCache(&KC, &VC, &KLENS, &LAYER, &KR, &VR);  // context_attention.cpp:136
    launchBuildCausalMasks(&M, &LENS, &KLENS);
    launchScaleMaskAndSoftmax(&QK, &M, &SC, 1.0f / std::sqrt((float)hd));
    launchTransposeOutRemovePadding(&Q, &PO, &TO);
    // top-K + sampling over the rows of qk ([bs * heads * mq, mk], K = 5) as Llama<T>::Sampling
    const int rows = bs * heads * mq, TOPK = 5;
    Dev<int> tid(rows * TOPK), oid(rows), seql(rows);
    Dev<float> tval(rows * TOPK);
    Dev<uint8_t> fin(rows);
    std::vector<uint8_t> fin_h(rows, 0);
    for (int r = 0; r < rows; r += 7) fin_h[r] = 1;
    fin.put(fin_h);
    seql.put(std::vector<int>(rows, 4));
    oid.put(std::vector<int>(rows, -1));
    TensorWrapper<float> PROBS(GPU, FP32, {rows, mk}, qk.p), TVAL(GPU, FP32, {rows, TOPK}, tval.p);
    TensorWrapper<int> TID(GPU, INT32, {rows, TOPK}, tid.p), OID(GPU, INT32, {rows}, oid.p), SEQ(GPU, INT32, {rows}, seql.p);
    TensorWrapper<bool> FIN(GPU, BOOL, {rows}, reinterpret_cast<bool*>(fin.p));
    launchTopKforBeamSearch(&PROBS, &TID, &TVAL, &TID, &TVAL);
    LLMI_CALL(llmi_device_sync());
    {
        std::vector<int> t = tid.get();
        save(dir + "/out_topk_ids.bin", std::vector<float>(t.begin(), t.end()));
        save(dir + "/out_topk_vals.bin", tval.get());
    }
    IntDict sp{{"step", 3}, {"end_id", 2}, {"vocab_size", mk}};
    launchSampling(&TID, &TVAL, &SEQ, &FIN, &OID, sp);
    LLMI_CALL(llmi_device_sync());
    {
        std::vector<int> o = oid.get(), sq = seql.get();
        std::vector<uint8_t> f = fin.get();
        save(dir + "/out_sample_id.bin", std::vector<float>(o.begin(), o.end()));
        save(dir + "/out_sample_seq.bin", std::vector<float>(sq.begin(), sq.end()));
        save(dir + "/out_sample_fin.bin", std::vector<float>(f.begin(), f.end()));
    }
    save(dir + "/out_kr.bin", kr.get());
    save(dir + "/out_vr.bin", vr.get());

    {
        std::vector<int> po = d_po.get(), cum = d_cum.get();
        save(dir + "/out_po.bin", std::vector<float>(po.begin(), po.begin() + tokens));
        save(dir + "/out_cum.bin", std::vector<float>(cum.begin(), cum.end()));
    }
    save(dir + "/out_q.bin", q.get());
    save(dir + "/out_k.bin", k.get());
    save(dir + "/out_v.bin", v.get());
    save(dir + "/out_kc.bin", kc.get());
    save(dir + "/out_vc.bin", vc.get());
    save(dir + "/out_mask.bin", mask.get());
    save(dir + "/out_score.bin", score.get());
    save(dir + "/out_tout.bin", tout.get());
    std::printf("{\"context_ops\": \"ok\", \"tokens\": %d}\n", tokens);
    return 0;
}
