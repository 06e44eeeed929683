"""Context-phase operators (context_ops.hip through the C ABI) against
oracle/context_ops.py on the same inputs: a ragged batch with padding and history,
fp32 and fp16 storage, and a 7B-width single sequence.

Bars: bit-exact for the mask, KV append and transpose (pure moves / integer tests);
RoPE and the softmax within the relative-L2 / absolute tolerances written below."""
import math

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import context_ops as C  # noqa: E402

DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from llmi import ops as O
    return O


def T(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    return t if dtype is None else t.to(dtype)


def N(t):
    torch.cuda.synchronize()
    return t.detach().float().cpu().numpy()


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


LENS, HIST = [5, 3, 7], [0, 4, 2]
HEADS, KVH, D = 4, 2, 128


def ragged(seed=0):
    rng = np.random.default_rng(seed)
    n = sum(LENS)
    qkv = rng.standard_normal((n, (HEADS + 2 * KVH) * D)).astype(np.float32)
    return qkv, C.padding_offset(LENS, max(LENS))


@pytest.mark.parametrize("dt", [torch.float32, torch.float16])
def test_rope_qkv_prefill_ragged(ops, dt):
    qkv, po = ragged()
    if dt == torch.float16:
        qkv = qkv.astype(np.float16).astype(np.float32)
    q, k, v = ops.launchAddFusedQKVBiasTransposeAndRoPE(T(qkv, dt), T(po), T(np.array(HIST, np.int32)), len(LENS),
                                                        max(LENS), HEADS, KVH, D)
    wq, wk, wv = C.rope_qkv_prefill(qkv, po, np.array(HIST), len(LENS), max(LENS), HEADS, KVH, D)
    tol = 1e-6 if dt == torch.float32 else 1e-3  # fp16: one rounding of the stored result
    assert rel(N(q), wq) < tol and rel(N(k), wk) < tol
    np.testing.assert_array_equal(N(v), wv.astype(np.float16).astype(np.float32) if dt == torch.float16 else wv)


@pytest.mark.parametrize("dt", [torch.float32, torch.float16])
def test_kv_append_bit_exact(ops, dt):
    rng = np.random.default_rng(2)
    b, max_q, max_seq, layers, layer = len(LENS), max(LENS), 24, 3, 1
    ks = rng.standard_normal((b, KVH, max_q, D)).astype(np.float32)
    vs = rng.standard_normal((b, KVH, max_q, D)).astype(np.float32)
    kc = rng.standard_normal((layers, b, KVH, max_seq, D)).astype(np.float32)
    vc = rng.standard_normal((layers, b, KVH, max_seq, D)).astype(np.float32)
    if dt == torch.float16:
        ks, vs, kc, vc = (a.astype(np.float16).astype(np.float32) for a in (ks, vs, kc, vc))
    gk, gv = T(kc, dt), T(vc, dt)
    ops.launchConcatKVCache(T(ks, dt), T(vs, dt), layer, T(np.array(LENS, np.int32)), T(np.array(HIST, np.int32)),
                            gk, gv)
    wk, wv = C.kv_append(ks, vs, layer, LENS, HIST, kc.copy(), vc.copy())
    np.testing.assert_array_equal(N(gk), wk)
    np.testing.assert_array_equal(N(gv), wv)


@pytest.mark.parametrize("dt", [torch.float32, torch.float16])
def test_causal_mask_bit_exact(ops, dt):
    ql, kl = np.array(LENS, np.int32), np.array([h + n for h, n in zip(HIST, LENS)], np.int32)
    m = ops.launchBuildCausalMasks(T(ql), T(kl), int(ql.max()), int(kl.max()), dtype=dt)
    np.testing.assert_array_equal(N(m), C.causal_mask(ql, kl, int(ql.max()), int(kl.max())))
    one = ops.launchBuildCausalMasks(T(np.array([1], np.int32)), T(np.array([1], np.int32)), 1, 1, dtype=dt)
    assert N(one).tolist() == [[[1.0]]]


@pytest.mark.parametrize("dt", [torch.float32, torch.float16])
def test_masked_softmax(ops, dt):
    rng = np.random.default_rng(3)
    ql = np.array(LENS, np.int32)
    kl = np.array([h + n for h, n in zip(HIST, LENS)], np.int32)
    mq, mk = int(ql.max()), int(kl.max())
    qk = (rng.standard_normal((len(LENS), HEADS, mq, mk)) * 8).astype(np.float32)
    mask = C.causal_mask(ql, kl, mq, mk)
    if dt == torch.float16:
        qk = qk.astype(np.float16).astype(np.float32)
    got = N(ops.launchScaleMaskAndSoftmax(T(qk, dt), T(mask, dt), 1 / math.sqrt(D)))
    want = C.masked_softmax(qk, mask, 1 / math.sqrt(D))
    atol = 1e-6 if dt == torch.float32 else 1e-3
    np.testing.assert_allclose(got, want, rtol=0, atol=atol)
    # wide rows (k_len past one workgroup's 256 threads), in place
    qk2 = (rng.standard_normal((1, 2, 3, 2500)) * 4).astype(np.float32)
    m2 = C.causal_mask([3], [2500], 3, 2500)
    t2 = T(qk2)
    ops.launchScaleMaskAndSoftmax(t2, T(m2), 0.25, out=t2)
    np.testing.assert_allclose(N(t2), C.masked_softmax(qk2, m2, 0.25), rtol=0, atol=1e-6)


@pytest.mark.parametrize("dt", [torch.float32, torch.float16])
def test_transpose_remove_pad_bit_exact(ops, dt):
    rng = np.random.default_rng(4)
    src = rng.standard_normal((len(LENS), HEADS, max(LENS), D)).astype(np.float32)
    if dt == torch.float16:
        src = src.astype(np.float16).astype(np.float32)
    po = C.padding_offset(LENS, max(LENS))
    got = ops.launchTransposeOutRemovePadding(T(src, dt), T(po), sum(LENS))
    np.testing.assert_array_equal(N(got), C.transpose_remove_pad(src, po, sum(LENS)))


def chain(ops, qkv, lens, hist, heads, kvh, max_seq):
    """The reference's context attention, every step an llmi operator (the GQA head
    expansion, the reference's repeat_kv, is torch plumbing here)."""
    b, mq = len(lens), max(lens)
    po = C.padding_offset(lens, mq)
    q, k, v = ops.launchAddFusedQKVBiasTransposeAndRoPE(T(qkv), T(po), T(np.array(hist, np.int32)), b, mq, heads,
                                                        kvh, D)
    kc = torch.zeros(1, b, kvh, max_seq, D, device=DEV)
    vc = torch.zeros_like(kc)
    ops.launchConcatKVCache(k, v, 0, T(np.array(lens, np.int32)), T(np.array(hist, np.int32)), kc, vc)
    kl = [h + n for h, n in zip(hist, lens)]
    mk = max(kl)
    g = heads // kvh
    kk = kc[0, :, :, :mk].repeat_interleave(g, dim=1)
    vv = vc[0, :, :, :mk].repeat_interleave(g, dim=1)
    qk = ops.launchLinearStridedBatchGemm(q, kk, trans_b=True)
    mask = ops.launchBuildCausalMasks(T(np.array(lens, np.int32)), T(np.array(kl, np.int32)), mq, mk)
    p = ops.launchScaleMaskAndSoftmax(qk, mask, 1 / math.sqrt(D))
    o = ops.launchLinearStridedBatchGemm(p, vv)
    return N(ops.launchTransposeOutRemovePadding(o.contiguous(), T(po), sum(lens)))


def test_context_attention_chain_ragged(ops):
    qkv, _ = ragged(5)
    got = chain(ops, qkv, LENS, HIST, HEADS, KVH, 16)
    want = C.context_attention(qkv, LENS, HIST, HEADS, KVH, D, np.zeros((1, 3, KVH, 16, D), np.float32),
                               np.zeros((1, 3, KVH, 16, D), np.float32))
    assert rel(got, want) < 1e-5


def test_context_attention_chain_7b_width():
    """Llama-2-7B heads (32 x 128), one 512-token sequence, no history (config 3 shape)."""
    from llmi import ops
    rng = np.random.default_rng(6)
    n, h = 512, 32
    qkv = rng.standard_normal((n, 3 * h * D)).astype(np.float32)
    got = chain(ops, qkv, [n], [0], h, h, n)
    want = C.context_attention(qkv, [n], [0], h, h, D, np.zeros((1, 1, h, n, D), np.float32),
                               np.zeros((1, 1, h, n, D), np.float32))
    assert rel(got, want) < 1e-5


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
@pytest.mark.parametrize("dt", [torch.float32, torch.float16])
def test_strided_batch_gemm(ops, ta, tb, dt):
    """Ragged tile edges (m, n, k not multiples of 64 / 16), 2 x 3 batch."""
    rng = np.random.default_rng(8)
    m, n, k = 70, 45, 37
    a = rng.standard_normal((2, 3, k, m) if ta else (2, 3, m, k)).astype(np.float32)
    b = rng.standard_normal((2, 3, n, k) if tb else (2, 3, k, n)).astype(np.float32)
    if dt == torch.float16:
        a, b = a.astype(np.float16).astype(np.float32), b.astype(np.float16).astype(np.float32)
    got = N(ops.launchLinearStridedBatchGemm(T(a, dt), T(b, dt), trans_a=ta, trans_b=tb))
    oa = np.swapaxes(a, -1, -2) if ta else a
    ob = np.swapaxes(b, -1, -2) if tb else b
    want = np.matmul(oa.astype(np.float64), ob.astype(np.float64))
    assert got.shape == (2, 3, m, n)
    assert rel(got, want) < (1e-6 if dt == torch.float32 else 1e-3)


@pytest.mark.parametrize("shape,tb", [((512, 512, 128), True), ((512, 128, 512), False)])
@pytest.mark.parametrize("dt", [torch.float32, torch.float16])
def test_strided_batch_gemm_attention_shapes_on_mfma(ops, shape, tb, dt):
    """The context layer's QK^T ([heads, q, d] x [heads, k, d]^T) and PV ([heads, q, k] x
    [heads, k, d]) at a 512-token 7B-width shape: the MFMA path (fp32 split into hi/lo fp16
    planes on both operands, three products) against float64, timed with HIP events: the
    MFMA kernel runs these in 16-33 us on MI355X (r03 bmm_probe), the sequential-FMA
    kernel it replaced took 100-720 us, so 80 us is a regression bar."""
    rng = np.random.default_rng(9)
    m, n, k = shape
    a = rng.standard_normal((1, 32, m, k)).astype(np.float32)
    b = rng.standard_normal((1, 32, n, k) if tb else (1, 32, k, n)).astype(np.float32)
    if dt == torch.float16:
        a, b = a.astype(np.float16).astype(np.float32), b.astype(np.float16).astype(np.float32)
    ta_, tb_ = T(a, dt), T(b, dt)
    got = N(ops.launchLinearStridedBatchGemm(ta_, tb_, trans_b=tb))
    ob = np.swapaxes(b, -1, -2) if tb else b
    want = np.matmul(a.astype(np.float64), ob.astype(np.float64))
    r = rel(got, want)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(20):
        ops.launchLinearStridedBatchGemm(ta_, tb_, trans_b=tb)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f"bmm {shape} tb={tb} {dt}: rel-L2 {r:.2e}, {us:.1f} us ({2 * 32 * m * n * k / us / 1e6:.1f} TFLOP/s)")
    assert r < (1e-6 if dt == torch.float32 else 1e-3)
    assert us < 80.0


@pytest.mark.parametrize("scale", [1e20, 1e6, 1e-6, 1e-30])
def test_strided_batch_gemm_fp32_range(ops, scale):
    """fp32 operands outside fp16's range (|v| > 65504) or below its normals (< 6e-5) on
    the MFMA path: each 32-deep K slab is scaled by a power of two before the hi/lo split
    (context_ops.hip), so results stay finite and fp32-faithful. Rows of A and columns of
    B span 12 decades (scale * 10^[-6, 6]) so every slab mixes magnitudes; float64 bar
    1e-6 rel-L2 per output row. The largest scale keeps every exact product sum inside
    fp32's range (1e20 * 1e6 * 1e3 * sqrt(96) ~ 1e30): at 1e30 some exact outputs
    exceed 3.4e38 and are inf in any fp32 GEMM, the reference's cuBLAS SGEMM included."""
    rng = np.random.default_rng(11)
    m, n, k = 64, 48, 96
    a = rng.standard_normal((1, 2, m, k)) * scale * 10.0 ** rng.uniform(-6, 6, (1, 2, m, 1))
    b = rng.standard_normal((1, 2, k, n)) * 10.0 ** rng.uniform(-3, 3, (1, 2, 1, n))
    a, b = a.astype(np.float32), b.astype(np.float32)
    got = N(ops.launchLinearStridedBatchGemm(T(a), T(b)))
    want = np.matmul(a.astype(np.float64), b.astype(np.float64))
    assert np.isfinite(got).all()
    err = np.linalg.norm(got - want, axis=-1) / np.linalg.norm(want, axis=-1)
    assert err.max() < 1e-6, err.max()


@pytest.mark.parametrize("dt", [torch.float32, torch.float16, torch.int32, torch.int64])
def test_tp_allreduce_single_rank(ops, dt):
    """llmi_tp_comm_create / llmi_tp_allreduce / llmi_tp_comm_destroy over RCCL with one
    rank (this box has one GPU): the sum over one rank is the input, bit for bit; the
    multi-rank reduction is exercised by bench.py --gpus N through the engine."""
    x = (torch.arange(4099, device=DEV) % 97 - 48).to(dt)
    ref = x.clone()
    with ops.TPComm(ops.tp_unique_id(), 1, 0, torch.cuda.current_device()) as comm:
        comm.all_reduce(x)
        torch.cuda.synchronize()
    assert torch.equal(x, ref)


def test_padding_offset_reference_example(ops):
    """cal_paddingoffset.cu:13-25's worked example: lengths [5, 4, 7, 6], max_q_len 8."""
    po, cum = ops.launchCalPaddingoffset(T(np.array([5, 4, 7, 6], np.int32)), 8)
    np.testing.assert_array_equal(N(po).astype(np.int32), C.padding_offset([5, 4, 7, 6], 8))
    assert N(cum).astype(int).tolist() == [0, 5, 9, 16, 22]


@pytest.mark.parametrize("cache_dt", [np.float32, np.float16])
@pytest.mark.parametrize("heads,kvh,lens,hist", [
    (4, 2, [5, 3, 7], [0, 4, 2]),          # GQA, ragged, history
    (8, 8, [33, 1, 64, 20], [31, 0, 3, 65]),  # chunks across 32-key blocks, one-token sequence
    (8, 1, [70], [0]),                     # MQA, one sequence past two query blocks
    (8, 2, [130, 65, 17], [0, 40, 100]),   # past two 64-query blocks, partly filled waves
])
def test_context_attention_qkv_fused_matches_oracle(ops, cache_dt, heads, kvh, lens, hist):
    """llmi_context_attention_qkv (RoPE + the k / v store into the cache + the ragged flash
    attention, what LLaMAContextAttentionLayer runs for head size 128) against the oracle's
    composition of the reference's unfused launchers (oracle/context_ops.py:
    context_attention): the attention output within 1e-5 rel-L2 (fp32 cache) / 1e-4 (fp16
    cache: both read the same rounded cache; a new k may round to the neighbouring fp16
    where the two RoPE restatements differ in the last fp32 bit), the new cache
    slots within 1e-6 (fp32) / one fp16 rounding (fp16), history slots untouched."""
    rng = np.random.default_rng(len(lens) * 7 + heads)
    d, layers, layer = 128, 2, 1
    n, batch, max_q = sum(lens), len(lens), max(lens)
    max_seq = max(h + q for h, q in zip(hist, lens)) + 5
    qkv = rng.standard_normal((n, (heads + 2 * kvh) * d)).astype(np.float32)
    kc = (rng.standard_normal((layers, batch, kvh, max_seq, d)) * 0.5).astype(cache_dt)
    vc = (rng.standard_normal((layers, batch, kvh, max_seq, d)) * 0.5).astype(cache_dt)
    ok, ov = kc.copy(), vc.copy()
    want = C.context_attention(qkv, lens, np.array(hist), heads, kvh, d, ok, ov, layer=layer)
    po = C.padding_offset(lens, max_q)
    tdt = torch.float32 if cache_dt == np.float32 else torch.float16
    tk, tv = T(kc, tdt), T(vc, tdt)
    got = N(ops.context_attention_qkv(T(qkv), T(po), T(np.array(hist, np.int32)), T(np.array(lens, np.int32)),
                                      batch, max_q, heads, kvh, tk, tv, layer=layer))
    e = rel(got, want)
    print(f"fused context attention heads {heads} kv {kvh} lens {lens} cache {cache_dt.__name__}: rel-L2 {e:.2e}")
    assert e < (1e-5 if cache_dt == np.float32 else 1e-4)
    gk, gv = N(tk), N(tv)
    for b, (h0, q) in enumerate(zip(hist, lens)):
        np.testing.assert_array_equal(gk[layer, b, :, :h0], kc[layer, b, :, :h0].astype(np.float32))
        np.testing.assert_array_equal(gv[layer, b, :, :h0], vc[layer, b, :, :h0].astype(np.float32))
        slot_tol = 1e-6 if cache_dt == np.float32 else 1e-3
        assert rel(gk[layer, b, :, h0:h0 + q], ok[layer, b, :, h0:h0 + q]) < slot_tol
        np.testing.assert_array_equal(gv[layer, b, :, h0:h0 + q], ov[layer, b, :, h0:h0 + q].astype(np.float32))
    np.testing.assert_array_equal(gk[0], kc[0].astype(np.float32))  # other layers untouched


@pytest.mark.parametrize("m", [16, 100, 300, 512])
def test_ffn_fused_matches_fp64(ops, m):
    """llmi_ffn (gate_up with the SiLU*up epilogue writing the down GEMM's fp16 input planes,
    then down; gemm2 below 256 rows, gemm3 above) against float64 numpy of
    W_down (silu(W_gate x) * (W_up x)) with the same fp16 weights: the fp32-faithful planes
    keep it within 1e-5 rel-L2; an unsupported shape raises instead of launching."""
    rng = np.random.default_rng(m)
    hidden, inter = 512, 1024
    x = rng.standard_normal((m, hidden)).astype(np.float32)
    wgu = (rng.standard_normal((2 * inter, hidden)) / math.sqrt(hidden)).astype(np.float16)
    wd = (rng.standard_normal((hidden, inter)) / math.sqrt(inter)).astype(np.float16)
    got = N(ops.ffn(T(x), T(wgu), T(wd)))
    x64, g64, d64 = x.astype(np.float64), wgu.astype(np.float64), wd.astype(np.float64)
    gu = x64 @ g64.T
    g, u = gu[:, :inter], gu[:, inter:]
    want = ((g / (1.0 + np.exp(-g))) * u) @ d64.T
    e = rel(got, want)
    print(f"fused ffn m {m}: rel-L2 vs fp64 {e:.2e}")
    assert e < 1e-5
    from llmi._lib import LlmiError
    with pytest.raises(LlmiError):
        ops.ffn(T(x[:8]), T(wgu), T(wd))  # m < 16: the caller's three-launch path


@pytest.mark.parametrize("m", [16, 300, 512])
@pytest.mark.parametrize("gdt", [np.float16, np.float32])
def test_linear_residual_matches_composition(ops, m, gdt):
    """llmi_linear_residual (o_proj + launchFusedAddBiasResidualRMSNorm as one call; the
    residual epilogue sums the K slices in slice order, then adds the residual) against the
    separate launches on the same inputs: the updated residual is bit-identical (same
    additions in the same order), the normalised rows within 1e-6 rel-L2 (the row's sum of
    squares is reduced in another order); gamma None returns the residual, out False only
    updates it; an unsupported shape raises before launching. K 2048 at 512 rows takes the
    8-slice split."""
    rng = np.random.default_rng(m)
    n, k, eps = 512, 2048, 1e-5
    x = rng.standard_normal((m, k)).astype(np.float32)
    w = (rng.standard_normal((n, k)) / math.sqrt(k)).astype(np.float16)
    r0 = rng.standard_normal((m, n)).astype(np.float32)
    gamma = (1.0 + 0.1 * rng.standard_normal(n)).astype(gdt)
    r = T(r0)
    y = ops.linear_residual(T(x), T(w), r, T(gamma), eps)
    r_ref, y_ref = T(r0), ops.launchLinearGemm(T(x), T(w))
    ops.launchFusedAddBiasResidualRMSNorm(r_ref, y_ref, T(gamma), eps)
    np.testing.assert_array_equal(N(r), N(r_ref))
    e = rel(N(y), N(y_ref))
    print(f"linear_residual m {m} gamma {np.dtype(gdt).name}: normalised rows rel-L2 vs separate launches {e:.2e}")
    assert e < 1e-6
    # float64 restatement of the pair (the projection's own error bar: llmi_linear's 1e-5)
    r64 = r0.astype(np.float64) + x.astype(np.float64) @ w.astype(np.float64).T
    assert rel(N(r), r64) < 1e-5
    r2 = T(r0)
    copy = ops.linear_residual(T(x), T(w), r2, None, eps)
    np.testing.assert_array_equal(N(copy), N(r2))
    r3 = T(r0)
    assert ops.linear_residual(T(x), T(w), r3, T(gamma), eps, out=False) is None
    np.testing.assert_array_equal(N(r3), N(r_ref))
    from llmi._lib import LlmiError
    with pytest.raises(LlmiError):
        ops.linear_residual(T(x[:8]), T(w), T(r0[:8]), T(gamma), eps)  # m < 16


@pytest.mark.parametrize("m", [16, 300, 512])
def test_ffn_residual_matches_composition(ops, m):
    """llmi_ffn_residual (the FFN + launchAddResidual + the next layer's launchRMSNorm as one
    call) against llmi_ffn followed by those launches: residual bit-identical, normalised
    rows within 1e-6 rel-L2, and within 1e-5 of float64."""
    rng = np.random.default_rng(100 + m)
    hidden, inter, eps = 512, 1024, 1e-6
    x = rng.standard_normal((m, hidden)).astype(np.float32)
    wgu = (rng.standard_normal((2 * inter, hidden)) / math.sqrt(hidden)).astype(np.float16)
    wd = (rng.standard_normal((hidden, inter)) / math.sqrt(inter)).astype(np.float16)
    r0 = rng.standard_normal((m, hidden)).astype(np.float32)
    gamma = (1.0 + 0.1 * rng.standard_normal(hidden)).astype(np.float16)
    r = T(r0)
    xt = T(x)
    y = ops.ffn_residual(xt, T(wgu), T(wd), r, T(gamma), eps)
    f = ops.ffn(T(x), T(wgu), T(wd))
    ops.launchAddResidual(T(r0), f)  # f = r0 + ffn(x): the next layer's input
    np.testing.assert_array_equal(N(r), N(f))
    r_ref = torch.empty_like(f)
    ops.launchRMSNorm(f, T(gamma), eps, r_ref)
    e = rel(N(y), N(f))
    print(f"ffn_residual m {m}: normalised rows rel-L2 vs separate launches {e:.2e}")
    assert e < 1e-6
    x64, g64, d64 = x.astype(np.float64), wgu.astype(np.float64), wd.astype(np.float64)
    gu = x64 @ g64.T
    g, u = gu[:, :inter], gu[:, inter:]
    r64 = r0.astype(np.float64) + ((g / (1.0 + np.exp(-g))) * u) @ d64.T
    assert rel(N(r), r64) < 1e-5
    np.testing.assert_array_equal(N(xt), x)  # x read, never written (out is a new tensor here)


@pytest.mark.parametrize("cache_dt", [np.float32, np.float16])
def test_context_attention_fused_7b_ragged_timing(ops, cache_dt):
    """The fused core at the context decoder's bench shape (Llama-2-7B heads, ragged lens
    200 / 150 / 100 / 62, no history) against the oracle, timed with HIP events: the f32
    MFMA kernel (context_ops.hip ctx_attn_mfma_kernel). Bar: the oracle's 1e-5 / 1e-4, and
    40 us per layer -- the VALU form it replaced took ~43 us (r04n kernel stats)."""
    rng = np.random.default_rng(21)
    lens, hist, heads, d = [200, 150, 100, 62], [0, 0, 0, 0], 32, 128
    n, batch, max_q = sum(lens), len(lens), max(lens)
    qkv = rng.standard_normal((n, 3 * heads * d)).astype(np.float32)
    kc = np.zeros((1, batch, heads, max_q, d), cache_dt)
    vc = np.zeros((1, batch, heads, max_q, d), cache_dt)
    want = C.context_attention(qkv, lens, np.array(hist), heads, heads, d, kc.copy(), vc.copy(), layer=0)
    po = C.padding_offset(lens, max_q)
    tdt = torch.float32 if cache_dt == np.float32 else torch.float16
    tk, tv = T(kc, tdt), T(vc, tdt)
    args = (T(qkv), T(po), T(np.array(hist, np.int32)), T(np.array(lens, np.int32)), batch, max_q, heads, heads, tk, tv)
    got = N(ops.context_attention_qkv(*args, layer=0))
    e = rel(got, want)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(20):
        ops.context_attention_qkv(*args, layer=0)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f"fused context attention 7B ragged {lens} cache {cache_dt.__name__}: rel-L2 {e:.2e}, {us:.1f} us "
          f"(RoPE + cache store + attention)")
    assert e < (1e-5 if cache_dt == np.float32 else 1e-4)
    assert us < 60.0


@pytest.mark.parametrize("cache_dt", [np.float32, np.float16])
@pytest.mark.parametrize("lens,hist", [([200, 150, 100, 62], [0, 0, 0, 0]), ([40, 9, 33], [0, 7, 20])])
def test_context_attention_proj_matches_linear_then_qkv(ops, cache_dt, lens, hist):
    """llmi_context_attention_proj (the q/k/v projection's K slices summed by the RoPE kernel)
    against llmi_linear followed by llmi_context_attention_qkv on the same inputs: the same
    additions in the same order, so the attention output and the cache slots are bitwise equal
    (7B-width heads at the bench's ragged shape: 2-slice split; fewer rows: other splits)."""
    rng = np.random.default_rng(sum(lens))
    heads, kvh, d, hidden = 32, 32, 128, 4096
    n, batch, max_q = sum(lens), len(lens), max(lens)
    max_seq = max(h + q for h, q in zip(hist, lens))
    x = rng.standard_normal((n, hidden)).astype(np.float32)
    w = (rng.standard_normal(((heads + 2 * kvh) * d, hidden)) / math.sqrt(hidden)).astype(np.float16)
    kc = (rng.standard_normal((1, batch, kvh, max_seq, d)) * 0.5).astype(cache_dt)
    vc = (rng.standard_normal((1, batch, kvh, max_seq, d)) * 0.5).astype(cache_dt)
    po = C.padding_offset(lens, max_q)
    tdt = torch.float32 if cache_dt == np.float32 else torch.float16
    idx = (T(po), T(np.array(hist, np.int32)), T(np.array(lens, np.int32)), batch, max_q, heads, kvh)
    k1, v1, k2, v2 = T(kc, tdt), T(vc, tdt), T(kc, tdt), T(vc, tdt)
    got = N(ops.context_attention_proj(T(x), T(w), *idx, k1, v1))
    qkv = ops.launchLinearGemm(T(x), T(w))
    want = N(ops.context_attention_qkv(qkv, *idx, k2, v2))
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(N(k1), N(k2))
    np.testing.assert_array_equal(N(v1), N(v2))


def test_linear_stream_k_shape_matches_fp64(ops):
    """A q/k/v-shaped projection whose 256 x 256 tiles leave CUs idle (m 512, n 12288: 96
    tiles): on the 2-slice split by default (stream-K measured slower for q/k/v; with
    LLMI_SK_LINEAR=1 the same call takes gemm3_sk_kernel): against float64 within
    llmi_linear's 1e-5 and twice in a row bitwise equal (repeatable sums)."""
    rng = np.random.default_rng(31)
    m, n, k = 512, 12288, 1024
    x = rng.standard_normal((m, k)).astype(np.float32)
    w = (rng.standard_normal((n, k)) / math.sqrt(k)).astype(np.float16)
    y1 = N(ops.launchLinearGemm(T(x), T(w)))
    y2 = N(ops.launchLinearGemm(T(x), T(w)))
    np.testing.assert_array_equal(y1, y2)
    want = x.astype(np.float64) @ w.astype(np.float64).T
    e = rel(y1, want)
    print(f"stream-K linear {m}x{n}x{k}: rel-L2 vs fp64 {e:.2e}")
    assert e < 1e-5


def test_ffn_stream_k_shape_matches_fp64(ops):
    """llmi_ffn with a gate_up of 96 tiles (m 512, inter 6144): the SiLU*up epilogue after the
    stream-K sum, against float64 within 1e-5, repeatable bitwise."""
    rng = np.random.default_rng(32)
    m, hidden, inter = 512, 1024, 6144
    x = rng.standard_normal((m, hidden)).astype(np.float32)
    wgu = (rng.standard_normal((2 * inter, hidden)) / math.sqrt(hidden)).astype(np.float16)
    wd = (rng.standard_normal((hidden, inter)) / math.sqrt(inter)).astype(np.float16)
    got = N(ops.ffn(T(x), T(wgu), T(wd)))
    np.testing.assert_array_equal(got, N(ops.ffn(T(x), T(wgu), T(wd))))
    x64, g64, d64 = x.astype(np.float64), wgu.astype(np.float64), wd.astype(np.float64)
    gu = x64 @ g64.T
    g, u = gu[:, :inter], gu[:, inter:]
    want = ((g / (1.0 + np.exp(-g))) * u) @ d64.T
    e = rel(got, want)
    print(f"stream-K ffn m {m} hidden {hidden} inter {inter}: rel-L2 vs fp64 {e:.2e}")
    assert e < 1e-5
    # every partial arrived: no sticky error bit on this stream, and reading clears it
    assert ops.stream_errors() == 0
    assert ops.stream_errors() == 0


@pytest.mark.parametrize("mode", [1, 2])
def test_ffn_stream_k_fault_raises_and_next_call_is_clean(ops, mode):
    """A stream-K piece that never publishes (mode 1) or publishes 2.5 s late, after its owner
    gave up (mode 2; the late flag must not satisfy a later launch's wait): llmi_ffn's result
    is flagged (bit 16) and ops.ffn raises; the next call is bitwise the clean result."""
    from llmi._lib import LlmiError
    rng = np.random.default_rng(32)
    m, hidden, inter = 512, 1024, 6144
    x = rng.standard_normal((m, hidden)).astype(np.float32)
    wgu = (rng.standard_normal((2 * inter, hidden)) / math.sqrt(hidden)).astype(np.float16)
    wd = (rng.standard_normal((hidden, inter)) / math.sqrt(inter)).astype(np.float16)
    tx, tgu, td = T(x), T(wgu), T(wd)
    clean = N(ops.ffn(tx, tgu, td))
    ops.debug_stream_k(mode, 1)
    try:
        with pytest.raises(LlmiError, match="stream-K partial never arrived"):
            ops.ffn(tx, tgu, td)
    finally:
        ops.debug_stream_k(0, 0)
    assert ops.stream_errors() == 0  # read and cleared by the raise
    np.testing.assert_array_equal(N(ops.ffn(tx, tgu, td)), clean)
    np.testing.assert_array_equal(N(ops.ffn(tx, tgu, td)), clean)


@pytest.mark.parametrize("trans_a,trans_b", [(False, False), (True, False), (True, True), (False, True)])
@pytest.mark.parametrize("m", [3, 32])
def test_linear_trans_forms_match_fp64(ops, trans_a, trans_b, m):
    """launchLinearGemm (llmi_linear_trans) in every (trans_a, trans_b) form of linear.cu:38-99
    on a non-square, non-symmetric fp16 weight: against float64 within 1e-6 (rel-L2)."""
    rng = np.random.default_rng(40 + m)
    k, n = 1024, 1536
    x = rng.standard_normal((m, k)).astype(np.float32)
    w = (rng.standard_normal((n, k)) / math.sqrt(k)).astype(np.float16)  # [out, in]
    xa = x.T.copy() if trans_a else x
    wb = w if trans_b else w.T.copy()
    got = N(ops.launchLinearGemm(T(xa), T(wb), trans_a=trans_a, trans_b=trans_b))
    want = x.astype(np.float64) @ w.astype(np.float64).T
    e = rel(got, want)
    print(f"linear m {m} trans_a {trans_a} trans_b {trans_b}: rel-L2 vs fp64 {e:.2e}")
    assert got.shape == (m, n) and e < 1e-6


def test_ffn_without_stream_k_matches_fp64():
    """LLMI_SK=0 (the knob that turns gemm3 stream-K off) in a child process: llmi_ffn at the
    stream-K shape on the plain 172-tile launch, against float64 within the same 1e-5."""
    import subprocess
    import sys
    import os
    code = r'''
import math, numpy as np, torch, sys
sys.path.insert(0, "llm-inference_amd")
from llmi import ops
rng = np.random.default_rng(32)
m, hidden, inter = 512, 1024, 6144
x = rng.standard_normal((m, hidden)).astype(np.float32)
wgu = (rng.standard_normal((2 * inter, hidden)) / math.sqrt(hidden)).astype(np.float16)
wd = (rng.standard_normal((hidden, inter)) / math.sqrt(inter)).astype(np.float16)
T = lambda a: torch.from_numpy(a).cuda()
got = ops.ffn(T(x), T(wgu), T(wd)).cpu().numpy().astype(np.float64)
gu = x.astype(np.float64) @ wgu.astype(np.float64).T
g, u = gu[:, :inter], gu[:, inter:]
want = ((g / (1.0 + np.exp(-g))) * u) @ wd.astype(np.float64).T
print(np.linalg.norm(got - want) / np.linalg.norm(want))
'''
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LLMI_SK="0")
    r = subprocess.run([sys.executable, "-c", code], cwd=repo, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    e = float(r.stdout.strip().splitlines()[-1])
    print(f"ffn with LLMI_SK=0: rel-L2 vs fp64 {e:.2e}")
    assert e < 1e-5
