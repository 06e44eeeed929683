"""Operator-level parity on the MI355X: every llmi kernel (through the C ABI)
against the numpy oracle / golden fixtures on the same inputs.

Bars: bit-exact for the generator, embedding gather, KV slot index and argmax;
fp32 kernels within the relative-L2 tolerance written in each test."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from llmi import _lib  # noqa: E402
from oracle import llama_ref as R  # noqa: E402
from oracle import prng  # noqa: E402

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from llmi import ops as O
    return O


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def T(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    return t if dtype is None else t.to(dtype)


def N(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


# ----------------------------------------------------------------- generator
def test_device_generator_bit_exact(ops):
    seed, tid = 5, prng.layer_tid(1, prng.KIND_DOWN)
    out = torch.empty(128, 200, dtype=torch.float16, device=DEV)
    ops.synth_fill(out, _lib.SYN_LINEAR, seed, tid, 128, 200, 7, 33, 11008)
    np.testing.assert_array_equal(N(out).view(np.uint16),
                                  prng.linear_fp16(seed, tid, 128, 200, 7, 33, 11008).view(np.uint16))
    q = torch.empty(32, 64, dtype=torch.int8, device=DEV)
    ops.synth_fill(q, _lib.SYN_INT8, seed, tid, 32, 64, 0, 0, 64)
    np.testing.assert_array_equal(N(q), prng.int8_weight(seed, tid, 32, 64))
    s = torch.empty(32, dtype=torch.float16, device=DEV)
    ops.synth_fill(s, _lib.SYN_INT8_SCALE, seed, tid, 32, 1, 0, 0, 1)
    np.testing.assert_array_equal(N(s).view(np.uint16), prng.int8_row_scale(seed, tid, 32).view(np.uint16))
    g = torch.empty(4096, dtype=torch.float32, device=DEV)
    ops.synth_fill(g, _lib.SYN_GAMMA, seed, tid, 1, 4096, 0, 0, 4096)
    np.testing.assert_array_equal(N(g), prng.gamma_fp16(seed, tid, 4096).astype(np.float32))


# --------------------------------------------------------------- embedding
@pytest.mark.parametrize("tdt", [np.float16, np.float32])
def test_embedding_bit_exact(ops, tdt):
    table = prng.embed_fp16(3, prng.GLOBAL_EMBED, 1000, 512).astype(tdt)
    ids = np.array([0, 999, 5, 5, 123], np.int32)
    out = N(ops.launchInputEmbedding(T(ids), T(table)))
    np.testing.assert_array_equal(out, table[ids].astype(np.float32))


# ----------------------------------------------------------------- rmsnorm
def test_rmsnorm_golden_and_residual_save(ops):
    f = np.load(os.path.join(G, "f1_ops.npz"))
    g = prng.gamma_fp16(int(f["seed"]), prng.layer_tid(0, prng.KIND_ATTN_NORM), 4096)
    x = T(f["x"])
    resid = torch.empty_like(x)
    ops.launchRMSNorm(x, T(g), 1e-5, decoder_residual=resid)
    assert rel(N(x), f["rms_out"]) < 1e-6
    np.testing.assert_array_equal(N(resid), f["x"])


def test_add_residual_rmsnorm_and_add_residual(ops):
    rng = np.random.default_rng(0)
    r0 = rng.standard_normal((3, 4096)).astype(np.float32)
    o0 = rng.standard_normal((3, 4096)).astype(np.float32)
    g = prng.gamma_fp16(1, 7, 4096)
    r, o = T(r0), T(o0)
    ops.launchFusedAddBiasResidualRMSNorm(r, o, T(g), 1e-5)
    np.testing.assert_allclose(N(r), r0 + o0, rtol=0, atol=0)
    assert rel(N(o), R.rmsnorm(r0 + o0, g, 1e-5)) < 1e-6
    a, b = T(r0), T(o0)
    ops.launchAddResidual(a, b)
    np.testing.assert_array_equal(N(b), o0 + r0)


# -------------------------------------------------------------------- GEMV
@pytest.mark.parametrize("wdt", ["f16", "f32", "i8"])
@pytest.mark.parametrize("n,k,m", [(256, 4096, 1), (77, 11008, 1), (4096, 512, 2), (33, 1376, 3), (1, 5120, 1)])
def test_linear_gemv(ops, wdt, n, k, m):
    rng = np.random.default_rng(n * k + m)
    x = rng.standard_normal((m, k)).astype(np.float32)
    tid = prng.layer_tid(0, prng.KIND_O)
    scales = None
    if wdt == "i8":
        w = prng.int8_weight(9, tid, n, k)
        s = prng.int8_row_scale(9, tid, n)
        wf = R.dequant(w, s)
        scales = T(s)
        wt = T(w)
    else:
        w = prng.linear_fp16(9, tid, n, k)
        wf = w.astype(np.float32)
        wt = T(w if wdt == "f16" else wf)
    y = N(ops.launchLinearGemm(T(x), wt, scales))
    ref = x.astype(np.float64) @ wf.astype(np.float64).T
    assert rel(y, ref) < 2e-6


@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("norm", [False, True])
def test_linear_fused_epilogues(ops, epi, norm):
    """llmi_linear_fused (the batch-1 LlamaSelfDecoder path): optional RMSNorm prologue with
    an fp16 gamma, then store / + resid / silu(gate) * up, against float64 numpy."""
    import ctypes as C
    rng = np.random.default_rng(epi * 2 + int(norm))
    k, inter = 4096, 1024
    n = 2 * inter if epi == 2 else 1536
    x = rng.standard_normal(k).astype(np.float32)
    w = prng.linear_fp16(3, prng.layer_tid(1, prng.KIND_GATE), n, k)
    g = (1.0 + 0.1 * rng.standard_normal(k)).astype(np.float16)
    res = rng.standard_normal(n).astype(np.float32)
    xn = x.astype(np.float64)
    if norm:
        xn = xn / np.sqrt(np.mean(xn * xn) + 1e-5) * g.astype(np.float64)
    acc = w.astype(np.float64) @ xn
    if epi == 0:
        want = acc
    elif epi == 1:
        want = acc + res
    else:
        gate, up = acc[:inter], acc[inter:]
        want = gate / (1.0 + np.exp(-gate)) * up
    xt, wt, gt, rt = T(x), T(w), T(g), T(res)
    y = torch.zeros(len(want), dtype=torch.float32, device=DEV)
    _lib.call("llmi_linear_fused", C.c_void_p(xt.data_ptr()), C.c_void_p(wt.data_ptr()), _lib.F16, None,
              C.c_void_p(y.data_ptr()), n, k, C.c_void_p(gt.data_ptr()) if norm else None, _lib.F16, 1e-5, epi,
              C.c_void_p(rt.data_ptr()) if epi == 1 else None, None)
    assert rel(N(y), want) < 2e-6


def test_linear_golden_q_proj(ops):
    f = np.load(os.path.join(G, "f1_ops.npz"))
    w = prng.linear_fp16(int(f["seed"]), prng.layer_tid(0, prng.KIND_Q), 256, 4096)
    y = N(ops.launchLinearGemm(T(f["x"]), T(w)))
    assert rel(y, f["linear_out"]) < 1e-6


# -------------------------------------------------------------- SiLU * mul
def test_silu_mul_golden(ops):
    f = np.load(os.path.join(G, "f1_ops.npz"))
    gu = f["silu_in"].reshape(2, 2, 512)
    out = N(ops.launchAct(T(gu)))
    assert rel(out, f["silu_mul_out"]) < 1e-6


# -------------------------------------------------------------------- RoPE
def test_rope_golden_positions(ops):
    f = np.load(os.path.join(G, "f1_ops.npz"))
    q, k = f["rope_q"][0], f["rope_k"][0]  # [heads, npos, d]
    for i, p in enumerate(f["rope_pos"]):
        qkv = np.concatenate([q[:, i].reshape(-1), k[:, i].reshape(-1), np.zeros(32 * 128, np.float32)])
        t = T(qkv)
        ops.launchRoPE(t, int(p), 32, 32)
        out = N(t)
        assert rel(out[:4096], f["rope_q_out"][0][:, i].reshape(-1)) < 2e-6, p
        assert rel(out[4096:8192], f["rope_k_out"][0][:, i].reshape(-1)) < 2e-6, p


# --------------------------------------------------------------- attention
def _attn_case(ops, heads, kv_heads, ctx, cache_dt, rope, max_seq=2048, layer=1, seed=0):
    d = 128
    rng = np.random.default_rng(seed + ctx)
    L = 2
    kc = (rng.standard_normal((L, kv_heads, max_seq, d)) * 0.5).astype(np.float32)
    vc = rng.standard_normal((L, kv_heads, max_seq, d)).astype(np.float32)
    kc, vc = kc.astype(cache_dt), vc.astype(cache_dt)
    qkv = rng.standard_normal((heads + 2 * kv_heads) * d).astype(np.float32)
    pos = ctx - 1
    ktd, vtd = T(kc), T(vc)
    ws = ops.attn_workspace(heads, max_seq)
    out = N(ops.launchDecoderMaskedMHA(T(qkv), ktd, vtd, layer, pos, heads, kv_heads, ws, rope=rope))
    q = qkv[:heads * d].reshape(heads, d)
    k = qkv[heads * d:(heads + kv_heads) * d].reshape(kv_heads, d)
    v = qkv[(heads + kv_heads) * d:].reshape(kv_heads, d)
    if rope:
        cos, sin = R.rope_cos_sin([pos], d, 10000.0)
        q, k = R.apply_rope(q, cos[0], sin[0]), R.apply_rope(k, cos[0], sin[0])
    kref, vref = kc[layer].copy(), vc[layer].copy()
    kref[:, pos] = k.astype(cache_dt)
    vref[:, pos] = v.astype(cache_dt)
    ref = R.attention_decode(q, kref.astype(np.float32), vref.astype(np.float32), ctx).reshape(-1)
    assert rel(out, ref) < 2e-6, (heads, kv_heads, ctx, cache_dt, rope, rel(out, ref))
    # the cache slot written is exactly `pos` of `layer` (index bit-exact), nothing
    # else changed; the written values are bit-exact without RoPE and within one
    # cache ulp with it (fp32 rotation arithmetic may contract differently)
    kn, vn = N(ktd), N(vtd)
    if rope:
        np.testing.assert_allclose(kn[layer][:, pos].astype(np.float32), kref[:, pos].astype(np.float32),
                                   rtol=2e-3 if cache_dt == np.float16 else 1e-6, atol=1e-6)
    else:
        np.testing.assert_array_equal(kn[layer][:, pos], kref[:, pos])
    np.testing.assert_array_equal(vn[layer][:, pos], vref[:, pos])
    mask = np.ones(kn.shape[:3], bool)
    mask[layer, :, pos] = False
    np.testing.assert_array_equal(kn[mask], kc[mask])
    np.testing.assert_array_equal(vn[mask], vc[mask])


@pytest.mark.parametrize("ctx", [1, 2, 63, 64, 65, 200, 1000, 2048])
@pytest.mark.parametrize("cache_dt", [np.float16, np.float32])
def test_attention_decode_mha(ops, ctx, cache_dt):
    _attn_case(ops, 32, 32, ctx, cache_dt, rope=False)


@pytest.mark.parametrize("ctx", [1, 129, 2048])
def test_attention_decode_fused_rope_and_gqa(ops, ctx):
    _attn_case(ops, 32, 32, ctx, np.float16, rope=True)
    _attn_case(ops, 8, 2, ctx, np.float32, rope=True, seed=1)


def test_attention_repeated_calls_leave_counters_clean(ops):
    for _ in range(3):
        _attn_case(ops, 4, 4, 700, np.float32, rope=False, max_seq=1024)


# ------------------------------------------------------------------ argmax
def test_argmax_ties_lowest_index(ops):
    rng = np.random.default_rng(2)
    lg = rng.standard_normal(32000).astype(np.float32)
    assert int(N(ops.argmax(T(lg)))[0]) == int(np.argmax(lg))
    lg[[7, 31999, 100]] = 50.0
    assert int(N(ops.argmax(T(lg)))[0]) == 7
    lg = -np.abs(lg) - 1
    assert int(N(ops.argmax(T(lg)))[0]) == int(np.argmax(lg))
