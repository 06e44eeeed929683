"""CPU: the context-operator oracle (oracle/context_ops.py) pinned to the golden-pinned
model oracle and to the reference's own worked examples."""
import math

import numpy as np

from oracle import context_ops as C
from oracle import llama_ref as R


def test_padding_offset_matches_reference_example():
    # cal_paddingoffset.cu:13-25: input lengths [5, 4, 7, 6], max_q_len 8
    po = C.padding_offset([5, 4, 7, 6], 8)
    np.testing.assert_array_equal(po, [0] * 5 + [3] * 4 + [7] * 7 + [8] * 6)


def test_rope_angles_equal_model_oracle():
    for pos in (0, 1, 127, 128, 2047):
        c, s = C.rope_angles(pos, 128, 10000.0)
        rc, rs = R.rope_cos_sin(np.array([pos]), 128, 10000.0)
        np.testing.assert_array_equal(c, rc[0, :64])
        np.testing.assert_array_equal(s, rs[0, :64])


def test_causal_mask_hand_worked():
    m = C.causal_mask([2, 3], [2, 5], 3, 5)
    want0 = [[1, 0, 0, 0, 0], [1, 1, 0, 0, 0], [0, 0, 0, 0, 0]]
    # k_len 5, q_len 3 (2 history positions): every history key is visible, as in
    # modeling_llama.py's cached forward (the reference's :29 would also require k >= 2)
    want1 = [[1, 1, 1, 0, 0], [1, 1, 1, 1, 0], [1, 1, 1, 1, 1]]
    np.testing.assert_array_equal(m[0], want0)
    np.testing.assert_array_equal(m[1], want1)


def test_causal_mask_equals_reference_formula_without_history():
    """The reference's own :29 test (with its k >= klen - qlen term) on batches with no
    history: identical to the restated mask (the term only differs when klen > qlen)."""
    rng = np.random.default_rng(7)
    for _ in range(20):
        lens = rng.integers(1, 12, size=4)
        mq = mk = int(lens.max())
        q = np.arange(mq)[:, None]
        k = np.arange(mk)[None, :]
        ref = np.asarray([(q < l) & (k < l) & (k <= q) & (k >= 0) for l in lens], np.float32)
        np.testing.assert_array_equal(C.causal_mask(lens, lens, mq, mk), ref)


def test_masked_softmax_rows():
    rng = np.random.default_rng(0)
    qk = rng.standard_normal((1, 2, 3, 5)).astype(np.float32)
    mask = C.causal_mask([3], [5], 3, 5)
    p = C.masked_softmax(qk, mask, 0.5)
    assert np.all(p[mask[:, None].repeat(2, 1) == 0] == 0)
    np.testing.assert_allclose(p.sum(-1), 1.0, atol=2e-6)


def test_context_attention_equals_model_oracle_prefill():
    """One sequence, no history: the unfused chain == llama_ref.attention_prefill with
    llama_ref's RoPE (both pinned by the golden vectors), MHA and GQA."""
    rng = np.random.default_rng(1)
    d, n = 128, 9
    for heads, kvh in ((4, 4), (4, 2)):
        qkv = rng.standard_normal((n, (heads + 2 * kvh) * d)).astype(np.float32)
        kc = np.zeros((1, 1, kvh, 16, d), np.float32)
        vc = np.zeros_like(kc)
        got = C.context_attention(qkv, [n], [0], heads, kvh, d, kc, vc)

        x = qkv.reshape(n, heads + 2 * kvh, d)
        cos, sin = R.rope_cos_sin(np.arange(n), d, 10000.0)
        q = np.stack([R.apply_rope(x[t, :heads], cos[t], sin[t]) for t in range(n)])
        k = np.stack([R.apply_rope(x[t, heads:heads + kvh], cos[t], sin[t]) for t in range(n)])
        v = x[:, heads + kvh:]
        want = R.attention_prefill(q, k.transpose(1, 0, 2), v.transpose(1, 0, 2), 0).reshape(n, heads * d)
        err = np.linalg.norm(got - want) / np.linalg.norm(want)
        assert err < 2e-6, err
        np.testing.assert_array_equal(kc[0, 0, :, :n], k.transpose(1, 0, 2))
        np.testing.assert_array_equal(vc[0, 0, :, :n], v.transpose(1, 0, 2))
        assert math.isfinite(err)
