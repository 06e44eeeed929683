"""CPU checks of oracle/sampling.py on the reference unit tests' own inputs
(tests/unittests/test_topk.cu, test_sampling.cu, test_repeat_kv.cu print rather than
check, so the expected values here are worked by hand from the kernels' definitions),
plus argument validation of the three C-ABI entry points (no GPU needed: they return
before any launch)."""
import numpy as np

from oracle import sampling as S


def test_topk_reference_unittest_input():
    # test_topk.cu:11-46: batch 1, beamwidth 2, vocab 30000, K 5, probs[i] = i
    probs = np.arange(60000, dtype=np.float32).reshape(2, 30000)
    ids, vals = S.topk(probs, 5)
    np.testing.assert_array_equal(ids, [[29999, 29998, 29997, 29996, 29995]] * 2)
    np.testing.assert_array_equal(vals[1], 30000 + np.array([29999, 29998, 29997, 29996, 29995], np.float32))


def test_topk_ties_and_short_rows():
    x = np.array([[1.0, 3.0, 3.0, -2.0]], np.float32)
    ids, vals = S.topk(x, 3)
    assert ids.tolist() == [[1, 2, 0]] and vals.tolist() == [[3.0, 3.0, 1.0]]
    ids, vals = S.topk(x, 6)  # vocab < K: init() padding (topK.h:15-20)
    assert ids[0, 4:].tolist() == [-1, -1] and np.allclose(vals[0, 4:], 1e-20)


def test_sampling_reference_unittest_input():
    # test_sampling.cu:25-34: ids i, values K-1-(i%K), seqlen 4, not finished
    bs, K = 3, 3
    ids = np.arange(bs * K, dtype=np.int32).reshape(bs, K)
    vals = (K - 1 - (np.arange(bs * K) % K)).astype(np.float32).reshape(bs, K)
    out, after, seq, fin = S.sampling(ids, vals, [4] * bs, [0] * bs, step=1, end_id=2, vocab=32000)
    e = np.exp(np.array([0.0, -1.0, -2.0], np.float32))
    np.testing.assert_allclose(after, np.tile(e, (bs, 1)), rtol=1e-6)
    for b in range(bs):
        u = float(S.uniform(1, b))
        c = np.cumsum(e) / e.sum()
        assert out[b] == ids[b, int(np.searchsorted(c, u))]
    assert seq.tolist() == [5] * bs
    assert fin.tolist() == [int(o == 2) for o in out]


def test_sampling_finished_rows_untouched_and_uniform_range():
    ids = np.array([[7, 8]], np.int32)
    vals = np.array([[1.0, 0.5]], np.float32)
    out, after, seq, fin = S.sampling(ids, vals, [9], [1], step=3, end_id=0, vocab=100)
    assert out[0] == -1 and seq[0] == 9 and fin[0] == 1 and np.array_equal(after, vals)
    u = np.array([S.uniform(s, r) for s in range(50) for r in range(8)])
    assert (u > 0).all() and (u <= 1).all() and 0.4 < u.mean() < 0.6


def test_repeat_kv_reference_unittest_input():
    # test_repeat_kv.cu:11-49: 2 layers, batch 1, heads = kv = 2, max_seq 4, max_k 2, d 2, ctx 2
    k = np.arange(2 * 1 * 2 * 4 * 2, dtype=np.float32).reshape(2, 1, 2, 4, 2)
    kd, vd = S.repeat_kv(k, k, 0, [2], heads=2, max_k_len=2)
    assert kd.reshape(-1).tolist() == [0, 1, 2, 3, 8, 9, 10, 11]
    np.testing.assert_array_equal(kd, vd)
    kd, _ = S.repeat_kv(k, k, 1, [1], heads=4, max_k_len=2)  # GQA 4 q heads on 2 kv heads
    assert kd[0, :, 0].tolist() == [[16, 17], [16, 17], [24, 25], [24, 25]] and (kd[0, :, 1] == 0).all()


def test_c_abi_argument_checks():
    from llmi import _lib
    L = _lib.lib()
    assert L.llmi_topk(None, _lib.F32, 1, 10, 5, None, None, None) == -1
    assert b"topk" in L.llmi_last_error()
    assert L.llmi_sampling(None, None, _lib.F32, 1, 5, None, None, None, 0, 0, 10, None) == -1
    assert b"sampling" in L.llmi_last_error()
    assert L.llmi_repeat_kv(None, None, _lib.F16, 0, None, 1, 2, 4, 3, 2, 2, None, None, None) == -1
    assert b"repeat_kv" in L.llmi_last_error()


def test_xorwow_restatement_properties():
    """oracle/xorwow.py: the GF(2) one-step matrix reproduces curand()'s v update, a
    2^5-step jump by 5 squarings equals 32 steps, and the subsequence jump composes
    (jump(a) then jump(b) == jump(a + b) for disjoint bits)."""
    from oracle import xorwow as X
    cols = [X._v_step(1 << c) for c in range(160)]
    v, d = X.init(12345)
    x = X._pack(v)
    assert X._apply(cols, x) == X._v_step(x)
    c32 = cols
    for _ in range(5):
        c32 = X._square(c32)
    y = x
    for _ in range(32):
        y = X._v_step(y)
    assert X._apply(c32, x) == y
    j = X.seq_jumps()
    assert X._apply(j[1], X._apply(j[0], x)) == X._apply(j[0], X._apply(j[1], x))
    v3, d3 = X.init_state(12345, 3)
    assert X._pack(v3) == X._apply(j[1], X._apply(j[0], x)) and d3 == d


def test_curand_uniform_c_abi_matches_oracle():
    """llmi_curand_uniform (csrc/xorwow.h + the C++ jump table, host side) equals the
    Python restatement bit for bit, for subsequences 0 (no jump) and > 0 (table)."""
    import ctypes as C
    from llmi import _lib
    from oracle import xorwow as X
    L = _lib.lib()
    out = C.c_float()
    for seed in (0, 1, 7, 512, 2047, 2 ** 40 + 3):
        for sub in (0, 1, 2, 5, 255, 4096, 65535):
            assert L.llmi_curand_uniform(seed, sub, C.byref(out)) == 0
            assert np.float32(out.value) == X.curand_uniform(seed, sub), (seed, sub)
    assert L.llmi_curand_uniform(0, 65536, C.byref(out)) == -1
