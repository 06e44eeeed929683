"""llmi_topk / llmi_sampling / llmi_repeat_kv (sampling.hip, context_ops.hip) through the
C ABI against oracle/sampling.py on the same inputs.

Bars: top-K ids and values bit-exact (pure selection); repeat_kv bit-exact (a move);
sampling ids exact except rows whose threshold lands within 1e-6 of a boundary (device
expf vs numpy exp may differ by an ulp there -- counted and bounded), exp values within
rtol 1e-6 (f32) / one fp16 ulp (f16)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import sampling as S  # noqa: E402

DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from llmi import ops as O
    return O


def _logits(rows, vocab, dtype, seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((rows, vocab)) * 3).astype(dtype)
    x[:, rng.integers(0, vocab, 4)] = x.max() + 1  # a tie at the top of every row
    return x


@pytest.mark.parametrize("dtype", [np.float32, np.float16])
@pytest.mark.parametrize("rows,vocab,k", [(1, 32000, 5), (3, 30000, 1), (2, 32000, 16), (4, 4097, 7), (2, 7, 9)])
def test_topk_matches_oracle(ops, dtype, rows, vocab, k):
    x = _logits(rows, vocab, dtype, rows * 7 + k)
    ids, vals = ops.launchTopKforBeamSearch(torch.from_numpy(x).to(DEV), k)
    oid, oval = S.topk(x, k)
    np.testing.assert_array_equal(ids.cpu().numpy(), oid)
    np.testing.assert_array_equal(vals.cpu().numpy(), oval)


def test_topk_reference_unittest_input(ops):
    probs = torch.arange(60000, dtype=torch.float32, device=DEV).view(2, 30000)
    ids, vals = ops.launchTopKforBeamSearch(probs, 5)
    assert ids.cpu().tolist() == [[29999, 29998, 29997, 29996, 29995]] * 2
    assert vals[1].cpu().tolist() == [59999.0, 59998.0, 59997.0, 59996.0, 59995.0]


def test_topk1_is_greedy_argmax(ops):
    x = torch.from_numpy(_logits(1, 32000, np.float32, 5)).to(DEV)
    ids, _ = ops.launchTopKforBeamSearch(x, 1)
    assert int(ids[0, 0]) == int(ops.argmax(x[0])[0]) == int(torch.argmax(x[0]))


@pytest.mark.parametrize("dtype,rtol", [(np.float32, 1e-6), (np.float16, 1e-3)])
def test_sampling_matches_oracle(ops, dtype, rtol):
    rows, k, vocab, end_id = 131, 8, 32000, 17
    x = _logits(rows, 2048, dtype, 11) * dtype(0.3)
    oid, oval = S.topk(x, k)
    oid[5, 2] = end_id  # make one row likely to finish
    oval[5] = oval[5, 0]  # flat row: every candidate equally likely
    fin = (np.arange(rows) % 9 == 4).astype(np.uint8)
    seq = np.arange(rows, dtype=np.int32) + 3
    mismatched = 0
    for step in (1, 2, 513):
        t_ids = torch.from_numpy(oid).to(DEV)
        t_val = torch.from_numpy(oval.copy()).to(DEV)
        t_seq = torch.from_numpy(seq).to(DEV)
        t_fin = torch.from_numpy(fin).to(DEV)
        t_out = torch.full((rows,), -1, dtype=torch.int32, device=DEV)
        ops.launchSampling(t_ids, t_val, t_seq, t_fin, t_out, step, end_id, vocab)
        e_out, e_val, e_seq, e_fin = S.sampling(oid, oval, seq, fin, step, end_id, vocab)
        got_val = t_val.cpu().numpy()
        np.testing.assert_allclose(got_val.astype(np.float32), e_val.astype(np.float32), rtol=rtol, atol=0)
        got = t_out.cpu().numpy()
        for b in np.nonzero(got != e_out)[0]:
            assert S.sampling_margin(e_val, step, b) < 1e-6, (step, b, got[b], e_out[b])
            mismatched += 1
        ok = got == e_out
        np.testing.assert_array_equal(t_seq.cpu().numpy()[ok], e_seq[ok])
        np.testing.assert_array_equal(t_fin.cpu().numpy()[ok], e_fin[ok])
        assert (got[fin == 1] == -1).all()
    assert mismatched <= 1


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_repeat_kv_matches_oracle(ops, dtype):
    layers, batch, kv, max_seq, d, heads, max_k = 3, 3, 4, 96, 128, 32, 80
    rng = np.random.default_rng(3)
    npd = np.float32 if dtype == torch.float32 else np.float16
    kc = rng.standard_normal((layers, batch, kv, max_seq, d)).astype(npd)
    vc = rng.standard_normal((layers, batch, kv, max_seq, d)).astype(npd)
    ctx = np.array([80, 1, 57], np.int32)
    kd = torch.full((batch, heads, max_k, d), 7.0, dtype=dtype, device=DEV)
    vd = torch.full_like(kd, -7.0)
    ops.launchRepeatKVCache(torch.from_numpy(kc).to(DEV), torch.from_numpy(vc).to(DEV),
                            torch.from_numpy(ctx).to(DEV), 2, kd, vd)
    ek, ev = S.repeat_kv(kc, vc, 2, ctx, heads, max_k, np.full(kd.shape, 7, npd), np.full(vd.shape, -7, npd))
    np.testing.assert_array_equal(kd.cpu().numpy(), ek)
    np.testing.assert_array_equal(vd.cpu().numpy(), ev)


def test_repeat_kv_reference_unittest_input(ops):
    k = torch.arange(32, dtype=torch.float32, device=DEV).view(2, 1, 2, 4, 2)
    kd = torch.zeros(1, 2, 2, 2, device=DEV)
    vd = torch.zeros_like(kd)
    ops.launchRepeatKVCache(k, k, torch.tensor([2], device=DEV), 0, kd, vd)
    assert kd.view(-1).cpu().tolist() == [0, 1, 2, 3, 8, 9, 10, 11] == vd.view(-1).cpu().tolist()
