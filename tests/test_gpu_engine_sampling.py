"""In-engine top-k sampling (llmi_engine_set_sampling: Llama<T>::Sampling, llama.cpp:245-262)
against the oracle run token by token with oracle/sampling.py's topk + sampling at
step = seed + position. Bars: sampled token ids bit-exact; k = 1 reproduces greedy; the
graph and eager paths agree."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import llama_ref as R  # noqa: E402
from oracle import sampling as S  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fixture():
    return np.load(os.path.join(REPO, "tests", "golden", "tiny.npz"), allow_pickle=False)


def _engine_tokens(k, seed, n, use_graph=True, prefill=False):
    import llmi
    from llmi.engine import Engine, preset
    f = _fixture()
    cfg = preset("tiny")
    cfg.kv_dtype = llmi.F32
    with Engine(cfg) as e:
        e.load_synthetic(int(f["seed"]))
        e.set_sampling(k, seed)
        return e.generate(f["prompt"], n, use_graph=use_graph, prefill=prefill)


def _oracle_tokens(k, seed, n):
    f = _fixture()
    o = R.LlamaOracle(R.LlamaConfig(hidden=512, heads=4, kv_heads=4, inter=1024, layers=2, max_seq=64),
                      seed=int(f["seed"]))
    prompt = [int(t) for t in f["prompt"]]
    seq = list(prompt)
    out = []
    for p in range(len(prompt) + n - 1):
        logits = o.forward_token(seq[p], p)
        if p + 1 < len(prompt):
            continue
        ids, vals = S.topk(np.asarray(logits, np.float32)[None], k)
        tok, _, _, _ = S.sampling(ids, vals, [0], [0], seed + p + 1, -1, logits.shape[-1])
        seq.append(int(tok[0]))
        out.append(int(tok[0]))
    return np.array(out, np.int32)


@pytest.mark.parametrize("k,seed", [(5, 11), (16, 12345)])
def test_engine_sampling_matches_oracle(k, seed):
    got = _engine_tokens(k, seed, 10)
    assert (got != _fixture()["tokens"][:10]).any()  # really sampled, not the greedy sequence
    np.testing.assert_array_equal(got, _oracle_tokens(k, seed, 10))
    np.testing.assert_array_equal(_engine_tokens(k, seed, 10, use_graph=False), got)


def test_engine_sampling_k1_is_greedy():
    f = _fixture()
    np.testing.assert_array_equal(_engine_tokens(1, 7, 8), f["tokens"][:8])
    np.testing.assert_array_equal(_engine_tokens(0, 7, 8), f["tokens"][:8])


def test_engine_sampling_argument_checks():
    import llmi
    from llmi._lib import LlmiError
    from llmi.engine import Engine, preset
    with Engine(preset("tiny")) as e:
        with pytest.raises(LlmiError, match="k must be"):
            e.set_sampling(17, 0)


@pytest.mark.parametrize("k,seed", [(5, 11), (16, 12345)])
def test_engine_sampling_after_prefill_matches_decode_path(k, seed):
    """firstTokenGen samples too: the token after a batched prefill is drawn at step
    seed + prompt_len, exactly as the token-by-token path draws it."""
    got = _engine_tokens(k, seed, 10, prefill=True)
    np.testing.assert_array_equal(got, _engine_tokens(k, seed, 10))
    np.testing.assert_array_equal(got, _oracle_tokens(k, seed, 10))
