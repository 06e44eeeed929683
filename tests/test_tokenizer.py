"""Tokenizer: include/llmi/tokenizer.h against the CPU
restatement oracle/tokenizer.py, both pinned by the reference's own known answer:
llama.cpp:382 hard-codes the ids of "Hey, are you conscious? Can you talk to me?"
(from the HF tokenizer; the vocabulary is the reference's llama2-7b-tokenizer.bin,
copied to tests/golden as a data fixture)."""
import json
import os
import subprocess

import pytest

from oracle import tokenizer as T

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VOCAB = os.path.join(REPO, "tests", "golden", "llama2-7b-tokenizer.bin")
# llama.cpp:382 (BOS = 1 first; Encode does not add it)
REF_PROMPT = "Hey, are you conscious? Can you talk to me?"
REF_IDS = [1, 18637, 29892, 526, 366, 19861, 29973, 1815, 366, 5193, 304, 592, 29973]
CASES = [REF_PROMPT, "Hello world", "  leading and  double  spaces ", "naïve café — déjà vu",
         "数学 and emoji 🙂", "tab\tand <n> newline-ish", "1234567890 3.14159", "<FLM_FIX_TOKEN_42>x",
         "The quick brown fox jumps over the lazy dog.", "a"]


@pytest.fixture(scope="module")
def vocab():
    return T.Vocab(VOCAB)


def test_oracle_matches_reference_known_answer(vocab):
    assert vocab.meta["bos_token_id"] == "1" and vocab.meta["eos_token_id"] == "2"
    assert [1] + vocab.encode(REF_PROMPT) == REF_IDS
    assert vocab.decode(REF_IDS[1:]) == " " + REF_PROMPT


@pytest.fixture(scope="module")
def cpp(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("tok") / "test_tokenizer")
    r = subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-I", os.path.join(REPO, "include"),
                        os.path.join(REPO, "tests", "cpp", "test_tokenizer.cpp"), "-o", exe],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_cpp_tokenizer_matches_oracle(cpp, vocab):
    r = subprocess.run([cpp, VOCAB], input="\n".join(CASES) + "\n", capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    outs = [json.loads(l) for l in r.stdout.splitlines()]
    assert len(outs) == len(CASES)
    for case, out in zip(CASES, outs):
        assert out["ids"] == vocab.encode(case), case
        assert out["text"] == vocab.decode(out["ids"]), case
    assert [1] + outs[0]["ids"] == REF_IDS
    # plain text round-trips (the reference's decode keeps the blank prefix as a space)
    assert outs[1]["text"] == " Hello world"
    assert outs[8]["text"] == " " + CASES[8]


def test_cpp_tokenizer_rejects_missing_file(cpp):
    r = subprocess.run([cpp, "/nonexistent/tokenizer.bin"], input="x\n", capture_output=True, text=True)
    assert r.returncode != 0 and "cannot open" in r.stderr
