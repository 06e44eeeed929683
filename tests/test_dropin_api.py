"""Drop-in boundary at the layer and model level: the
reference's call syntax and its user_entry.cpp compile against include/llmi/*.h,
and Llama<T>::Response (tokenize -> one batched prefill -> graph decode) gives the
token-by-token decode path's tokens.

The reference's user_entry.cpp is read from /root/reference at test time (this
container only; nothing of it is committed) and built with only its two src/
includes replaced by "llmi/model.h"."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(REPO, "llm-inference_amd", "lib")
VOCAB = os.path.join(REPO, "tests", "golden", "llama2-7b-tokenizer.bin")
REF_ENTRY = "/root/reference/user_entry.cpp"


def _build(src, out):
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-I", os.path.join(REPO, "include"), src, "-L", LIBDIR, "-lllmi",
           f"-Wl,-rpath,{LIBDIR}", "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return out


@pytest.mark.skipif(not os.path.exists(REF_ENTRY), reason="the reference checkout is only in the build container")
def test_reference_user_entry_compiles_with_include_edits_only(tmp_path):
    src = open(REF_ENTRY, encoding="utf-8").read()
    old = '#include "src/utils/model_utils.h"\n#include "src/models/basemodel.h"'
    assert old in src
    edited = tmp_path / "user_entry.cpp"
    edited.write_text(src.replace(old, '#include "llmi/model.h"'), encoding="utf-8")
    _build(str(edited), str(tmp_path / "user_entry"))


def test_reference_call_syntax_compiles(tmp_path):
    exe = _build(os.path.join(REPO, "tests", "cpp", "test_dropin.cpp"), str(tmp_path / "test_dropin"))
    assert subprocess.run([exe], timeout=60).returncode == 0


@pytest.mark.gpu
def test_llama_response_prefill_equals_decode_path(tmp_path):
    exe = _build(os.path.join(REPO, "tests", "cpp", "test_dropin.cpp"), str(tmp_path / "test_dropin"))
    r = subprocess.run([exe, VOCAB], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, (r.stdout, r.stderr)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    # llama.cpp:382's ids: BOS + the tokenizer's encoding of the reference's query
    assert out["prompt"] == [1, 18637, 29892, 526, 366, 19861, 29973, 1815, 366, 5193, 304, 592, 29973]
    assert len(out["prefill_tokens"]) == 24 and out["prefill_tokens"] == out["decode_tokens"]
    assert out["pieces"] == 24 and out["answer_matches_pieces"] and out["answer_matches_decode"]


@pytest.mark.gpu
def test_user_entry_example_chats(tmp_path):
    """examples/user_entry.cpp: CreateDummyLLMModel<float> (the reference's dummy geometry:
    7B widths, 3 layers, 64 positions), two rounds of MakeInput -> Response -> MakeHistory."""
    exe = _build(os.path.join(REPO, "examples", "user_entry.cpp"), str(tmp_path / "user_entry"))
    r = subprocess.run([exe, VOCAB], input="Hey, are you conscious?\nCan you talk to me?\nexit\n",
                       capture_output=True, text=True, timeout=300)
    print(r.stdout[-2000:])
    assert r.returncode == 0, r.stderr
    assert r.stdout.count("llama:") == 2 and r.stdout.count("please input the question") == 3
