"""Host-side C++ under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only; GPU
sanitizers are not available on this pool): the caching allocator's pool policy
(fake raw backend) and the tokenizer (file parsing, BPE merges, byte fallback,
fix tokens, decode) -- the host code of include/llmi/ that runs no GPU kernel."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
         "-fno-sanitize-recover=all", "-Wall", "-I", os.path.join(REPO, "include")]


def _build(tmp_path, name):
    exe = str(tmp_path / f"{name}_asan")
    r = subprocess.run(FLAGS + [os.path.join(REPO, "tests", "cpp", f"{name}.cpp"), "-o", exe],
                       capture_output=True, text=True)
    if r.returncode != 0 and "libasan" in r.stderr:
        pytest.skip("no ASan runtime in this toolchain")
    assert r.returncode == 0, r.stderr
    return exe


def test_allocator_under_asan_ubsan(tmp_path):
    r = subprocess.run([_build(tmp_path, "test_allocator")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "allocator ok" in r.stdout, (r.stdout, r.stderr)


def test_tokenizer_under_asan_ubsan(tmp_path):
    vocab = os.path.join(REPO, "tests", "golden", "llama2-7b-tokenizer.bin")
    text = "Hey, are you conscious?\nnaïve café 🙂 数学\n<FLM_FIX_TOKEN_42>x\n  a  b \n\n" + "long " * 400 + "\n"
    r = subprocess.run([_build(tmp_path, "test_tokenizer"), vocab], input=text, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    assert len(r.stdout.splitlines()) == 6 and "ERROR" not in r.stderr
