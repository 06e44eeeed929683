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


def _flm(*fields):
    """A minimal .flm vocabulary file: version 0, then the given int32 / float32 fields."""
    import struct
    out = struct.pack("<i", 0)
    for f in fields:
        out += struct.pack("<f", f) if isinstance(f, float) else struct.pack("<i", f)
    return out


@pytest.mark.parametrize("name,data", [
    ("truncated", None),                                   # the real file cut short
    ("negative_id", _flm(1, 1, ord("a"), -5, 0.0)),
    ("huge_count", _flm(0x7FFFFFFF)),
    ("negative_len", _flm(1, -3)),
    ("oversized_len", _flm(1, 1 << 20)),
    ("id_too_large", _flm(1, 1, ord("a"), 1 << 30, 0.0)),
])
def test_tokenizer_rejects_malformed_files_under_asan(tmp_path, name, data):
    """The vocabulary file is external data (Tokenizer::Initialize, tokenizer.h:137-167 in the
    reference reads it unchecked): malformed counts, lengths and ids, and short reads, raise a
    clean error without touching memory out of bounds."""
    f = tmp_path / f"{name}.bin"
    if data is None:
        with open(os.path.join(REPO, "tests", "golden", "llama2-7b-tokenizer.bin"), "rb") as src:
            data = src.read()[:100_000]
    f.write_bytes(data)
    r = subprocess.run([_build(tmp_path, "test_tokenizer"), str(f)], input="hello\n", capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "Tokenizer:" in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
