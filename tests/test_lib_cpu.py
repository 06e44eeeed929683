"""CPU-side checks of the C ABI (no GPU needed): the library loads, exports
every symbol include/llmi.h declares, the host twin of the synthetic-weight
generator is bit-identical to the numpy oracle PRNG, and argument errors come
back as codes + messages (LLM_CHECK convention)."""
import ctypes as C

import numpy as np
import pytest

from llmi import _lib
from llmi._lib import call, lib
from llmi.engine import preset, synth_prompt
from oracle import prng


def test_library_exports_every_header_symbol():
    L = lib()
    names = _lib.header_functions()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(names) == set(_lib._SIGS), set(names) ^ set(_lib._SIGS)


def _host_fill(kind, dtype, seed, tid, rows, cols, row0=0, col0=0, ld=0):
    out = np.zeros((rows, cols), dtype)
    dt = {np.float16: _lib.F16, np.float32: _lib.F32, np.int8: _lib.I8}[dtype]
    call("llmi_synth_fill_host", out.ctypes.data, dt, kind, seed, tid, rows, cols, row0, col0, ld)
    return out


@pytest.mark.parametrize("seed", [0, 7, 2**40 + 3])
def test_host_generator_matches_numpy_prng(seed):
    tid = prng.layer_tid(3, prng.KIND_GATE)
    a = _host_fill(_lib.SYN_LINEAR, np.float16, seed, tid, 64, 96, 5, 17, 4096)
    b = prng.linear_fp16(seed, tid, 64, 96, 5, 17, 4096)
    np.testing.assert_array_equal(a.view(np.uint16), b.view(np.uint16))
    a32 = _host_fill(_lib.SYN_LINEAR, np.float32, seed, tid, 64, 96, 5, 17, 4096)
    np.testing.assert_array_equal(a32, b.astype(np.float32))
    e = _host_fill(_lib.SYN_EMBED, np.float16, seed, prng.GLOBAL_EMBED, 8, 512)
    np.testing.assert_array_equal(e.view(np.uint16), prng.embed_fp16(seed, prng.GLOBAL_EMBED, 8, 512).view(np.uint16))
    g = _host_fill(_lib.SYN_GAMMA, np.float16, seed, tid, 1, 4096, 0, 0, 4096)
    np.testing.assert_array_equal(g[0].view(np.uint16), prng.gamma_fp16(seed, tid, 4096).view(np.uint16))
    q = _host_fill(_lib.SYN_INT8, np.int8, seed, tid, 16, 64, 3, 32, 5120)
    np.testing.assert_array_equal(q, prng.int8_weight(seed, tid, 16, 64, 3, 32, 5120))
    s = _host_fill(_lib.SYN_INT8_SCALE, np.float16, seed, tid, 40, 1, 9, 0, 1)
    np.testing.assert_array_equal(s[:, 0].view(np.uint16), prng.int8_row_scale(seed, tid, 40, 9).view(np.uint16))


def test_prompt_ids_match():
    np.testing.assert_array_equal(synth_prompt(13, 8, 32000), prng.prompt_ids(13, 8, 32000))


def test_presets():
    c = preset("llama2-7b")
    assert (c.hidden, c.heads, c.kv_heads, c.head_dim, c.inter, c.layers, c.vocab) == \
        (4096, 32, 32, 128, 11008, 32, 32000)
    assert abs(c.rms_eps - 1e-5) < 1e-12 and c.rope_base == 10000.0
    c13 = preset("llama2-13b")
    assert (c13.hidden, c13.heads, c13.inter, c13.layers) == (5120, 40, 13824, 40)
    with pytest.raises(_lib.LlmiError, match="unknown name"):
        preset("gpt-2")


def test_errors_are_codes_with_messages():
    L = lib()
    rc = L.llmi_linear(None, None, _lib.F16, None, None, 0, 1, 1, None)
    assert rc == -1
    assert "[llmi][ERROR]" in L.llmi_last_error().decode()
    rc = L.llmi_synth_fill_host(None, _lib.F32, _lib.SYN_INT8, 0, 0, 1, 1, 0, 0, 0)
    assert rc == -1 and b"int8" in L.llmi_last_error()
    x = C.c_void_p(16)  # never dereferenced: the checks come first
    rc = L.llmi_linear_fused(x, x, _lib.F16, None, x, 8, 64, None, _lib.F16, 1e-5, 3, None, None)
    assert rc == -1 and b"epilogue" in L.llmi_last_error()
    rc = L.llmi_linear_fused(x, x, _lib.F16, None, x, 8, 64, None, _lib.F16, 1e-5, 1, x, None)
    assert rc == -1 and b"resid != y" in L.llmi_last_error()
    cfg = preset("tiny", tp_world=3)
    h = C.c_void_p()
    rc = L.llmi_engine_create(C.byref(cfg), 0, None, C.byref(h))
    assert rc == -1 and b"divide by tp_world" in L.llmi_last_error()
