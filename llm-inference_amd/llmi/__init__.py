"""llmi: MI355X-native Llama-2 decode engine (host-side Python handle).

The compute lives in libllmi.so (HIP kernels for gfx950 + C ABI,
include/llmi.h). `llmi.engine.Engine` drives the native decode loop;
`llmi.ops` exposes the per-launcher operator API on torch device tensors.
"""
from ._lib import F16, F32, I8, I32, Config, LlmiError, lib  # noqa: F401

__all__ = ["lib", "Config", "LlmiError", "F16", "F32", "I8", "I32"]
