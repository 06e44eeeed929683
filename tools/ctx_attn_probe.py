#!/usr/bin/env python3
"""HIP-event timing of llmi_context_attention alone (the fused context-attention core) at
7B heads: ragged lens 200/150/100/62 and one 512-row sequence, fp32 and fp16 caches.
LLMI_LIB_PATH selects a library variant. Prints one JSON line.

    python tools/ctx_attn_probe.py [--iters 50]
"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm-inference_amd"))

from llmi import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    heads, d = 32, 128
    out = {"lib": os.environ.get("LLMI_LIB_PATH", "default")}
    g = torch.Generator(device="cuda").manual_seed(0)
    for lens in ([200, 150, 100, 62], [512]):
        b, mq = len(lens), max(lens)
        q = torch.randn(b, heads, mq, d, device="cuda", generator=g)
        res = torch.empty(sum(lens), heads * d, device="cuda")
        hist = torch.zeros(b, dtype=torch.int32, device="cuda")
        ql = torch.tensor(lens, dtype=torch.int32, device="cuda")
        for dt, code in ((torch.float32, 0), (torch.float16, 1)):
            kc = torch.randn(1, b, heads, mq, d, device="cuda", generator=g).to(dt)
            vc = torch.randn(1, b, heads, mq, d, device="cuda", generator=g).to(dt)
            st = torch.cuda.current_stream().cuda_stream

            def run():
                _lib.call("llmi_context_attention", C.c_void_p(q.data_ptr()), C.c_void_p(kc.data_ptr()),
                          C.c_void_p(vc.data_ptr()), code, 0, C.c_void_p(hist.data_ptr()),
                          C.c_void_p(ql.data_ptr()), b, heads, heads, mq, mq, d, C.c_float(d ** -0.5),
                          C.c_void_p(res.data_ptr()), C.c_void_p(st))
            for _ in range(5):
                run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            out[f"us_{'x'.join(map(str, lens))}_{'f32' if code == 0 else 'f16'}"] = round(
                e0.elapsed_time(e1) / a.iters * 1e3, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
