#!/usr/bin/env python3
"""Config 5 kernels: Llama-2-13B-shape int8 (W8A16) engine, each decode kernel
timed with layers cycled (weights from HBM), plus a short graph decode loop."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm-inference_amd"))

import llmi  # noqa: E402
from llmi.engine import Engine, preset, synth_prompt  # noqa: E402


def main():
    layers = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    wdt = llmi.I8 if (len(sys.argv) < 3 or sys.argv[2] == "i8") else llmi.F16
    cfg = preset("llama2-13b", layers=layers, max_seq=512)
    cfg.weight_dtype = wdt
    out = {"lib": os.environ.get("LLMI_LIB_PATH", "default"), "layers": layers, "wdt": int(wdt)}
    with Engine(cfg) as e:
        e.load_synthetic(0)
        p = synth_prompt(0, 8, cfg.vocab)
        eager = len(sys.argv) > 3 and sys.argv[3] == "eager"  # rocprofv3 cannot trace graph replays
        e.generate(p, 64, use_graph=not eager)
        if not eager:
            e.set_prompt(p)
            e.sync()
            t0 = time.perf_counter()
            e.decode(256)
            e.sync()
            out["loop_us_per_token"] = round((time.perf_counter() - t0) / 256 * 1e6, 1)
        for k in ("qkv", "attn", "o", "gate_up", "down", "lm_head"):
            us, b = e.time_kernel(k, 64)
            out[k] = {"us": round(us, 2), "GBps": round(b / us / 1e3, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
