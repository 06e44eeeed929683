#!/usr/bin/env python3
"""Time the batched prefill (config 3: Llama-2-7B, 512 prompt rows) on one GPU,
both GEMM precisions, and print JSON (ms, TFLOP/s on the algorithmic FLOPs).
    python tools/prefill_probe.py [rows] [iters] [exact|exact8|fast]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm-inference_amd"))

from llmi.engine import Engine, preset, synth_prompt  # noqa: E402


def prefill_flops(cfg, m):
    lin = cfg.hidden * ((cfg.heads + 2 * cfg.kv_heads) * cfg.head_dim) + cfg.hidden * cfg.hidden \
        + 3 * cfg.hidden * cfg.inter
    attn = 2 * 2 * cfg.heads * cfg.head_dim * (m * (m + 1) // 2)
    return cfg.layers * (2 * m * lin + attn) + 2 * cfg.hidden * cfg.vocab


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    modes = {"exact": (1,), "exact8": (2,), "fast": (0,)}.get(sys.argv[3] if len(sys.argv) > 3 else "", (1, 2, 0))
    cfg = preset("llama2-7b", max_seq=m + 64)
    prompt = synth_prompt(1, m, cfg.vocab)
    out = {"m": m, "flops": prefill_flops(cfg, m)}
    with Engine(cfg) as e:
        e.load_synthetic(0)
        for exact in modes:
            ts = []
            for i in range(iters + 1):
                e.set_prompt(prompt)
                e.sync()
                t0 = time.perf_counter()
                e.prefill(m, exact)
                e.sync()
                ts.append(time.perf_counter() - t0)
            ms = 1e3 * min(ts[1:])
            key = {1: "exact", 2: "exact8", 0: "fast"}[exact]
            out[key] = {"ms": ms, "tflops": out["flops"] / (ms * 1e-3) / 1e12, "token": int(e.tokens()[m])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
