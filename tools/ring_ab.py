#!/usr/bin/env python3
"""Decode mode 0 (five launches per layer) vs mode 1 (attention + persistent ring layer)
on the bench workload: Llama-2-7B fp16, fp16 KV, 8-token prompt, graph-replayed decode to
2048 positions. Prints one JSON line per mode (tokens/s, us/token, the ring launch's
HIP-event time when mode 1) and whether the two modes generated the same tokens.

    python tools/ring_ab.py [--max-seq 2048] [--reps 2] [--layers 32]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm-inference_amd"))

import llmi  # noqa: E402
from llmi.engine import Engine, preset, synth_prompt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-seq", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--modes", default="0,1")
    a = ap.parse_args()
    cfg = preset("llama2-7b", layers=a.layers, max_seq=a.max_seq)
    cfg.kv_dtype = llmi.F16
    prompt = synth_prompt(0, 8, cfg.vocab)
    toks = {}
    with Engine(cfg) as e:
        e.load_synthetic(0)
        for mode in [int(m) for m in a.modes.split(",")]:
            e.set_decode_mode(mode)
            e.set_prompt(prompt)
            e.decode(a.max_seq)  # graph capture + warm
            e.sync()
            best = None
            for _ in range(a.reps):
                e.set_prompt(prompt)
                e.sync()
                t0 = time.perf_counter()
                e.decode(a.max_seq)
                e.sync()
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            toks[mode] = e.tokens(a.max_seq + 1)
            out = {"mode": mode, "layers": a.layers, "forwards": a.max_seq,
                   "tokens_per_s": round((a.max_seq - 7) / best, 2),
                   "us_per_forward": round(best / a.max_seq * 1e6, 2)}
            kern = ("ring", "attn") if mode == 1 else ("o", "gate_up", "down", "qkv", "attn")
            for k in kern:
                us, b = e.time_kernel(k, iters=64)
                out[f"{k}_us"] = round(us, 2)
                out[f"{k}_GBps"] = round(b / (us * 1e-6) / 1e9, 1)
            print(json.dumps(out), flush=True)
    if len(toks) == 2:
        t0, t1 = toks[0], toks[1]
        same = int((t0 == t1).sum())
        print(json.dumps({"tokens_equal": bool((t0 == t1).all()), "equal_count": same, "n": int(len(t0))}), flush=True)


if __name__ == "__main__":
    main()
