#!/usr/bin/env python3
"""Same-process A/B of engine options on the bench workload (Llama-2-7B fp16, fp16 KV, 8 prompt
ids, graph-replayed forwards at positions 0..max_seq-1), alternating the variants pass by pass
so box drift hits all of them alike.

    python tools/decode_ab.py --option kpar --values 0,1 [--tp-world 8] [--passes 3] [--layers 32] [--max-seq 2048]

One JSON line per (pass, value): us per token and tok/s (generated tokens as bench.py counts them).
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
    ap.add_argument("--option", default="kpar")
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--tp-world", type=int, default=1, help="> 1: rank 0, exchange looped back (mode --exchange)")
    ap.add_argument("--exchange", type=int, default=1)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--max-seq", type=int, default=2048)
    ap.add_argument("--preset", default="llama2-7b")
    ap.add_argument("--int8", action="store_true")
    ap.add_argument("--fixed", default="", help="options set once for every variant: name=value[,name=value]")
    a = ap.parse_args()
    cfg = preset(a.preset, layers=a.layers, max_seq=a.max_seq, tp_rank=0, tp_world=a.tp_world)
    cfg.kv_dtype = llmi.F16
    if a.int8:
        cfg.weight_dtype = llmi.I8
    vals = [int(v) for v in a.values.split(",")]
    prompt = synth_prompt(0, 8, cfg.vocab)
    with Engine(cfg) as e:
        e.load_synthetic(0)
        for kv in filter(None, a.fixed.split(",")):
            k, v = kv.split("=")
            e.set_option(k, int(v))
        if a.tp_world > 1:
            e.xchg_loopback()
            e.set_exchange(a.exchange)
        toks = {}
        for v in vals:  # capture + warm every variant once
            e.set_option(a.option, v)
            e.set_prompt(prompt)
            e.decode(a.max_seq)
            e.sync()
            toks[v] = e.tokens(a.max_seq + 1)[:64].tolist()
        same = all(toks[v] == toks[vals[0]] for v in vals)
        for p in range(a.passes):
            for v in vals:
                e.set_option(a.option, v)
                e.set_prompt(prompt)
                e.decode(a.max_seq)  # every split count's graph captured outside the timed region
                e.set_prompt(prompt)
                e.sync()
                t0 = time.perf_counter()
                e.decode(a.max_seq)
                e.sync()
                dt = time.perf_counter() - t0
                print(json.dumps({"pass": p, a.option: v, "layers": a.layers, "us_per_token": round(dt / a.max_seq * 1e6, 2),
                                  "tok_s": round((a.max_seq - 8 + 1) / dt, 2), "tokens_equal_first64": same}), flush=True)


if __name__ == "__main__":
    main()
