#!/usr/bin/env python3
"""Price one tensor-parallel rank of Llama-2-7B on ONE GPU.

    python tools/tp_loopback_probe.py [--worlds 2,4,8] [--modes 0,1,2] [--max-seq 2048] [--layers 32]

For each TP degree W: an engine holding rank 0's real 1/W shard (32 layers, fp16, fp16 KV),
its exchange looped back onto its own inbox (llmi_engine_xchg_loopback: the push writes the
same W x 32 KB a real push writes, the flags of all W ranks are raised locally, the reduce
sums W slots), then the bench workload -- 8 prompt ids, graph-replayed forwards at positions
0..max_seq-1 -- timed per exchange mode:
  0: no exchange at all (the compute-only floor of a rank),
  1: one-shot exchange launches (2 L + 1 per token),
  2: the exchange fused into the o_proj / down / lm_head launches.
No xGMI latency is in these numbers (the writes stay in local HBM): they are the per-rank
launch structure's cost, a lower bound for a real W-GPU rank. One JSON line per (W, mode).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm-inference_amd"))

from llmi.engine import Engine, preset, synth_prompt  # noqa: E402
import llmi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--modes", default="0,1,2")
    ap.add_argument("--max-seq", type=int, default=2048)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--decode-mode", type=int, default=0)
    ap.add_argument("--eager", action="store_true", help="launch eagerly (rocprofv3 kernel traces of graph "
                                                          "replays crash on ROCm 7.2)")
    args = ap.parse_args()
    for W in [int(w) for w in args.worlds.split(",")]:
        cfg = preset("llama2-7b", max_seq=args.max_seq, layers=args.layers, tp_rank=0, tp_world=W)
        cfg.kv_dtype = llmi.F16
        with Engine(cfg, device=0) as e:
            e.load_synthetic(0)
            if W > 1:
                e.xchg_loopback()
            if args.decode_mode:
                e.set_decode_mode(args.decode_mode)
            prompt = synth_prompt(0, 8, cfg.vocab)
            wbytes, _ = e.bytes_per_token()
            for mode in ([int(m) for m in args.modes.split(",")] if W > 1 else [0]):
                if W > 1:
                    e.set_exchange(mode)
                best = None
                for rep in range(args.reps + 1):  # first pass: capture + warm-up
                    e.set_prompt(prompt)
                    e.sync()
                    t0 = time.perf_counter()
                    e.decode(args.max_seq, use_graph=not args.eager)
                    e.sync()
                    dt = time.perf_counter() - t0
                    if rep > 0:
                        best = dt if best is None else min(best, dt)
                us_tok = best / args.max_seq * 1e6
                print(json.dumps({"tp_world": W, "exchange_mode": mode, "decode_mode": args.decode_mode, "graph": not args.eager,
                                  "layers": args.layers, "max_seq": args.max_seq,
                                  "us_per_token_per_rank": round(us_tok, 2),
                                  "us_per_layer": round(us_tok / args.layers, 2),
                                  "weight_bytes_per_token_per_rank": wbytes,
                                  "weight_GBps": round(wbytes / (us_tok * 1e-6) / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
