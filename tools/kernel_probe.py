#!/usr/bin/env python3
"""Launch the engine's hot kernels in isolation (eager, HIP-event timed) on the
Llama-2-7B shapes -- the target of the rocprofv3 --pmc passes (profiles/).

    python tools/kernel_probe.py [--layers 2] [--iters 20] [--kernels gate_up,qkv,...]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm-inference_amd"))

from llmi.engine import Engine, preset, synth_prompt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--ctx", type=int, default=2048)
    ap.add_argument("--kernels", default="qkv,attn,o,gate_up,down,lm_head")
    ap.add_argument("--loop", action="store_true", help="also time a graph-replayed decode loop")
    ap.add_argument("--attn-sweep", default="", help="comma list of ctx values to time attention at")
    ap.add_argument("--prefill", action="store_true",
                    help="reach ctx with one batched prefill instead of ctx eager decode steps (few dispatches: "
                         "for rocprofv3 --pmc passes)")
    a = ap.parse_args()
    cfg = preset("llama2-7b", layers=a.layers, max_seq=a.ctx)
    with Engine(cfg) as e:
        e.load_synthetic(0)
        if a.prefill:
            e.set_prompt(synth_prompt(0, a.ctx, cfg.vocab))
            e.prefill(a.ctx)  # leaves cur_pos = ctx - 1: attention runs at full ctx
        else:
            e.set_prompt(synth_prompt(0, 8, cfg.vocab))
            e.decode(a.ctx, use_graph=False)  # leaves cur_pos = ctx - 1: attention runs at full ctx
        out = {"lib": os.environ.get("LLMI_LIB_PATH", "default")}
        if a.loop:
            import time
            e.set_prompt(synth_prompt(0, 8, cfg.vocab))
            e.decode(a.ctx)  # graph build + warm
            e.sync()
            e.set_prompt(synth_prompt(0, 8, cfg.vocab))
            t0 = time.perf_counter()
            e.decode(a.ctx)
            e.sync()
            dt = time.perf_counter() - t0
            out["loop_us_per_token"] = round(dt / a.ctx * 1e6, 2)
            out["loop_layers"] = a.layers
            e.set_prompt(synth_prompt(0, 8, cfg.vocab))
            e.decode(a.ctx, use_graph=False)
        if a.attn_sweep:
            e.set_prompt(synth_prompt(0, 8, cfg.vocab))
            done, sweep = 0, {}
            for c in [int(v) for v in a.attn_sweep.split(",")]:
                e.decode(c - done)
                done = c
                sweep[c] = e.time_kernel("attn", a.iters)[0]
            out["attn_us_by_ctx"] = sweep
            e.set_prompt(synth_prompt(0, 8, cfg.vocab))
            e.decode(a.ctx, use_graph=False)
        for k in a.kernels.split(","):
            us, b = e.time_kernel(k, a.iters)
            out[k] = {"avg_us": round(us, 2), "bytes": b, "GBps": round(b / us / 1e3, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
