#!/usr/bin/env python3
"""One-device rehearsal of tensor-parallel decode's launch structure: the in-process group
(llmi_group_*: W rank engines stepped phase by phase on one stream) at Llama-2-7B width,
graph-replayed greedy decode, per exchange form:
  mode 0  in-place reduction kernel (1 launch per exchange for the whole group),
  mode 1  one-shot peer exchange as launches (W pushes + W reduces per exchange),
  mode 2  the push fused into every rank's o_proj / down / lm_head tail (W reduces).
All W ranks run on the SAME GPU one after another, so the time per token is the sum of
every rank's kernels: it shows what the exchange launches cost, not a scaling number.

    python tools/group_tp_probe.py [--layers 8] [--worlds 2,4,8] [--tokens 64]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm-inference_amd"))

import llmi  # noqa: E402
from llmi.engine import TPGroup, preset, synth_prompt  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--tokens", type=int, default=64)
    a = ap.parse_args()
    for w in [int(x) for x in a.worlds.split(",")]:
        cfg = preset("llama2-7b", layers=a.layers, max_seq=a.tokens + 16)
        cfg.kv_dtype = llmi.F16
        prompt = synth_prompt(0, 8, cfg.vocab)
        out = {"world": w, "layers": a.layers, "forwards": a.tokens}
        toks = {}
        with TPGroup(cfg, w) as g:
            g.load_synthetic(0)
            for mode in (0, 1, 2, 0, 1, 2):
                g.set_exchange(mode)
                g.generate(prompt, 8)  # graph capture + warm
                best = out.get(f"us_per_forward_mode{mode}", 1e30)
                t0 = time.perf_counter()
                t = g.generate(prompt, a.tokens - 7)
                dt = (time.perf_counter() - t0) / a.tokens * 1e6
                out[f"us_per_forward_mode{mode}"] = round(min(best, dt), 2)
                toks[mode] = t
        out["tokens_equal_across_modes"] = bool((toks[0] == toks[1]).all() and (toks[0] == toks[2]).all())
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
