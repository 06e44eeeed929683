#!/usr/bin/env python3
"""Run a few short decodes with whichever libllmi.so LLMI_LIB_PATH selects and save tokens,
logits and the final hidden state, so two builds can be compared bit for bit:
    LLMI_LIB_PATH=... python tools/lib_bitwise.py out_a.npz
    python tools/lib_bitwise.py out_b.npz
    python tools/lib_bitwise.py --compare out_a.npz out_b.npz"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm-inference_amd"))


def run(out):
    import llmi
    from llmi.engine import Engine, preset, synth_prompt
    res = {}
    cases = [("7b2", preset("llama2-7b", layers=2, max_seq=200), llmi.F16, llmi.F16),
             ("13b_i8", preset("llama2-13b", layers=2, max_seq=200), llmi.I8, llmi.F16),
             ("7b2_f32kv", preset("llama2-7b", layers=2, max_seq=200), llmi.F16, llmi.F32)]
    for name, cfg, wdt, kv in cases:
        cfg.weight_dtype, cfg.kv_dtype = wdt, kv
        with Engine(cfg) as e:
            e.load_synthetic(7)
            toks = e.generate(synth_prompt(3, 8, cfg.vocab), 150)  # ctx 158: three split counts
            res[name + "_tokens"], res[name + "_logits"], res[name + "_hidden"] = toks, e.logits(), e.hidden()
    np.savez(out, **res)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = [k for k in A.files if not np.array_equal(A[k], B[k])]
    print("bitwise equal" if not bad else "DIFFER: " + ", ".join(bad))
    return not bad


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    run(sys.argv[1])
