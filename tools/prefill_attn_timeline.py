#!/usr/bin/env python3
"""Per-workgroup timeline of the transposed prefill attention kernel (diagnostics).

Runs one 7B prefill of `rows` prompt rows with llmi_debug_prefill_stamps on: the last
layer's launch leaves, per workgroup, [start, first block landed, loop end, end, smid,
query block | head << 16, key blocks] (100 MHz s_memrealtime ticks). Prints one JSON line:
the kernel span, the spread of starts, and per query block (= key blocks on the critical
path) the mean prologue / loop / epilogue times in us.
    python tools/prefill_attn_timeline.py [rows] [exact]"""
import collections
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm-inference_amd"))

import torch  # noqa: E402

from llmi import _lib  # noqa: E402
from llmi.engine import Engine, preset, synth_prompt  # noqa: E402


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    exact = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    cfg = preset("llama2-7b", max_seq=m + 64)
    prompt = synth_prompt(1, m, cfg.vocab)
    buf = torch.zeros(8 * 4096, dtype=torch.int64, device="cuda")
    with Engine(cfg) as e:
        e.load_synthetic(0)
        e.set_prompt(prompt)
        e.prefill(m, exact)  # warm
        e.sync()
        buf.zero_()
        torch.cuda.synchronize()
        _lib.check(_lib.lib().llmi_debug_prefill_stamps(ctypes.c_void_p(buf.data_ptr())), "stamps")
        e.set_prompt(prompt)
        e.prefill(m, exact)
        e.sync()
        _lib.check(_lib.lib().llmi_debug_prefill_stamps(None), "stamps")
    st = buf.view(-1, 8).cpu().numpy()
    st = st[st[:, 0] != 0]
    t0 = st[:, 0].min()
    us = lambda x: float(x) / 100.0  # noqa: E731  (100 MHz ticks -> us)
    by_qb = collections.defaultdict(list)
    for r in st:
        by_qb[int(r[5]) & 0xFFFF].append(r)
    rows = {}
    for qb, rs in sorted(by_qb.items()):
        n = len(rs)
        rows[qb] = {"wgs": n, "key_blocks": int(rs[0][6]),
                    "start": round(sum(us(r[0] - t0) for r in rs) / n, 2),
                    "prologue": round(sum(us(r[1] - r[0]) for r in rs) / n, 2),
                    "loop": round(sum(us(r[2] - r[1]) for r in rs) / n, 2),
                    "epilogue": round(sum(us(r[3] - r[2]) for r in rs) / n, 2),
                    "end_max": round(max(us(r[3] - t0) for r in rs), 2)}
    out = {"rows": m, "exact": exact, "workgroups": int(len(st)),
           "span_us": round(us(st[:, 3].max() - t0), 2),
           "start_spread_us": round(us(st[:, 0].max() - t0), 2),
           "distinct_cus": int(len(set(int(x) for x in st[:, 4]))),
           "per_query_block": rows}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
