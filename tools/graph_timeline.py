#!/usr/bin/env python3
"""Timeline of ONE graph-replayed decode token (rocprofv3 cannot trace graph replays on
this image: profiles/r02_graph_trace_segfault.log). Every stamped launch of the captured
step writes {start, end, CU} per workgroup into its own region (llmi_engine_debug_timeline,
s_memrealtime at 100 MHz), so the replay itself reports each kernel's span (first
workgroup start -> last workgroup end) and the gap to the next kernel's first workgroup --
the in-graph kernel boundary that the eager traces can only infer.

    python tools/graph_timeline.py [--ctx 8,512,1024,2047] [--layers 32] [--out f.json]

Launch order per token: step_start (unstamped), then per layer qkv, attn, o, gate_up,
down, then lm_head.
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm-inference_amd"))
from llmi import _lib  # noqa: E402
from llmi.engine import Engine, preset, synth_prompt  # noqa: E402
from llmi.timeline import analyse, slot_wgs  # noqa: E402

def wg_detail(host, stride, layer):
    """Per-workgroup start / end (us from the launch's first start), the XCD (blockIdx % 8,
    round-robin dispatch) and the hardware CU id, for layer `layer`'s q/k/v, o and down, plus
    per-XCD completion quantiles: where a launch's tail comes from."""
    out = {}
    for k, off in (("qkv", 0), ("attn", 1), ("o", 2), ("down", 4), ("qkv_attn_part", 0)):
        s = 5 * layer + off
        rows = host[s * stride:(s + 1) * stride].astype(np.int64)
        sel = rows[:, 0] > 0
        if off == 0:  # the fused q/k/v + attention launch: its attention blocks set mark 1
            sel &= (rows[:, 1] > 0) if k == "qkv_attn_part" else (rows[:, 1] == 0)
        idx = np.nonzero(sel)[0]
        if not len(idx):
            continue
        v = rows[idx]
        t0 = rows[rows[:, 0] > 0][:, 0].min()  # the launch's first start (fused: either part)
        start, end = (v[:, 0] - t0) / 100.0, (v[:, 3] - t0) / 100.0
        xcd = idx % 8
        per_xcd = {}
        for x in range(8):
            e = end[xcd == x]
            if len(e):
                per_xcd[str(x)] = [round(float(q), 2) for q in np.quantile(e, [0, 0.5, 0.9, 1.0])]
        out[k] = {"n": int(len(idx)), "end_quantiles_us": [round(float(q), 2) for q in
                                                            np.quantile(end, [0, 0.1, 0.5, 0.9, 0.99, 1.0])],
                  "start_max_us": round(float(start.max()), 2),
                  # kernel-defined marks (attention: [1] q rotated + K/V rows in registers,
                  # [2] P V done), quantiles [min, p50, max] in us from the launch's first start
                  "mark_quantiles_us": {str(m): [round(float(q), 2) for q in np.quantile((v[v[:, m] > 0, m] - t0) / 100.0,
                                                                                       [0, 0.5, 1.0])]
                                        for m in (1, 2) if (v[:, m] > 0).any()},
                  "end_quantiles_by_xcd_us [min, p50, p90, max]": per_xcd,
                  "wg": [[int(i), round(float(a), 2), round(float(b), 2), int(r[4])]
                         for i, a, b, r in zip(idx, start, end, v)]}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", default="8,512,1024,2047")
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--preset", default="llama2-7b")
    ap.add_argument("--out", default="")
    ap.add_argument("--tp-world", type=int, default=1,
                    help="> 1: rank 0 of that TP degree, exchange looped back (llmi_engine_xchg_loopback)")
    ap.add_argument("--exchange", type=int, default=0, help="with --tp-world: exchange mode 0 / 1 / 2")
    ap.add_argument("--wg-layer", type=int, default=-1,
                    help="also dump layer L's per-workgroup {start, end, xcd, cu} for q/k/v, o and down, "
                         "with completion quantiles per XCD (VERDICT r04 item 3a)")
    ap.add_argument("--set", default="", help="engine options name=value[,name=value] (llmi_engine_set_option)")
    a = ap.parse_args()
    lib = _lib.lib()
    cfg = preset(a.preset, layers=a.layers, max_seq=2048, tp_rank=0, tp_world=a.tp_world)
    n_slots = 5 * a.layers + 1
    stride = slot_wgs(cfg)
    nbytes = n_slots * stride * 64
    buf = C.c_void_p()
    assert lib.llmi_device_alloc(C.byref(buf), C.c_size_t(nbytes)) == 0
    host = np.zeros((n_slots * stride, 8), np.uint64)
    res = {"preset": a.preset, "layers": a.layers, "slot_wgs": stride, "clock": "s_memrealtime 100 MHz",
           "mode": "hipGraph replay (one captured graph per active split count)", "ctx": {}}
    with Engine(cfg) as e:
        e.load_synthetic(0)
        for kv in filter(None, a.set.split(",")):
            k, v = kv.split("=")
            e.set_option(k, int(v))
        if a.tp_world > 1:
            e.xchg_loopback()
            e.set_exchange(a.exchange)
        e.set_prompt(synth_prompt(0, 8, cfg.vocab))
        _lib.call("llmi_engine_debug_timeline", e._h, buf, C.c_size_t(nbytes), stride)
        pos = 0
        for c in sorted(int(x) for x in a.ctx.split(",")):
            if c - 1 > pos:
                e.decode(c - 1 - pos)  # graph replays up to the position before the stamped one
                pos = c - 1
            e.sync()
            lib.llmi_device_memset(buf, 0, C.c_size_t(nbytes))
            e.decode(1)  # the stamped replay: position c - 1, context c
            pos += 1
            e.sync()
            lib.llmi_memcpy(host.ctypes.data_as(C.c_void_p), buf, C.c_size_t(nbytes), 1)
            r = analyse(host, n_slots, stride, a.layers)
            if a.wg_layer >= 0:
                r["workgroups"] = wg_detail(host, stride, a.wg_layer)
            res["ctx"][str(c)] = r
            print(c, json.dumps(r), flush=True)
        lib.llmi_engine_debug_timeline(e._h, None, C.c_size_t(0), 0)
    lib.llmi_device_free(buf)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
