#!/usr/bin/env python3
"""Stamped timeline of one decode-mode-1 token (graph replay): per ring launch, the phase
marks every workgroup records (ring.hip stamp indices: 0 loader start, 1 o_proj sums
issued, 2 every CU's o_proj arrived, 3 gate_up done, 4 down sums issued, 5 every CU's
down arrived, 6 q/k/v done, 7 loaders drained), relative to the launch's first start, in
us (100 MHz clock). Reports min / median / max over workgroups, averaged over layers,
plus the attention spans and the gaps between launches.

    python tools/ring_timeline.py [--ctx 1024] [--layers 32]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm-inference_amd"))

import llmi  # noqa: E402
from llmi import _lib  # noqa: E402
from llmi.engine import Engine, preset, synth_prompt  # noqa: E402
from llmi.timeline import slot_wgs  # noqa: E402

NAMES = ["loader_start", "o_issued", "o_all_arrived", "gate_up_done", "down_issued", "down_all_arrived",
         "qkv_done", "loader_end"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--max-seq", type=int, default=2048)
    ap.add_argument("--prof", action="store_true",
                    help="the library was built with -DLLMI_RING_PROF=1 (LLMI_LIB_PATH): report wait totals")
    ap.add_argument("--prof2", action="store_true",
                    help="the library was built with -DLLMI_RING_PROF=2: consumer wave 0's O-phase marks")
    a = ap.parse_args()
    cfg = preset("llama2-7b", layers=a.layers, max_seq=a.max_seq)
    cfg.kv_dtype = llmi.F16
    lib = _lib.lib()
    with Engine(cfg) as e:
        e.load_synthetic(0)
        e.set_decode_mode(1)
        e.set_prompt(synth_prompt(0, 8, cfg.vocab))
        stride = slot_wgs(cfg)
        n_slots = 2 * cfg.layers + 2
        nbytes = n_slots * stride * 64
        buf = C.c_void_p()
        _lib.call("llmi_device_alloc", C.byref(buf), C.c_size_t(nbytes))
        try:
            _lib.call("llmi_engine_debug_timeline", e._h, buf, C.c_size_t(nbytes), stride)
            e.decode(a.ctx - 1)
            e.sync()
            _lib.call("llmi_device_memset", buf, 0, C.c_size_t(nbytes))
            e.decode(1)
            e.sync()
            host = np.zeros((n_slots * stride, 8), np.uint64)
            _lib.call("llmi_memcpy", host.ctypes.data_as(C.c_void_p), buf, C.c_size_t(nbytes), 1)
        finally:
            lib.llmi_engine_debug_timeline(e._h, None, C.c_size_t(0), 0)
            lib.llmi_device_free(buf)
    spans = []   # (name, start, end)
    phase = []   # per layer: [8 marks][min, med, max] relative to the ring start
    for s in range(n_slots):
        rows = host[s * stride:(s + 1) * stride].astype(np.int64)
        if s == 0 or s == n_slots - 1 or s % 2 == 1:  # gemv / attention: idx 0 start, idx 3 end
            v = rows[rows[:, 0] > 0]
            if len(v):
                spans.append(("qkv" if s == 0 else "lm_head" if s == n_slots - 1 else "attn", v[:, 0].min(),
                              v[:, 3].max()))
            continue
        if a.prof:  # wait totals per workgroup (ticks), mean over workgroups and layers
            v = rows[:256]
            phase.append(v.mean(axis=0))
            continue
        v = rows[rows[:, 0] > 0]
        if not len(v):
            continue
        t0 = v[:, 0].min()
        spans.append(("ring", t0, v[:, 1:8].max()))
        marks = []
        for i in range(8):
            col = v[:, i]
            col = col[col > 0] - t0
            marks.append([float(np.min(col)), float(np.median(col)), float(np.max(col))] if len(col) else [0, 0, 0])
        phase.append(marks)
    if a.prof2:
        ph = np.array(phase) / 100.0  # [layers][8 marks][min, med, max], us
        names = ["cons_start", "merge_loads_landed", "head_merged", "wo_pieces_done", "atomics_issued",
                 "arrived", "all_arrived", "gathered"]
        m = ph.mean(axis=0)
        print(json.dumps({"ctx": a.ctx, "prof2_us_min_med_max": {k: [round(float(x), 2) for x in m[i]]
                                                                  for i, k in enumerate(names)}}))
        return
    if a.prof:
        m = np.array(phase).mean(axis=0) / 100.0
        names = ["loader0_free_wait", "loader0_land_wait", "loader1_free_wait", "loader1_land_wait",
                 "cons0_full_wait_O", "cons0_full_wait_G", "cons0_full_wait_D", "cons0_full_wait_Q"]
        print(json.dumps({"ctx": a.ctx, "layers": a.layers, "prof_us_mean_per_wg": {k: round(float(x), 2)
                                                                                    for k, x in zip(names, m)}}))
        return
    ph = np.array(phase) / 100.0  # us
    mean = ph.mean(axis=0)
    out = {"ctx": a.ctx, "layers": a.layers, "ring_launches": len(phase),
           "phase_us_min_med_max": {NAMES[i]: [round(x, 2) for x in mean[i]] for i in range(8)}}
    starts = np.array([s[1] for s in spans])
    ends = np.array([s[2] for s in spans])
    gaps = (starts[1:] - ends[:-1]) / 100.0
    for k in ("qkv", "attn", "ring", "lm_head"):
        idx = [i for i, s in enumerate(spans) if s[0] == k]
        if idx:
            out[f"{k}_span_us_mean"] = round(float(np.mean((ends[idx] - starts[idx]) / 100.0)), 2)
    out["gap_us_mean"] = round(float(gaps.mean()), 2)
    out["token_us"] = round(float((ends[-1] - starts[0]) / 100.0), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
