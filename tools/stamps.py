#!/usr/bin/env python3
"""Per-workgroup timeline of one launch of an engine kernel (Llama-2-7B shapes,
ctx 2048): WgStamp records {start, mark1, mark2, end, cu} per workgroup.

    python tools/stamps.py [--kernels attn,o,attn_o,qkv,gate_up,down] [--ctx 2048]

Prints per kernel: span (first start -> last end), dispatch ramp (start
quantiles), workgroup duration quantiles, end quantiles, marks if used.
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

MAXWG = 1 << 15


def q(v):
    return [round(float(x), 2) for x in np.quantile(v, [0, 0.1, 0.5, 0.9, 1.0])]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", default="qkv,attn,o,attn_o,gate_up,down")
    ap.add_argument("--ctx", type=int, default=2048)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--out", default="")
    ap.add_argument("--ring-grid", type=int, default=256, help="workgroups of the ring layer (CUs)")
    ap.add_argument("--preset", default="llama2-7b")
    ap.add_argument("--int8", action="store_true", help="int8 W8A16 weights (config 5)")
    a = ap.parse_args()
    lib = _lib.lib()
    cfg = preset(a.preset, layers=a.layers, max_seq=a.ctx)
    if a.int8:
        import llmi
        cfg.weight_dtype = llmi.I8
    buf = C.c_void_p()
    nbytes = MAXWG * 8 * 8
    assert lib.llmi_device_alloc(C.byref(buf), C.c_size_t(nbytes)) == 0
    res = {}
    with Engine(cfg) as e:
        e.load_synthetic(0)
        e.set_prompt(synth_prompt(0, 8, cfg.vocab))
        e.decode(a.ctx, use_graph=False)
        assert lib.llmi_engine_debug_stamps(e._h, buf) == 0
        host = np.zeros((MAXWG, 8), np.uint64)
        for k in a.kernels.split(","):
            zero = np.zeros((MAXWG, 8), np.uint64)
            lib.llmi_memcpy(buf, zero.ctypes.data_as(C.c_void_p), C.c_size_t(nbytes), 0)
            e.time_kernel(k, 1)
            lib.llmi_memcpy(host.ctypes.data_as(C.c_void_p), buf, C.c_size_t(nbytes), 1)
            rows = host[: a.ring_grid] if k == "ring" else host
            v = rows[rows[:, 0] > 0].astype(np.int64)
            t0 = v[:, 0].min()
            st = (v[:, 0] - t0) / 100.0
            en = (v[:, 3] - t0) / 100.0
            r = {"wgs": int(len(v)), "span_us": round(float(en.max()), 2), "start_q": q(st), "dur_q": q(en - st),
                 "end_q": q(en), "cus": int(len(np.unique(v[:, 4])))}
            for m in (1, 2, 5, 6, 7):
                sel = v[:, m] > 0
                if sel.any():
                    r[f"mark{m}_q"] = q((v[sel, m] - t0) / 100.0)
            if k == "ring":  # per-piece cadence of workgroup 0: {issued, published, consumed}
                nwg = a.ring_grid
                pc = host[nwg:nwg + 1000].reshape(-1)[: 3 * 2000].reshape(-1, 3).astype(np.int64)
                pc = pc[pc[:, 0] > 0]
                if len(pc):
                    rel = (pc - t0) / 100.0
                    r["wg0_pieces"] = len(pc)
                    r["wg0_issue_us"] = [round(float(x), 2) for x in rel[:, 0][::8]]
                    r["wg0_land_minus_issue_q"] = q(rel[:, 1] - rel[:, 0])
                    r["wg0_consume_minus_publish_q"] = q(rel[:, 2] - rel[:, 1])
                    r["wg0_table_us"] = [[round(float(x), 3) for x in row] for row in rel]
            res[k] = r
            print(k, json.dumps(r), flush=True)
        lib.llmi_engine_debug_stamps(e._h, None)
    lib.llmi_device_free(buf)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
