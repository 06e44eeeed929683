#!/usr/bin/env python3
"""Build profiles/pmc_traffic.json (read by bench.py) from the rocprofv3 --pmc
FETCH_SIZE / WRITE_SIZE counter CSVs of tools/kernel_probe.py, with the gfx950
correction of MI355X_MICROARCH.md §HBM (FETCH_SIZE x2; both in KB).

    python tools/make_traffic.py <fetch.csv> <write.csv> <tag> [i8]
(7B fp16 kernels from tools/kernel_probe.py, 13B int8 ones -- i8_* -- from tools/int8_probe.py)
"""
import collections
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# attention at ctx 2048 (kernel_probe --ctx 2048): 2 * 2048 * 32 * 128 * 2 B of K/V + the new slot
ALG = {"qkv": 100663296, "gate_up": 180355072, "down": 90177536, "lm_head": 262144000, "attn": 33570816,
       "o": 33554432, "qkv_attn": 100663296 + 33570816,
       # config 5 (tools/int8_probe.py, Llama-2-13B shape): int8 weights + fp16 row scales
       "i8_qkv": 15360 * 5120 + 15360 * 2, "i8_o": 5120 * 5120 + 5120 * 2,
       "i8_gate_up": 27648 * 5120 + 27648 * 2, "i8_down": 5120 * 13824 + 5120 * 2}


def role(name):
    for epi, r in ((", 2, 0,", "i8_qkv"), (", 2, 2,", "i8_gate_up"), (", 2, 4,", "i8_down")):
        if "gemv_kernel<signed char" in name and epi in name:
            return r
    if "attn_oproj_kernel<signed char" in name:
        return "i8_o"
    if "gemv_kernel<__half, 2, 2," in name:
        return "gate_up"
    if "gemv_kernel<__half, 2, 0," in name:
        return "qkv"
    if "gemv_kernel<__half, 2, 3," in name:
        return "lm_head"
    if "gemv_kernel<__half, 2, 4," in name:
        return "down"
    if "attn_decode_kernel<__half>" in name or "attn_decode_kernel<__half, " in name:
        return "attn"
    if "attn_oproj_kernel<__half" in name or "attn_oproj2_kernel<__half" in name:
        return "o"
    if "qkv_attn_kernel<__half, __half, 4, 4, __half, false>" in name:
        return "qkv_attn"
    return None


def per_role(path, counter):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row.get("Counter_Name") == counter and role(row["Kernel_Name"]):
            acc[role(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    fetch_csv, write_csv, tag = sys.argv[1:4]
    i8 = len(sys.argv) > 4 and sys.argv[4] == "i8"  # the int8 probe: keep only its i8_* kernels
    out_path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    old = json.load(open(out_path)) if os.path.exists(out_path) else {"kernels": {}}
    fetch, write = per_role(fetch_csv, "FETCH_SIZE"), per_role(write_csv, "WRITE_SIZE")
    kern = dict(old.get("kernels", {}))
    src = {}
    for k, f in fetch.items():
        if k.startswith("i8_") != i8:
            continue
        w = write.get(k, 0.0)
        b = int(2 * f * 1024 + w * 1024)
        kern[k] = {"hbm_bytes_per_launch": b, "algorithmic_bytes": ALG[k], "traffic_over_algorithmic": round(b / ALG[k], 4),
                   "fetch_kb": round(f, 1), "write_kb": round(w, 1), "pass": tag}
        src[k] = tag
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) on tools/kernel_probe.py; bytes = "
                     "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halving); per-kernel pass tag in 'pass' "
                     f"(profiles/<tag>_pmc_*.csv)", "kernels": kern}
    for k, v in kern.items():
        v.setdefault("pass", "r01b")
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
