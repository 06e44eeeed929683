#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV per (kernel, grid) -- o_proj and down_proj
share one GEMV instantiation and differ only in grid size / order.

    python tools/trace_summary.py <kernel_trace.csv> > summary.json
"""
import collections
import csv
import json
import re
import sys


def short(name):
    m = re.search(r"(\w+_kernel)(<[^()]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:80]


def main():
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(sys.argv[1])):
        dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
        key = f'{short(row["Kernel_Name"])} grid={row.get("Grid_Size_X", row.get("Grid_Size", "?"))}x{row.get("Grid_Size_Y", "")}'
        acc[key].append(dur)
    out = {}
    for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        out[k] = {"calls": len(v), "avg_us": round(sum(v) / len(v) / 1e3, 2), "median_us": round(v[len(v) // 2] / 1e3, 2),
                  "min_us": round(v[0] / 1e3, 2), "max_us": round(v[-1] / 1e3, 2), "total_ms": round(sum(v) / 1e6, 1)}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
