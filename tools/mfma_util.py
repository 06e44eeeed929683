#!/usr/bin/env python3
"""MFMA busy fraction per prefill kernel from a rocprofv3 --pmc pass with
SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_F16 and GRBM_GUI_ACTIVE:
busy = MFMA_BUSY / (256 CUs * 4 SIMDs * GUI_ACTIVE / 8 XCDs); MOPS_F16 counts
units of 512 FLOP.     python tools/mfma_util.py <counter_collection.csv> <out.json>"""
import collections
import csv
import json
import re
import sys


def short(name):
    m = re.search(r"(\w+_kernel(?:I\w+E|<[^>]*>))", name)
    n = name if not m else m.group(1)
    return re.sub(r"\(.*", "", n.replace("void llmi::(anonymous namespace)::", ""))


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for row in csv.DictReader(open(sys.argv[1])):
        acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {"note": "SQ_VALU_MFMA_BUSY_CYCLES summed over SIMDs; GRBM_GUI_ACTIVE summed over the 8 XCDs; busy "
                   "fraction = MFMA_BUSY / (256 CUs * 4 SIMDs * GUI_ACTIVE / 8); MOPS_F16 in units of 512 FLOP "
                   "(MFMA work = 2x the algorithmic FLOPs in the exact mode); per-launch means", "kernels": {}}
    for k, c in acc.items():
        mean = {n: sum(v) / len(v) for n, v in c.items()}
        g, b, mops = mean.get("GRBM_GUI_ACTIVE", 0), mean.get("SQ_VALU_MFMA_BUSY_CYCLES", 0), mean.get(
            "SQ_INSTS_VALU_MFMA_MOPS_F16", 0)
        out["kernels"][k] = {**{n: round(v) for n, v in mean.items()},
                             "mfma_busy_frac": round(b / (256 * 4 * g / 8), 4) if g else None,
                             "mfma_work_flop": mops * 512}
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
