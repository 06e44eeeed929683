#!/usr/bin/env python3
"""MFMA busy fraction per prefill kernel launch shape from a rocprofv3 --pmc pass with
SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_F16 and GRBM_GUI_ACTIVE.

Dispatches are grouped by (kernel, workgroups, MFMA work): one template instance serves
several GEMM shapes and both precisions (the lo plane doubles the MFMA work).
  busy (chip)        = MFMA_BUSY / (256 CUs * 4 SIMDs * GUI_ACTIVE / 8 XCDs)
  busy (active CUs)  = MFMA_BUSY / (min(workgroups, 256) * 4 * GUI_ACTIVE / 8) for the
                       one-workgroup-per-CU GEMMs (gemm3: 136 KB of LDS per workgroup)
MOPS_F16 counts units of 512 FLOP.
    python tools/mfma_util.py <counter_collection.csv> <out.json>"""
import collections
import csv
import json
import re
import sys

# Llama-2-7B prefill at M = 512: (kernel, workgroups) -> GEMM
SHAPES = {("gemm3_kernel<2>", 172): "gate_up", ("gemm3_silu_bal_kernel", 256): "gate_up (fp8-lo, every CU)",
          ("gemm3_kernel<5>", 192): "qkv (2 K slices)",
          ("gemm3_kernel<5>", 256): "down (8 K slices)", ("gemm2_kernel<128, 2, 5>", 256): "o_proj (2 K slices)",
          ("gemm2_kernel<128, 1, 5>", 256): "o_proj (2 K slices)"}


def short(name):
    m = re.search(r"(\w+_kernel(?:I\w+E|<[^>]*>)?)", name)
    n = name if not m else m.group(1)
    return re.sub(r"\(.*", "", n.replace("void llmi::(anonymous namespace)::", ""))


def main():
    disp = collections.defaultdict(dict)
    for row in csv.DictReader(open(sys.argv[1])):
        d = disp[row["Dispatch_Id"]]
        d["name"] = short(row["Kernel_Name"])
        d["wgs"] = int(row["Grid_Size"]) // max(1, int(row["Workgroup_Size"]))
        d[row["Counter_Name"]] = float(row["Counter_Value"])
    groups = collections.defaultdict(list)
    for d in disp.values():
        groups[(d["name"], d["wgs"], round(d.get("SQ_INSTS_VALU_MFMA_MOPS_F16", 0)))].append(d)
    out = {"note": __doc__.split("\n\n")[1].strip(), "kernels": []}
    for (name, wgs, mops), ds in sorted(groups.items(), key=lambda kv: -kv[0][2]):
        g = sum(x.get("GRBM_GUI_ACTIVE", 0) for x in ds) / len(ds)
        b = sum(x.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for x in ds) / len(ds)
        e = {"kernel": name, "gemm": SHAPES.get((name, wgs)), "workgroups": wgs, "launches": len(ds),
             "GRBM_GUI_ACTIVE": round(g), "SQ_VALU_MFMA_BUSY_CYCLES": round(b), "mfma_work_flop": mops * 512,
             "mfma_busy_frac_chip": round(b / (256 * 4 * g / 8), 4) if g else None}
        if name.startswith("gemm3") and g:
            e["mfma_busy_frac_active_cus"] = round(b / (min(wgs, 256) * 4 * g / 8), 4)
        out["kernels"].append(e)
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
