#!/usr/bin/env python3
"""Turn rocprofv3 --pmc CSV output (FETCH_SIZE / WRITE_SIZE passes) into per-kernel
HBM bytes per launch, with the gfx950 correction of MI355X_MICROARCH.md §HBM:
FETCH_SIZE reports 1/2 of the bytes of a wide coalesced streaming read (x2);
WRITE_SIZE is exact for 16-B streaming stores. Both are in KB (x1024).

    python tools/pmc_summarize.py <fetch_counter_collection.csv> <write_counter_collection.csv> out.json
"""
import collections
import csv
import json
import sys

KMAP = {"gemv_kernel": None, "attn_decode_kernel": "attn"}


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row.get("Counter_Name") != counter:
            continue
        acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    if len(sys.argv) != 4:
        raise SystemExit("usage: pmc_summarize.py <fetch.csv> <write.csv> <out.json>")
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) on tools/kernel_probe.py; "
                     "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE halving)",
           "kernels_raw": {}}
    for k, f in fetch.items():
        w = write.get(k, 0.0)
        out["kernels_raw"][k] = {"fetch_kb": f, "write_kb": w, "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024)}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
