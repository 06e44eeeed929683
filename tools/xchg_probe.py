#!/usr/bin/env python3
"""Time the one-shot peer exchange (csrc/xchg.hip) between two rank processes that share
ONE GPU (the only multi-process setting a one-GPU box offers): each exchange is one kernel
per rank that writes the 32 KB residual partial into both inboxes, raises flags and waits for
the other process. Prints the per-exchange latency, eager and graph-replayed, and the
graph-replayed decode per token with the exchange as its own launches (mode 1) and fused
into the producing launches (mode 2; XCHG_LAYERS layers, default 1). Cross-GPU xGMI
latency needs the multi-GPU bench (tp_exchange in its JSON line).

    python tools/xchg_probe.py [preset] [world]"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    pname = sys.argv[1] if len(sys.argv) > 1 else "tiny"
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    worker = os.path.join(REPO, "tests", "helpers", "xchg_worker.py")
    fixture = os.path.join(REPO, "tests", "golden", "tiny.npz")
    with tempfile.TemporaryDirectory() as rdv:
        env = dict(os.environ, XCHG_TIME="1", XCHG_LAYERS=os.environ.get("XCHG_LAYERS", "1"))
        procs = [subprocess.Popen([sys.executable, worker, str(r), str(world), "0", rdv, fixture, pname, "8"], env=env)
                 for r in range(world)]
        rcs = [p.wait(timeout=300) for p in procs]
        assert all(rc == 0 for rc in rcs), rcs
        res = [np.load(os.path.join(rdv, f"out_{r}.npz")) for r in range(world)]
        out = {"preset": pname, "world": world, "device": "one GPU, two processes",
               "us_per_exchange_eager": [round(float(r["us_xchg"]), 2) for r in res],
               "us_per_exchange_graph": [round(float(r["us_xchg_graph"]), 2) for r in res],
               "layers": int(env["XCHG_LAYERS"]),
               # graph-replayed decode, us per token: exchange launches (1) vs fused into the producers (2)
               "loop_us_mode1": [round(float(r["us_loop_mode1"]), 2) for r in res],
               "loop_us_mode2": [round(float(r["us_loop_mode2"]), 2) for r in res]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
