#!/usr/bin/env python3
"""Per-phase timeline of one dataflow layer launch (layer.hip) from in-kernel
s_memrealtime stamps: when each phase's workgroups start, pass their wait and
finish. Prints JSON (us, relative to the first workgroup start)."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "llm-inference_amd"))
os.environ.setdefault("LLMI_FUSED", "1")

from llmi.engine import Engine, preset, synth_prompt  # noqa: E402

NAMES = ["qkv", "attn", "o", "gate_up", "down"]


def main():
    ctx = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    cfg = preset("llama2-7b", layers=2, max_seq=2048)
    out = {"ctx": ctx}
    with Engine(cfg) as e:
        e.load_synthetic(0)
        e.generate(synth_prompt(0, 8, cfg.vocab), ctx - 8)
        st, ph = e.layer_stamps()
        out["layer_us_timed"] = e.time_kernel("layer", 50)[0]
        out["parts_us"] = {k: e.time_kernel(k, 50)[0] for k in NAMES}
        out["fused_alone_us"] = {k: e.time_kernel("f_" + k, 50)[0] for k in NAMES}
        out["fused_alone_plain_us"] = {k: e.time_kernel("p_" + k, 50)[0] for k in NAMES}
    b = 0
    phases = {}
    for name, n in zip(NAMES, ph.tolist()):
        s = st[b:b + n]
        b += n
        live = s[:, 1] > 0  # early-exit workgroups (inactive KV splits) never pass a wait
        s = s[live] if live.any() else s
        q = lambda a, p: float(np.percentile(a, p))
        phases[name] = {
            "wgs": int(n),
            "start_min": q(s[:, 0], 0), "start_med": q(s[:, 0], 50), "start_max": q(s[:, 0], 100),
            "wait_pass_med": q(s[:, 1], 50), "wait_pass_max": q(s[:, 1], 100),
            "end_min": q(s[:, 2], 0), "end_med": q(s[:, 2], 50), "end_max": q(s[:, 2], 100),
            "wait_us_med": q(s[:, 1] - s[:, 0], 50), "body_us_med": q(s[:, 2] - s[:, 1], 50),
        }
    out["phases"] = phases
    if os.environ.get("LLMI_STAMPS_NPZ"):
        np.savez_compressed(os.environ["LLMI_STAMPS_NPZ"], stamps=st, phase_wgs=ph)
    out["span_us"] = float(st[:, 2].max())
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
