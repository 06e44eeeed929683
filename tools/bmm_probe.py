"""Time llmi_batched_matmul (launchLinearStridedBatchGemm) at the context layer's
attention shapes with HIP events; run under rocprofv3 --kernel-trace --stats for the
per-kernel durations. Usage: python tools/bmm_probe.py [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "llm-inference_amd"))
from llmi import ops  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    rng = np.random.default_rng(9)
    for dt in (torch.float32, torch.float16):
        for (m, n, k), tb in (((512, 512, 128), True), ((512, 128, 512), False)):
            a = torch.from_numpy(rng.standard_normal((1, 32, m, k)).astype(np.float32)).to("cuda", dt)
            bs = (1, 32, n, k) if tb else (1, 32, k, n)
            b = torch.from_numpy(rng.standard_normal(bs).astype(np.float32)).to("cuda", dt)
            for _ in range(3):
                ops.launchLinearStridedBatchGemm(a, b, trans_b=tb)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(reps):
                ops.launchLinearStridedBatchGemm(a, b, trans_b=tb)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / reps * 1e3
            print(f"bmm m={m} n={n} k={k} tb={tb} {dt}: {us:.1f} us "
                  f"({2 * 32 * m * n * k / us / 1e6:.1f} TFLOP/s)", flush=True)


if __name__ == "__main__":
    main()
