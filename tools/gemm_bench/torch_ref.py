#!/usr/bin/env python3
"""hipBLASLt reference point for the prefill GEMM shapes: torch.matmul of fp16
A[M, K] by W[N, K]^T (fp32 accumulate, fp16 out) timed with HIP events. Not part
of the product: it only tells gemm_bench's numbers what the vendor library does."""
import json
import sys

import torch


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    shapes = [("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096), ("down", 4096, 11008),
              ("sq4096", 4096, 4096)]
    variants = [("randn", torch.float16)]
    if len(sys.argv) > 2 and sys.argv[2] == "all":  # + zero-filled fp16 and random bf16 (power vs schedule)
        variants += [("zeros", torch.float16), ("randn", torch.bfloat16)]
    for (name, n, k), (data, dt) in [(s, v) for s in shapes for v in variants]:
        mm = 4096 if name == "sq4096" else m
        if data == "zeros":
            a = torch.zeros(mm, k, device="cuda", dtype=dt)
            w = torch.zeros(n, k, device="cuda", dtype=dt)
        else:
            a = torch.randn(mm, k, device="cuda", dtype=dt)
            w = torch.randn(n, k, device="cuda", dtype=dt) * 0.05
        for _ in range(3):
            torch.matmul(a, w.t())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        iters = 20
        e0.record()
        for _ in range(iters):
            torch.matmul(a, w.t())
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        print(json.dumps({"shape": name, "data": data, "dtype": str(dt), "m": mm, "n": n, "k": k, "torch_us": round(us, 2),
                          "torch_tflops": round(2.0 * mm * n * k / us * 1e-6, 1)}), flush=True)


if __name__ == "__main__":
    main()
