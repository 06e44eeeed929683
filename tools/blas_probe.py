"""Library GEMM rates at the 7B prefill projection shapes (M = 512 rows): torch.matmul
(hipBLASLt / rocBLAS underneath) in fp16, timed with HIP events. A go/no-go probe for
running the prefill's hi/lo-split projections as plain library GEMMs."""
import json
import sys

import torch


def rate(m, n, k, reps=20, dt=torch.float16):
    a = torch.randn(m, k, device="cuda", dtype=dt)
    b = torch.randn(k, n, device="cuda", dtype=dt)
    for _ in range(3):
        torch.matmul(a, b)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        torch.matmul(a, b)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    return us, 2 * m * n * k / us / 1e6


def main():
    out = []
    for name, n, k in (("qkv", 12288, 4096), ("o", 4096, 4096), ("gate_up", 22016, 4096), ("down", 4096, 11008),
                       ("gate_up_k2", 22016, 8192), ("qkv_k2", 12288, 8192)):
        for lt in (False, True):
            torch.backends.cuda.preferred_blas_library("cublaslt" if lt else "cublas")
            us, tf = rate(512, n, k)
            r = {"gemm": name, "m": 512, "n": n, "k": k, "lib": "hipblaslt" if lt else "rocblas", "us": round(us, 1),
                 "tflops": round(tf, 1)}
            print(json.dumps(r), flush=True)
            out.append(r)
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
