#!/bin/bash
# gate_up (512 rows, random data) plain lo8 vs balanced lo8, and plain fp16 planes vs balanced,
# three alternating passes in one call (same box, same clocks).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for pass in 1 2 3; do
  for pm in 3 4 2 5; do
    timeout -k 10 60 ./tools/gemm_bench/gemm_bench_lo8 512 30 0 gate_up $pm 0 | grep -v timeline >> gpurun_out/ab_bal.jsonl || exit 1
  done
done
cat gpurun_out/ab_bal.jsonl
