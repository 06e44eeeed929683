#!/bin/bash
# per-token RoPE workgroup size A/B (LLMI_ROPE_THREADS 256 vs the default 1024)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_prefill.py tests/test_gpu_context_ops.py tests/test_gpu_ctx_history.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_rope.log 2>&1
rc=$?; tail -1 $OUT/pytest_rope.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_rope.log | head; exit $rc; }
g++ -std=c++17 -O2 -I include tools/ctx_decoder_bench.cpp -L llm-inference_amd/lib -lllmi -Wl,-rpath,$PWD/llm-inference_amd/lib -o /tmp/cdb || exit 1
: > $OUT/rope_ab.jsonl
for pass in 1 2; do
  for n in 1024 256; do
    r=$(LLMI_ROPE_THREADS=$n timeout -k 10 200 python -u tools/prefill_probe.py 512 5 2> $OUT/rope_ab.err) || { tail -5 $OUT/rope_ab.err; exit 1; }
    c=$(LLMI_ROPE_THREADS=$n timeout -k 10 120 /tmp/cdb 32 3 200 150 100 62) || exit 1
    echo "{\"threads\": $n, \"prefill\": $r, \"ctx\": $c}" | tee -a $OUT/rope_ab.jsonl
  done
done
