#!/bin/bash
# row-kernel block size A/B on the engine prefill (LLMI_RN256=1: 256 threads a row)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_prefill.py tests/test_gpu_context_ops.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_rn2.log 2>&1
rc=$?; tail -2 $OUT/pytest_rn2.log; [ $rc -eq 0 ] || exit $rc
: > $OUT/pf_rn.jsonl
for pass in 1 2; do
  for v in 0 1; do
    r=$(LLMI_RN256=$v timeout -k 10 200 python -u tools/prefill_probe.py 512 5 2> $OUT/pf_rn.err) || { tail -5 $OUT/pf_rn.err; exit 1; }
    echo "{\"rn256\": $v, \"r\": $r}" | tee -a $OUT/pf_rn.jsonl
  done
done
