#!/bin/bash
# prefill attention split sweep (LLMI_PF_CHUNK key blocks per chunk), fp8-lo and exact modes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_prefill.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_pf_chunk.log 2>&1; rc=$?
tail -3 $OUT/pytest_pf_chunk.log
[ $rc -eq 0 ] || exit $rc
: > $OUT/pf_chunk.jsonl
for pass in 1 2; do
  for cb in 0 1 2 4 8; do
    r=$(LLMI_PF_CHUNK=$cb timeout -k 10 200 python -u tools/prefill_probe.py 512 5 exact8 2> $OUT/pf_chunk.err) || { echo "probe $cb failed"; tail -20 $OUT/pf_chunk.err; exit 1; }
    echo "{\"chunk\": $cb, \"pass\": $pass, \"r\": $r}" | tee -a $OUT/pf_chunk.jsonl
  done
done
