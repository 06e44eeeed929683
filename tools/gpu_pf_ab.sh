#!/bin/bash
# prefill A/B of lib variants, alternating: VARIANTS="default nopin" bash tools/gpu_pf_ab.sh <tag>
set -o pipefail
TAG=${1:-pfab}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
L=$PWD/llm-inference_amd/lib
: > $OUT/pf_ab_$TAG.jsonl
for pass in 1 2 3; do
  for v in ${VARIANTS:-default}; do
    lib=$L/libllmi.so; [ "$v" != default ] && lib=$L/libllmi_$v.so
    r=$(LLMI_LIB_PATH=$lib timeout -k 10 200 python -u tools/prefill_probe.py 512 5 ${MODE:-exact8} 2> $OUT/pf_ab.err) || { echo "probe $v failed"; tail -20 $OUT/pf_ab.err; exit 1; }
    echo "{\"variant\": \"$v\", \"pass\": $pass, \"r\": $r}" | tee -a $OUT/pf_ab_$TAG.jsonl
  done
done
