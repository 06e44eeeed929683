#!/bin/bash
# int8 13B probe A/B of lib variants, alternating: VARIANTS="default i8w4" bash tools/gpu_i8_ab.sh <tag>
set -o pipefail
TAG=${1:-i8ab}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
L=$PWD/llm-inference_amd/lib
: > $OUT/i8_ab_$TAG.jsonl
for pass in 1 2; do
  for v in ${VARIANTS:-default}; do
    lib=$L/libllmi.so; [ "$v" != default ] && lib=$L/libllmi_$v.so
    r=$(LLMI_LIB_PATH=$lib timeout -k 10 200 python -u tools/int8_probe.py 8 2> $OUT/i8_ab.err) || { echo "probe $v failed"; tail -20 $OUT/i8_ab.err; exit 1; }
    echo "{\"variant\": \"$v\", \"pass\": $pass, \"r\": $r}" | tee -a $OUT/i8_ab_$TAG.jsonl
  done
done
