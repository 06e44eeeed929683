#!/bin/bash
# alternate lib variants on the 8-layer 7B probe loop: VARIANTS="default ks2" bash tools/gpu_ab_libs.sh <tag>
set -o pipefail
TAG=${1:-ab}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
L=$PWD/llm-inference_amd/lib
: > $OUT/ab_$TAG.jsonl
for pass in 1 2; do
  for v in ${VARIANTS:-default}; do
    lib=$L/libllmi.so; [ "$v" != default ] && lib=$L/libllmi_$v.so
    LLMI_LIB_PATH=$lib timeout -k 10 200 python -u tools/kernel_probe.py --layers ${LAYERS:-8} --loop --iters 64 --kernels ${KERNELS:-down,gate_up,o,qkv} > $OUT/ab_one.json 2> $OUT/ab_one.err || { echo "probe $v failed"; tail -20 $OUT/ab_one.err; exit 1; }
    echo "{\"variant\": \"$v\", \"pass\": $pass, \"r\": $(cat $OUT/ab_one.json)}" | tee -a $OUT/ab_$TAG.jsonl
  done
done
echo done
