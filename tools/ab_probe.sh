#!/bin/bash
# A/B kernel probes of library variants: bash tools/ab_probe.sh <tag> <variant>...  (default = lib/libllmi.so)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
for v in "$@"; do
  if [ "$v" = default ]; then unset LLMI_LIB_PATH; else export LLMI_LIB_PATH=$PWD/llm-inference_amd/lib/libllmi_$v.so; fi
  if [ -n "$PROBE7B" ]; then
    timeout -k 10 120 python3 tools/kernel_probe.py --layers 2 --iters 200 --loop --attn-sweep 8,512,2047 > gpurun_out/ab_${TAG}_7b_$v.json 2>&1 || exit 1
    echo "7b $v"; cat gpurun_out/ab_${TAG}_7b_$v.json
  fi
  timeout -k 10 120 python3 tools/int8_probe.py 8 > gpurun_out/ab_${TAG}_i8_$v.json 2>&1 || exit 1
  echo "i8 $v"; cat gpurun_out/ab_${TAG}_i8_$v.json
done
