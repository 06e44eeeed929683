#!/bin/bash
# A/B of library variants on the 13B int8 probe (tools/int8_probe.py), two alternating passes:
#   bash tools/ab_int8.sh <tag> <variant>...   (default = lib/libllmi.so; others lib/libllmi_<v>.so)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
for pass in 1 2; do
  for v in "$@"; do
    if [ "$v" = default ]; then unset LLMI_LIB_PATH; else export LLMI_LIB_PATH=$PWD/llm-inference_amd/lib/libllmi_$v.so; fi
    out=gpurun_out/abi8_${TAG}_${v}_p$pass.json
    timeout -k 10 200 python3 tools/int8_probe.py ${LAYERS:-8} > $out 2> gpurun_out/abi8_${TAG}.err || { echo "int8 probe $v failed"; tail -5 gpurun_out/abi8_${TAG}.err; exit 1; }
    echo "$v p$pass $(cat $out)"
  done
done
