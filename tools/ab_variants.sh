#!/bin/bash
# A/B of library variants in one process each, two passes in alternating order:
#   bash tools/ab_variants.sh <tag> <variant>...   (default = lib/libllmi.so; others lib/libllmi_<v>.so)
# env: LAYERS (8), KERNELS (qkv,attn,o,gate_up,down), CTX (2048)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
for pass in 1 2; do
  for v in "$@"; do
    if [ "$v" = default ]; then unset LLMI_LIB_PATH; else export LLMI_LIB_PATH=$PWD/llm-inference_amd/lib/libllmi_$v.so; fi
    out=gpurun_out/ab_${TAG}_${v}_p$pass.json
    timeout -k 10 150 python3 tools/kernel_probe.py --layers ${LAYERS:-8} --iters 200 --loop --ctx ${CTX:-2048} \
      --kernels ${KERNELS:-qkv,attn,o,gate_up,down} > $out 2> gpurun_out/ab_${TAG}.err || { echo "probe $v failed"; tail -5 gpurun_out/ab_${TAG}.err; exit 1; }
    echo "$v p$pass $(cat $out)"
  done
done
