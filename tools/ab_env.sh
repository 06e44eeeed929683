#!/bin/bash
# A/B of one environment switch in one process each, two passes in alternating order:
#   VAR=LLMI_GEMV_TICKETS bash tools/ab_env.sh <tag> <value>...
# env: LAYERS (8), KERNELS (qkv,attn,o,gate_up,down), CTX (2048)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
for pass in 1 2; do
  for v in "$@"; do
    out=gpurun_out/abenv_${TAG}_${v}_p$pass.json
    env "$VAR=$v" timeout -k 10 150 python3 tools/kernel_probe.py --layers ${LAYERS:-8} --iters 200 --loop --ctx ${CTX:-2048} \
      --kernels ${KERNELS:-qkv,attn,o,gate_up,down} > $out 2> gpurun_out/abenv_${TAG}.err || { echo "probe $v failed"; tail -5 gpurun_out/abenv_${TAG}.err; exit 1; }
    echo "$VAR=$v p$pass $(cat $out)"
  done
done
