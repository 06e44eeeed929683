#!/bin/bash
# GPU session: gpu tests, kernel probe under env variants, bench line.
# Usage (on the gpurun box): bash tools/exp_sweep.sh <tag> [VAR=a,b,c ...]
set -o pipefail
TAG=${1:-exp}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
if [ -z "$NO_TESTS" ]; then
  echo "[$(date +%T)] pytest -m gpu"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed $?"; tail -30 $OUT/pytest_gpu_$TAG.log; exit 1; }
  tail -2 $OUT/pytest_gpu_$TAG.log
fi
for spec in "$@"; do
  var=${spec%%=*}; vals=${spec#*=}
  for v in ${vals//,/ }; do
    echo "[$(date +%T)] probe $var=$v"
    n=$(basename "$v")
    env $var=$v timeout -k 10 200 python3 tools/kernel_probe.py --layers 8 --iters 100 --loop --kernels ${KERNELS:-qkv,attn,o,attn_o,gate_up,down} > $OUT/probe_${TAG}_${var}_$n.json 2> $OUT/probe_${TAG}.err || { echo "probe failed $?"; tail -20 $OUT/probe_${TAG}.err; exit 1; }
    cat $OUT/probe_${TAG}_${var}_$n.json
  done
done
if [ -z "$NO_BENCH" ]; then
  echo "[$(date +%T)] bench"
  timeout -k 10 600 python bench.py --steps 2 --warmup 1 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed $?"; tail -20 $OUT/bench_$TAG.err; exit 1; }
  cat $OUT/bench_$TAG.json
fi
echo "[$(date +%T)] done"
