#!/bin/bash
# GPU session: full gpu test suite, then a short bench line.
#   gpurun -- bash tools/gpu_check.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-check}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
echo "[$(date +%T)] pytest -m gpu ${2:+-k $2}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${2:+-k "$2"} > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|rel-L2|passed|failed" $OUT/pytest_gpu_$TAG.log | tail -60
[ $rc -eq 0 ] || { tail -40 $OUT/pytest_gpu_$TAG.log; exit $rc; }
if [ -z "$NO_BENCH" ]; then
  echo "[$(date +%T)] bench"
  timeout -k 10 600 python -u bench.py --steps ${STEPS:-3} --warmup 1 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed $?"; tail -20 $OUT/bench_$TAG.err; exit 1; }
  cat $OUT/bench_$TAG.json
fi
echo "[$(date +%T)] done"
