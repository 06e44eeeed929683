#!/bin/bash
# full GPU suite + smoke + default bench line:  bash tools/gpu_suite.sh <tag>   (NO_BENCH=1 skips the bench)
set -o pipefail
TAG=${1:-suite}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_gpu_$TAG.log | tail -20
[ $rc -eq 0 ] || { tail -60 $OUT/pytest_gpu_$TAG.log; exit $rc; }
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke_$TAG.log; exit 1; }
tail -1 $OUT/smoke_$TAG.log
if [ -z "$NO_BENCH" ]; then
  echo "[$(date +%T)] bench"
  timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed $?"; tail -20 $OUT/bench_$TAG.err; exit 1; }
  cat $OUT/bench_$TAG.json
fi
echo "[$(date +%T)] done"
