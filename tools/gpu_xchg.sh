#!/bin/bash
# TP exchange session: xchg tests (group + two processes, modes 1/2), then the probe at 7B width.
set -o pipefail
TAG=${1:-xchg}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
echo "[$(date +%T)] pytest xchg"
timeout -k 10 600 python -u -m pytest tests/test_gpu_xchg.py tests/test_gpu_tp_group.py -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/pytest_xchg_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest_xchg_$TAG.log | tail -40
[ $rc -eq 0 ] || { tail -40 $OUT/pytest_xchg_$TAG.log; exit $rc; }
echo "[$(date +%T)] probe 7B width, 2 layers, 2 processes"
XCHG_LAYERS=2 timeout -k 10 300 python -u tools/xchg_probe.py llama2-7b 2 > $OUT/xchg_probe_$TAG.json 2> $OUT/xchg_probe_$TAG.err || { echo "probe failed $?"; tail -20 $OUT/xchg_probe_$TAG.err; exit 1; }
cat $OUT/xchg_probe_$TAG.json
echo "[$(date +%T)] done"
