#!/bin/bash
# ring tests, A/B and stamped timeline:  bash tools/gpu_ring2.sh <tag> [pytest -k]
set -o pipefail
TAG=${1:-ring}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
echo "[$(date +%T)] pytest ring"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py -x -v -s -p no:cacheprovider --timeout 200 --timeout-method thread ${2:+-k "$2"} > $OUT/pytest_ring_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|rel-L2|passed|failed|Error" $OUT/pytest_ring_$TAG.log | tail -40
[ $rc -eq 0 ] || { tail -40 $OUT/pytest_ring_$TAG.log; exit $rc; }
echo "[$(date +%T)] ring timeline"
timeout -k 10 200 python -u tools/ring_timeline.py > $OUT/ring_tl_$TAG.json 2> $OUT/ring_tl_$TAG.err || { echo "tl failed $?"; tail -20 $OUT/ring_tl_$TAG.err; exit 1; }
cat $OUT/ring_tl_$TAG.json
echo "[$(date +%T)] ring A/B"
timeout -k 10 300 python -u tools/ring_ab.py ${AB_ARGS:---modes 1} > $OUT/ring_ab_$TAG.jsonl 2> $OUT/ring_ab_$TAG.err || { echo "ab failed $?"; tail -20 $OUT/ring_ab_$TAG.err; exit 1; }
cat $OUT/ring_ab_$TAG.jsonl
echo "[$(date +%T)] done"
