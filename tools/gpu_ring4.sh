#!/bin/bash
# ring variants: tests on the default lib, then A/B + timeline per lib variant, wait profiles
set -o pipefail
TAG=${1:-ring}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
L=$PWD/llm-inference_amd/lib
echo "[$(date +%T)] pytest ring"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_ring_$TAG.log 2>&1 || { tail -30 $OUT/pytest_ring_$TAG.log; exit 1; }
tail -1 $OUT/pytest_ring_$TAG.log
for v in ${VARIANTS:-default}; do
  lib=$L/libllmi.so; [ "$v" != default ] && lib=$L/libllmi_$v.so
  echo "[$(date +%T)] variant $v"
  LLMI_LIB_PATH=$lib timeout -k 10 200 python -u tools/ring_timeline.py > $OUT/ring_tl_${TAG}_$v.json 2> $OUT/ring_tl_${TAG}_$v.err || { echo "tl failed $?"; tail -20 $OUT/ring_tl_${TAG}_$v.err; exit 1; }
  cat $OUT/ring_tl_${TAG}_$v.json
  LLMI_LIB_PATH=$lib timeout -k 10 300 python -u tools/ring_ab.py --modes 1 --reps 1 > $OUT/ring_ab_${TAG}_$v.jsonl 2> $OUT/ring_ab_${TAG}_$v.err || { echo "ab failed $?"; tail -20 $OUT/ring_ab_${TAG}_$v.err; exit 1; }
  cat $OUT/ring_ab_${TAG}_$v.jsonl
done
for pv in ${PROFS:-}; do
  flag=--prof; [ "$pv" = prof2 ] && flag=--prof2
  echo "[$(date +%T)] profile $pv"
  LLMI_LIB_PATH=$L/libllmi_$pv.so timeout -k 10 200 python -u tools/ring_timeline.py $flag > $OUT/ring_${pv}_$TAG.json 2> $OUT/ring_${pv}_$TAG.err || { echo "prof failed $?"; tail -20 $OUT/ring_${pv}_$TAG.err; exit 1; }
  cat $OUT/ring_${pv}_$TAG.json
done
echo "[$(date +%T)] done"
