#!/bin/bash
# ring: tests, stamped timeline, wait-time profile (libllmi_prof.so), A/B
set -o pipefail
TAG=${1:-ring}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
echo "[$(date +%T)] pytest ring"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ring.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_ring_$TAG.log 2>&1 || { tail -30 $OUT/pytest_ring_$TAG.log; exit 1; }
tail -1 $OUT/pytest_ring_$TAG.log
echo "[$(date +%T)] ring timeline"
timeout -k 10 200 python -u tools/ring_timeline.py > $OUT/ring_tl_$TAG.json 2> $OUT/ring_tl_$TAG.err || { echo "tl failed $?"; tail -20 $OUT/ring_tl_$TAG.err; exit 1; }
cat $OUT/ring_tl_$TAG.json
echo "[$(date +%T)] ring wait profile"
LLMI_LIB_PATH=$PWD/llm-inference_amd/lib/libllmi_prof.so timeout -k 10 200 python -u tools/ring_timeline.py --prof > $OUT/ring_prof_$TAG.json 2> $OUT/ring_prof_$TAG.err || { echo "prof failed $?"; tail -20 $OUT/ring_prof_$TAG.err; exit 1; }
cat $OUT/ring_prof_$TAG.json
echo "[$(date +%T)] ring A/B"
timeout -k 10 300 python -u tools/ring_ab.py ${AB_ARGS:---modes 1} > $OUT/ring_ab_$TAG.jsonl 2> $OUT/ring_ab_$TAG.err || { echo "ab failed $?"; tail -20 $OUT/ring_ab_$TAG.err; exit 1; }
cat $OUT/ring_ab_$TAG.jsonl
echo "[$(date +%T)] done"
