#!/bin/bash
# prefill session: prefill tests, then the 512-row probe (3 modes) twice
set -o pipefail
TAG=${1:-pf}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
echo "[$(date +%T)] pytest prefill"
timeout -k 10 600 python -u -m pytest tests/test_gpu_prefill.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_pf_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|rel-L2|passed|failed" $OUT/pytest_pf_$TAG.log | tail -30
[ $rc -eq 0 ] || { tail -30 $OUT/pytest_pf_$TAG.log; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python -u tools/prefill_probe.py 512 5 >> $OUT/pf_probe_$TAG.jsonl 2>> $OUT/pf_probe_$TAG.err || { echo "probe failed"; tail -20 $OUT/pf_probe_$TAG.err; exit 1; }
done
cat $OUT/pf_probe_$TAG.jsonl
echo "[$(date +%T)] done"
