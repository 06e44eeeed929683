#!/bin/bash
# round-4 session: context decoder with the residual entry points (tests + ragged timing),
# then the fused-exchange tail v2 (exchange tests, group probe, two-process probe).
# A test failure (rc 1) goes on to the next step; a timeout / abort / fault ends the script.
set -o pipefail
TAG=${1:-r04u}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
fatal() { case $1 in 0|1) return 1;; *) echo "fatal rc $1 at $2"; return 0;; esac; }
echo "[$(date +%T)] pytest ctx"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ctx_history.py tests/test_gpu_context_ops.py tests/test_cpp_api.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_ctx_$TAG.log 2>&1
rc=$?; grep -E "FAILED|ERROR|rel-L2|passed|failed" $OUT/pytest_ctx_$TAG.log | tail -30
fatal $rc pytest_ctx && exit $rc
g++ -std=c++17 -O2 -I include tools/ctx_decoder_bench.cpp -L llm-inference_amd/lib -lllmi -Wl,-rpath,$PWD/llm-inference_amd/lib -o /tmp/cdb || exit 1
: > $OUT/ctx_bench_$TAG.jsonl
for uf in 0 1 0; do
  for lens in "512" "200 150 100 62"; do
    LLMI_CTX_UNFUSED=$uf timeout -k 10 120 /tmp/cdb 32 3 $lens >> $OUT/ctx_bench_$TAG.jsonl; rc=$?
    fatal $rc ctx_bench && exit $rc
  done
done
cat $OUT/ctx_bench_$TAG.jsonl
echo "[$(date +%T)] pytest xchg"
timeout -k 10 400 python -u -m pytest tests/test_gpu_xchg.py tests/test_gpu_tp_group.py tests/test_gpu_bench_rehearsal.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $OUT/pytest_xchg_$TAG.log 2>&1
rc=$?; tail -3 $OUT/pytest_xchg_$TAG.log
fatal $rc pytest_xchg && exit $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/group_tp_probe.py > $OUT/group_tp_$TAG.jsonl 2> $OUT/group_tp_$TAG.err; rc=$?
cat $OUT/group_tp_$TAG.jsonl
fatal $rc group_probe && exit $rc
XCHG_LAYERS=2 timeout -k 10 300 python -u tools/xchg_probe.py llama2-7b 2 > $OUT/xchg_probe_$TAG.jsonl 2>&1; rc=$?
tail -5 $OUT/xchg_probe_$TAG.jsonl
echo "[$(date +%T)] done"
exit $rc
