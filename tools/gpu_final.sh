#!/bin/bash
# Round evidence in one call: GPU suite, smoke, the default bench line, an eager kernel
# trace of one bench step, a kernel trace of the fp8-lo prefill.   bash tools/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-final}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed $?"; tail -40 $OUT/pytest_gpu_$TAG.log; exit 1; }
tail -2 $OUT/pytest_gpu_$TAG.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke failed $?"; tail -20 $OUT/smoke_$TAG.log; exit 1; }
tail -3 $OUT/smoke_$TAG.log
step bench
timeout -k 10 900 python -u bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed $?"; tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
step "kernel trace (eager bench step)"
rm -rf /tmp/prof_trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_trace -o trace --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-side --eager > $OUT/prof_trace_$TAG.log 2>&1 || { echo "trace failed $?"; tail -20 $OUT/prof_trace_$TAG.log; exit 1; }
find /tmp/prof_trace -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_$TAG.csv \;
step "kernel trace (fp8-lo prefill)"
rm -rf /tmp/pf8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pf8 -o pf --output-format csv -- python3 tools/prefill_probe.py 512 2 exact8 > $OUT/pf8_trace_$TAG.log 2>&1 || { echo "pf8 trace failed $?"; exit 1; }
find /tmp/pf8 -name '*kernel_stats.csv' -exec cp {} $OUT/pf8_kernel_stats_$TAG.csv \;
step done
