#!/bin/bash
# The one GPU runner (replaces the per-experiment gpu_*.sh / ab_*.sh scripts of rounds 1-4).
#   bash tools/gpu.sh <tag> <step> [<step> ...]
# Steps, run in order; the first failure ends the call (nothing more touches the GPU):
#   pytest            the whole GPU suite              pytest=<args>  e.g. pytest=tests/test_gpu_ring.py
#   smoke             __graft_entry__.smoke()
#   bench             bench.py (BENCH_ARGS env: extra flags)
#   trace             rocprofv3 kernel trace of one eager bench step (+ tools/trace_summary.py)
#   pmc               FETCH_SIZE and WRITE_SIZE passes (separate runs) on the decode kernels
#   pftrace           rocprofv3 kernel trace of a 512-row prefill (PF_MODE env: exact | exact8 | fast, default exact8)
#   mfma              MFMA-busy PMC pass on the prefill GEMMs / attention
#   lds               LDS bank-conflict / LDS-instruction PMC pass on the prefill GEMMs / attention
#   cmd=<command>     any other command, under a 600-s limit, output in gpurun_out/cmd_<tag>_<n>.log
# Every output lands in gpurun_out/<step>_<tag>.*; copy what is judged into profiles/.
set -o pipefail
TAG=${1:?usage: tools/gpu.sh <tag> <step> ...}
shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
n=0
step() { echo "[$(date +%T)] $*"; }
fail() { echo "FAILED ($1): $2"; tail -40 "$3"; exit 1; }
for s in "$@"; do
  n=$((n + 1))
  case "$s" in
    pytest|pytest=*)
      args=${s#pytest}; args=${args#=}; [ -z "$args" ] && args=tests
      step "pytest -m gpu $args"
      timeout -k 10 1100 python -u -m pytest $args -m gpu -x -v -p no:cacheprovider --timeout 300 \
        --timeout-method thread > $OUT/pytest_$TAG.log 2>&1 || fail $? pytest $OUT/pytest_$TAG.log
      grep -E "passed|failed" $OUT/pytest_$TAG.log | tail -2 ;;
    smoke)
      step smoke
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 \
        || fail $? smoke $OUT/smoke_$TAG.log
      tail -1 $OUT/smoke_$TAG.log ;;
    bench)
      step "bench ${BENCH_ARGS:-}"
      timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err \
        || fail $? bench $OUT/bench_$TAG.err
      cat $OUT/bench_$TAG.json ;;
    trace)
      step "kernel trace (eager bench step)"
      rm -rf /tmp/prof_trace
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_trace -o trace --output-format csv -- \
        python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-side --eager > $OUT/trace_$TAG.log 2>&1 \
        || fail $? trace $OUT/trace_$TAG.log
      find /tmp/prof_trace -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_$TAG.csv \;
      python3 tools/trace_summary.py $(find /tmp/prof_trace -name '*kernel_trace.csv' | head -1) \
        > $OUT/trace_summary_$TAG.json || echo "trace summary failed" ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        step "pmc $c"
        rm -rf /tmp/pmc_$c
        timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex 'gemv_kernel|attn_decode_kernel|attn_oproj2?_kernel|qkv_attn_kernel' \
          -d /tmp/pmc_$c -o pmc --output-format csv -- python3 tools/kernel_probe.py --ctx 2048 --prefill --iters 8 \
          --kernels gate_up,qkv,lm_head,attn,o,down,qkv_attn > $OUT/pmc_${c}_$TAG.log 2>&1 || fail $? pmc $OUT/pmc_${c}_$TAG.log
        find /tmp/pmc_$c -name '*counter_collection.csv' -exec cp {} $OUT/pmc_${c}_$TAG.csv \;
      done ;;
    pftrace)
      step "kernel trace (prefill, mode ${PF_MODE:-exact8})"
      rm -rf /tmp/prof_pf
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_pf -o pf --output-format csv -- \
        python3 tools/prefill_probe.py 512 3 ${PF_MODE:-exact8} > $OUT/pftrace_$TAG.log 2>&1 || fail $? pftrace $OUT/pftrace_$TAG.log
      find /tmp/prof_pf -name '*kernel_stats.csv' -exec cp {} $OUT/prefill_kernel_stats_$TAG.csv \; ;;
    mfma)
      step "pmc mfma (prefill)"
      rm -rf /tmp/pmc_m
      timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE \
        --kernel-include-regex 'gemm[23]?_(sk_)?kernel|attn_prefill' -d /tmp/pmc_m -o pmc --output-format csv -- \
        python3 tools/prefill_probe.py 512 3 ${PF_MODE:-exact} > $OUT/mfma_$TAG.log 2>&1 || fail $? mfma $OUT/mfma_$TAG.log
      find /tmp/pmc_m -name '*counter_collection.csv' -exec cp {} $OUT/pmc_mfma_$TAG.csv \; ;;
    lds)
      step "pmc lds (prefill GEMMs / attention)"
      rm -rf /tmp/pmc_l
      timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE \
        --kernel-include-regex 'gemm[23]?_(sk_)?kernel|attn_prefill' -d /tmp/pmc_l -o pmc --output-format csv -- \
        python3 tools/prefill_probe.py 512 3 ${PF_MODE:-exact} > $OUT/lds_$TAG.log 2>&1 || fail $? lds $OUT/lds_$TAG.log
      find /tmp/pmc_l -name '*counter_collection.csv' -exec cp {} $OUT/pmc_lds_$TAG.csv \; ;;
    cmd=*)
      c=${s#cmd=}
      step "$c"
      timeout -k 10 600 bash -c "$c" > $OUT/cmd_${TAG}_$n.log 2>&1 || fail $? "$c" $OUT/cmd_${TAG}_$n.log
      tail -30 $OUT/cmd_${TAG}_$n.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
step done
