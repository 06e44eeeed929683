#!/bin/bash
# PMC passes over gemm_bench (one shape, one precision); summaries under gpurun_out/gemm_pmc_<tag>/
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B=$R/tools/gemm_bench/${BIN:-gemm_bench_l0}
SHAPE=${SHAPE:-gate_up}
TAG=${TAG:-a}
O=$R/gpurun_out/gemm_pmc_$TAG
mkdir -p $O
timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d $O/kt -o kt -- $B 512 5 0 $SHAPE 1 > $O/kt.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/p1 -o p1 -- $B 512 5 0 $SHAPE 1 > $O/p1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $O/p2 -o p2 -- $B 512 5 0 $SHAPE 1 > $O/p2.log 2>&1
find $O -name "*.csv" | head -20
