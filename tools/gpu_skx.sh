#!/bin/bash
# stream-K cost split (timing-only libs): kernel stats of the ragged context bench with q/k/v on
# stream-K too (LLMI_SK_LINEAR=1), for the default lib, skx1 (no slot payload), skx2 (no hand-off)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
L=$PWD/llm-inference_amd/lib
for v in default skx1 skx2; do
  name=libllmi.so; [ "$v" != default ] && name=libllmi_$v.so
  g++ -std=c++17 -O2 -I include tools/ctx_decoder_bench.cpp -L $L -l:$name -Wl,-rpath,$L -o /tmp/cdb_$v || exit 1
  rm -rf /tmp/ctr
  LLMI_SK_LINEAR=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ctr -o ctr --output-format csv -- /tmp/cdb_$v 32 1 200 150 100 62 > $OUT/skx_$v.log 2>&1 || { echo "trace $v failed"; tail -5 $OUT/skx_$v.log; exit 1; }
  find /tmp/ctr -name '*kernel_stats.csv' -exec cp {} $OUT/skx_stats_$v.csv \;
  echo "== $v"; grep gemm3 $OUT/skx_stats_$v.csv | cut -d, -f1-4
done
