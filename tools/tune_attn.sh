#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out; mkdir -p $OUT
for lib in llm-inference_amd/lib/libllmi*.so; do
  LLMI_LIB_PATH=$PWD/$lib timeout -k 10 180 python3 tools/kernel_probe.py --layers 2 --iters 100 --kernels attn --attn-sweep 8,64,65,128,256,512,1024,2047 >> $OUT/tune_$1.jsonl 2>> $OUT/tune_$1.err || { echo "probe failed on $lib"; tail -5 $OUT/tune_$1.err; exit 1; }
  tail -1 $OUT/tune_$1.jsonl
done
