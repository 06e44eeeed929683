L=$PWD/llm-inference_amd/lib
for v in base NOWAIT NOSOFT; do
  if [ $v = base ]; then lib=$L/libllmi.so; else lib=$L/libllmi_$v.so; fi
  echo "== $v"; LLMI_LIB_PATH=$lib timeout -k 10 120 python tools/prefill_attn_timeline.py 512 1 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); q=d['per_query_block']
print(d['span_us'], [(k, v['prologue'], v['loop'], v['epilogue']) for k,v in q.items()])" || exit 1
done
