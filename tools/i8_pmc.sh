set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/pmci8_$c
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-include-regex 'gemv_kernel|attn_oproj_kernel' -d /tmp/pmci8_$c -o pmc --output-format csv -- python3 tools/int8_probe.py 8 i8 eager > gpurun_out/pmci8_${c}.log 2>&1 || exit 1
  find /tmp/pmci8_$c -name '*counter_collection.csv' -exec cp {} gpurun_out/pmci8_${c}_r06p.csv \;
done
