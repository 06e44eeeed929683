cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_prefill.py -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_pf.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_pf.log | grep -v "^$"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/prefill_probe.py 512 3
rm -rf /tmp/pp; timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/pp -o pf --output-format csv -- python3 tools/prefill_probe.py 512 1 > gpurun_out/pp.log 2>&1 && find /tmp/pp -name '*kernel_stats.csv' -exec cp {} gpurun_out/prefill_stats_g2.csv \; ; head -12 gpurun_out/prefill_stats_g2.csv | cut -c1-150
