# RF engine: bit-exact tests vs the numpy oracle, fit-time A/B (EM_RF_DERIVE=0 vs 1), kernel stats
set -o pipefail
mkdir -p gpurun_out/rfd
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_forest.py tests/test_trees_property_gpu.py tests/test_train_gpu.py -k "forest or rf or tree" -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/rfd/t.log 2>&1 || { grep -E "PASSED|FAILED|Error|assert" gpurun_out/rfd/t.log | tail -30; exit 3; }
grep -cE "PASSED" gpurun_out/rfd/t.log; tail -1 gpurun_out/rfd/t.log
for r in 1; do
  for d in 0 1; do
    EM_RF_DERIVE=$d timeout -k 10 200 python tools/rf_bench.py > gpurun_out/rfd/b_${d}_$r.log 2>&1 || { tail -5 gpurun_out/rfd/b_${d}_$r.log; exit 4; }
    grep '^{' gpurun_out/rfd/b_${d}_$r.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('derive=$d', 'rows', j['rows'], 'fit_ms %.2f' % (j['fit_s']*1e3), 'nodes_split', j['nodes_split'], 'val_acc %.4f' % j['val']['acc'])"
  done
done
EM_RF_DERIVE=1 timeout -k 10 200 python tools/rf_bench.py --rows 700000 > gpurun_out/rfd/b_700k.log 2>&1 || exit 5
grep '^{' gpurun_out/rfd/b_700k.log | tail -1 | cut -c1-200
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rfd/prof -o run -- python3 tools/rf_bench.py --repeat 2 > gpurun_out/rfd/prof.log 2>&1 || exit 6
head -8 gpurun_out/rfd/prof/run_kernel_stats.csv | cut -c1-120
