# RF fused partition + child histograms: bit-exact tests vs the numpy oracle, fit-time A/B (EM_RF_FUSE=0 vs 1)
set -o pipefail
mkdir -p gpurun_out/rff
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_forest.py tests/test_trees_property_gpu.py tests/test_train_gpu.py -k "forest or rf or tree" -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/rff/t.log 2>&1 || { grep -E "PASSED|FAILED|Error|assert" gpurun_out/rff/t.log | tail -30; exit 3; }
tail -1 gpurun_out/rff/t.log
EM_RF_FUSE=0 timeout -k 10 400 python -u -m pytest tests/test_forest.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/rff/t0.log 2>&1 || { tail -20 gpurun_out/rff/t0.log; exit 4; }
tail -1 gpurun_out/rff/t0.log
for r in 1 2; do
  for d in 0 1; do
    EM_RF_FUSE=$d timeout -k 10 200 python tools/rf_bench.py > gpurun_out/rff/b_${d}_$r.log 2>&1 || { tail -5 gpurun_out/rff/b_${d}_$r.log; exit 5; }
    grep '^{' gpurun_out/rff/b_${d}_$r.log | tail -1 | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('fuse=$d', 'rows', j['rows'], 'fit_ms %.2f' % (j['fit_s']*1e3), 'nodes_split', j['nodes_split'], 'val_acc %.4f' % j['val']['acc'])"
  done
done
timeout -k 10 200 python tools/rf_bench.py --rows 700000 > gpurun_out/rff/b_700k.log 2>&1 || exit 6
grep '^{' gpurun_out/rff/b_700k.log | tail -1 | cut -c1-200
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rff/prof -o run -- python3 tools/rf_bench.py --repeat 2 > gpurun_out/rff/prof.log 2>&1 || exit 7
head -8 gpurun_out/rff/prof/run_kernel_stats.csv | cut -c1-120
