# RF: oracle tests (both histogram kernels), bench with the MFMA histogram on/off, kernel stats
set -o pipefail
mkdir -p gpurun_out/rf
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_forest.py -x -q -m gpu --timeout 180 --timeout-method thread > gpurun_out/rf/t.log 2>&1 || { tail -30 gpurun_out/rf/t.log; exit 3; }
tail -1 gpurun_out/rf/t.log
EM_RF_MFMA=0 timeout -k 10 300 python tools/rf_bench.py --rows 700000 > gpurun_out/rf/atomic.json 2>/dev/null || exit 4
timeout -k 10 300 python tools/rf_bench.py --rows 700000 > gpurun_out/rf/mfma.json 2>/dev/null || exit 5
python -c "import json;a=json.loads(open('gpurun_out/rf/atomic.json').read().splitlines()[-1]);b=json.loads(open('gpurun_out/rf/mfma.json').read().splitlines()[-1]);print('atomic fit',a['fit_s'],'acc',a['val']['acc'],' mfma fit',b['fit_s'],'acc',b['val']['acc'], 'nodes', a['nodes_split'], b['nodes_split'])"
cd /tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rf/prof -o run --output-format csv -- python tools/rf_bench.py --rows 700000 --repeat 2 > gpurun_out/rf/prof.log 2>&1 || exit 6
