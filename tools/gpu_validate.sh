# Full validation of the tree as the driver sees it: GPU suite, smoke(), default bench
set -o pipefail
mkdir -p gpurun_out/val
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/val/gpu_tests.log 2>&1 || { tail -40 gpurun_out/val/gpu_tests.log; exit 3; }
tail -1 gpurun_out/val/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/val/smoke.log 2>&1 || { tail -20 gpurun_out/val/smoke.log; exit 4; }
tail -1 gpurun_out/val/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/val/bench_default.json 2> gpurun_out/val/bench_default.err || { tail -20 gpurun_out/val/bench_default.err; exit 5; }
grep '^{' gpurun_out/val/bench_default.json | tail -1
