# session-3 baseline: GPU tests, driver-shape bench, step composition
set -o pipefail
mkdir -p gpurun_out/e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e/pytest.log 2>&1 || { tail -30 gpurun_out/e/pytest.log; exit 3; }
tail -2 gpurun_out/e/pytest.log
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/e/bench20.json 2> gpurun_out/e/bench20.err || exit 4
timeout -k 10 120 python bench.py --steps 1000 --warmup 10 --no-eval > gpurun_out/e/bench1000.json 2> gpurun_out/e/bench1000.err || exit 5
timeout -k 10 120 python tools/step_parts.py > gpurun_out/e/parts.jsonl 2> gpurun_out/e/parts.err || exit 6
cat gpurun_out/e/bench20.json gpurun_out/e/parts.jsonl
