# v6 default: full GPU tests, driver-shape bench, 200-step bench, rocprof kernel stats, step parts
set -o pipefail
mkdir -p gpurun_out/g
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g/pytest.log 2>&1 || { tail -40 gpurun_out/g/pytest.log; exit 3; }
tail -2 gpurun_out/g/pytest.log
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/g/bench20.json 2> gpurun_out/g/bench20.err || exit 4
timeout -k 10 120 python bench.py --steps 200 --warmup 10 > gpurun_out/g/bench200.json 2> gpurun_out/g/bench200.err || exit 5
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/g/prof -o run --output-format csv -- python bench.py --steps 200 --warmup 10 --no-eval > gpurun_out/g/prof.log 2>&1 || exit 6
STEP_PARTS_B=1048576,2097152,4194304 timeout -k 10 120 python tools/step_parts.py > gpurun_out/g/parts.jsonl 2>&1 || exit 7
cat gpurun_out/g/bench20.json gpurun_out/g/parts.jsonl
