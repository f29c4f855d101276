#!/bin/bash
# Round-5 batch 25: GEMM tests after removing the superseded skinny-K store forms; quick wide bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/g27
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > $O/pytest_gemm.log 2>&1 || { tail -40 $O/pytest_gemm.log; exit 2; }
tail -1 $O/pytest_gemm.log
timeout -k 10 300 python bench.py --model mlp-wide --steps 10 --warmup 3 > $O/wide.json 2> $O/wide.err || { tail $O/wide.err; exit 3; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"acc": [0-9.]*' $O/wide.json | tr '\n' ' '; echo
echo rc=0
