#!/bin/bash
# Round-5 batch 18: GEMM tests after restoring the NT trainer paths (MN forms kept for gemm()), wide bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/g20
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_gbdt.py -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --model mlp-wide --steps 10 --warmup 3 > $O/wide_$r.json 2> $O/wide_$r.err || { tail $O/wide_$r.err; exit 4; }
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/wide_$r.json | tr '\n' ' '; echo
done
echo rc=0
