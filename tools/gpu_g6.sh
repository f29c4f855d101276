#!/bin/bash
# Round-5 batch 6: RF predict (full-tree staging) tests + bench; DP proxy budget (nowait / flags / copy).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/g6
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_forest.py tests/test_xgmi_proxy_gpu.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
for r in 1 2; do timeout -k 10 200 python tools/rf_bench.py > $O/rf_bench_$r.jsonl 2>&1 || { tail $O/rf_bench_$r.jsonl; exit 3; }; grep -o '"predict_s": [0-9.e-]*' $O/rf_bench_$r.jsonl; done
timeout -k 10 300 python tools/xgmi_budget.py > $O/xgmi_budget.jsonl 2> $O/xgmi_budget.err || { tail $O/xgmi_budget.err; exit 4; }
cat $O/xgmi_budget.jsonl
echo rc=0
