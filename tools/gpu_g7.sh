#!/bin/bash
# Round-5 batch 7: LL exchange -- xGMI proxy / IPC / DP tests, DP budget.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/g7
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_xgmi_proxy_gpu.py tests/test_xgmi_gpu.py tests/test_dp_gpu.py tests/test_train_gpu.py -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/xgmi_budget.py > $O/xgmi_budget.jsonl 2> $O/xgmi_budget.err || { tail $O/xgmi_budget.err; exit 4; }
cat $O/xgmi_budget.jsonl
echo rc=0
