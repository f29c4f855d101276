set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/g1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_xgmi_proxy_gpu.py tests/test_xgmi_gpu.py tests/test_dp_gpu.py tests/test_train_gpu.py tests/test_fused_mlp_gpu.py > gpurun_out/g1/pytest.log 2>&1 || { tail -50 gpurun_out/g1/pytest.log; exit 3; }
tail -3 gpurun_out/g1/pytest.log
timeout -k 10 300 python tools/xgmi_budget.py > gpurun_out/g1/xgmi_budget.jsonl 2> gpurun_out/g1/xgmi_budget.err || { tail -20 gpurun_out/g1/xgmi_budget.err; exit 4; }
cat gpurun_out/g1/xgmi_budget.jsonl
