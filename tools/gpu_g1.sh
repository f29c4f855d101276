set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/g1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_xgmi_proxy_gpu.py tests/test_xgmi_gpu.py tests/test_dp_gpu.py tests/test_train_gpu.py tests/test_fused_mlp_gpu.py > gpurun_out/g1/pytest.log 2>&1 || { tail -50 gpurun_out/g1/pytest.log; exit 3; }
tail -3 gpurun_out/g1/pytest.log
timeout -k 10 300 python tools/xgmi_budget.py > gpurun_out/g1/xgmi_budget.jsonl 2> gpurun_out/g1/xgmi_budget.err || { tail -20 gpurun_out/g1/xgmi_budget.err; exit 4; }
cat gpurun_out/g1/xgmi_budget.jsonl
timeout -k 10 200 python tools/adam_probe.py > gpurun_out/g1/adam_probe.jsonl 2>&1 || { tail -20 gpurun_out/g1/adam_probe.jsonl; exit 5; }
cat gpurun_out/g1/adam_probe.jsonl
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_forest.py -m gpu > gpurun_out/g1/pytest_rf.log 2>&1 || { tail -30 gpurun_out/g1/pytest_rf.log; exit 6; }
tail -2 gpurun_out/g1/pytest_rf.log
for i in 1 2; do timeout -k 10 120 python tools/rf_bench.py >> gpurun_out/g1/rf_bench.jsonl 2>&1 || exit 7; done
cat gpurun_out/g1/rf_bench.jsonl
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_gemm_accum_gpu.py tests/test_gemm_property_gpu.py tests/test_perf_guard_gpu.py > gpurun_out/g1/pytest_gemm.log 2>&1 || { tail -30 gpurun_out/g1/pytest_gemm.log; exit 8; }
tail -2 gpurun_out/g1/pytest_gemm.log
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gbdt.py -m gpu > gpurun_out/g1/pytest_gbdt.log 2>&1 || { tail -30 gpurun_out/g1/pytest_gbdt.log; exit 10; }
tail -2 gpurun_out/g1/pytest_gbdt.log
