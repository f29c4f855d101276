set -o pipefail
L=$PWD/euromillioner_amd/lib/ab
mkdir -p gpurun_out/tr
EUROM_FUSED_V=8 timeout -k 10 300 python -u -m pytest tests/test_fused_mlp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tr/pytest.log 2>&1 || { tail -30 gpurun_out/tr/pytest.log; exit 2; }
tail -1 gpurun_out/tr/pytest.log
EUROM_FUSED_V=8 EUROM_NATIVE_LIB=$L/trace.so timeout -k 10 120 python tools/fused_trace.py > gpurun_out/tr/trace_pipe1.txt 2>&1 || { tail gpurun_out/tr/trace_pipe1.txt; exit 3; }
tail -9 gpurun_out/tr/trace_pipe1.txt
ARMS="v6|EUROM_FUSED_V=6;v8|EUROM_FUSED_V=8" ROUNDS=3 bash tools/gpu_ab.sh
timeout -k 10 400 python -u -m pytest tests/test_dp_gpu.py::test_bench_xgmi_fault_falls_back_to_rccl tests/test_train_gpu.py::test_rccl_step_replays_from_a_hipgraph -x -v --timeout 200 --timeout-method thread > gpurun_out/tr/pytest_fallback.log 2>&1 || { tail -40 gpurun_out/tr/pytest_fallback.log; exit 5; }
tail -3 gpurun_out/tr/pytest_fallback.log
