set -o pipefail
O=gpurun_out/wc; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gemm_accum_gpu.py tests/test_train_gpu.py tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
ARMS="seq|EUROM_WIDE_CONCURRENT=0;conc|EUROM_WIDE_CONCURRENT=1" ROUNDS=3 BENCH_ARGS="--model mlp-wide --steps 10 --warmup 3 --no-eval" bash tools/gpu_ab.sh
