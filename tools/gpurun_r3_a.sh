set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r3a
timeout -k 10 400 python -u -m pytest tests/test_fused_mlp_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3a/t_fused.log 2>&1 || { tail -40 gpurun_out/r3a/t_fused.log; exit 3; }
tail -3 gpurun_out/r3a/t_fused.log
ARMS="old|EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/old.so EUROM_FUSED_ADAM=0;split|EUROM_FUSED_ADAM=0;fused|EUROM_FUSED_ADAM=1" ROUNDS=3 bash tools/gpu_ab.sh || exit 4
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3a/bench_driver.json 2> gpurun_out/r3a/bench_driver.err || { tail gpurun_out/r3a/bench_driver.err; exit 5; }
grep '^{' gpurun_out/r3a/bench_driver.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver-shape', d['value']/1e9, d['ms_per_step'], d['val']['acc'])"
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3a/t_gemm.log 2>&1 || { tail -40 gpurun_out/r3a/t_gemm.log; exit 6; }
tail -3 gpurun_out/r3a/t_gemm.log
