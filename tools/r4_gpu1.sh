set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4a
timeout -k 10 300 python -u -m pytest tests/test_fused_mlp_gpu.py -x -v --timeout 120 --timeout-method thread -k "not f32" > gpurun_out/r4a/pytest.log 2>&1 || { tail -30 gpurun_out/r4a/pytest.log; exit 3; }
tail -3 gpurun_out/r4a/pytest.log
rm -rf gpurun_out/ab
ARMS="v7|X=1;v6|EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/v6.so" ROUNDS=3 BENCH_ARGS="--steps 100 --warmup 5" bash tools/gpu_ab.sh || exit 4
cp gpurun_out/ab/results.jsonl gpurun_out/r4a/ab.jsonl
