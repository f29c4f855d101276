set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4d; mkdir -p $O
L=$PWD/euromillioner_amd/lib/ab
timeout -k 10 300 python -u -m pytest tests/test_fused_mlp_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -2 $O/pytest.log
TL_B=1048576 TL_SHARED=1 EUROM_NATIVE_LIB=$L/stamps.so timeout -k 10 120 python tools/fused_timeline.py > $O/tl_s.txt 2>&1 || { tail $O/tl_s.txt; exit 4; }
cat $O/tl_s.txt
rm -rf gpurun_out/ab
ARMS="shared|X=1;units|EUROM_NATIVE_LIB=$L/v6u.so;v7s|EUROM_NATIVE_LIB=$L/v7s.so;r3|EUROM_NATIVE_LIB=$L/r3.so" ROUNDS=2 BENCH_ARGS="--steps 100 --warmup 5 --no-eval" bash tools/gpu_ab.sh || exit 5
cp gpurun_out/ab/results.jsonl $O/ab.jsonl
