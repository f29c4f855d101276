set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4c; mkdir -p $O
L=$PWD/euromillioner_amd/lib/ab
timeout -k 10 300 python -u -m pytest tests/test_fused_mlp_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 3; }
tail -2 $O/pytest.log
EUROM_NATIVE_LIB=$L/v7s.so timeout -k 10 300 python -u -m pytest tests/test_fused_mlp_gpu.py -x -q --timeout 120 --timeout-method thread -k "not f32" > $O/pytest7.log 2>&1 || { tail -30 $O/pytest7.log; exit 3; }
tail -2 $O/pytest7.log
TL_B=1048576 TL_SHARED=1 EUROM_NATIVE_LIB=$L/stamps.so timeout -k 10 120 python tools/fused_timeline.py > $O/tl_s.txt 2>&1 || { tail $O/tl_s.txt; exit 4; }
TL_B=1048576 TL_SHARED=1 TL_V7=1 EUROM_NATIVE_LIB=$L/stamps7s.so timeout -k 10 120 python tools/fused_timeline.py > $O/tl_7s.txt 2>&1 || { tail $O/tl_7s.txt; exit 4; }
cat $O/tl_s.txt $O/tl_7s.txt
rm -rf gpurun_out/ab
ARMS="shared|X=1;units|EUROM_NATIVE_LIB=$L/v6u.so;v7s|EUROM_NATIVE_LIB=$L/v7s.so" ROUNDS=2 BENCH_ARGS="--steps 100 --warmup 5 --no-eval" bash tools/gpu_ab.sh || exit 5
cp gpurun_out/ab/results.jsonl $O/ab.jsonl
timeout -k 10 400 python -u -m pytest tests/test_trees_property_gpu.py tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread -k "gbdt or GBDT" > $O/pytest_gbdt.log 2>&1 || { tail -30 $O/pytest_gbdt.log; exit 6; }
tail -2 $O/pytest_gbdt.log
timeout -k 10 300 python tools/gbdt_bench.py hip > $O/gbdt_bench.jsonl 2>&1 || { tail $O/gbdt_bench.jsonl; exit 7; }
EM_GBDT_GRAPH=0 timeout -k 10 300 python tools/gbdt_bench.py reference > $O/gbdt_bench_eager.jsonl 2>&1 || { tail $O/gbdt_bench_eager.jsonl; exit 8; }
cat $O/gbdt_bench.jsonl $O/gbdt_bench_eager.jsonl
