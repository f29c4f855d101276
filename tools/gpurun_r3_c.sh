set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r3c
timeout -k 10 500 python -u -m pytest tests/test_fused_mlp_gpu.py tests/test_gbdt.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r3c/t.log 2>&1 || { tail -40 gpurun_out/r3c/t.log; exit 3; }
tail -3 gpurun_out/r3c/t.log
ARMS="old|EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/old.so EUROM_FUSED_ADAM=0;split|EUROM_FUSED_ADAM=0;fused|EUROM_FUSED_ADAM=1" ROUNDS=3 bash tools/gpu_ab.sh || exit 4
timeout -k 10 300 python tools/gbdt_bench.py 262k > gpurun_out/r3c/gbdt.jsonl 2> gpurun_out/r3c/gbdt.err || { tail gpurun_out/r3c/gbdt.err; exit 5; }
cat gpurun_out/r3c/gbdt.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3c/gbdt_prof -o run -- python tools/gbdt_bench.py 262k > gpurun_out/r3c/gbdt_prof.log 2>&1 || { tail gpurun_out/r3c/gbdt_prof.log; exit 6; }
