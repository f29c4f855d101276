set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4b; mkdir -p $O
L=$PWD/euromillioner_amd/lib/ab
TL_B=1048576 TL_V7=1 EUROM_NATIVE_LIB=$L/stamps7.so timeout -k 10 120 python tools/fused_timeline.py > $O/tl_v7.txt 2>&1 || { tail $O/tl_v7.txt; exit 3; }
TL_B=1048576 TL_V7=0 EUROM_NATIVE_LIB=$L/stamps6.so timeout -k 10 120 python tools/fused_timeline.py > $O/tl_v6.txt 2>&1 || { tail $O/tl_v6.txt; exit 4; }
cat $O/tl_v7.txt $O/tl_v6.txt
rm -rf gpurun_out/ab
ARMS="v7|X=1;v6|EUROM_NATIVE_LIB=$L/v6.so;v6s3|EUROM_NATIVE_LIB=$L/v6s3.so" ROUNDS=2 BENCH_ARGS="--steps 100 --warmup 5 --no-eval" bash tools/gpu_ab.sh || exit 5
cp gpurun_out/ab/results.jsonl $O/ab.jsonl
