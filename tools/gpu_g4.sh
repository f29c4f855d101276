#!/bin/bash
# Round-5 batch 4: softmax packing A/B (headline), GBDT tests at 128-row chunks, the headline-batch
# gradient test, RF predict kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/g4
mkdir -p $O
L=$PWD/euromillioner_amd/lib/ab
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fused_mlp_gpu.py tests/test_gbdt.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/rfprof -o rf -- python3 $GRAFT_REPO_ROOT/tools/rf_bench.py --repeat 1 > $GRAFT_REPO_ROOT/$O/rf_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/rf_prof.log; exit 3; }
cd $GRAFT_REPO_ROOT
find $O/rfprof -name "*kernel_stats.csv" -exec head -12 {} \; | cut -c1-160
ARMS="base|EUROM_X=0;nopk|EUROM_NATIVE_LIB=$L/nopk.so;noslp|EUROM_NATIVE_LIB=$L/noslp.so;nopk_slp|EUROM_NATIVE_LIB=$L/nopk_slp.so" ROUNDS=3 BENCH_ARGS="--steps 100 --warmup 5 --no-eval" timeout -k 10 600 bash tools/gpu_ab.sh > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 4; }
cp gpurun_out/ab/results.jsonl $O/ab_headline.jsonl
cat $O/ab_headline.jsonl
for v in shipped nopk noslp nopk_slp; do
  if [ $v = shipped ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
  env $E timeout -k 10 120 python tools/ab_hash.py >> $O/hash.jsonl 2>&1 || { tail $O/hash.jsonl; exit 5; }
done
cat $O/hash.jsonl
echo rc=0
