#!/bin/bash
# Round-5 same-box A/Bs: headline step (fused-kernel b2 placement, Adam slab-reduction shapes) and the
# GBDT reference fit (histogram chunk size).  Side libraries: tools/build_variant.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/g2
L=$PWD/euromillioner_amd/lib/ab
ARMS="base|EUROM_X=0;b2early|EUROM_NATIVE_LIB=$L/b2early.so;swap_orig|EUROM_NATIVE_LIB=$L/swap_orig.so;swap_b2e|EUROM_NATIVE_LIB=$L/swap_b2e.so;adam_g32|EUROM_NATIVE_LIB=$L/adam_g32.so;adam_nt|EUROM_NATIVE_LIB=$L/adam_nt.so" ROUNDS=3 BENCH_ARGS="--steps 100 --warmup 5 --no-eval" timeout -k 10 900 bash tools/gpu_ab.sh > gpurun_out/g2/ab.log 2>&1 || { tail -20 gpurun_out/g2/ab.log; exit 3; }
cp gpurun_out/ab/results.jsonl gpurun_out/g2/ab_headline.jsonl
for r in 1 2; do
  for v in base gbdt_chunk128 gbdt_chunk256; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/gbdt_bench.py reference > gpurun_out/g2/gbdt_${v}_$r.jsonl 2>&1 || { tail gpurun_out/g2/gbdt_${v}_$r.jsonl; exit 4; }
    echo "$v $r $(grep -o '"hip_s": [0-9.]*' gpurun_out/g2/gbdt_${v}_$r.jsonl)"
  done
done
cat gpurun_out/g2/ab_headline.jsonl
EUROM_NATIVE_LIB=$L/stamps.so TL_B=1048576 timeout -k 10 200 python tools/fused_timeline.py > gpurun_out/g2/timeline.txt 2>&1 || { tail -20 gpurun_out/g2/timeline.txt; exit 5; }
cat gpurun_out/g2/timeline.txt
for v in shipped b2early swap_orig swap_b2e adam_g32 adam_nt; do
  if [ $v = shipped ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
  env $E timeout -k 10 120 python tools/ab_hash.py >> gpurun_out/g2/hash.jsonl 2>&1 || { tail gpurun_out/g2/hash.jsonl; exit 6; }
done
cat gpurun_out/g2/hash.jsonl
timeout -k 10 300 python tools/gemm_bench.py --cases fwd_hidden_ct,fwd_hidden,dgrad_hidden_nt,wgrad_hidden_nt,transpose,fwd_in,fwd_out > gpurun_out/g2/gemm_bench.jsonl 2>&1 || { tail gpurun_out/g2/gemm_bench.jsonl; exit 7; }
cat gpurun_out/g2/gemm_bench.jsonl
timeout -k 10 200 python tools/xgmi_budget.py > gpurun_out/g2/xgmi_budget.jsonl 2> gpurun_out/g2/xgmi_budget.err || { tail gpurun_out/g2/xgmi_budget.err; exit 8; }
cat gpurun_out/g2/xgmi_budget.jsonl
timeout -k 10 120 python -u -m pytest -x -v --timeout 110 --timeout-method thread tests/test_forest.py -m gpu -k "predict" > gpurun_out/g2/pytest_rf.log 2>&1 || { tail -30 gpurun_out/g2/pytest_rf.log; exit 9; }
for r in 1 2; do timeout -k 10 200 python tools/rf_bench.py --rows 1000000 > gpurun_out/g2/rf_bench_$r.jsonl 2>&1 || { tail gpurun_out/g2/rf_bench_$r.jsonl; exit 10; }; cat gpurun_out/g2/rf_bench_$r.jsonl; done
echo rc=0
