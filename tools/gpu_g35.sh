#!/bin/bash
# Round-5 batch 33: max-memory-clause scheduling for the Adam, GBDT and RF kernels (side builds) vs the default:
# headline step (Adam), GBDT reference fit, RF fit/predict; 3 interleaved rounds each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/euromillioner_amd/lib/ab
O=gpurun_out/g35
mkdir -p $O
rm -f gpurun_out/ab/results.jsonl
ARMS="base|X=0;adam_mc|EUROM_NATIVE_LIB=$L/adam_mc.so" ROUNDS=3 bash tools/gpu_ab.sh || exit 2
cp gpurun_out/ab/results.jsonl $O/ab_adam_mc.jsonl
for r in 1 2 3; do
  for v in base gbdt_mc; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_${v}_$r.jsonl 2>&1 || { tail $O/gbdt_${v}_$r.jsonl; exit 3; }
    echo "$v $r $(grep -o '"hip_s": [0-9.]*, "hip_test_logloss": [0-9.]*, "hip_trees_per_s": [0-9.]*' $O/gbdt_${v}_$r.jsonl)"
  done
done
for r in 1 2 3; do
  for v in base rf_mc; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/rf_bench.py > $O/rf_${v}_$r.jsonl 2>&1 || { tail $O/rf_${v}_$r.jsonl; exit 4; }
    echo "$v $r $(grep -o '"fit_s": [0-9.]*\|"predict_s": [0-9.]*' $O/rf_${v}_$r.jsonl | tr '\n' ' ')"
  done
done
echo rc=0
