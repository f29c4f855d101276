#!/bin/bash
# Round-5 batch 34: fused train kernel without machine-scheduler memory clustering (fused_nocluster) vs the
# shipped build (3 interleaved headline rounds + parameter hash); GBDT max-memory-clause confirmation (3 rounds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/euromillioner_amd/lib/ab
O=gpurun_out/g36
mkdir -p $O
rm -f gpurun_out/ab/results.jsonl
ARMS="base|X=0;fused_nocluster|EUROM_NATIVE_LIB=$L/fused_nocluster.so" ROUNDS=3 bash tools/gpu_ab.sh || exit 2
cp gpurun_out/ab/results.jsonl $O/ab_nocluster.jsonl
EUROM_NATIVE_LIB=$L/fused_nocluster.so timeout -k 10 200 python tools/ab_hash.py > $O/hash_nocluster.jsonl 2>&1 || { tail $O/hash_nocluster.jsonl; exit 3; }
grep '^{' $O/hash_nocluster.jsonl
for r in 1 2 3; do
  for v in gbdt_mc base; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_${v}_$r.jsonl 2>&1 || { tail $O/gbdt_${v}_$r.jsonl; exit 4; }
    echo "$v $r $(grep -o '"hip_s": [0-9.]*, "hip_test_logloss": [0-9.]*, "hip_trees_per_s": [0-9.]*' $O/gbdt_${v}_$r.jsonl)"
  done
done
echo rc=0
