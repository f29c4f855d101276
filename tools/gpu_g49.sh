#!/bin/bash
# Round-5 batch 47: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs host memory (=0) vs the
# runtime default: GBDT reference fit (launch-chain bound) and the headline step; 3 interleaved rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/g49
mkdir -p $O
for r in 1 2 3; do
  for v in default dev1 dev0; do
    case $v in default) E="X=0";; dev1) E="HIP_FORCE_DEV_KERNARG=1";; dev0) E="HIP_FORCE_DEV_KERNARG=0";; esac
    env $E timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_${v}_$r.jsonl 2>&1 || { tail $O/gbdt_${v}_$r.jsonl; exit 3; }
    echo "$v $r $(grep -o '"hip_s": [0-9.]*, "hip_test_logloss": [0-9.]*, "hip_trees_per_s": [0-9.]*' $O/gbdt_${v}_$r.jsonl)"
  done
done
rm -f gpurun_out/ab/results.jsonl
ARMS="default|X=0;dev1|HIP_FORCE_DEV_KERNARG=1;dev0|HIP_FORCE_DEV_KERNARG=0" ROUNDS=2 bash tools/gpu_ab.sh || exit 2
cp gpurun_out/ab/results.jsonl $O/ab_kernarg.jsonl
echo rc=0
