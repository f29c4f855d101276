#!/bin/bash
# Round-5 batch 29: GBDT (scratch-free hist kernel, split prefetch sized by block) base vs HEAD (gbdt_prev) vs 1024-thread blocks and up to 16 row phases (shorter per-thread
# RMW chains; LDS budget 128 KB = gbdt_t1024, 72 KB = gbdt_prev) vs the 512-thread / 8-phase base.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/g31
mkdir -p $O
L=$R/euromillioner_amd/lib/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gbdt.py -m gpu > $O/pytest_t1024.log 2>&1 || { tail -40 $O/pytest_t1024.log; exit 2; }
tail -1 $O/pytest_t1024.log
for r in 1 2 3; do
  for v in base gbdt_t1024 gbdt_prev; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_${v}_$r.jsonl 2>&1 || { tail $O/gbdt_${v}_$r.jsonl; exit 3; }
    echo "$v $r $(grep -o '"hip_s": [0-9.]*, "hip_test_logloss": [0-9.]*, "hip_trees_per_s": [0-9.]*' $O/gbdt_${v}_$r.jsonl)"
  done
done
echo rc=0
