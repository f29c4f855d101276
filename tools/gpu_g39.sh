#!/bin/bash
# Round-5 batch 37: GBDT split launch with 8 / 16 partial loads in flight per thread (66 / 128 VGPRs) instead
# of 32 (256 VGPRs + AGPRs): tests on the 8-deep build, 3 interleaved rounds of the reference fit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/euromillioner_amd/lib/ab
O=gpurun_out/g39
mkdir -p $O
EUROM_NATIVE_LIB=$L/gbdt_split8.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gbdt.py -m gpu > $O/pytest_split8.log 2>&1 || { tail -40 $O/pytest_split8.log; exit 2; }
tail -1 $O/pytest_split8.log
for r in 1 2 3; do
  for v in base gbdt_split8 gbdt_split16; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_${v}_$r.jsonl 2>&1 || { tail $O/gbdt_${v}_$r.jsonl; exit 3; }
    echo "$v $r $(grep -o '"hip_s": [0-9.]*, "hip_test_logloss": [0-9.]*, "hip_trees_per_s": [0-9.]*' $O/gbdt_${v}_$r.jsonl)"
  done
done
echo rc=0
