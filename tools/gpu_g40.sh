#!/bin/bash
# Round-5 batch 38: base = split launch prefetch 8 (adopted); gbdt_hsplit4 = the in-pass root split with 4 loads in flight per
# thread (69 VGPRs) instead of 16; gbdt_split4 = the split launch with 4: tests + 3 interleaved rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/euromillioner_amd/lib/ab
O=gpurun_out/g40
mkdir -p $O
EUROM_NATIVE_LIB=$L/gbdt_hsplit4.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gbdt.py -m gpu > $O/pytest_hsplit4.log 2>&1 || { tail -40 $O/pytest_hsplit4.log; exit 2; }
tail -1 $O/pytest_hsplit4.log
for r in 1 2 3; do
  for v in base gbdt_hsplit4 gbdt_split4; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_${v}_$r.jsonl 2>&1 || { tail $O/gbdt_${v}_$r.jsonl; exit 3; }
    echo "$v $r $(grep -o '"hip_s": [0-9.]*, "hip_test_logloss": [0-9.]*, "hip_trees_per_s": [0-9.]*' $O/gbdt_${v}_$r.jsonl)"
  done
done
echo rc=0
