#!/bin/bash
# Round-5 batch 14: GBDT update-in-histogram with the previous tree staged in LDS: tests, A/B vs the
# histogram, stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/g16
mkdir -p $O
L=$PWD/euromillioner_amd/lib/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gbdt.py -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
EUROM_NATIVE_LIB=$L/gbdt_nofsplit.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gbdt.py -m gpu > $O/pytest_nofsplit.log 2>&1 || { tail -30 $O/pytest_nofsplit.log; exit 3; }
tail -1 $O/pytest_nofsplit.log
for r in 1 2 3; do
  for v in base gbdt_nofsplit; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_${v}_$r.jsonl 2>&1 || { tail $O/gbdt_${v}_$r.jsonl; exit 4; }
    echo "$v $r $(grep -o '"hip_test_logloss": [0-9.]*, "hip_trees_per_s": [0-9.]*' $O/gbdt_${v}_$r.jsonl)"
  done
done
EUROM_NATIVE_LIB=$L/gbdt_stamps.so timeout -k 10 200 python tools/gbdt_stamps.py > $O/gbdt_stamps.jsonl 2>&1 || { tail $O/gbdt_stamps.jsonl; exit 5; }
grep '^{' $O/gbdt_stamps.jsonl
echo rc=0
