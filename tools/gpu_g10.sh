#!/bin/bash
# Round-5 batch 10: RF predict variants (12 waves x 2 groups vs 8 waves x 3 groups; leaf-read schedules).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/g10
mkdir -p $O
L=$PWD/euromillioner_amd/lib/ab
for v in rf_v2 rf8 rf8v2; do
  EUROM_NATIVE_LIB=$L/$v.so timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_forest.py -m gpu -k predict > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 2; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for r in 1 2 3; do
  for v in base rf_v2 rf8 rf8v2; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/rf_bench.py > $O/rf_${v}_$r.jsonl 2>&1 || { tail $O/rf_${v}_$r.jsonl; exit 3; }
    echo "$v $r $(grep -o '"predict_s": [0-9.e-]*' $O/rf_${v}_$r.jsonl)"
  done
done

EUROM_NATIVE_LIB=$L/gbdt_stamps.so timeout -k 10 200 python tools/gbdt_stamps.py > $O/gbdt_stamps.jsonl 2>&1 || { tail $O/gbdt_stamps.jsonl; exit 4; }
grep '^{' $O/gbdt_stamps.jsonl
for v in gbdt_h512c256 gbdt_h512c128; do
  EUROM_NATIVE_LIB=$L/$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gbdt.py -m gpu > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 5; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for r in 1 2 3; do
  for v in base gbdt_h512c256 gbdt_h512c128; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_${v}_$r.jsonl 2>&1 || { tail $O/gbdt_${v}_$r.jsonl; exit 6; }
    echo "$v $r $(grep -o '"hip_trees_per_s": [0-9.]*' $O/gbdt_${v}_$r.jsonl)"
  done
done
echo rc=0
