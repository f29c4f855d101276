#!/bin/bash
# Round-5 batch 8: GBDT histogram batched updates (A/B vs the previous loop, batch 8, chunk 64/256) + tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/g8
mkdir -p $O
L=$PWD/euromillioner_amd/lib/ab
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gbdt.py -m gpu > $O/pytest_gbdt.log 2>&1 || { tail -30 $O/pytest_gbdt.log; exit 2; }
tail -1 $O/pytest_gbdt.log
for r in 1 2 3; do
  for v in base gbdt_old gbdt_b8 gbdt_b4c256 gbdt_b4c64; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_${v}_$r.jsonl 2>&1 || { tail $O/gbdt_${v}_$r.jsonl; exit 4; }
    echo "$v $r $(grep -o '"hip_trees_per_s": [0-9.]*' $O/gbdt_${v}_$r.jsonl)"
  done
done

timeout -k 10 300 python tools/xgmi_budget.py > $O/xgmi_budget.jsonl 2> $O/xgmi_budget.err || { tail $O/xgmi_budget.err; exit 5; }
cat $O/xgmi_budget.jsonl
echo rc=0
