#!/bin/bash
# Round-5 batch 11: adopted GBDT 512-thread histogram + RF select-addressed leaf reads: tests, benches,
# GBDT host-overhead profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/g11
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gbdt.py tests/test_forest.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
for r in 1 2; do timeout -k 10 200 python tools/rf_bench.py > $O/rf_bench_$r.jsonl 2>&1 || exit 3; grep -o '"predict_s": [0-9.e-]*' $O/rf_bench_$r.jsonl; done
for r in 1 2; do timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_bench_$r.jsonl 2>&1 || exit 4; grep -o '"hip_s": [0-9.]*, "hip_test_logloss": [0-9.]*, "hip_trees_per_s": [0-9.]*' $O/gbdt_bench_$r.jsonl; done
timeout -k 10 300 python tools/gbdt_fit_profile.py > $O/gbdt_fit_profile.txt 2>&1 || { tail -20 $O/gbdt_fit_profile.txt; exit 5; }
head -60 $O/gbdt_fit_profile.txt
echo rc=0
