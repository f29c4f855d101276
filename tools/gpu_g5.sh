#!/bin/bash
# Round-5 batch 5: RF predict (12-wave streamed kernel) tests + bench + trace; DP proxy kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/g5
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_forest.py -m gpu > $O/pytest_rf.log 2>&1 || { tail -30 $O/pytest_rf.log; exit 2; }
tail -1 $O/pytest_rf.log
for r in 1 2; do timeout -k 10 200 python tools/rf_bench.py > $O/rf_bench_$r.jsonl 2>&1 || { tail $O/rf_bench_$r.jsonl; exit 3; }; grep -o '"predict_s": [0-9.e-]*' $O/rf_bench_$r.jsonl; done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/rfprof -o rf --output-format csv -- python3 $R/tools/rf_bench.py --repeat 1 > $R/$O/rf_prof.log 2>&1 || { tail -20 $R/$O/rf_prof.log; exit 4; }
XB_ROUNDS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/xgprof -o xg --output-format csv -- python3 $R/tools/xgmi_budget.py > $R/$O/xg_prof.log 2>&1 || { tail -20 $R/$O/xg_prof.log; exit 5; }
cd $R
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-4 $f | head -12 | cut -c1-150; done
echo rc=0
