set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dp_gpu.py -x -v --timeout 200 --timeout-method thread -k "wide" > $O/pytest_dp.log 2>&1 || { tail -30 $O/pytest_dp.log; exit 3; }
grep -E "PASS|SKIP|FAIL" $O/pytest_dp.log | tail -6
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/wo -o run -- python tools/wide_overlap.py > $O/wide_overlap.jsonl 2> $O/wide_overlap.err || { tail $O/wide_overlap.err; exit 4; }
cat $O/wide_overlap.jsonl
f=$(ls $O/wo/*/run_kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find $O/wo -name "*kernel_trace.csv" | head -1)
python tools/wide_overlap.py report $f > $O/wide_overlap_report.jsonl && cat $O/wide_overlap_report.jsonl
timeout -k 10 240 python tools/xgmi_budget.py > $O/xgmi_budget.jsonl 2>&1 || { tail -20 $O/xgmi_budget.jsonl; exit 5; }
cat $O/xgmi_budget.jsonl
