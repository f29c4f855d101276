#!/bin/bash
# Round-5 final evidence pass: full GPU suite + smoke, driver-shape bench, headline kernel trace + 2 PMC passes,
# the DP=8 exchange proxy, RF and GBDT benches.  Outputs under gpurun_out/g43/ (copied to profiles/r5/); + the wide step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/g43; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 4; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail $O/bench_driver.err; exit 5; }
grep '^{' $O/bench_driver.json | cut -c1-300
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 200 --warmup 5 --no-eval > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 6; }
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc1 -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-eval --graph 0 > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 7; }
cd $R
timeout -k 10 300 python tools/xgmi_budget.py > $O/xgmi_budget_dp8_proxy.jsonl 2> $O/xgmi_budget.err || { tail -20 $O/xgmi_budget.err; exit 8; }
cat $O/xgmi_budget_dp8_proxy.jsonl
for i in 1 2; do timeout -k 10 120 python tools/rf_bench.py >> $O/rf_bench.jsonl 2>&1 || exit 9; done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rf_trace -o run -- python3 $R/tools/rf_bench.py > $O/rf_trace.log 2>&1 || { tail $O/rf_trace.log; exit 10; }
cd $R
for i in 1 2; do timeout -k 10 200 python tools/gbdt_bench.py reference >> $O/gbdt_bench.jsonl 2>&1 || exit 11; done
cat $O/rf_bench.jsonl $O/gbdt_bench.jsonl | cut -c1-250
timeout -k 10 300 python bench.py --model mlp-wide --steps 10 --warmup 3 > $O/bench_wide.json 2> $O/bench_wide.err || { tail $O/bench_wide.err; exit 12; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/bench_wide.json | tr '\n' ' '; echo
echo rc=0
