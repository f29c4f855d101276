set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gbdt.py tests/test_trees_property_gpu.py tests/test_train_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "gbdt or GBDT or hip" > $O/pytest_gbdt.log 2>&1 || { tail -30 $O/pytest_gbdt.log; exit 6; }
tail -2 $O/pytest_gbdt.log
timeout -k 10 300 python tools/gbdt_bench.py > $O/gbdt_bench.jsonl 2>&1 || { tail $O/gbdt_bench.jsonl; exit 7; }
EM_GBDT_SMALL=0 timeout -k 10 300 python tools/gbdt_bench.py reference > $O/gbdt_bench_level_graph.jsonl 2>&1 || { tail $O/gbdt_bench_level_graph.jsonl; exit 8; }
EM_GBDT_SMALL=0 EM_GBDT_GRAPH=0 timeout -k 10 300 python tools/gbdt_bench.py reference > $O/gbdt_bench_level_eager.jsonl 2>&1 || { tail $O/gbdt_bench_level_eager.jsonl; exit 8; }
grep case $O/gbdt_bench*.jsonl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/gbdtprof -o run -- python tools/gbdt_bench.py reference > $O/gbdt_ref_prof.log 2>&1 || { tail $O/gbdt_ref_prof.log; exit 11; }
timeout -k 10 240 python tools/xgmi_budget.py > $O/xgmi_budget.jsonl 2>&1 || { tail -20 $O/xgmi_budget.jsonl; exit 5; }
grep round $O/xgmi_budget.jsonl
timeout -k 10 300 python bench.py --device-data-gb -1 --batch 268435456 --steps 10 --warmup 2 > $O/bench_mega_fill_p09.json 2> $O/bench_mega_fill_p09.err || { tail $O/bench_mega_fill_p09.err; exit 9; }
tail -1 $O/bench_mega_fill_p09.json
timeout -k 10 300 python bench.py --device-data-gb -1 --batch 268435456 --steps 10 --warmup 2 --planted 0.7 > $O/bench_mega_fill_p07.json 2> $O/bench_mega_fill_p07.err || { tail $O/bench_mega_fill_p07.err; exit 10; }
tail -1 $O/bench_mega_fill_p07.json
