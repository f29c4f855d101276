set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gbdt.py tests/test_trees_property_gpu.py tests/test_train_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "gbdt or GBDT or hip" > $O/pytest_gbdt.log 2>&1 || { tail -30 $O/pytest_gbdt.log; exit 6; }
tail -2 $O/pytest_gbdt.log
for rnd in 1 2; do
  EM_GBDT_GRAPH=0 timeout -k 10 200 python tools/gbdt_bench.py > $O/gbdt_fused_eager_$rnd.jsonl 2>&1 || { tail $O/gbdt_fused_eager_$rnd.jsonl; exit 7; }
  timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_fused_graph_$rnd.jsonl 2>&1 || { tail $O/gbdt_fused_graph_$rnd.jsonl; exit 7; }
done
for f in $O/gbdt_*_?.jsonl; do echo "$f"; grep -o '"case": "[a-z_0-9]*"\|"hip_s": [0-9.]*\|"hip_test_logloss": [0-9.]*\|"hip_exact_s": [0-9.]*' $f | tr '\n' ' '; echo; done
EM_GBDT_GRAPH=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gbdtprof -o run -- python tools/gbdt_bench.py reference > $O/gbdt_prof.log 2>&1 || { tail $O/gbdt_prof.log; exit 9; }
