set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gbdt.py tests/test_forest.py tests/test_trees_property_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_trees.log 2>&1 || { tail -30 $O/pytest_trees.log; exit 6; }
tail -2 $O/pytest_trees.log
for rnd in 1 2; do
  EM_GBDT_GRAPH=0 timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_fused_eager_$rnd.jsonl 2>&1 || { tail $O/gbdt_fused_eager_$rnd.jsonl; exit 7; }
  timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_fused_graph_$rnd.jsonl 2>&1 || { tail $O/gbdt_fused_graph_$rnd.jsonl; exit 7; }
  EM_GBDT_FUSE=0 EM_GBDT_GRAPH=0 timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_sep_eager_$rnd.jsonl 2>&1 || { tail $O/gbdt_sep_eager_$rnd.jsonl; exit 8; }
done
for f in $O/gbdt_*_?.jsonl; do echo "$f $(grep -o '"hip_s": [0-9.]*' $f) $(grep -o '"hip_test_logloss": [0-9.]*' $f)"; done
EM_GBDT_GRAPH=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gbdtprof -o run -- python tools/gbdt_bench.py reference > $O/gbdt_prof.log 2>&1 || { tail $O/gbdt_prof.log; exit 9; }
for rnd in 1 2; do
  timeout -k 10 120 python tools/rf_bench.py > $O/rf_new_$rnd.jsonl 2>&1 || { tail $O/rf_new_$rnd.jsonl; exit 10; }
  EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/rf_old.so timeout -k 10 120 python tools/rf_bench.py > $O/rf_old_$rnd.jsonl 2>&1 || { tail $O/rf_old_$rnd.jsonl; exit 11; }
done
for f in $O/rf_*_?.jsonl; do echo "$f $(grep -o '"fit_s": [0-9.]*' $f | tr '\n' ' ')"; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rfprof -o run -- python tools/rf_bench.py --repeat 2 > $O/rf_prof.log 2>&1 || { tail $O/rf_prof.log; exit 12; }
