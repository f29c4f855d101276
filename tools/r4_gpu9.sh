set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gbdt.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gbdt.log 2>&1 || { tail -30 $O/pytest_gbdt.log; exit 6; }
tail -2 $O/pytest_gbdt.log
for rnd in 1 2; do
  timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_small_$rnd.jsonl 2>&1 || { tail $O/gbdt_small_$rnd.jsonl; exit 7; }
  EM_GBDT_SMALL=0 timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_level_graph_$rnd.jsonl 2>&1 || { tail $O/gbdt_level_graph_$rnd.jsonl; exit 8; }
  EM_GBDT_SMALL=0 EM_GBDT_GRAPH=0 timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_level_eager_$rnd.jsonl 2>&1 || { tail $O/gbdt_level_eager_$rnd.jsonl; exit 8; }
done
for f in $O/gbdt_*_?.jsonl; do echo "$f $(grep -o '"hip_s": [0-9.]*' $f)"; done
EM_GBDT_SMALL_STAMPS=$PWD/$O/small_stamps.jsonl timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_stamps_run.jsonl 2>&1 || { tail $O/gbdt_stamps_run.jsonl; exit 9; }
tail -2 $O/small_stamps.jsonl | cut -c1-600
