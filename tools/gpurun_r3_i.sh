set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3i; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gbdt.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 3; }
tail -2 $O/t.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gbdt_prof -o run -- python tools/gbdt_bench.py 262k > $O/gbdt_prof.log 2>&1 || { tail $O/gbdt_prof.log; exit 6; }
grep '^{' $O/gbdt_prof.log
timeout -k 10 300 python tools/gbdt_bench.py > $O/gbdt_all.jsonl 2> $O/gbdt_all.err || { tail $O/gbdt_all.err; exit 7; }
cat $O/gbdt_all.jsonl
