set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3l; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gbdt.py tests/test_small_ops_property_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 3; }
tail -2 $O/t.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gbdt_prof -o run -- python tools/gbdt_bench.py 262k > $O/gbdt_prof.log 2>&1 || { tail $O/gbdt_prof.log; exit 6; }
grep '^{' $O/gbdt_prof.log
