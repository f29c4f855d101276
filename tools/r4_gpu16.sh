set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_forest.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_rf.log 2>&1 || { tail -30 $O/pytest_rf.log; exit 6; }
tail -2 $O/pytest_rf.log
for rnd in 1 2; do
  timeout -k 10 120 python tools/rf_bench.py > $O/rf_ybits_$rnd.jsonl 2>&1 || { tail $O/rf_ybits_$rnd.jsonl; exit 7; }
  EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/rf_ybits_cntsep.so timeout -k 10 120 python tools/rf_bench.py > $O/rf_ybitscntsep_$rnd.jsonl 2>&1 || { tail $O/rf_ybitscntsep_$rnd.jsonl; exit 8; }
  EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/rf_noybits.so timeout -k 10 120 python tools/rf_bench.py > $O/rf_noybits_$rnd.jsonl 2>&1 || { tail $O/rf_noybits_$rnd.jsonl; exit 8; }
done
for f in $O/rf_*_?.jsonl; do echo "$f $(grep -o '"fit_s": [0-9.]*' $f | tr '\n' ' ')"; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rfprof -o run -- python tools/rf_bench.py --repeat 2 > $O/rf_prof.log 2>&1 || { tail $O/rf_prof.log; exit 12; }
timeout -k 10 300 python -u -m pytest tests/test_gbdt.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gbdt.log 2>&1 || { tail -30 $O/pytest_gbdt.log; exit 13; }
tail -1 $O/pytest_gbdt.log
for rnd in 1 2 3; do timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_$rnd.jsonl 2>&1 || { tail $O/gbdt_$rnd.jsonl; exit 14; }; done
grep -h -o '"hip_s": [0-9.]*' $O/gbdt_?.jsonl
