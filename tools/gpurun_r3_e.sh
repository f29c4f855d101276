set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gbdt.py tests/test_fused_mlp_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 3; }
tail -2 $O/t.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gbdt_prof -o run -- python tools/gbdt_bench.py 262k > $O/gbdt_prof.log 2>&1 || { tail $O/gbdt_prof.log; exit 6; }
grep '^{' $O/gbdt_prof.log
ARMS="old|EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/old.so;split|EUROM_FUSED_ADAM=0" ROUNDS=3 bash tools/gpu_ab.sh || exit 4
timeout -k 10 400 python -u -m pytest tests/test_dp_gpu.py -x -v --timeout 300 --timeout-method thread -k wide > $O/t_dp.log 2>&1 || { tail -40 $O/t_dp.log; exit 7; }
tail -6 $O/t_dp.log
timeout -k 10 300 python tools/wide_overlap.py > $O/overlap.jsonl 2> $O/overlap.err || { tail $O/overlap.err; exit 8; }
cat $O/overlap.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/overlap_prof -o run -- python tools/wide_overlap.py > $O/overlap_prof.log 2>&1 || { tail $O/overlap_prof.log; exit 9; }
