set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gbdt.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/t_gbdt.log 2>&1 || { tail -40 $O/t_gbdt.log; exit 3; }
tail -2 $O/t_gbdt.log
timeout -k 10 300 python tools/gbdt_bench.py 262k > $O/gbdt.jsonl 2> $O/gbdt.err || { tail $O/gbdt.err; exit 5; }
cat $O/gbdt.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gbdt_prof -o run -- python tools/gbdt_bench.py 262k > $O/gbdt_prof.log 2>&1 || { tail $O/gbdt_prof.log; exit 6; }
for arm in "old|EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/old.so" "split|EUROM_FUSED_ADAM=0"; do
  name=${arm%%|*}; envs=${arm#*|}
  env $envs timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- python bench.py --steps 200 --warmup 5 --no-eval > $O/$name.log 2>&1 || { tail -30 $O/$name.log; exit 7; }
done
timeout -k 10 300 python bench.py --dtype fp32 --steps 20 --warmup 5 > $O/fp32.json 2> $O/fp32.err || { tail $O/fp32.err; exit 8; }
grep '^{' $O/fp32.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fp32', d['value']/1e6, 'M/s', d['ms_per_step'], d['val']['acc'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fp32_prof -o run -- python bench.py --dtype fp32 --steps 20 --warmup 5 --no-eval > $O/fp32_prof.log 2>&1 || { tail $O/fp32_prof.log; exit 9; }
