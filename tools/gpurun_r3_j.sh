set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3j; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gbdt.py tests/test_gemm_f32_gpu.py tests/test_gemm_gpu.py tests/test_train_gpu.py tests/test_gemm_accum_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 3; }
tail -2 $O/t.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gbdt_prof -o run -- python tools/gbdt_bench.py 262k > $O/gbdt_prof.log 2>&1 || { tail $O/gbdt_prof.log; exit 6; }
grep '^{' $O/gbdt_prof.log
timeout -k 10 300 python tools/gbdt_bench.py > $O/gbdt_all.jsonl 2> $O/gbdt_all.err || { tail $O/gbdt_all.err; exit 7; }
cat $O/gbdt_all.jsonl
timeout -k 10 300 python bench.py --dtype fp32 --steps 20 --warmup 5 > $O/fp32.json 2> $O/fp32.err || { tail $O/fp32.err; exit 8; }
grep '^{' $O/fp32.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fp32', d['value']/1e6, 'M/s', d['ms_per_step'], d['val']['acc'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fp32_prof -o run -- python bench.py --dtype fp32 --steps 20 --warmup 5 --no-eval > $O/fp32_prof.log 2>&1 || { tail $O/fp32_prof.log; exit 9; }
timeout -k 10 300 python bench.py --model mlp-wide --steps 10 --warmup 3 > $O/wide.json 2> $O/wide.err || { tail $O/wide.err; exit 10; }
grep '^{' $O/wide.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('wide', d['value']/1e6, 'M/s', d['ms_per_step'], d['val']['acc'])"
