#!/bin/bash
# Round-5 batch 15: 256-tile GEMM with MN-contiguous operands (wide MLP without transposed copies):
# GEMM tests, per-GEMM A/B (MN vs NT), wide bench new vs HEAD tree (same box), kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/g17
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > $O/pytest_gemm.log 2>&1 || { tail -40 $O/pytest_gemm.log; exit 2; }
tail -1 $O/pytest_gemm.log
timeout -k 10 300 python tools/gemm_bench.py --no-lib --iters 10 --cases dgrad_hidden_nt,dgrad_hidden,wgrad_hidden_nt,wgrad_hidden,fwd_hidden > $O/gemm_bench.jsonl 2>&1 || { tail $O/gemm_bench.jsonl; exit 3; }
grep '^{' $O/gemm_bench.jsonl
for r in 1 2; do
  timeout -k 10 300 python bench.py --model mlp-wide --steps 10 --warmup 3 > $O/wide_new_$r.json 2> $O/wide_new_$r.err || { tail $O/wide_new_$r.err; exit 4; }
  grep -o '"value": [0-9.]*, "unit": "[^"]*", "n_gpus": 1, "steps": 10, "warmup": 3, "warmup_extra_steps": [0-9]*, "warmup_min_ms": [0-9.]*, "ms_per_step": [0-9.]*' $O/wide_new_$r.json
  (cd gpurun_ab/head && EUROM_NATIVE_LIB=$R/euromillioner_amd/lib/ab/gemm_head.so timeout -k 10 300 python bench.py --model mlp-wide --steps 10 --warmup 3 > $O/wide_head_$r.json 2> $O/wide_head_$r.err) || { tail $O/wide_head_$r.err; exit 5; }
  grep -o '"value": [0-9.]*, "unit": "[^"]*", "n_gpus": 1, "steps": 10, "warmup": 3, "warmup_extra_steps": [0-9]*, "warmup_min_ms": [0-9.]*, "ms_per_step": [0-9.]*' $O/wide_head_$r.json
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --model mlp-wide --steps 10 --warmup 3 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 6; }
echo rc=0
