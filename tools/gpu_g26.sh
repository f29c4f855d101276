#!/bin/bash
# Round-5 batch 24: skinny-K GEMM with the in-place row image (36 KB LDS, 4 blocks / CU) vs the staged one
# (k64crow1): GEMM tests, per-kernel A/B, wide-step A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/g26
mkdir -p $O
L=$R/euromillioner_amd/lib/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > $O/pytest_gemm.log 2>&1 || { tail -40 $O/pytest_gemm.log; exit 2; }
tail -1 $O/pytest_gemm.log
for r in 1 2; do
  for v in base k64crow1; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/gemm_bench.py --no-lib --iters 20 --cases fwd_in,fwd_in_ct,dgrad_out_ct > $O/k64_${v}_$r.jsonl 2>&1 || { tail $O/k64_${v}_$r.jsonl; exit 3; }
    grep '^{' $O/k64_${v}_$r.jsonl | sed "s/^/$v /" | cut -c1-110
  done
done
for r in 1 2; do
  for v in base k64crow1; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 300 python bench.py --model mlp-wide --steps 10 --warmup 3 --no-eval > $O/wide_${v}_$r.json 2> $O/wide_${v}_$r.err || { tail $O/wide_${v}_$r.err; exit 4; }
    echo "$v $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/wide_${v}_$r.json | tr '\n' ' ')"
  done
done
echo rc=0
