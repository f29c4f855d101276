#!/bin/bash
# Round-5 batch 27: relu-dgrad epilogue with the activity words hoisted (one round trip) vs per 32-row block
# (gemm_prev): GEMM tests, per-GEMM A/B (3 rounds), wide-step A/B (2 rounds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/g29
mkdir -p $O
L=$R/euromillioner_amd/lib/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > $O/pytest_gemm.log 2>&1 || { tail -40 $O/pytest_gemm.log; exit 2; }
tail -1 $O/pytest_gemm.log
for r in 1 2 3; do
  for v in base gemm_prev; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/gemm_bench.py --no-lib --iters 10 --cases dgrad_hidden_bits > $O/g_${v}_$r.jsonl 2>&1 || { tail $O/g_${v}_$r.jsonl; exit 3; }
    grep '^{' $O/g_${v}_$r.jsonl | sed "s/^/$v /" | cut -c1-110
  done
done
for r in 1 2; do
  for v in base gemm_prev; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 300 python bench.py --model mlp-wide --steps 10 --warmup 3 --no-eval > $O/wide_${v}_$r.json 2> $O/wide_${v}_$r.err || { tail $O/wide_${v}_$r.err; exit 4; }
    echo "$v $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/wide_${v}_$r.json | tr '\n' ' ')"
  done
done
echo rc=0
