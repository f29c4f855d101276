#!/bin/bash
# Same-box A/B of the wide-MLP step: the shipped library vs lib/ab/gemm_head.so (tools/build_variant.sh with
# FILE=csrc/gemm.hip SRC=<old gemm.hip>), GEMM GPU tests first, then two alternating rounds and a kernel trace each.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/wab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
for rnd in 1 2; do
  timeout -k 10 200 python bench.py --model mlp-wide --steps 10 --warmup 3 > $O/new_$rnd.json 2>/dev/null || exit 4
  EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/gemm_head.so timeout -k 10 200 python bench.py --model mlp-wide --steps 10 --warmup 3 > $O/head_$rnd.json 2>/dev/null || exit 5
done
for f in $O/*_?.json; do echo "$f $(grep '^{' $f | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_new -o run -- python bench.py --model mlp-wide --steps 10 --warmup 3 > $O/trn.log 2>&1 || exit 6
EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/gemm_head.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_head -o run -- python bench.py --model mlp-wide --steps 10 --warmup 3 > $O/trh.log 2>&1 || exit 7
