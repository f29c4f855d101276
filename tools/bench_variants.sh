#!/bin/bash
# Sanity run of bench.py's less-common modes (torch baseline, per-layer GEMM engine, BCE, wide with the bf16
# wire, eager launches, smaller batch); one summary line per mode.  Through gpurun: bash tools/bench_variants.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/bv; mkdir -p $O
while IFS= read -r a; do
  [ -z "$a" ] && continue
  echo "== $a"
  timeout -k 10 300 python bench.py $a > $O/o.json 2> $O/o.err; rc=$?
  echo "rc=$rc"
  grep '^{' $O/o.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config'].get('engine'), (d.get('val') or {}).get('acc'))" || tail -3 $O/o.err
  [ $rc -ge 124 ] && exit $rc
done <<'LIST'
--impl torch --steps 5 --warmup 2 --no-eval
--impl gemm --steps 10 --warmup 2 --no-eval
--loss bce --steps 20 --warmup 5
--model mlp-wide --comm-dtype bf16 --steps 5 --warmup 2 --no-eval
--graph 0 --steps 20 --warmup 5 --no-eval
--batch 262144 --steps 20 --warmup 5 --no-eval
LIST
