#!/bin/bash
# Same-box A/B of how the driver-shape window (20 timed steps) is split into hipGraph launches.
# A short head graph starts the GPU while the host is still launching the long one.
# Output: gpurun_out/graph_plan/results.jsonl (plan, value, ms_per_step, median)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/graph_plan
mkdir -p $O
: > $O/results.jsonl
PLANS=${PLANS:-"20 1,19 2,18 1,1,18 4,16"}
for r in $(seq 1 ${ROUNDS:-3}); do
  for p in $PLANS; do
    timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 --no-eval --graph-chunks $p > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 3; }
    grep '^{' $O/b.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'round': $r, 'plan': '$p', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'median': d['ms_per_step_median']}))" >> $O/results.jsonl || exit 4
  done
done
cat $O/results.jsonl
