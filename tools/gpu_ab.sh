#!/bin/bash
# Same-box interleaved A/B of bench.py arms (cdna_hip_programming.md §5.4 rule 24).
#   ARMS="name1|ENV=a ENV2=b;name2|ENV=c" ROUNDS=3 BENCH_ARGS="--steps 100 --warmup 5 --no-eval" bash tools/gpu_ab.sh
# One line per (round, arm) in gpurun_out/ab/results.jsonl; any failing run stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ab
mkdir -p $OUT
ROUNDS=${ROUNDS:-3}
BENCH_ARGS=${BENCH_ARGS:---steps 100 --warmup 5 --no-eval}
IFS=';' read -ra LIST <<< "$ARMS"
for r in $(seq 1 $ROUNDS); do
  for arm in "${LIST[@]}"; do
    name=${arm%%|*}; envs=${arm#*|}
    env $envs timeout -k 10 180 python bench.py $BENCH_ARGS > $OUT/${name}_$r.json 2> $OUT/${name}_$r.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "arm $name round $r failed rc=$rc"; tail -20 $OUT/${name}_$r.err; exit $rc; fi
    python - "$name" "$r" $OUT/${name}_$r.json >> $OUT/results.jsonl <<'PY'
import json, sys
name, r, path = sys.argv[1:4]
d = [json.loads(l) for l in open(path) if l.startswith("{")][-1]
print(json.dumps({"arm": name, "round": int(r), "value": d["value"], "ms_per_step": d["ms_per_step"],
                  "median_ms": d.get("ms_per_step_median"), "val_acc": (d.get("val") or {}).get("acc")}))
PY
    tail -1 $OUT/results.jsonl
  done
done
