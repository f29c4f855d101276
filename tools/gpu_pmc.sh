#!/bin/bash
# PMC counters for the fused train kernel (separate rocprofv3 runs; --pmc never combined with sys/runtime traces)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
ARGS="--steps 6 --warmup 2 --graph 0 --no-eval --warmup-ms 0"
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $OUT/set$i -o run -- python3 bench.py $ARGS > $OUT/set$i.log 2>&1
  rc=$?; echo "SET$i RC=$rc ($set)"
  case $rc in 0) ;; *) tail -5 $OUT/set$i.log; exit $rc;; esac
done
