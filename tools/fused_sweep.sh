#!/bin/bash
# Compile-time tuning sweep of the fused train kernel on the GPU box: rebuild with each -D set,
# run a short bench, print one line per variant.  Usage: tools/fused_sweep.sh "A=1 B=2" "A=0" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
i=0
for v in "$@"; do
  i=$((i+1))
  defs=""
  for d in $v; do defs="$defs --define $d"; done
  python -m euromillioner_amd._build $defs > gpurun_out/sweep/build$i.log 2>&1 || { echo "BUILD FAIL $v"; exit 1; }
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-eval > gpurun_out/sweep/bench$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "BENCH RC=$rc for $v"; tail -3 gpurun_out/sweep/bench$i.log; exit $rc; fi
  python3 -c "import json,sys; j=json.loads(open('gpurun_out/sweep/bench$i.log').read().strip().splitlines()[-1]); print('%-40s %.3f G samples/s  %.4f ms' % (sys.argv[1], j['value']/1e9, j['ms_per_step']))" "$v"
done
