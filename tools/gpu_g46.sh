#!/bin/bash
# Round-5 batch 44: wide-MLP step kernel trace on the final round-5 tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/g46
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --model mlp-wide --steps 10 --warmup 3 --no-eval > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 2; }
grep '^{' $O/trace.log | cut -c1-200
echo rc=0
