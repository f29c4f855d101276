#!/bin/bash
# Round-5 batch 9: GBDT reference-fit kernel trace (per-kernel durations and inter-kernel gaps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/g9
mkdir -p $O
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/gb -o gb --output-format csv -- python3 $R/tools/gbdt_bench.py reference > $R/$O/gb.log 2>&1 || { tail -20 $R/$O/gb.log; exit 3; }
cd $R
grep -o '"hip_s": [0-9.]*' $O/gb.log
echo rc=0
