#!/bin/bash
# Round-5 batch 46: host-side profile of the GBDT reference fit on the final kernels (tools/gbdt_fit_profile.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/g48
mkdir -p $O
timeout -k 10 300 python tools/gbdt_fit_profile.py > $O/gbdt_fit_profile.txt 2>&1 || { tail -20 $O/gbdt_fit_profile.txt; exit 2; }
head -60 $O/gbdt_fit_profile.txt
echo rc=0
