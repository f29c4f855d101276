#!/bin/bash
# Round-5 batch 42: GBDT round phase stamps on the final kernels (GBDT_STAMPS side build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/euromillioner_amd/lib/ab
O=gpurun_out/g44
mkdir -p $O
EUROM_NATIVE_LIB=$L/gbdt_stamps.so timeout -k 10 200 python tools/gbdt_stamps.py > $O/gbdt_stamps.jsonl 2>&1 || { tail $O/gbdt_stamps.jsonl; exit 2; }
grep '^{' $O/gbdt_stamps.jsonl
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/$O/trace -o run -- python3 $OLDPWD/tools/gbdt_bench.py reference > $OLDPWD/$O/trace.log 2>&1 || { tail $OLDPWD/$O/trace.log; exit 3; }
echo rc=0
