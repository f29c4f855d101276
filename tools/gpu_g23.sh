#!/bin/bash
# Round-5 batch 21: pp16 GEMM segment timers (G_STAMPS side build): per-tile prologue / epilogue share of
# the wide layers' GEMMs (forward plain and with C^T).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/g23
mkdir -p $O
L=$PWD/euromillioner_amd/lib/ab
for ct in 0 1; do
  STAMP_CT=$ct EUROM_NATIVE_LIB=$L/gstamps.so timeout -k 10 200 python tools/gemm_stamps.py > $O/stamps_ct$ct.jsonl 2>&1 || { tail $O/stamps_ct$ct.jsonl; exit 2; }
  grep '^{' $O/stamps_ct$ct.jsonl
done
echo rc=0
