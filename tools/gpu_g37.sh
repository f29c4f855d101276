#!/bin/bash
# Round-5 batch 35: fused train kernel built with -fno-honor-nans/-infinities (NaN-free max: 16 fewer v_max per
# tile loop) and additionally -fno-signed-zeros, vs the shipped build: parameter hashes + 3 headline rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/euromillioner_amd/lib/ab
O=gpurun_out/g37
mkdir -p $O
for v in fused_nonan fused_nonan_nsz; do
  EUROM_NATIVE_LIB=$L/$v.so timeout -k 10 200 python tools/ab_hash.py > $O/hash_$v.jsonl 2>&1 || { tail $O/hash_$v.jsonl; exit 3; }
  grep '^{' $O/hash_$v.jsonl
done
rm -f gpurun_out/ab/results.jsonl
ARMS="base|X=0;fused_nonan|EUROM_NATIVE_LIB=$L/fused_nonan.so;fused_nonan_nsz|EUROM_NATIVE_LIB=$L/fused_nonan_nsz.so" ROUNDS=3 bash tools/gpu_ab.sh || exit 2
cp gpurun_out/ab/results.jsonl $O/ab_fastmath.jsonl
echo rc=0
