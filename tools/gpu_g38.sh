#!/bin/bash
# Round-5 batch 36: fused train kernel with the AMDGPU register-pressure trackers off, and with bottom-up pre-RA
# scheduling, vs the shipped build: parameter hashes + 3 headline rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/euromillioner_amd/lib/ab
O=gpurun_out/g38
mkdir -p $O
for v in fused_trk0 fused_bottomup; do
  EUROM_NATIVE_LIB=$L/$v.so timeout -k 10 200 python tools/ab_hash.py > $O/hash_$v.jsonl 2>&1 || { tail $O/hash_$v.jsonl; exit 3; }
  grep '^{' $O/hash_$v.jsonl
done
rm -f gpurun_out/ab/results.jsonl
ARMS="base|X=0;fused_trk0|EUROM_NATIVE_LIB=$L/fused_trk0.so;fused_bottomup|EUROM_NATIVE_LIB=$L/fused_bottomup.so" ROUNDS=3 bash tools/gpu_ab.sh || exit 2
cp gpurun_out/ab/results.jsonl $O/ab_sched2.jsonl
echo rc=0
