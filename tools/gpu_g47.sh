#!/bin/bash
# Round-5 batch 45: fused-kernel knobs re-tested under the max-memory-clause schedule: ring-wait s_sleep 0 / 2
# (1 shipped), forward-wave priority 2 (1 shipped); 3 interleaved headline rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/euromillioner_amd/lib/ab
O=gpurun_out/g47
mkdir -p $O
rm -f gpurun_out/ab/results.jsonl
ARMS="base|X=0;f_sleep0|EUROM_NATIVE_LIB=$L/f_sleep0.so;f_sleep2|EUROM_NATIVE_LIB=$L/f_sleep2.so;f_fprio2|EUROM_NATIVE_LIB=$L/f_fprio2.so" ROUNDS=3 bash tools/gpu_ab.sh || exit 2
cp gpurun_out/ab/results.jsonl $O/ab_knobs.jsonl
echo rc=0
