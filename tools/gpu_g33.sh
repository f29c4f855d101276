#!/bin/bash
# Round-5 batch 31: the fused train kernel under the LLVM AMDGPU scheduler strategies max-ilp and
# max-memory-clause (side builds of csrc/mlp_fused.hip) vs the default, 3 interleaved rounds of the
# 1M-sample step (bench.py --steps 100 --warmup 5 --no-eval), plus bitwise parameter hashes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/euromillioner_amd/lib/ab
O=gpurun_out/g33
mkdir -p $O
rm -f gpurun_out/ab/results.jsonl
ARMS="base|X=0;sched_ilp|EUROM_NATIVE_LIB=$L/sched_ilp.so;sched_memclause|EUROM_NATIVE_LIB=$L/sched_memclause.so" ROUNDS=3 bash tools/gpu_ab.sh || exit 2
cp gpurun_out/ab/results.jsonl $O/ab_sched.jsonl
echo rc=0
