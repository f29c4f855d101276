#!/bin/bash
# Same-box A/B of LLVM AMDGPU scheduler options on the wide-MLP GEMMs and the headline fused kernel.
# Side libraries first (CPU):
#   FILE=csrc/gemm.hip bash tools/build_variant.sh g1 -mllvm -amdgpu-sched-strategy=max-ilp
#   FILE=csrc/gemm.hip bash tools/build_variant.sh g2 -mllvm -amdgpu-sched-strategy=max-memory-clause
#   FILE=csrc/gemm.hip bash tools/build_variant.sh g3 -mllvm -amdgpu-use-amdgpu-trackers
#   bash tools/build_variant.sh s3 <flags to compare against the shipped mlp_fused.hip build>
# then through gpurun: bash tools/sched_ab.sh   (results: gpurun_out/abw, gpurun_out/abh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/euromillioner_amd/lib/ab
rm -rf gpurun_out/ab gpurun_out/abw gpurun_out/abh
ARMS="base|X=1;g1|EUROM_NATIVE_LIB=$L/g1.so;g2|EUROM_NATIVE_LIB=$L/g2.so;g3|EUROM_NATIVE_LIB=$L/g3.so" ROUNDS=3 \
  BENCH_ARGS="--model mlp-wide --steps 20 --warmup 3 --no-eval" bash tools/gpu_ab.sh || exit 3
mv gpurun_out/ab gpurun_out/abw
ARMS="base|X=1;s3|EUROM_NATIVE_LIB=$L/s3.so" ROUNDS=5 bash tools/gpu_ab.sh || exit 4
mv gpurun_out/ab gpurun_out/abh
