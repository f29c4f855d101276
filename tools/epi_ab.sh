#!/bin/bash
# One-launch vs two-launch optimizer step: per-workgroup epilogue timeline (FUSED_STAMPS side build) and a
# same-box A/B.  Build the side library first (on the CPU):
#   bash tools/build_variant.sh stamps -DFUSED_STAMPS=1
# then run through gpurun: bash tools/epi_ab.sh   (outputs under gpurun_out/epi and gpurun_out/ab)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/euromillioner_amd/lib/ab
mkdir -p gpurun_out/epi
EUROM_NATIVE_LIB=$L/stamps.so timeout -k 10 200 python tools/epi_timeline.py > gpurun_out/epi/stamps.txt 2>&1 || { tail -20 gpurun_out/epi/stamps.txt; exit 3; }
cat gpurun_out/epi/stamps.txt
rm -rf gpurun_out/ab
ARMS="split|EUROM_FUSED_ADAM=0;fused|EUROM_FUSED_ADAM=1" ROUNDS=${ROUNDS:-3} bash tools/gpu_ab.sh || exit 5
