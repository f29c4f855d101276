# v6 compile-time sweep (EM_FUSED_V6=1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export EM_FUSED_V6=1
mkdir -p gpurun_out/v6
bash tools/fused_sweep.sh "V6_F1P=1" "V6_F1P=2" "V6_F1P=1" "V6_F1P=2" > gpurun_out/v6/sweep.txt 2>&1
cat gpurun_out/v6/sweep.txt
