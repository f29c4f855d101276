# RCCL fallback of the fused DP step replayed from a hipGraph (world-1 RCCL group on the box's GPU)
set -o pipefail
mkdir -p gpurun_out/rg
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -k "rccl or dp_code_path" -x -v --timeout 120 --timeout-method thread > gpurun_out/rg/t.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/rg/t.log | tail -30
exit $rc
