# Fixed cost of the fused step: train/Adam parts at small batches + v6 phase stamps (V4_STAMPS build)
set -o pipefail
mkdir -p gpurun_out/fixed
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export EM_FUSED_V6=1
STEP_PARTS_B=8192,65536,262144,1048576 timeout -k 10 120 python tools/step_parts.py > gpurun_out/fixed/parts.txt 2>gpurun_out/fixed/parts.err || { tail -5 gpurun_out/fixed/parts.err; exit 3; }
cat gpurun_out/fixed/parts.txt
python -m euromillioner_amd._build --define V4_STAMPS=1 > gpurun_out/fixed/build.log 2>&1 || { tail -5 gpurun_out/fixed/build.log; exit 4; }
TL_B=8192,65536,1048576 timeout -k 10 120 python tools/dev/stamps_timeline.py > gpurun_out/fixed/stamps.txt 2>gpurun_out/fixed/stamps.err || { tail -5 gpurun_out/fixed/stamps.err; exit 5; }
cat gpurun_out/fixed/stamps.txt
