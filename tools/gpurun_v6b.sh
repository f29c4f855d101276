# v6 phase stamps (steady clock)
set -o pipefail
mkdir -p gpurun_out/v6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
python -m euromillioner_amd._build --define V4_STAMPS=1 > gpurun_out/v6/build_st.log 2>&1 || exit 2
EM_FUSED_V6=1 TL_B=1048576 timeout -k 10 120 python tools/dev/stamps_timeline.py > gpurun_out/v6/timeline.txt 2>&1 || { cat gpurun_out/v6/timeline.txt; exit 3; }
cat gpurun_out/v6/timeline.txt
