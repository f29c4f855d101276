# V4_STAMPS timeline (steady clock) + compile-time sweep of stagger/prio/sleep
set -o pipefail
mkdir -p gpurun_out/f
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
python -m euromillioner_amd._build --define V4_STAMPS=1 > gpurun_out/f/build_st.log 2>&1 || exit 2
timeout -k 10 120 python tools/dev/stamps_timeline.py > gpurun_out/f/timeline.txt 2>&1 || { cat gpurun_out/f/timeline.txt; exit 3; }
cat gpurun_out/f/timeline.txt
bash tools/fused_sweep.sh "V4_MIX=1" "V4_STAGGER=4" "V4_STAGGER=16" "V4_PRIO=1" "V4_SLEEP=1" "V4_STAGGER=16 V4_PRIO=1" > gpurun_out/f/sweep.txt 2>&1
cat gpurun_out/f/sweep.txt
