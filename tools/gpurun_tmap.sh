# V6_TMAP A/B (XCD-major stream numbering) + stamps of the variant
set -o pipefail
mkdir -p gpurun_out/tmap
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/fused_sweep.sh "V6_TMAP=0" "V6_TMAP=1" "V6_TMAP=0" "V6_TMAP=1" > gpurun_out/tmap/sweep.txt 2>&1 || { cat gpurun_out/tmap/sweep.txt; exit 3; }
cat gpurun_out/tmap/sweep.txt
export EM_FUSED_V6=1
python -m euromillioner_amd._build --define V4_STAMPS=1 --define V6_TMAP=1 > gpurun_out/tmap/build.log 2>&1 || exit 4
TL_B=1048576 timeout -k 10 120 python tools/dev/stamps_timeline.py > gpurun_out/tmap/stamps.txt 2>gpurun_out/tmap/stamps.err || { tail -5 gpurun_out/tmap/stamps.err; exit 5; }
cat gpurun_out/tmap/stamps.txt
