# GBDT histogram A/B (EM_GBDT_HIST_STAGE=0 old byte-load form vs 1 staged form) + per-case kernel stats
set -o pipefail
mkdir -p gpurun_out/gbdt
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gbdt.py tests/test_dist.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/gbdt/t.log 2>&1 || { tail -40 gpurun_out/gbdt/t.log; exit 3; }
tail -2 gpurun_out/gbdt/t.log
for i in 1 2; do
  for s in 0 1; do
    EM_GBDT_HIST_STAGE=$s timeout -k 10 300 python tools/gbdt_bench.py hip > gpurun_out/gbdt/s${s}_$i.jsonl 2>&1 || exit 4
    echo "stage=$s"; cat gpurun_out/gbdt/s${s}_$i.jsonl
  done
done
R=$PWD
cd /tmp
for c in reference synthetic; do
  for s in 0 1; do
    EM_GBDT_HIST_STAGE=$s timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/gbdt/prof_${c}_$s -o run -- python3 $R/tools/gbdt_bench.py $c > $R/gpurun_out/gbdt/prof_${c}_$s.log 2>&1 || exit 5
  done
done
