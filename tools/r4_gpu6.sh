set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 200 python tools/power_probe.py > $O/power_probe.jsonl 2>&1 || { tail -20 $O/power_probe.jsonl; exit 3; }
cat $O/power_probe.jsonl
bash tools/r4_gpu5.sh
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gbdtprof -o run -- python tools/gbdt_bench.py reference > $O/gbdt_ref.jsonl 2>&1 || { tail $O/gbdt_ref.jsonl; exit 9; }
f=$(find $O/gbdtprof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats_gbdt_reference.csv; head -25 $O/kernel_stats_gbdt_reference.csv
