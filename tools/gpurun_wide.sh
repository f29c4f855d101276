# wide-MLP bench refresh + kernel stats
set -o pipefail
mkdir -p gpurun_out/wide
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --model mlp-wide --steps 10 --warmup 3 > gpurun_out/wide/bench_wide.jsonl 2> gpurun_out/wide/bench_wide.err || exit 3
cat gpurun_out/wide/bench_wide.jsonl | cut -c1-300
R=$PWD
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/wide/prof -o run -- python3 $R/bench.py --model mlp-wide --steps 5 --warmup 2 --graph 0 --no-eval > $R/gpurun_out/wide/prof.log 2>&1 || exit 4
