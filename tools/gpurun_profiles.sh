# round-2 profile refresh: headline bench (driver K/W and 200 steps), kernel stats of the headline step,
# 1-GPU multi-rank rehearsal (dp2/dp4 gloo, shared task), RF bench + stats, wide-MLP DP launch order
set -o pipefail
mkdir -p gpurun_out/p2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/p2/bench20.json 2> gpurun_out/p2/bench20.err || exit 3
timeout -k 10 120 python bench.py --steps 200 --warmup 10 > gpurun_out/p2/bench200.json 2> gpurun_out/p2/bench200.err || exit 3
timeout -k 10 120 python bench.py --steps 1000 --warmup 10 --no-eval > gpurun_out/p2/bench1000.json 2> gpurun_out/p2/bench1000.err || exit 3
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/p2/prof_fused -o run --output-format csv -- python bench.py --steps 200 --warmup 10 --no-eval > gpurun_out/p2/prof_fused.log 2>&1 || exit 4
for n in 2 4; do
  timeout -k 10 300 python bench.py --gpus $n --dist-backend gloo --steps 100 --warmup 10 > gpurun_out/p2/dp$n.json 2> gpurun_out/p2/dp$n.err || exit 5
done
timeout -k 10 300 python tools/rf_bench.py --rows 700000 > gpurun_out/p2/rf.json 2>/dev/null || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p2/prof_rf -o run --output-format csv -- python tools/rf_bench.py --rows 700000 --repeat 2 > gpurun_out/p2/prof_rf.log 2>&1 || exit 7
timeout -k 10 300 python tools/wide_dp_trace.py --out gpurun_out/p2/wide > gpurun_out/p2/wide.log 2>&1 || exit 8
echo profiles-done
