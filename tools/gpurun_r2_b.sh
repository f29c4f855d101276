# fixed vs marginal cost of the fused step: bench at several batch sizes + a kernel trace of graph replays
set -o pipefail
mkdir -p gpurun_out/r2b
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for b in 1048576 2097152 4194304 16777216; do
  timeout -k 10 120 python bench.py --batch $b --draws-per-gpu 41943040 --steps 100 --warmup 5 --no-eval > gpurun_out/r2b/b_$b.json 2>gpurun_out/r2b/b_$b.err || exit 3
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r2b/prof -o run --output-format csv -- python bench.py --steps 200 --warmup 5 --no-eval > gpurun_out/r2b/prof.log 2>&1 || exit 4
echo done
