# multi-step hipGraph chunks: headline bench (driver's K/W) at several --graph-steps + a kernel trace
set -o pipefail
mkdir -p gpurun_out/r2c
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for gs in 1 10 20; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --graph-steps $gs > gpurun_out/r2c/b20_gs$gs.json 2>gpurun_out/r2c/b20_gs$gs.err || exit 3
done
timeout -k 10 120 python bench.py --steps 200 --warmup 5 > gpurun_out/r2c/b200.json 2>gpurun_out/r2c/b200.err || exit 3
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r2c/prof -o run --output-format csv -- python bench.py --steps 200 --warmup 5 --no-eval > gpurun_out/r2c/prof.log 2>&1 || exit 4
echo done
