# after the compile-time staging lead: GEMM GPU tests, GEMM vs hipBLASLt, wide-MLP benches
set -o pipefail
mkdir -p gpurun_out/gfix
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_property_gpu.py tests/test_gemm_accum_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/gfix/t.log 2>&1 || { tail -30 gpurun_out/gfix/t.log; exit 3; }
tail -1 gpurun_out/gfix/t.log
timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gfix/gemm_bench.log 2>&1 || exit 4
grep '^{' gpurun_out/gfix/gemm_bench.log | cut -c1-170
timeout -k 10 200 python bench.py --model mlp-wide --steps 10 --warmup 3 > gpurun_out/gfix/wide.json 2> gpurun_out/gfix/wide.err || { tail -5 gpurun_out/gfix/wide.err; exit 5; }
grep '^{' gpurun_out/gfix/wide.json | cut -c1-300
timeout -k 10 300 python bench.py --model mlp-wide --device-data-gb 100 --accum 16 --steps 4 --warmup 1 > gpurun_out/gfix/wide_mega.json 2> gpurun_out/gfix/wide_mega.err || { tail -5 gpurun_out/gfix/wide_mega.err; exit 6; }
grep '^{' gpurun_out/gfix/wide_mega.json | cut -c1-300
