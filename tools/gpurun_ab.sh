# same-box A/B of the in-tree native build vs euromillioner_amd/lib/ab/base.so (+ fused-MLP GPU tests first)
set -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fused_mlp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/t_fused.log 2>&1 || { tail -30 gpurun_out/ab/t_fused.log; exit 3; }
tail -2 gpurun_out/ab/t_fused.log
for i in 1 2 3; do
  EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/base.so timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-eval > gpurun_out/ab/a$i.json 2>/dev/null || exit 4
  timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-eval > gpurun_out/ab/b$i.json 2>/dev/null || exit 5
  python -c "import json;a=json.load(open('gpurun_out/ab/a$i.json'));b=json.load(open('gpurun_out/ab/b$i.json'));print(f'base {a[\"ms_per_step\"]*1e3:.2f} us (med {a[\"ms_per_step_median\"]*1e3:.2f})  new {b[\"ms_per_step\"]*1e3:.2f} us (med {b[\"ms_per_step_median\"]*1e3:.2f})')"
done


