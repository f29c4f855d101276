# v5 fused kernel: GPU numerics tests under EM_FUSED_V5=1, then a same-box A/B of v4 vs v5
set -o pipefail
mkdir -p gpurun_out/v5
export TMPDIR=/tmp
EM_FUSED_V5=1 timeout -k 10 300 python -u -m pytest tests/test_fused_mlp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/v5/t_fused.log 2>&1 || { tail -40 gpurun_out/v5/t_fused.log; exit 3; }
tail -2 gpurun_out/v5/t_fused.log
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 10 > gpurun_out/v5/a$i.json 2>/dev/null || exit 4
  EM_FUSED_V5=1 timeout -k 10 120 python bench.py --steps 200 --warmup 10 > gpurun_out/v5/b$i.json 2>/dev/null || exit 5
  python -c "import json;a=json.load(open('gpurun_out/v5/a$i.json'));b=json.load(open('gpurun_out/v5/b$i.json'));print(f'v4 {a[\"ms_per_step\"]*1e3:.2f} us acc {a[\"val\"][\"acc\"]:.4f}   v5 {b[\"ms_per_step\"]*1e3:.2f} us acc {b[\"val\"][\"acc\"]:.4f}')"
done
EM_FUSED_V5=1 timeout -k 10 120 python tools/step_parts.py > gpurun_out/v5/parts.txt 2>&1 && grep -v amdgpu gpurun_out/v5/parts.txt
EM_FUSED_V5=1 EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/stamps.so timeout -k 10 120 python tools/fused_phases.py > gpurun_out/v5/phases.txt 2>&1; grep -v amdgpu gpurun_out/v5/phases.txt | head -14
