# Adam slab kernel A/B: fused tests, step parts with base vs new library
set -o pipefail
mkdir -p gpurun_out/adam
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_fused_mlp_gpu.py tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/adam/t.log 2>&1 || { tail -30 gpurun_out/adam/t.log; exit 3; }
tail -1 gpurun_out/adam/t.log
for i in 1 2; do
  EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/base.so STEP_PARTS_B=1048576 timeout -k 10 120 python tools/step_parts.py > gpurun_out/adam/b$i.txt 2>/dev/null || exit 4
  STEP_PARTS_B=1048576 timeout -k 10 120 python tools/step_parts.py > gpurun_out/adam/n$i.txt 2>/dev/null || exit 5
  echo "base $(sed -n 1p gpurun_out/adam/b$i.txt)"; echo "new  $(sed -n 1p gpurun_out/adam/n$i.txt)"
done
