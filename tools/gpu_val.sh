set -o pipefail
mkdir -p gpurun_out/val
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 5 > gpurun_out/val/dp2.json 2> gpurun_out/val/dp2.err || { tail -20 gpurun_out/val/dp2.err; exit 3; }
grep '^{' gpurun_out/val/dp2.json | cut -c1-300
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/val/pytest.log 2>&1 || { tail -40 gpurun_out/val/pytest.log; exit 4; }
tail -3 gpurun_out/val/pytest.log
