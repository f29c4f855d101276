set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_device_gen_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_dg.log 2>&1 &&
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/b1.json 2> gpurun_out/b1.err &&
timeout -k 10 180 python bench.py --steps 200 --warmup 10 > gpurun_out/b1_200.json 2> gpurun_out/b1_200.err &&
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 100 --warmup 10 > gpurun_out/b2.json 2> gpurun_out/b2.err &&
timeout -k 10 300 python bench.py --gpus 4 --dist-backend gloo --steps 100 --warmup 10 > gpurun_out/b4.json 2> gpurun_out/b4.err
echo "rc=$?"
