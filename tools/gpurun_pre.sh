# step-counter advance in the train kernel + ticket-free Adam: fused/xgmi/train tests, step parts A/B
set -o pipefail
mkdir -p gpurun_out/pre
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_fused_mlp_gpu.py tests/test_train_gpu.py tests/test_xgmi_gpu.py tests/test_small_ops_property_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pre/t.log 2>&1 || { tail -40 gpurun_out/pre/t.log; exit 3; }
tail -1 gpurun_out/pre/t.log
STEP_PARTS_B=1048576 timeout -k 10 120 python tools/step_parts.py > gpurun_out/pre/parts.txt 2>/dev/null || exit 4
cat gpurun_out/pre/parts.txt
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/pre/bench20_$i.json 2> gpurun_out/pre/bench20_$i.err || exit 5
  grep '^{' gpurun_out/pre/bench20_$i.json | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench20', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,2), 'us', d.get('val',{}).get('acc'))"
done
timeout -k 10 120 python bench.py --steps 1000 --warmup 10 --no-eval > gpurun_out/pre/bench1000.json 2> gpurun_out/pre/bench1000.err || exit 6
grep '^{' gpurun_out/pre/bench1000.json | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench1000', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,2), 'us')"
