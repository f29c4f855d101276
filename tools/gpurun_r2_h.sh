# refresh after the v6 work: full GPU tests, driver-shape bench x2, 1000-step bench, rocprof stats,
# 1-GPU multi-rank rehearsal (gloo dp2/dp4, shared task)
set -o pipefail
mkdir -p gpurun_out/h
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/h/pytest.log 2>&1 || { tail -40 gpurun_out/h/pytest.log; exit 3; }
tail -2 gpurun_out/h/pytest.log
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/h/bench20_$i.json 2> gpurun_out/h/bench20_$i.err || exit 4
done
timeout -k 10 120 python bench.py --steps 1000 --warmup 10 --no-eval > gpurun_out/h/bench1000.json 2> gpurun_out/h/bench1000.err || exit 5
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/h/prof -o run --output-format csv -- python bench.py --steps 200 --warmup 10 --no-eval > gpurun_out/h/prof.log 2>&1 || exit 6
for n in 2 4; do
  timeout -k 10 300 python bench.py --gpus $n --dist-backend gloo --steps 100 --warmup 10 > gpurun_out/h/dp$n.json 2> gpurun_out/h/dp$n.err || exit 7
done
python - <<'PY'
import json
for f in ['bench20_1','bench20_2','bench1000','dp2','dp4']:
    d=json.loads([l for l in open(f"gpurun_out/h/{f}.json") if l.startswith("{")][-1])
    print(f, round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,2), 'us/step', 'acc', d.get('val',{}).get('acc'), d['config'].get('grad_allreduce'))
PY
