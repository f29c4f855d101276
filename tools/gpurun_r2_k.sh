# 1-GPU rehearsal of bench.py --gpus 8 (gloo ranks sharing the card; xGMI one-shot gradient path)
set -o pipefail
mkdir -p gpurun_out/k
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python bench.py --gpus 8 --dist-backend gloo --steps 50 --warmup 5 > gpurun_out/k/dp8.json 2> gpurun_out/k/dp8.err || { tail -20 gpurun_out/k/dp8.err; exit 4; }
python - <<'PY'
import json
d=json.loads([l for l in open('gpurun_out/k/dp8.json') if l.startswith('{')][-1])
print('dp8', round(d['value']/1e9,3), 'G/s aggregate on ONE GPU', round(d['ms_per_step']*1e3,1), 'us/step', 'acc', d['val']['acc'], d['config']['grad_allreduce'], 'n_gpus', d['n_gpus'])
PY
