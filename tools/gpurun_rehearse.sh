# 1-GPU multi-rank rehearsal of the bench (gloo ranks sharing the card): xGMI path and forced RCCL fallback
set -o pipefail
mkdir -p gpurun_out/reh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 20 --warmup 3 > gpurun_out/reh/dp2.json 2> gpurun_out/reh/dp2.err || { tail -20 gpurun_out/reh/dp2.err; exit 3; }
grep '^{' gpurun_out/reh/dp2.json | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('dp2', j['n_gpus'], j['config']['grad_allreduce'], j['config']['hipgraph'], '%.2f G/s' % (j['value']/1e9), 'val_acc', j['val'].get('acc'))"
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --comm rccl --steps 20 --warmup 3 > gpurun_out/reh/dp2r.json 2> gpurun_out/reh/dp2r.err || { tail -20 gpurun_out/reh/dp2r.err; exit 4; }
grep '^{' gpurun_out/reh/dp2r.json | python -c "import json,sys; j=json.loads(sys.stdin.read()); print('dp2 rccl-path', j['n_gpus'], j['config']['grad_allreduce'], j['config']['hipgraph'], '%.2f G/s' % (j['value']/1e9), 'val_acc', j['val'].get('acc'))"
