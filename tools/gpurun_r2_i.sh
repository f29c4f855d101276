# headline at the driver shape with and without the 250 ms clock warmup (v6)
set -o pipefail
mkdir -p gpurun_out/i
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --warmup-ms 0 > gpurun_out/i/nowarm_$i.json 2>/dev/null || exit 4
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/i/warm_$i.json 2>/dev/null || exit 5
done
python - <<'PY'
import json
for f in ['nowarm_1','warm_1','nowarm_2','warm_2']:
    d=json.loads(open(f'gpurun_out/i/{f}.json').read().strip().splitlines()[-1])
    print(f, round(d['value']/1e9,3), 'G/s', round(d['ms_per_step']*1e3,2), 'us', 'extra', d['warmup_extra_steps'], 'acc', round(d['val']['acc'],4))
PY
