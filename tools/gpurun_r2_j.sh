# v6 refresh of the HBM-resident data runs: 1M steps streamed over 200 GiB, and 256M-sample mega-batches
set -o pipefail
mkdir -p gpurun_out/j
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --device-data-gb 200 --steps 50 --warmup 5 > gpurun_out/j/mega_data.json 2> gpurun_out/j/mega_data.err || exit 4
timeout -k 10 300 python bench.py --device-data-gb 200 --batch 268435456 --steps 10 --warmup 2 > gpurun_out/j/mega_batch.json 2> gpurun_out/j/mega_batch.err || exit 5
python - <<'PY'
import json
for f in ['mega_data','mega_batch']:
    d=json.loads(open(f'gpurun_out/j/{f}.json').read().strip().splitlines()[-1])
    print(f, round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],3), 'ms/step', 'acc', d['val'].get('acc'), 'gen', d['datagen'])
PY
