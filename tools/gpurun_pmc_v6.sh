# PMC of the v6 train kernel: two passes (<= 8 SQ counters each), then a summary
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_pmc.sh "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MFMA GRBM_GUI_ACTIVE GRBM_COUNT" || exit 3
python - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob('gpurun_out/pmc/set*')):
    f = glob.glob(d + '/**/*counter_collection.csv', recursive=True)
    if not f: print(d, 'no csv'); continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if 'v6_kernel' in r.get('Kernel_Name', ''):
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
    for k, v in acc.items():
        print(d.split('/')[-1], k, 'n=%d' % len(v), 'median %.4g' % sorted(v)[len(v) // 2])
PY
