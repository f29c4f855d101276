# GEMM box-variance check: forward GEMM vs hipBLASLt twice, then one PMC pass of the forward shape
set -o pipefail
mkdir -p gpurun_out/gvar
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
(rocm-smi --showclocks --showpower --showtemp > gpurun_out/gvar/smi_before.txt 2>&1 || true)
for i in 1 2; do
  timeout -k 10 120 python tools/gemm_bench.py --cases fwd_hidden,square_8192,wgrad_hidden_nt > gpurun_out/gvar/bench$i.log 2>&1 || { tail -5 gpurun_out/gvar/bench$i.log; exit 3; }
  grep '^{' gpurun_out/gvar/bench$i.log | cut -c1-170
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/gvar/pmc -o run -- python3 tools/gemm_one.py --case fwd --iters 3 > gpurun_out/gvar/pmc.log 2>&1 || exit 4
(rocm-smi --showclocks --showpower --showtemp > gpurun_out/gvar/smi_after.txt 2>&1 || true)
python - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/gvar/pmc/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'gemm256' in r['Kernel_Name']:
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(acc.items()):
    print(k, 'median %.4g' % sorted(v)[len(v) // 2])
PY
