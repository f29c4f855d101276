# fused small-n GBDT: GPU tests, then the reference-config bench with the fused path on and off
set -o pipefail
mkdir -p gpurun_out/gb
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gbdt.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gb/t.log 2>&1 || { tail -40 gpurun_out/gb/t.log; exit 3; }
tail -1 gpurun_out/gb/t.log
for i in 1 2; do
  timeout -k 10 200 python tools/gbdt_bench.py reference_calendar > gpurun_out/gb/fused_$i.json 2>/dev/null || exit 4
  EM_GBDT_FUSED=0 timeout -k 10 200 python tools/gbdt_bench.py reference_calendar > gpurun_out/gb/kern_$i.json 2>/dev/null || exit 5
  echo "fused: $(cat gpurun_out/gb/fused_$i.json)"; echo "kernels: $(cat gpurun_out/gb/kern_$i.json)"
done
