# GEMM schedule A/B on one box: race/identity tests with the new default, then the large shapes
# alternating EM_GEMM_BAL=0 / 1 (same process layout, 3 rounds each).
set -o pipefail
mkdir -p gpurun_out/gab
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gab/t_gemm.log 2>&1 || { tail -30 gpurun_out/gab/t_gemm.log; exit 3; }
tail -2 gpurun_out/gab/t_gemm.log
C=${GAB_CASES:-fwd_hidden_ct,fwd_hidden,square_8192,dgrad_hidden_nt,wgrad_hidden_nt}
timeout -k 10 120 python tools/gemm_bench.py --cases $C --iters 50 > gpurun_out/gab/lib.jsonl 2>&1 || exit 4
for i in 1 2 3; do
  for b in 0 1; do
    EM_GEMM_BAL=$b timeout -k 10 120 python tools/gemm_bench.py --cases $C --iters 50 --no-lib > gpurun_out/gab/bal${b}_$i.jsonl 2>&1 || exit 5
  done
done
python - <<'PY'
import json, glob, collections
r = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/gab/bal*_*.jsonl")):
    b = f.split("bal")[1][0]
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line); r[(d["case"], b)].append(d["ours_tflops"])
lib = {json.loads(l)["case"]: json.loads(l)["lib_tflops"] for l in open("gpurun_out/gab/lib.jsonl") if l.startswith("{")}
for (c, b), v in sorted(r.items()):
    print(f"{c:18s} BAL={b}  TF {' '.join(f'{x:7.1f}' for x in v)}   lib {lib.get(c)}")
PY
