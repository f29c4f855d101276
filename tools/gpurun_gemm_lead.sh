# pp16 staging lead A/B (needs a --define G_LEAD=-1 build): race screen + numerics with EM_GEMM_LEAD=1, then alternating bench rounds
set -o pipefail
mkdir -p gpurun_out/glead
export TMPDIR=/tmp
EM_GEMM_LEAD=1 timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/glead/t.log 2>&1 || { tail -30 gpurun_out/glead/t.log; exit 3; }
tail -1 gpurun_out/glead/t.log
C=fwd_hidden,fwd_hidden_ct,square_8192,wgrad_hidden_nt,dgrad_hidden_nt
for i in 1 2; do
  for l in 0 1; do
    EM_GEMM_LEAD=$l timeout -k 10 120 python tools/gemm_bench.py --cases $C --iters 40 --no-lib > gpurun_out/glead/l${l}_$i.jsonl 2>&1 || exit 4
    echo "LEAD=$l $(grep -o '"case": "[a-z_0-9]*"\|"ours_tflops": [0-9.]*' gpurun_out/glead/l${l}_$i.jsonl | sed 's/"case": //; s/"ours_tflops": //' | tr '\n' ' ')"
  done
done
