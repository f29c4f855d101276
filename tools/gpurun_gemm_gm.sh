# GEMM tile-grouping A/B (EM_GEMM_GM)
set -o pipefail
mkdir -p gpurun_out/ggm
export TMPDIR=/tmp
C=${GM_CASES:-fwd_hidden,fwd_hidden_ct,square_8192,wgrad_hidden_nt,dgrad_hidden_nt}
for i in 1 2; do
  for gm in ${GM_LIST:-1 2 4 8}; do
    EM_GEMM_GM=$gm timeout -k 10 120 python tools/gemm_bench.py --cases $C --iters 40 --no-lib > gpurun_out/ggm/gm${gm}_$i.jsonl 2>&1 || exit 4
    echo "GM=$gm $(grep -o '"case": "[a-z_0-9]*"\|"ours_tflops": [0-9.]*' gpurun_out/ggm/gm${gm}_$i.jsonl | sed 's/"case": //; s/"ours_tflops": //' | tr '\n' ' ')"
  done
done
