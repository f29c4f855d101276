# GEMM compile-time sweep: one build per define set (args), 2 rounds, our kernel only
set -o pipefail
mkdir -p gpurun_out/gdefs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for r in 1 2; do
  for v in "$@"; do
    i=$((i+1))
    defs=""
    for d in $v; do defs="$defs --define $d"; done
    python -m euromillioner_amd._build $defs > gpurun_out/gdefs/build$i.log 2>&1 || { echo "BUILD FAIL $v"; exit 3; }
    timeout -k 10 120 python tools/gemm_bench.py --cases fwd_hidden,fwd_hidden_ct,dgrad_hidden_nt,wgrad_hidden_nt,square_8192 --no-lib > gpurun_out/gdefs/b$i.log 2>&1 || { tail -5 gpurun_out/gdefs/b$i.log; exit 4; }
    grep '^{' gpurun_out/gdefs/b$i.log | python -c "import json,sys; print('%-14s' % sys.argv[1], ' '.join('%s %.0f' % (j['case'], j['ours_tflops']) for j in map(json.loads, sys.stdin)))" "$v"
  done
done
