# GEMM A/B on one box: current gemm.hip (runtime staging-lead flag), compile-time lead 0, and the
# gemm.hip of commit 7dda647 (before the G_STAMPS / EM_GEMM_LEAD instrumentation); 2 rounds each
set -o pipefail
mkdir -p gpurun_out/gsweep
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
cp csrc/gemm.hip gpurun_out/gsweep/gemm_current.hip
run() {  # label, build args...
  local label=$1; shift
  python -m euromillioner_amd._build "$@" > gpurun_out/gsweep/build_$label.log 2>&1 || { echo "BUILD FAIL $label"; tail -5 gpurun_out/gsweep/build_$label.log; exit 3; }
  timeout -k 10 120 python tools/gemm_bench.py --cases fwd_hidden,square_8192,wgrad_hidden_nt --no-lib > gpurun_out/gsweep/b_$label.log 2>&1 || { tail -5 gpurun_out/gsweep/b_$label.log; exit 4; }
  grep '^{' gpurun_out/gsweep/b_$label.log | python -c "import json,sys; print('$label', ' '.join('%s %.0f' % (j['case'], j['ours_tflops']) for j in map(json.loads, sys.stdin)))"
}
for r in 1 2; do
  cp gpurun_out/gsweep/gemm_current.hip csrc/gemm.hip
  run cur$r
  run ct0_$r --define G_LEAD=0
  cp tools/dev/gemm_7dda647.hip csrc/gemm.hip
  run old$r
done
cp gpurun_out/gsweep/gemm_current.hip csrc/gemm.hip
