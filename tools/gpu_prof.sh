#!/bin/bash
# rocprofv3 kernel-trace + stats of the headline bench (fused) and the torch comparison.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/fused -o run -- \
  python3 bench.py --steps 20 --warmup 3 --graph 0 --no-eval > gpurun_out/prof/fused_bench.log 2>&1
rc=$?; echo "PROF_FUSED_RC=$rc"; tail -1 gpurun_out/prof/fused_bench.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --graph 0 --impl torch > gpurun_out/prof/torch_bench.log 2>&1
rc=$?; echo "TORCH_RC=$rc"; tail -1 gpurun_out/prof/torch_bench.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --graph 1 --no-eval > gpurun_out/prof/graph_bench.log 2>&1
rc=$?; echo "GRAPH_RC=$rc"; tail -1 gpurun_out/prof/graph_bench.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/wide -o run -- \
  python3 bench.py --model mlp-wide --steps 5 --warmup 2 --graph 0 --no-eval > gpurun_out/prof/wide_bench.log 2>&1
rc=$?; echo "PROF_WIDE_RC=$rc"; tail -1 gpurun_out/prof/wide_bench.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/rf -o run -- \
  python3 tools/rf_bench.py --repeat 2 > gpurun_out/prof/rf_bench.log 2>&1
rc=$?; echo "PROF_RF_RC=$rc"; tail -1 gpurun_out/prof/rf_bench.log
find gpurun_out/prof -name "*stats*" | head -20
