#!/bin/bash
# GPU validation run (used through gpurun): smoke -> pytest -m gpu -> short bench.
# Any GPU fault / abort / timeout stops the script (no further GPU steps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "SMOKE_RC=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest ${PYTEST_ARGS:-tests -m gpu} -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "PYTEST_RC=$rc"; tail -5 gpurun_out/pytest_gpu.log
fatal $rc && exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 30 --warmup 5} > gpurun_out/bench.log 2>&1
rc=$?; echo "BENCH_RC=$rc"; tail -2 gpurun_out/bench.log
exit $rc
