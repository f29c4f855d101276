# GPU test files given as arguments (default: the whole gpu suite), one pytest process
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED|passed|failed" gpurun_out/gpu_tests.log | tail -60
exit $rc
