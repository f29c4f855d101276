#!/bin/bash
# Round-5 batch 19: GBDT exact histogram with LDS fp64 atomic adds (ds_add_f64) vs read-modify-write
# (gbdt_rmw): tests + A/B; then a 2-rank bench.py rehearsal of the DP path (both ranks on the one GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/g21
mkdir -p $O
L=$R/euromillioner_amd/lib/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gbdt.py -m gpu > $O/pytest_gbdt.log 2>&1 || { tail -40 $O/pytest_gbdt.log; exit 2; }
tail -1 $O/pytest_gbdt.log
for r in 1 2 3; do
  for v in base gbdt_rmw; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_${v}_$r.jsonl 2>&1 || { tail $O/gbdt_${v}_$r.jsonl; exit 3; }
    echo "$v $r $(grep -o '"hip_s": [0-9.]*, "hip_test_logloss": [0-9.]*, "hip_trees_per_s": [0-9.]*' $O/gbdt_${v}_$r.jsonl)"
  done
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo > $O/bench_dp2.json 2> $O/bench_dp2.err || { tail -20 $O/bench_dp2.err; exit 4; }
grep '^{' $O/bench_dp2.json | cut -c1-400
echo rc=0
