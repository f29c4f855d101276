#!/bin/bash
# Round-5 same-box A/Bs: headline step (fused-kernel b2 placement, Adam slab-reduction shapes) and the
# GBDT reference fit (histogram chunk size).  Side libraries: tools/build_variant.sh.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/g2
L=$PWD/euromillioner_amd/lib/ab
ARMS="base|EUROM_X=0;b2early|EUROM_NATIVE_LIB=$L/b2early.so;adam_g32|EUROM_NATIVE_LIB=$L/adam_g32.so;adam_nt|EUROM_NATIVE_LIB=$L/adam_nt.so" ROUNDS=3 BENCH_ARGS="--steps 100 --warmup 5 --no-eval" timeout -k 10 900 bash tools/gpu_ab.sh > gpurun_out/g2/ab.log 2>&1 || { tail -20 gpurun_out/g2/ab.log; exit 3; }
cp gpurun_out/ab/results.jsonl gpurun_out/g2/ab_headline.jsonl
for r in 1 2; do
  for v in base gbdt_chunk128 gbdt_chunk256; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/gbdt_bench.py reference > gpurun_out/g2/gbdt_${v}_$r.jsonl 2>&1 || { tail gpurun_out/g2/gbdt_${v}_$r.jsonl; exit 4; }
    echo "$v $r $(grep -o '"hip_s": [0-9.]*' gpurun_out/g2/gbdt_${v}_$r.jsonl)"
  done
done
cat gpurun_out/g2/ab_headline.jsonl
EUROM_NATIVE_LIB=$L/stamps.so TL_B=1048576 timeout -k 10 200 python tools/fused_timeline.py > gpurun_out/g2/timeline.txt 2>&1 || { tail -20 gpurun_out/g2/timeline.txt; exit 5; }
cat gpurun_out/g2/timeline.txt
