#!/bin/bash
# One GPU call that refreshes every committed profile summary (see profiles/README.md):
#   rocprofv3 --kernel-trace --stats for the headline fused MLP, the wide MLP, the RF and GBDT engines,
#   derived PMC metrics (each --pmc set in its own run, never combined with traces).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/profiles
rm -rf $OUT && mkdir -p $OUT
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -1 $OUT/$name.log | cut -c1-160
  case $rc in 0) return 0;; *) exit $rc;; esac
}
run fused_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fused -o run -- python3 bench.py --steps 20 --warmup 3 --graph 0 --no-eval
run wide_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/wide -o run -- python3 bench.py --model mlp-wide --steps 5 --warmup 2 --graph 0 --no-eval
run rf_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rf -o run -- python3 tools/rf_bench.py --repeat 2
run gbdt_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/gbdt -o run -- python3 tools/gbdt_bench.py
run fused_pmc 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/fused_pmc -o run -- python3 bench.py --steps 6 --warmup 2 --graph 0 --no-eval
run fused_pmc2 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/fused_pmc2 -o run -- python3 bench.py --steps 6 --warmup 2 --graph 0 --no-eval
run wide_pmc 400 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE FETCH_SIZE --output-format csv -d $OUT/wide_pmc -o run -- python3 bench.py --model mlp-wide --steps 3 --warmup 1 --graph 0 --no-eval
run bench_headline 300 python3 bench.py --steps 100 --warmup 10
run bench_torch 300 python3 bench.py --steps 20 --warmup 3 --graph 0 --impl torch --no-eval
run bench_wide 300 python3 bench.py --model mlp-wide --steps 10 --warmup 3
run bench_mega_data 300 python3 bench.py --device-data-gb 200 --steps 50 --warmup 5
run bench_mega_batch 300 python3 bench.py --device-data-gb 200 --batch 268435456 --steps 10 --warmup 2
run bench_wide_mega 400 python3 bench.py --model mlp-wide --device-data-gb 100 --accum 16 --steps 4 --warmup 1
run gemm_bench 300 python3 tools/gemm_bench.py
run rf_bench 300 python3 tools/rf_bench.py
run gbdt_bench 300 python3 tools/gbdt_bench.py
echo ALL_OK
