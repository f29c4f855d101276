#!/bin/bash
# Round-5 batch 17: MN-operand GEMM with whole-line A units (G_WGRAD_AMN=2 vs 1): GEMM tests, per-GEMM
# A/B, LDS-conflict PMC of the wgrad forms; then the GBDT deep in-pass splits (tests + A/B vs gbdt_nodeep).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/g19
mkdir -p $O
L=$R/euromillioner_amd/lib/ab
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py > $O/pytest_gemm.log 2>&1 || { tail -40 $O/pytest_gemm.log; exit 2; }
tail -1 $O/pytest_gemm.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gbdt.py -m gpu > $O/pytest_gbdt.log 2>&1 || { tail -40 $O/pytest_gbdt.log; exit 3; }
tail -1 $O/pytest_gbdt.log
for r in 1 2; do
  timeout -k 10 200 python tools/gemm_bench.py --no-lib --iters 10 --cases wgrad_hidden_nt,wgrad_hidden > $O/gemm_base_$r.jsonl 2>&1 || { tail $O/gemm_base_$r.jsonl; exit 4; }
  grep '^{' $O/gemm_base_$r.jsonl | cut -c1-120
  EUROM_NATIVE_LIB=$L/gemm_amn1.so timeout -k 10 200 python tools/gemm_bench.py --no-lib --iters 10 --cases wgrad_hidden > $O/gemm_amn1_$r.jsonl 2>&1 || { tail $O/gemm_amn1_$r.jsonl; exit 5; }
  grep '^{' $O/gemm_amn1_$r.jsonl | cut -c1-120
done
for r in 1 2 3; do
  for v in base gbdt_nodeep; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/gbdt_bench.py reference > $O/gbdt_${v}_$r.jsonl 2>&1 || { tail $O/gbdt_${v}_$r.jsonl; exit 6; }
    echo "$v $r $(grep -o '"hip_s": [0-9.]*, "hip_test_logloss": [0-9.]*, "hip_trees_per_s": [0-9.]*' $O/gbdt_${v}_$r.jsonl)"
  done
done
cd /tmp
for c in wgrad_hidden wgrad_hidden_nt; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d $O/pmc_$c -o run -- python3 $R/tools/gemm_bench.py --no-lib --iters 2 --cases $c > $O/pmc_$c.log 2>&1 || { tail -5 $O/pmc_$c.log; exit 7; }
done
echo rc=0
