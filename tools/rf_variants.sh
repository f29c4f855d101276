#!/bin/bash
# Same-box RF variant timing: fit_s of tools/rf_bench.py and the per-kernel trace of one fit for the
# shipped library and every euromillioner_amd/lib/ab/rf_*.so side library (tools/build_variant.sh).
#   bash tools/rf_variants.sh [outdir]
set -e
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/rfvar}
mkdir -p $O
run() {  # name lib
  local n=$1 lib=$2
  EUROM_NATIVE_LIB=$lib timeout -k 10 120 python tools/rf_bench.py > $O/$n.jsonl 2>&1 || { tail $O/$n.jsonl; return 1; }
  EUROM_NATIVE_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$n -o run -- python tools/rf_bench.py --repeat 1 > $O/tr_$n.log 2>&1 || { tail $O/tr_$n.log; return 1; }
  echo "$n $(grep -o '"fit_s": [0-9.]*' $O/$n.jsonl) $(grep -o '"nodes_split": [0-9]*' $O/$n.jsonl)"
}
run base "" 
for l in euromillioner_amd/lib/ab/rf_*.so; do run $(basename $l .so) $PWD/$l; done
