#!/bin/bash
# PMC passes over one RF fit (tools/rf_bench.py --repeat 1): instruction mix and LDS pressure of
# rf_init_rows / rf_partition.  One rocprofv3 run per counter set, --pmc only (no traces).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=${1:-gpurun_out/rfpmc}
mkdir -p $O
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/set$i -o run -- python3 tools/rf_bench.py --repeat 1 > $O/set$i.log 2>&1
  rc=$?; echo "SET$i RC=$rc"
  [ $rc = 0 ] || { tail -5 $O/set$i.log; exit $rc; }
done
