# PMC passes comparing the 256x256 NT GEMM on the forward shape (M=65536, N=K=8192) with the
# weight-gradient shape (M=N=8192, K=65536): one rocprofv3 run per counter set (never with traces).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_shapes; mkdir -p $OUT
i=0
for c in fwd wgt; do
  timeout -k 10 60 python3 tools/gemm_one.py --case $c --iters 6 > $OUT/time_$c.log 2>&1 || exit $?
  tail -1 $OUT/time_$c.log
  for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/set$i -o run -- python3 tools/gemm_one.py --case $c --iters 3 > $OUT/set$i.log 2>&1
    rc=$?; echo "SET$i $c RC=$rc"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
