# PMC passes on the 256x256 GEMM (tools/gemm_one.py, forward 65536 x 8192 x 8192): one rocprofv3 run per
# counter set (never combined with traces).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_gemm; mkdir -p $OUT
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/set$i -o run -- python3 tools/gemm_one.py --iters 4 > $OUT/set$i.log 2>&1
  rc=$?; echo "SET$i RC=$rc"; tail -1 $OUT/set$i.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
