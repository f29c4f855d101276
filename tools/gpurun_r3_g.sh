set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3g; mkdir -p $O
EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/stamps.so TL_B=1048576 timeout -k 10 200 python tools/fused_timeline.py > $O/timeline.txt 2>&1 || { tail -20 $O/timeline.txt; exit 3; }
cat $O/timeline.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc1 -o run -- python bench.py --steps 20 --warmup 5 --no-eval --graph 0 > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 4; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc2 -o run -- python bench.py --steps 20 --warmup 5 --no-eval --graph 0 > $O/pmc2.log 2>&1 || { tail -20 $O/pmc2.log; exit 5; }
ls $O/pmc1 $O/pmc2
