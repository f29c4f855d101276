#!/bin/bash
# GPU measurements as named stages (run through gpurun; every GPU step has its own time
# limit and a failing step ends the script).  Outputs under gpurun_out/round/<stage>/.
#   bash tools/gpu_round.sh full            GPU suite + smoke() + driver-shape and default bench
#   bash tools/gpu_round.sh headline-prof   kernel trace + 2 PMC passes of the headline step, phase
#                                           stamps when the FUSED_STAMPS side build lib/ab/stamps.so exists
#   bash tools/gpu_round.sh gbdt            GBDT GPU tests, kernel trace of the 183k-row case, gbdt_bench
#   bash tools/gpu_round.sh fp32            bench.py --dtype fp32 + kernel trace
#   bash tools/gpu_round.sh wide            wide-MLP bench + kernel trace, one-GPU overlap rehearsal
#   bash tools/gpu_round.sh gbdt-ref        GBDT reference fit: GPU tests, bench, phase
#                                           stamps (needs lib/ab/gbdt_stamps.so: build_variant.sh -DGBDT_STAMPS=1)
#   bash tools/gpu_round.sh rf-ab           RF tests + rf_bench against lib/ab/rf_head.so (the committed
#                                           forest.hip: SRC=... build_variant.sh rf_head), kernel stats
#   bash tools/gpu_round.sh dp-proxy        one-GPU DP=8 small-MLP exchange proxy (tools/xgmi_budget.py)
#   bash tools/gpu_round.sh hbm-fill        HBM-filling 256M-sample runs on p = 0.9 and p = 0.7
#   bash tools/gpu_round.sh v8              K7 v8 (EUROM_FUSED_V=8): fused GPU tests, v6/v8 A/B, phase timeline
#   bash tools/gpu_round.sh pmc-ab          two PMC passes of the train kernel per arm of PMC_ARMS
#   bash tools/gpu_round.sh tests           pytest -m gpu over TESTS (default: the whole suite)
#   bash tools/gpu_round.sh ab              tools/gpu_ab.sh with ARMS / ROUNDS / BENCH_ARGS
#   bash tools/gpu_round.sh dp2             2-rank shared-GPU bench rehearsal + the 1-rank driver shape
#   bash tools/gpu_round.sh gbdt-host       host-side profile of the GBDT reference fit
#   bash tools/gpu_round.sh k7-trace        per-tile event trace of the v8 train kernel
# (round 6 folded the one-off tools/gpu_gNN.sh batch scripts of rounds 3-5 into these stages; git history
# keeps them)
# Several stages run in order: bash tools/gpu_round.sh gbdt fp32
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
summ() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', d['value'], d['ms_per_step'], (d.get('val') or {}).get('acc'))"; }
for stage in "$@"; do
  O=gpurun_out/round/$stage
  mkdir -p $O
  case $stage in
  full)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
    tail -1 $O/pytest.log
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 4; }
    tail -1 $O/smoke.log
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail $O/bench_driver.err; exit 5; }
    timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 6; }
    summ $O/bench_driver.json driver && summ $O/bench_default.json default || exit 7
    ;;
  headline-prof)
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 200 --warmup 5 --no-eval > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 9; }
    timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc1 -o run -- python bench.py --steps 20 --warmup 5 --no-eval --graph 0 > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 10; }
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc2 -o run -- python bench.py --steps 20 --warmup 5 --no-eval --graph 0 > $O/pmc2.log 2>&1 || { tail -20 $O/pmc2.log; exit 11; }
    if [ -f euromillioner_amd/lib/ab/stamps.so ]; then
      EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/stamps.so TL_B=1048576 timeout -k 10 200 python tools/fused_timeline.py > $O/timeline.txt 2>&1 || { tail -20 $O/timeline.txt; exit 12; }
      cat $O/timeline.txt
    fi
    ;;
  v8)
    # K7 v8 (three waves per SIMD): fused-kernel GPU tests on v8, same-box v6/v8 A/B, v8 phase timeline
    EUROM_FUSED_V=8 timeout -k 10 400 python -u -m pytest tests/test_fused_mlp_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_v8.log 2>&1 || { tail -40 $O/pytest_v8.log; exit 30; }
    tail -3 $O/pytest_v8.log
    ARMS=${V8_ARMS:-"v6|EUROM_FUSED_V=6;v8|EUROM_FUSED_V=8"} ROUNDS=${V8_ROUNDS:-3} bash tools/gpu_ab.sh || exit 31
    if [ -f euromillioner_amd/lib/ab/stamps.so ]; then
      EUROM_FUSED_V=8 EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/stamps.so TL_B=1048576 timeout -k 10 200 python tools/fused_timeline.py > $O/timeline_v8.txt 2>&1 || { tail -20 $O/timeline_v8.txt; exit 32; }
      cat $O/timeline_v8.txt
    fi
    ;;
  pmc-ab)
    # the same two PMC passes for each arm of PMC_ARMS="name|ENV=..;name2|ENV=.." (train-kernel counters, eager launches)
    IFS=';' read -ra LIST <<< "${PMC_ARMS:-v6|EUROM_FUSED_V=6;v8|EUROM_FUSED_V=8}"
    for arm in "${LIST[@]}"; do
      name=${arm%%|*}; envs=${arm#*|}
      for pass in 1 2; do
        if [ $pass = 1 ]; then C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE";
        else C="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"; fi
        env $envs timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/$name/p$pass -o run -- python bench.py --steps 20 --warmup 5 --no-eval --graph 0 > $O/${name}_p$pass.log 2>&1 || { tail -20 $O/${name}_p$pass.log; exit 40; }
      done
    done
    python tools/summarize_profiles.py pmc-ab $O > $O/pmc_ab.md 2>&1; cat $O/pmc_ab.md
    ;;
  gbdt)
    timeout -k 10 400 python -u -m pytest tests/test_gbdt.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 13; }
    tail -1 $O/pytest.log
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python tools/gbdt_bench.py 262k > $O/trace.log 2>&1 || { tail $O/trace.log; exit 14; }
    timeout -k 10 300 python tools/gbdt_bench.py > $O/gbdt_bench.jsonl 2> $O/gbdt_bench.err || { tail $O/gbdt_bench.err; exit 15; }
    cat $O/gbdt_bench.jsonl
    ;;
  fp32)
    timeout -k 10 300 python bench.py --dtype fp32 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 16; }
    summ $O/bench.json fp32 || exit 17
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --dtype fp32 --steps 20 --warmup 5 --no-eval > $O/trace.log 2>&1 || { tail $O/trace.log; exit 18; }
    ;;
  wide)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --model mlp-wide --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 19; }
    summ $O/bench.json wide || exit 20
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/overlap -o run -- python tools/wide_overlap.py > $O/overlap.jsonl 2> $O/overlap.err || { tail $O/overlap.err; exit 21; }
    python tools/wide_overlap.py report $O/overlap/run_kernel_trace.csv > $O/overlap_report.jsonl && cat $O/overlap.jsonl
    ;;
  gbdt-ref)
    timeout -k 10 400 python -u -m pytest tests/test_gbdt.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 22; }
    tail -1 $O/pytest.log
    for rnd in 1 2; do
      timeout -k 10 200 python tools/gbdt_bench.py reference > $O/eager_$rnd.jsonl 2>&1 || { tail $O/eager_$rnd.jsonl; exit 23; }
    done
    grep -h -o '"hip_s": [0-9.]*' $O/eager_?.jsonl
    if [ -f euromillioner_amd/lib/ab/gbdt_stamps.so ]; then
      EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/gbdt_stamps.so timeout -k 10 120 python tools/gbdt_stamps.py > $O/stamps.jsonl 2>&1 || { tail $O/stamps.jsonl; exit 24; }
      cat $O/stamps.jsonl
    fi
    ;;
  rf-ab)
    timeout -k 10 300 python -u -m pytest tests/test_forest.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 25; }
    tail -1 $O/pytest.log
    for rnd in 1 2; do
      timeout -k 10 120 python tools/rf_bench.py > $O/new_$rnd.jsonl 2>&1 || { tail $O/new_$rnd.jsonl; exit 26; }
      if [ -f euromillioner_amd/lib/ab/rf_head.so ]; then
        EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/rf_head.so timeout -k 10 120 python tools/rf_bench.py > $O/head_$rnd.jsonl 2>&1 || { tail $O/head_$rnd.jsonl; exit 26; }
      fi
    done
    for f in $O/*_?.jsonl; do echo "$f $(grep -o '"fit_s": [0-9.]*' $f)"; done
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python tools/rf_bench.py --repeat 2 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 27; }
    ;;
  dp-proxy)
    timeout -k 10 240 python tools/xgmi_budget.py > $O/xgmi_budget.jsonl 2>&1 || { tail -20 $O/xgmi_budget.jsonl; exit 28; }
    grep round $O/xgmi_budget.jsonl
    ;;
  hbm-fill)
    for pl in 0.9 0.7; do
      timeout -k 10 300 python bench.py --device-data-gb -1 --batch 268435456 --steps 10 --warmup 2 --planted $pl > $O/fill_$pl.json 2> $O/fill_$pl.err || { tail $O/fill_$pl.err; exit 29; }
      summ $O/fill_$pl.json fill_$pl || exit 30
    done
    ;;
  tests)
    # named GPU test files / node ids: TESTS="tests/test_gbdt.py tests/test_forest.py::test_x" (default: the suite)
    timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 41; }
    tail -1 $O/pytest.log
    ;;
  ab)
    # same-box interleaved bench A/B: ARMS="name|ENV=..;name2|EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/x.so"
    # (side libraries from tools/build_variant.sh), ROUNDS, BENCH_ARGS as in tools/gpu_ab.sh
    bash tools/gpu_ab.sh || exit 42
    cp gpurun_out/ab/results.jsonl $O/results.jsonl
    ;;
  dp2)
    # 2-rank bench.py rehearsal of the DP path with both ranks on the one GPU (gloo control plane; the fused
    # xGMI exchange carries the gradients), then the 1-rank driver shape
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo > $O/bench_dp2.json 2> $O/bench_dp2.err || { grep -v amdgpu.ids $O/bench_dp2.err | tail -20; exit 43; }
    grep '^{' $O/bench_dp2.json | cut -c1-600
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_dp1.json 2> $O/bench_dp1.err || { tail $O/bench_dp1.err; exit 44; }
    summ $O/bench_dp1.json dp1 || exit 45
    ;;
  gbdt-host)
    # host-side profile of the GBDT reference fit (tools/gbdt_fit_profile.py)
    timeout -k 10 300 python tools/gbdt_fit_profile.py > $O/gbdt_fit_profile.txt 2>&1 || { tail -20 $O/gbdt_fit_profile.txt; exit 46; }
    head -60 $O/gbdt_fit_profile.txt
    ;;
  k7-trace)
    # per-tile event trace of the v8 train kernel (needs lib/ab/trace.so: build_variant.sh trace -DFUSED_TRACE=1)
    EUROM_FUSED_V=8 EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/trace.so timeout -k 10 120 python tools/fused_trace.py > $O/trace.txt 2>&1 || { tail $O/trace.txt; exit 47; }
    tail -9 $O/trace.txt
    ;;
  *) echo "unknown stage $stage"; exit 2;;
  esac
done
