set -e
# A/B of two libem_native.so builds: BASE_LIB=<baseline .so> bash tools/ab_adam.sh (the in-tree build is "new")
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_fused_mlp_gpu.py tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/tests.log 2>&1
tail -1 gpurun_out/ab/tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base new; do
  if [ $v = base ]; then export EUROM_NATIVE_LIB=${BASE_LIB:?set BASE_LIB to the baseline libem_native.so}; else unset EUROM_NATIVE_LIB; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/prof_$v -o run -- python3 bench.py --steps 200 --warmup 10 --no-eval > gpurun_out/ab/bench_$v.json 2> gpurun_out/ab/bench_$v.err
done
for r in 1 2; do for v in base new; do
  if [ $v = base ]; then export EUROM_NATIVE_LIB=${BASE_LIB:?set BASE_LIB to the baseline libem_native.so}; else unset EUROM_NATIVE_LIB; fi
  timeout -k 10 120 python3 bench.py --steps 200 --warmup 10 --no-eval > gpurun_out/ab/b_${v}_$r.json 2>/dev/null
  echo $v $(python3 -c "import json,sys;d=json.loads(open('gpurun_out/ab/b_${v}_$r.json').read().strip().splitlines()[-1]);print(round(d['value']/1e9,3),round(d['ms_per_step'],4))")
done; done
find gpurun_out/ab -name '*kernel_stats.csv' | while read f; do echo $f; grep -i "adam\|mlp_fused" $f | cut -c1-200; done
