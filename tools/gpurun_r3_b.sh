set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r3b
for arm in "old|EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/old.so EUROM_FUSED_ADAM=0" "split|EUROM_FUSED_ADAM=0" "fused|EUROM_FUSED_ADAM=1"; do
  name=${arm%%|*}; envs=${arm#*|}
  export $envs
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b/$name -o run -- python bench.py --steps 200 --warmup 5 --no-eval > gpurun_out/r3b/$name.log 2>&1 || { tail -30 gpurun_out/r3b/$name.log; exit 3; }
  unset EUROM_NATIVE_LIB EUROM_FUSED_ADAM
  grep '^{' gpurun_out/r3b/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', d['ms_per_step'])"
done
