# A/B of lib/ab/new.so (tests + bench) against lib/ab/base.so
set -o pipefail
mkdir -p gpurun_out/v6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NEW=$PWD/euromillioner_amd/lib/ab/new.so; BASE=$PWD/euromillioner_amd/lib/ab/base.so
EUROM_NATIVE_LIB=$NEW timeout -k 10 300 python -u -m pytest tests/test_fused_mlp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/v6/t_new.log 2>&1 || { tail -30 gpurun_out/v6/t_new.log; exit 3; }
tail -1 gpurun_out/v6/t_new.log
one() {  # tag lib
  EUROM_NATIVE_LIB=$2 timeout -k 10 120 python bench.py --steps 200 --warmup 10 > gpurun_out/v6/$1.json 2>/dev/null || return 1
  python -c "import json;a=json.loads(open('gpurun_out/v6/$1.json').read().strip().splitlines()[-1]);print(f'$1 {a[\"value\"]/1e9:.3f} G/s med {a[\"ms_per_step_median\"]*1e3:.2f} us acc {a[\"val\"][\"acc\"]:.4f}')"
}
for i in 1 2; do one base_$i $BASE || exit 4; one new_$i $NEW || exit 5; done
