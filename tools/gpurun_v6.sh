# v6 producer/consumer fused kernel: GPU tests under EM_FUSED_V6=1, then same-box bench A/B:
# base (lib/ab/base.so) vs the in-tree build, both v6
set -o pipefail
mkdir -p gpurun_out/v6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_fused_mlp_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/v6/t_fused.log 2>&1 || { tail -40 gpurun_out/v6/t_fused.log; exit 3; }
tail -2 gpurun_out/v6/t_fused.log
one() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 200 --warmup 10 > gpurun_out/v6/$tag.json 2>/dev/null || return 1
  python -c "import json;a=json.load(open('gpurun_out/v6/$tag.json'));print(f'$tag {a[\"value\"]/1e9:.3f} G/s med {a[\"ms_per_step_median\"]*1e3:.2f} us acc {a[\"val\"][\"acc\"]:.4f}')"
}
for i in 1 2; do
  one base_$i EM_FUSED_V6=1 EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/base.so || exit 4
  one new_$i EM_FUSED_V6=1 || exit 5
done
