# A/B of two native builds on one box: bench.py alternately with EUROM_NATIVE_LIB=<a> and the in-tree lib.
# usage: bash tools/ab_bench.sh abtest/old.so [rounds]
set -o pipefail
A=$1; R=${2:-3}
for i in $(seq 1 $R); do
  EUROM_NATIVE_LIB=$PWD/$A timeout -k 10 120 python bench.py --steps 100 > gpurun_out/ab_a.json || exit $?
  timeout -k 10 120 python bench.py --steps 100 > gpurun_out/ab_b.json || exit $?
  python -c "import json;a=json.load(open('gpurun_out/ab_a.json'));b=json.load(open('gpurun_out/ab_b.json'));print(f'A {a[\"ms_per_step\"]*1e3:.2f} us  B {b[\"ms_per_step\"]*1e3:.2f} us')"
done
