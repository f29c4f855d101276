set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3full; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
tail -3 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 4; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail $O/bench_driver.err; exit 5; }
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail $O/bench_default.err; exit 6; }
for f in bench_driver bench_default; do grep '^{' $O/$f.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value']/1e9, d['ms_per_step'], d['ms_per_step_median'], d['val']['acc'])"; done
rm -rf gpurun_out/ab
ARMS="split|EUROM_FUSED_ADAM=0;fused|EUROM_FUSED_ADAM=1" ROUNDS=3 bash tools/gpu_ab.sh || exit 7
