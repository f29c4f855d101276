set -o pipefail
O=gpurun_out/gb; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gbdt.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  EM_GBDT_PRESPLIT=0 timeout -k 10 200 python tools/gbdt_bench.py reference > $O/off_$r.jsonl 2>&1 || { tail $O/off_$r.jsonl; exit 3; }
  timeout -k 10 200 python tools/gbdt_bench.py reference > $O/on_$r.jsonl 2>&1 || { tail $O/on_$r.jsonl; exit 4; }
done
for f in $O/off_?.jsonl $O/on_?.jsonl; do echo "$f $(grep -o '"hip_s": [0-9.]*' $f)"; done
L=$PWD/euromillioner_amd/lib/ab
ARMS="s8|EUROM_X=0;s6|EUROM_NATIVE_LIB=$L/r4.so;s4|EUROM_NATIVE_LIB=$L/r2.so" ROUNDS=3 bash tools/gpu_ab.sh
