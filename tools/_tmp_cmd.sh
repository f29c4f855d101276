set -o pipefail
O=gpurun_out/xg; mkdir -p $O
L=$PWD/euromillioner_amd/lib/ab
timeout -k 10 400 python -u -m pytest tests/test_xgmi_proxy_gpu.py tests/test_xgmi_gpu.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  XB_ROUNDS=1 timeout -k 10 240 python tools/xgmi_budget.py > $O/new_$r.jsonl 2>&1 || { tail -20 $O/new_$r.jsonl; exit 3; }
  XB_ROUNDS=1 EUROM_NATIVE_LIB=$L/adam_head.so timeout -k 10 240 python tools/xgmi_budget.py > $O/head_$r.jsonl 2>&1 || { tail -20 $O/head_$r.jsonl; exit 4; }
done
for f in $O/head_?.jsonl $O/new_?.jsonl; do echo "== $f"; grep '^{' $f | cut -c1-220; done
