set -o pipefail
O=gpurun_out/v9; mkdir -p $O
L=$PWD/euromillioner_amd/lib/ab
EUROM_FUSED_V=9 EUROM_NATIVE_LIB=$L/tracedyn.so timeout -k 10 120 python tools/fused_trace.py > $O/trace_v9dyn.txt 2>&1 || { tail $O/trace_v9dyn.txt; exit 3; }
tail -9 $O/trace_v9dyn.txt
ARMS="v6|EUROM_FUSED_V=6;v9|EUROM_FUSED_V=9;v9dyn|EUROM_FUSED_V=9 EUROM_NATIVE_LIB=$L/dyn1.so;v9dynb0|EUROM_FUSED_V=9 EUROM_NATIVE_LIB=$L/dyn1b0.so;v9dynf1|EUROM_FUSED_V=9 EUROM_NATIVE_LIB=$L/dyn1f1.so" ROUNDS=2 bash tools/gpu_ab.sh
