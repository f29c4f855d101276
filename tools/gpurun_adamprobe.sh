# Adam slab kernel: time vs number of slabs reduced, and the per-launch floor, for probe builds
# (lib/ab/pN.so: ADAM_PROBE bits 1 = no ticket, 2 = no image pack, 4 = no powf)
set -o pipefail
mkdir -p gpurun_out/adamp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base p1 p2 p4 p7 base; do
  EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/$v.so timeout -k 10 120 python tools/dev/adam_probe.py > gpurun_out/adamp/$v.txt 2> gpurun_out/adamp/$v.err || exit 4
  echo "$v $(cat gpurun_out/adamp/$v.txt)"
done
