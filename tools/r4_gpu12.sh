set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4m; mkdir -p $O
EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/gbdt_stamps.so EM_GBDT_GRAPH=0 timeout -k 10 120 python tools/gbdt_stamps.py > $O/stamps.jsonl 2>&1 || { tail $O/stamps.jsonl; exit 6; }
EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/gbdt_stamps.so EM_GBDT_GRAPH=0 timeout -k 10 120 python tools/gbdt_stamps.py >> $O/stamps.jsonl 2>&1 || { tail $O/stamps.jsonl; exit 6; }
grep split $O/stamps.jsonl
