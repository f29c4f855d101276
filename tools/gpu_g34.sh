#!/bin/bash
# Round-5 batch 32: the 256 GEMM under the LLVM AMDGPU scheduler strategies max-ilp / max-memory-clause
# (side builds of csrc/gemm.hip) vs the default: 8192^2 layers per GEMM, 3 interleaved rounds; then the
# fused train kernel's max-memory-clause build: parameter hash vs the shipped kernel + 3 more headline rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/euromillioner_amd/lib/ab
O=gpurun_out/g34
mkdir -p $O
for r in 1 2 3; do
  for v in base gemm_ilp gemm_memclause; do
    if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
    env $E timeout -k 10 200 python tools/gemm_bench.py --no-lib --iters 10 --cases fwd_hidden,dgrad_hidden_bits,wgrad_hidden_nt > $O/g_${v}_$r.jsonl 2>&1 || { tail $O/g_${v}_$r.jsonl; exit 3; }
    grep '^{' $O/g_${v}_$r.jsonl | sed "s/^/$v $r /" | cut -c1-100
  done
done
for v in base sched_memclause; do
  if [ $v = base ]; then E=""; else E="EUROM_NATIVE_LIB=$L/$v.so"; fi
  env $E timeout -k 10 200 python tools/ab_hash.py > $O/hash_$v.jsonl 2>&1 || { tail $O/hash_$v.jsonl; exit 4; }
  grep '^{' $O/hash_$v.jsonl
done
rm -f gpurun_out/ab/results.jsonl
ARMS="base|X=0;sched_memclause|EUROM_NATIVE_LIB=$L/sched_memclause.so" ROUNDS=3 bash tools/gpu_ab.sh || exit 5
cp gpurun_out/ab/results.jsonl $O/ab_sched_confirm.jsonl
echo rc=0
