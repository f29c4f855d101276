#!/bin/bash
# Round-5 batch 20: 2-rank bench.py rehearsal of the DP path with both ranks on the one GPU (gloo for the
# control plane; the fused xGMI exchange carries the gradients), then the 1-rank driver shape.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/g50
mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo > $O/bench_dp2.json 2> $O/bench_dp2.err || { grep -v amdgpu.ids $O/bench_dp2.err | tail -20; exit 4; }
grep '^{' $O/bench_dp2.json | cut -c1-600
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_dp1.json 2> $O/bench_dp1.err || { tail $O/bench_dp1.err; exit 5; }
grep '^{' $O/bench_dp1.json | cut -c1-300
echo rc=0
