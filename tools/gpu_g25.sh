#!/bin/bash
# Round-5 batch 23: store-shape micro-benchmark (bytes per row segment of a wave store instruction).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/g25
mkdir -p $O
timeout -k 10 120 ./tools/micro/store_shapes > $O/store_shapes.jsonl 2>&1 || { cat $O/store_shapes.jsonl; exit 2; }
cat $O/store_shapes.jsonl
echo rc=0
