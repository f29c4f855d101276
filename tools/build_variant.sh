#!/bin/bash
# Side library for same-box A/B runs: the current objects with csrc/mlp_fused.hip recompiled under extra
# -D flags, linked to euromillioner_amd/lib/ab/<name>.so (the shipped library is untouched).
#   bash tools/build_variant.sh <name> -DKNOB=1 ...      then  EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/<name>.so
set -e
cd "$(dirname "$0")/.."
name=$1; shift
python -c "import euromillioner_amd._build as b; b.build()" > /dev/null
OBJ=build/obj
mkdir -p build/ab euromillioner_amd/lib/ab
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result -Wno-unused-command-line-argument \
  -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form=1 "$@" -I csrc -c csrc/mlp_fused.hip -o build/ab/mlp_fused_$name.o
objs=$(ls $OBJ/*.hip.o | grep -v mlp_fused.hip.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o euromillioner_amd/lib/ab/$name.so $objs build/ab/mlp_fused_$name.o -lpthread
echo euromillioner_amd/lib/ab/$name.so
