#!/bin/bash
# Side library for same-box A/B runs: the current objects with one kernel source recompiled under extra
# -D flags, linked to euromillioner_amd/lib/ab/<name>.so (the shipped library is untouched).
#   bash tools/build_variant.sh <name> -DKNOB=1 ...      then  EUROM_NATIVE_LIB=$PWD/euromillioner_amd/lib/ab/<name>.so
# FILE=csrc/<x>.hip picks the source to vary (default csrc/mlp_fused.hip); SRC=<file> compiles another
# version of it in its place (e.g. `git show HEAD:csrc/mlp_fused.hip > build/ab/old.hip`).
set -e
cd "$(dirname "$0")/.."
name=$1; shift
FILE=${FILE:-csrc/mlp_fused.hip}
base=$(basename "$FILE")
python -c "import euromillioner_amd._build as b; b.build()" > /dev/null
flags=$(python -c "import euromillioner_amd._build as b, sys; print(' '.join(b.COMMON_FLAGS + b._file_flags(sys.argv[1])))" "$FILE")
OBJ=build/obj
mkdir -p build/ab euromillioner_amd/lib/ab
/opt/rocm/bin/hipcc $flags "$@" -I csrc -c "${SRC:-$FILE}" -o build/ab/${base}_$name.o
objs=$(ls $OBJ/*.hip.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o euromillioner_amd/lib/ab/$name.so $objs build/ab/${base}_$name.o -lpthread
echo euromillioner_amd/lib/ab/$name.so
