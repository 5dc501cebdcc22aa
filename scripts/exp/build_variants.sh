#!/bin/bash
# Experiment builds: scripts/exp/build_variants.sh SRC MACRO N... compiles minicv_amd/csrc/SRC with
# -DMACRO=N and links it against the product's other objects into libs/exp/N/ (screens only; the
# product build defines nothing).
set -e
cd "$(dirname "$0")/../.."
src=$1; macro=$2; shift 2
python -c "import __graft_entry__ as g; g.build()" > /dev/null
for n in "$@"; do
    mkdir -p build/exp/$n libs/exp/$n
    /opt/rocm/bin/hipcc -x hip -std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize \
        -fvisibility=hidden -Iinclude -Iminicv_amd/csrc -D$macro=$n -c minicv_amd/csrc/$src -o build/exp/$n/$src.o
    objs=$(ls build/native/*.o | grep -v "/$src.o")
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o libs/exp/$n/libMiniCVNative.so $objs build/exp/$n/$src.o
done
