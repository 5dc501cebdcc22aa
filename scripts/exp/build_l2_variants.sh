#!/bin/bash
# Experiment builds of match_l2.hip with -DMCV_EXP_L2=N linked against the product's other objects,
# into libs/exp/N/ (screens only; the product build defines nothing).
set -e
cd "$(dirname "$0")/../.."
python -c "import __graft_entry__ as g; g.build()" > /dev/null
for n in "$@"; do
    mkdir -p build/exp/$n libs/exp/$n
    /opt/rocm/bin/hipcc -x hip -std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize \
        -fvisibility=hidden -Iinclude -Iminicv_amd/csrc -DMCV_EXP_L2=$n -c minicv_amd/csrc/match_l2.hip -o build/exp/$n/match_l2.o
    objs=$(ls build/native/*.o | grep -v match_l2.hip.o)
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o libs/exp/$n/libMiniCVNative.so $objs build/exp/$n/match_l2.o
done
