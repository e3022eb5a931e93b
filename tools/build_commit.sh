#!/bin/bash
# Development: build libpfilter_hip.so of an earlier commit into pfilter-noetic_amd/var/NAME/ for A/B
# runs (PFILTER_HIP_LIB=pfilter-noetic_amd/var/NAME/libpfilter_hip.so).  tools/build_commit.sh REV NAME
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; NAME=$2
T=$(mktemp -d)
git -C $R archive $REV pfilter-noetic_amd/csrc include | tar -x -C $T
D=$R/pfilter-noetic_amd/var/$NAME
mkdir -p $D/obj
for f in $T/pfilter-noetic_amd/csrc/*.hip; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -c $f -o $D/obj/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libpfilter_hip.so $D/obj/*.o
rm -rf $D/obj $T
echo built $D/libpfilter_hip.so
