#!/bin/bash
# Development: build libpfilter_hip.so with extra compile flags into pfilter-noetic_amd/var/NAME/
# (load it with PFILTER_HIP_LIB=pfilter-noetic_amd/var/NAME/libpfilter_hip.so).
#   tools/build_variant.sh NAME "-DPF_KNN_MINW=8 ..."
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
D=$R/pfilter-noetic_amd/var/$NAME
mkdir -p $D/obj
for f in $R/pfilter-noetic_amd/csrc/*.hip; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC $* -c $f -o $D/obj/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libpfilter_hip.so $D/obj/*.o
rm -rf $D/obj
echo built $D/libpfilter_hip.so
