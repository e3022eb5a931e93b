#!/bin/bash
# k_lm_solve launch span A/B: the HEAD build (var/base) against the in-tree library, alternated
set -o pipefail
mkdir -p gpurun_out/lm
export PF_PROBE_FRAMES=${PF_PROBE_FRAMES:-200}
: > gpurun_out/lm/ab.txt
for r in 1 2; do
  PFILTER_HIP_LIB=pfilter-noetic_amd/var/base/libpfilter_hip.so timeout -k 10 200 python3 -u tools/probe_lm2.py 2>&1 | grep "launch span" >> gpurun_out/lm/ab.txt &&
  timeout -k 10 200 python3 -u tools/probe_lm2.py > gpurun_out/lm/probe_cur.txt 2>&1 && grep "launch span" gpurun_out/lm/probe_cur.txt >> gpurun_out/lm/ab.txt || exit 1
done
