#!/bin/bash
# LM probe of the in-tree library and of a variant (tools/build_variant.sh)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 100 python tools/probe_lm.py 2>&1 | tail -2
PFILTER_HIP_LIB=pfilter-noetic_amd/var/$1/libpfilter_hip.so timeout -k 10 100 python tools/probe_lm.py 2>&1 | tail -2
