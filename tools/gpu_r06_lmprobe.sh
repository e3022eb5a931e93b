#!/bin/bash
# k_lm_solve timelines (block 0 phases, every workgroup's publish / wait) on the headline configuration
set -o pipefail
mkdir -p gpurun_out/lm
timeout -k 10 240 python3 -u tools/probe_lm2.py > gpurun_out/lm/probe.txt 2>&1 &&
timeout -k 10 240 python3 -u tools/probe_lm3.py > gpurun_out/lm/probe3.txt 2>&1
