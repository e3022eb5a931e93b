#!/bin/bash
# PMC passes over the standalone kNN probe (one counter group per pass, each under its own limit).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT=gpurun_out/clspmc
mkdir -p $OUT
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 tools/cls_probe.py --iters 5 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_table.py $OUT k_cls_search
