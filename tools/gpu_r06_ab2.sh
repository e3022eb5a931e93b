#!/bin/bash
# round 6: tie / odometry / rgbds tests and headline A/B against a variant build (VAR)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${OUTDIR:-r06ab2}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_tie.py tests/test_gpu_odom.py tests/test_gpu_rgm.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not long_sequence and not full_sequence" > $OUT/pytest.txt 2>&1
rc=$?; tail -3 $OUT/pytest.txt; [ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --only-headline > $OUT/headline_$name.json 2> $OUT/headline_$name.err || { tail -5 $OUT/headline_$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/headline_$name.json').read().strip().splitlines()[-1]); print('$name value', d['value'], d.get('stage_us'))"
}
run new
run ${VAR} PFILTER_HIP_LIB=pfilter-noetic_amd/var/${VAR}/libpfilter_hip.so
run new2
run ${VAR}2 PFILTER_HIP_LIB=pfilter-noetic_amd/var/${VAR}/libpfilter_hip.so
