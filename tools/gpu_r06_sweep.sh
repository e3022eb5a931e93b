#!/bin/bash
# round 6: two-sweep stop ranking (PF_SWEEP2): tier profile on real keys, tie / odometry tests, headline A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/${OUTDIR:-r06sw}
mkdir -p $OUT
for v in tieprof6n tieprof6; do for c in 1 2; do
  PFILTER_HIP_LIB=pfilter-noetic_amd/var/$v/libpfilter_hip.so timeout -k 10 120 python3 tools/tie_prof.py pfilter-noetic_amd/var/keys3098.bin $c > $OUT/${v}_real$c.txt 2>&1 || { tail -5 $OUT/${v}_real$c.txt; exit 1; }
done; done
head -34 $OUT/tieprof6n_real1.txt; echo ===; head -34 $OUT/tieprof6_real1.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_tie.py tests/test_gpu_odom.py tests/test_gpu_rgm.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not long_sequence and not full_sequence" > $OUT/pytest.txt 2>&1
rc=$?; tail -3 $OUT/pytest.txt; [ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --only-headline > $OUT/headline_$name.json 2> $OUT/headline_$name.err || { tail -5 $OUT/headline_$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/headline_$name.json').read().strip().splitlines()[-1]); print('$name value', d['value'], d.get('stage_us'))"
}
run new PF_TIE_AUX=0
run old PF_TIE_AUX=0 PFILTER_HIP_LIB=pfilter-noetic_amd/var/old/libpfilter_hip.so
run sweep1 PF_TIE_AUX=0 PFILTER_HIP_LIB=pfilter-noetic_amd/var/sweep1/libpfilter_hip.so
run medglb PF_TIE_AUX=0 PFILTER_HIP_LIB=pfilter-noetic_amd/var/medglb/libpfilter_hip.so
run new2 PF_TIE_AUX=0
