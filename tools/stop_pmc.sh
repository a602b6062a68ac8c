#!/bin/bash
# SQ instruction counters of the stop-after-phase variants (one rocprofv3 run each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp R=2
OUT=gpurun_out/${STOPOUT:-stop}
mkdir -p $OUT
for v in stop0 stop1 stop2 stop3 stop4 stop5 stop6 stop7 stop8 stop13 stop9 full; do
  timeout -k 10 120 rocprofv3 --pmc ${COUNTERS:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE} --output-format csv -d $OUT/$v -o run -- python3 tools/ab_time.py build_variants/$v.so > $OUT/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(grep -h 'ms' $OUT/$v.log | tail -1)"
  case $rc in 124|134|137|139) exit $rc;; esac
done
