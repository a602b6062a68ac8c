#!/bin/bash
# PMC passes over the C3 rollout kernel (one counter group per pass; --pmc
# is never combined with tracing domains).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
LIB=${LIB:-manipulator_mujoco_amd/libmpcr.so}
OUT=gpurun_out/pmc
mkdir -p $OUT
if [ "${LIST:-0}" = 1 ]; then timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1; fi
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python tools/ab_time.py $LIB > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i ($grp) rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
