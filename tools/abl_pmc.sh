#!/bin/bash
# SQ instruction counters of every build_variants/*.so on the C3 workload
# (one rocprofv3 run each): per-function attribution with the
# -DMPCR_STOP_AFTER / -DMPCR_ABL_FUNC builds (diagnostic).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp R=2
OUT=gpurun_out/${ABLOUT:-abl}
mkdir -p $OUT
for so in build_variants/*.so; do
  v=$(basename $so .so)
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $OUT/$v -o run -- python3 tools/ab_time.py $so > $OUT/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
