#!/bin/bash
# SQ VALU counters of the collision ablation variants (build_variants/abl/*.so,
# -DMPCR_ABL_FUNC / -DMPCR_ABL_DEEP) on C3: which narrow-phase function costs
# how many VALU instructions per candidate-step (diagnostic; the ablated
# builds drop contacts, so their dynamics differ).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp R=2
OUT=gpurun_out/${ABLOUT:-r06_abl}
mkdir -p $OUT
for so in build_variants/abl/*.so; do
  v=$(basename $so .so)
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU --output-format csv -d $OUT/$v -o run -- python3 tools/ab_time.py $so > $OUT/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(grep -h 'ms' $OUT/$v.log | tail -1)"
  case $rc in 124|134|137|139) exit $rc;; esac
done
