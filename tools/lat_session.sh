#!/bin/bash
# A/B timing of build_variants/*.so (interleaved) + one SQ latency-level PMC pass
# on the first variant.  Diagnostic.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/lat
mkdir -p $OUT
for round in 1 2; do
  for v in "$@"; do
    R=20 timeout -k 10 120 python tools/ab_time.py build_variants/$v.so 2>&1 | grep -v amdgpu.ids
    rc=${PIPESTATUS[0]}; case $rc in 124|134|137|139) exit $rc;; esac
  done
done
if [ -n "${PMC:-}" ]; then
  R=2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_WAIT_ANY --output-format csv -d $OUT/pmc_$1 -o run -- python3 tools/ab_time.py build_variants/$1.so > $OUT/pmc_$1.log 2>&1
  echo "pmc rc=$?"
fi
