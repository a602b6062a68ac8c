#!/bin/bash
# Interleaved A/B timing of build_variants/<a>.so vs <b>.so on one workload
# (MODEL / N / H env as tools/ab_time.py), 3 rounds each.  Diagnostic.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2 3; do
  for v in "$@"; do
    R=${R:-20} timeout -k 10 200 python tools/ab_time.py build_variants/$v.so 2>&1 | grep -v amdgpu.ids
    rc=${PIPESTATUS[0]}; case $rc in 0) ;; *) echo "rc=$rc"; exit $rc;; esac
  done
done
