#!/bin/bash
# Interleaved A/B timing of every build_variants/*.so (2 rounds).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
for round in 1 2; do
  for so in build_variants/*.so; do
    timeout -k 10 120 python tools/ab_time.py "$so" 2>&1 | grep -v amdgpu.ids
    rc=${PIPESTATUS[0]}
    case $rc in 124|134|137|139) echo "fatal rc=$rc on $so"; exit $rc;; esac
  done
done
