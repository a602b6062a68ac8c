#!/bin/bash
# Kernel tolerance variants (build_variants/v_*.so, tools/build_variant.py):
# C4-shard parity triage against the oracle run with the same rules, and the
# dual-arm kernel time of each.  Diagnostic.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/tol
mkdir -p $OUT
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[tol] $name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -6
  case $rc in 124|134|137|139) exit $rc;; esac
}
MPCR_LIB=build_variants/v_base.so step tri_base 400 python tools/parity_triage.py dual_arm 4096 100 4 c4_base
MPCR_LIB=build_variants/v_mpr6.so ORACLE_FLOORS=1e-6,1e-5,1e-6,1e-6 step tri_mpr6 400 python tools/parity_triage.py dual_arm 4096 100 4 c4_mpr6
MPCR_LIB=build_variants/v_mpr6_band0.so ORACLE_FLOORS=1e-6,0,1e-6,1e-6 step tri_mpr6_band0 400 python tools/parity_triage.py dual_arm 4096 100 4 c4_mpr6_band0
MPCR_LIB=build_variants/v_exact.so ORACLE_EXACT=1 step tri_exact 400 python tools/parity_triage.py dual_arm 4096 100 4 c4_exact
MPCR_LIB=build_variants/v_exact.so ORACLE_EXACT=1 step tri_exact_c3 400 python tools/parity_triage.py scene_mjx 4096 50 3 c3_exactk
for v in v_base v_mpr6 v_mpr6_band0 v_exact; do
  MODEL=dual_arm N=4096 H=100 R=3 step time_$v 300 python tools/ab_time.py build_variants/$v.so
done
for v in v_base v_exact; do
  R=20 step time_c3_$v 200 python tools/ab_time.py build_variants/$v.so
done
step valu_rate 60 tools/micro/valu_rate
echo "[tol] done"
