#!/bin/bash
# Two waves per candidate (narrow variant, MPCR_WPC2_MAX_N): bitwise equality
# with one wave and the kernel time at the small-batch sizes.  Diagnostic.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/wpc
mkdir -p $OUT
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[wpc] $name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -2
  case $rc in 124|134|137|139) exit $rc;; esac
}
for nm in "1024 ur5e_hande_mjx" "1024 scene_mjx" "2048 scene_mjx" "512 scene_mjx" "4096 scene_mjx"; do
  set -- $nm
  for w in 0 4096; do
    MPCR_WPC2_MAX_N=$w N=$1 MODEL=$2 R=20 step t_$2_$1_w$w 200 python tools/ab_time.py manipulator_mujoco_amd/libmpcr.so
  done
done
echo "[wpc] done"
