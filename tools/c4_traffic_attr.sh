#!/bin/bash
# Where the C4 shard's HBM bytes come from (diagnostic, round 6): FETCH_SIZE /
# WRITE_SIZE passes of tools/ab_time.py on the dual arm 4096 x 100 with the
# shipped segmenting (7-step horizon segments over two candidate groups), with
# one launch per call (MPCR_SEG_STEPS=0: no segment state saved / restored; the
# second half of the batch waits for the first), and without the theta /
# thetadot outputs (THETA=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MODEL=dual_arm N=4096 H=100 R=1
OUT=gpurun_out/r06_c4traffic
mkdir -p $OUT
for v in "seg7:MPCR_SEG_STEPS=7" "seg0:MPCR_SEG_STEPS=0" "nothe:THETA=0" "seg50:MPCR_SEG_STEPS=50"; do
  name=${v%%:*}; envs=${v#*:}
  for c in FETCH_SIZE WRITE_SIZE; do
    (export $envs; timeout -k 10 180 rocprofv3 --pmc $c --output-format csv -d $OUT/${name}_$c -o run -- python3 tools/ab_time.py manipulator_mujoco_amd/libmpcr.so > $OUT/${name}_$c.log 2>&1)
    rc=$?
    echo "$name $c rc=$rc"
    case $rc in 124|134|137|139) exit $rc;; esac
  done
done
