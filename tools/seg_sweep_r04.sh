#!/bin/bash
# Dual-arm horizon segments: segment length x candidate groups at the C4 shard (4096 x 100) and the
# C5 rollout (8192 x 50), twice, interleaved (tools/ab_time.py; the engine reads MPCR_SEG_* at creation)
mkdir -p gpurun_out/r04
TAG=${TAG:-seg3}
for round in 1 2; do
  for sg in ${C4_SG:-"10 2" "7 2" "5 2" "4 2" "3 2"}; do
    set -- $sg
    MPCR_SEG_STEPS=$1 MPCR_SEG_GROUPS=$2 MODEL=dual_arm N=4096 H=100 R=5 timeout -k 10 200 python tools/ab_time.py manipulator_mujoco_amd/libmpcr.so > gpurun_out/r04/${TAG}_${round}_c4_$1_$2.log 2>&1 || exit 1
  done
  for sg in ${C5_SG:-"13 2" "10 2" "7 2" "5 2"}; do
    set -- $sg
    MPCR_SEG_STEPS=$1 MPCR_SEG_GROUPS=$2 MODEL=dual_arm N=8192 H=50 R=5 timeout -k 10 200 python tools/ab_time.py manipulator_mujoco_amd/libmpcr.so > gpurun_out/r04/${TAG}_${round}_c5_$1_$2.log 2>&1 || exit 1
  done
done
for f in gpurun_out/r04/${TAG}_*.log; do echo "$(basename $f .log) $(grep -o 'median [0-9.]* ms' $f)"; done > gpurun_out/r04/${TAG}_summary.txt
