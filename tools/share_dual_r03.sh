# dual-arm rank shares on one GPU (the shipped libmpcr.so): the C5 rollout per
# rank at 2 / 4 / 8 GPUs (8192 x 50 split) and the H = 100 shard sizes
set -o pipefail
for nh in "8192 50" "4096 50" "2048 50" "1024 50" "1024 100" "2048 100"; do
  set -- $nh
  MODEL=dual_arm N=$1 H=$2 R=5 timeout -k 10 200 python tools/ab_time.py manipulator_mujoco_amd/libmpcr.so 2>&1 | grep -v amdgpu.ids | sed "s/^/N=$1 H=$2 /" || exit $?
done
