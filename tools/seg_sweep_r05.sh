set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r05seg; mkdir -p $OUT
for r in 1 2; do
for sg in 7 10 13 25; do
  MPCR_SEG_STEPS=$sg MODEL=dual_arm N=4096 H=100 R=5 timeout -k 10 200 python tools/ab_time.py manipulator_mujoco_amd/libmpcr.so > $OUT/seg_${r}_$sg.log 2>&1 || exit $?
  echo "seg $sg $(grep median $OUT/seg_${r}_$sg.log | sed 's/\[.*\]//')"
done
done
