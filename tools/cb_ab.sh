set -u
mkdir -p gpurun_out/cbab
for round in 1 2; do
  for so in shipped cbties; do
    for cfg in "scene_mjx 4096 50" "dual_arm 4096 100" "dual_arm 1024 50"; do
      set -- $cfg
      MODEL=$1 N=$2 H=$3 R=5 timeout -k 10 200 python tools/ab_time.py build_variants/lut/$so.so > gpurun_out/cbab/${round}_${so}_$1_$2.log 2>&1 || exit $?
      echo "$so $1 $2x$3 $(grep median gpurun_out/cbab/${round}_${so}_$1_$2.log | sed 's/\[.*\]//; s/.*median/median/')"
    done
  done
done
