#!/bin/bash
# Support start table resolution A/B: libraries built with -DMPCR_LUT_R=<r>
# (the engine builds its table at that resolution since model format v9).
#   LUTOUT=r06lut LUTS="128:lut128 256:lut256" bash tools/lut_ab.sh   (build_variants/lut/<name>.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${LUTOUT:-r05lut}; mkdir -p $OUT
for round in 1 2; do
  for v in ${LUTS:-16:cur16 32:lut32 64:lut64}; do
    r=${v%%:*}; name=${v#*:}
    for cfg in "dual_arm 1024 50" "dual_arm 4096 100"; do
      set -- $cfg
      MODEL=$1 N=$2 H=$3 R=3 timeout -k 10 200 python tools/ab_time.py build_variants/lut/$name.so > $OUT/${round}_${name}_$2.log 2>&1 || exit $?
      echo "$name $(grep median $OUT/${round}_${name}_$2.log | sed 's/\[.*\]//')"
    done
  done
done
