set -o pipefail
mkdir -p gpurun_out/w2
for nh in "512 30" "1024 100" "2048 100"; do
  set -- $nh
  for thr in 0 4096; do
    MPCR_WPC2W_MAX_N=$thr MODEL=dual_arm N=$1 H=$2 R=3 SAVE=gpurun_out/w2/o_$1_$2_$thr.npz timeout -k 10 200 python tools/ab_time.py build_variants/w2.so 2>&1 | grep -v amdgpu.ids | sed "s/^/thr=$thr /" || exit $?
  done
done
