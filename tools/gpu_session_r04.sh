#!/bin/bash
# Round-4 measurement session on one MI355X: bench lines (C3 default, C2,
# C4 with the elite exchange, C3 strong-scaling mode on 1 GPU), the rocprofv3
# kernel-trace summary of the default bench command, and the PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ instruction counters) -- each pass its own run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "[session] $name: $*"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[session] $name rc=$rc"; tail -3 "$OUT/$name.log"
  if fatal $rc; then echo "[session] fatal rc=$rc in $name, stopping"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-tests,bench,prof,pmc,wavetime}
if [[ $STEPS == *host* ]]; then  # the box's CPU share: cgroup quota, affinity, nproc
  { cat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc; python -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())"; \
    grep -m1 "model name" /proc/cpuinfo; env | grep -E "OMP|MAX_JOBS" ; } > $OUT/host.log 2>&1
fi
if [[ $STEPS == *tests* ]]; then
  MPCR_PARITY_LOG=$OUT/parity.jsonl run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
fi
if [[ $STEPS == *abdual* ]]; then  # pacing A/B on the dual-arm shard (build_variants/{nopace,pace}.so)
  i=0
  for v in nopace pace nopace pace; do
    i=$((i+1)); MODEL=dual_arm N=4096 H=100 R=3 run ab_dual_${i}_$v 200 python tools/ab_time.py build_variants/$v.so
  done
fi
if [[ $STEPS == *triage* ]]; then  # parity triage: which candidates miss, then the per-step replay of them
  run triage_c3 300 python tools/parity_triage.py scene_mjx 4096 50 3 c3
  run diag_c3 300 python tools/diag_parity.py scene_mjx 4096 50 3 $(cat gpurun_out/triage_c3.txt)
  run triage_c2 300 python tools/parity_triage.py ur5e_hande_mjx 1024 50 2 c2
  run triage_c4 600 python tools/parity_triage.py dual_arm 4096 100 4 c4
fi
if [[ $STEPS == *exact* ]]; then  # the kernel against the MuJoCo-exact oracle (no kernel-matching floors)
  ORACLE_EXACT=1 run exact_c2 300 python tools/parity_triage.py ur5e_hande_mjx 1024 50 2 c2_exact
  ORACLE_EXACT=1 run exact_c3 300 python tools/parity_triage.py scene_mjx 4096 50 3 c3_exact
  ORACLE_EXACT=1 run exact_c4 600 python tools/parity_triage.py dual_arm 4096 100 4 c4_exact
fi
if [[ $STEPS == *mrank* ]]; then
  run mrank 400 python -u -m pytest tests/test_gpu_bench.py -v --timeout 300 --timeout-method thread
fi
if [[ $STEPS == *share* ]]; then  # one rank's share of C4 / C5 at 1..8 GPUs, timed on one GPU
  for nh in "8192 50" "4096 50" "2048 50" "1024 50" "4096 100" "2048 100" "1024 100"; do
    set -- $nh
    MODEL=dual_arm N=$1 H=$2 R=5 run share_dual_${1}x$2 300 python tools/ab_time.py manipulator_mujoco_amd/libmpcr.so
  done
  for n in 4096 2048 1024 512; do
    N=$n R=20 run share_c3_$n 200 python tools/ab_time.py manipulator_mujoco_amd/libmpcr.so
  done
  N=1024 MODEL=ur5e_hande_mjx R=20 run share_c2_1024 200 python tools/ab_time.py manipulator_mujoco_amd/libmpcr.so
fi
if [[ $STEPS == *micro* ]]; then
  run micro_build 120 hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o /tmp/valu_rate tools/micro/valu_rate.hip
  run micro_valu 60 /tmp/valu_rate
fi
if [[ $STEPS == *bench* ]]; then
  run bench_c3 300 python bench.py
  run bench_c2 300 python bench.py --config c2
  run bench_c4 300 python bench.py --config c4 --no-cpu-baseline --steps 5 --warmup 1
  run bench_c3_strong 300 python bench.py --scaling strong --no-cpu-baseline
fi
if [[ $STEPS == *prof* ]]; then
  run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-contact-report --steps 10 --warmup 2
fi
if [[ $STEPS == *pmc* ]]; then
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    run pmc$i 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py --no-cpu-baseline --no-contact-report --steps 3 --warmup 1
  done
fi
if [[ $STEPS == *pmcc4* ]]; then  # instruction mix / VALU busy of the dual-arm shard
  run pmc_c4 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_c4 -o run -- python3 bench.py --config c4 --no-cpu-baseline --no-contact-report --steps 2 --warmup 1
fi
if [[ $STEPS == *pmccfg* ]]; then  # HBM traffic passes of the C2 / C4 bench lines (+ C2's SQ pass)
  for cf in c2 c4; do
    for grp in FETCH_SIZE WRITE_SIZE; do
      run pmc_${cf}_$grp 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_${cf}_$grp -o run -- python3 bench.py --config $cf --no-cpu-baseline --no-contact-report --steps 2 --warmup 1
    done
  done
  run pmc_c2_sq 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_c2_sq -o run -- python3 bench.py --config c2 --no-cpu-baseline --no-contact-report --steps 2 --warmup 1
fi
if [[ $STEPS == *l2hit* ]]; then  # L2 hit rate of the dual-arm shard and the C3 launch
  run l2_c4 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/l2_c4 -o run -- python3 bench.py --config c4 --no-cpu-baseline --no-contact-report --steps 2 --warmup 1
  run l2_c3 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/l2_c3 -o run -- python3 bench.py --no-cpu-baseline --no-contact-report --steps 3 --warmup 1
fi
if [[ $STEPS == *lat* ]]; then  # memory-latency levels of the rollout kernel (C3 bench command)
  run pmc_lat 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_WAIT_ANY --output-format csv -d $OUT/pmc_lat -o run -- python3 bench.py --no-cpu-baseline --no-contact-report --steps 3 --warmup 1
fi
if [[ $STEPS == *c5* ]]; then
  run c5_dual 300 python tools/bench_mpc.py --model dual_arm --ticks 30
  run c5_planner 200 python tools/bench_mpc.py --model planner_scene --ticks 30
fi
if [[ $STEPS == *phase* ]]; then  # needs libmpcr_prof.so (python tools/phase_profile.py --build, CPU container)
  N=4096 H=100 run phase_c4 200 python tools/phase_profile.py dual_arm $OUT/phase_c4.json
  N=4096 H=50 run phase_c3 200 python tools/phase_profile.py scene_mjx $OUT/phase_c3.json
fi
if [[ $STEPS == *wavec4* ]]; then
  N=4096 H=100 run wavetime_c4 200 python tools/wavetime.py dual_arm $OUT/wavetime_c4.json
fi
if [[ $STEPS == *wpc* ]]; then  # one vs two waves per candidate (narrow variant) at the small-batch sizes
  for nm in "1024 ur5e_hande_mjx" "512 scene_mjx" "1024 scene_mjx" "2048 scene_mjx" "4096 scene_mjx"; do
    set -- $nm
    for w in 0 8192; do
      MPCR_WPC2_MAX_N=$w N=$1 MODEL=$2 R=20 run wpc_$2_$1_w$w 200 python tools/ab_time.py manipulator_mujoco_amd/libmpcr.so
    done
  done
fi
if [[ $STEPS == *wavetime* ]]; then
  N=4096 run wavetime 120 python tools/wavetime.py scene_mjx $OUT/wavetime_c3_4096.json
fi
if [[ $STEPS == *traffic* ]]; then  # HBM traffic attribution (build_variants/t_*.so, tools/build_traffic_variants.py)
  for v in ${TRAFFIC_VARIANTS:-t_ship t_jl96 t_cprev t_both t_nopace}; do
    for c in FETCH_SIZE WRITE_SIZE; do
      N=4096 R=3 run traffic_${v}_$c 120 rocprofv3 --pmc $c --output-format csv -d $OUT/traffic_${v}_$c -o run -- python3 tools/ab_time.py build_variants/$v.so
    done
  done
  for c in FETCH_SIZE WRITE_SIZE; do  # the shipped build without the theta / thetadot outputs
    THETA=0 N=4096 R=3 run traffic_t_ship_notheta_$c 120 rocprofv3 --pmc $c --output-format csv -d $OUT/traffic_t_ship_notheta_$c -o run -- python3 tools/ab_time.py build_variants/t_ship.so
  done
fi
echo "[session] done"
if [[ $STEPS == *mech* ]]; then  # which mechanism moves each well-conditioned GPU miss (tools/diag_f32.py --gpu)
  run mech_c4 600 python -u tools/diag_f32.py --gpu dual_arm 4096 100 4 ${MECH_K:-40}
  run mech_c3 400 python -u tools/diag_f32.py --gpu scene_mjx 4096 50 3 ${MECH_K:-40}
fi
if [[ $STEPS == *ab* ]]; then  # interleaved A/B timing of build_variants/*.so (C3 unless MODEL/N/H say otherwise)
  for round in 1 2 3; do
    for so in build_variants/*.so; do
      run ab_${round}_$(basename $so .so) 120 python tools/ab_time.py "$so"
    done
  done
  grep -h "median" $OUT/ab_*.log | sort > $OUT/ab_summary.txt
fi
if [[ $STEPS == *seg* ]]; then  # dual-arm horizon segments x candidate groups (env of the engine), C4 and C5 sizes
  for round in 1 2; do
    for sg in "0 1" "50 1" "25 1" "50 2" "25 2" "20 4" "25 4" "10 4"; do
      set -- $sg
      MPCR_SEG_STEPS=$1 MPCR_SEG_GROUPS=$2 MODEL=dual_arm N=4096 H=100 R=5 run seg_${round}_c4_$1_$2 200 python tools/ab_time.py manipulator_mujoco_amd/libmpcr.so
    done
    for sg in "0 1" "25 2" "25 4" "10 4"; do
      set -- $sg
      MPCR_SEG_STEPS=$1 MPCR_SEG_GROUPS=$2 MODEL=dual_arm N=8192 H=50 R=5 run seg_${round}_c5_$1_$2 200 python tools/ab_time.py manipulator_mujoco_amd/libmpcr.so
    done
  done
  for f in $OUT/seg_*.log; do echo "$(basename $f .log) $(grep median $f)"; done > $OUT/seg_summary.txt
fi
if [[ $STEPS == *bitwise* ]]; then  # the narrow kernel bitwise against the previous build (build_variants/ship.so)
  for M in scene_mjx ur5e_hande_mjx; do
    SAVE=$OUT/bw_old_$M.npz MODEL=$M N=4096 R=2 run bw_old_$M 120 python tools/ab_time.py build_variants/ship.so
    SAVE=$OUT/bw_new_$M.npz MODEL=$M N=4096 R=2 run bw_new_$M 120 python tools/ab_time.py manipulator_mujoco_amd/libmpcr.so
    run bw_cmp_$M 60 python -c "import numpy as np; a=np.load('$OUT/bw_old_$M.npz', allow_pickle=False); b=np.load('$OUT/bw_new_$M.npz', allow_pickle=False); print('$M bitwise', all(np.array_equal(a[k], b[k]) for k in ('c4','th','st')))"
  done
fi
if [[ $STEPS == *abc4* ]]; then  # dual-arm A/B of build_variants/*.so, one launch (no segments) and the default segments
  for round in 1 2; do
    for so in build_variants/*.so; do
      MPCR_SEG_STEPS=0 MODEL=dual_arm N=4096 H=100 R=3 run abc4_${round}_$(basename $so .so)_noseg 200 python tools/ab_time.py "$so"
    done
  done
  grep -h "median" $OUT/abc4_*.log | sort > $OUT/abc4_summary.txt
  for f in $OUT/abc4_*.log; do echo "$(basename $f .log) $(grep median $f | sed 's/.*median/median/')"; done > $OUT/abc4_summary.txt
fi
if [[ $STEPS == *steperr* ]]; then  # per-step error budget of the GPU's accumulated-drift misses (tools/step_errors.py)
  run steperr_c4 400 python -u tools/step_errors.py dual_arm 4096 100 4 ${STEPERR_CANDS:-928 3593 3162 2818 3136 2429 3470 628 2863 93 2112}
fi
if [[ $STEPS == *mechvar* ]]; then  # GPU well-conditioned misses of each build_variants/*.so on the C4 batch
  for so in build_variants/*.so; do
    MPCR_LIB=$so run mechvar_$(basename $so .so) 400 python -u tools/diag_f32.py --gpu dual_arm 4096 100 4 ${MECH_K:-0}
  done
  grep -H "GPU well-misses" $OUT/mechvar_*.log | grep -v "worst first" > $OUT/mechvar_summary.txt
fi
