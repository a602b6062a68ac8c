#!/bin/bash
# Round-6 measurement session on one MI355X.  STEPS picks the parts (comma
# list); every GPU step runs under its own time limit and the session stops
# at the first fatal exit (timeout, abort, segfault).  The libmpcr.so source
# hash of the build this session ran is written to $OUT/source_hash.txt, and
# tools/commit_profiles.py refuses to commit counters whose hash does not
# match the checkout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r06}
OUT=gpurun_out/$TAG
mkdir -p $OUT
python -c "from manipulator_mujoco_amd import build; print(build.source_hash())" > $OUT/source_hash.txt
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
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
STEPS=${STEPS:-tests}
IFS=, read -ra ST <<< "$STEPS"
has() { local s; for s in "${ST[@]}"; do [[ $s == "$1" ]] && return 0; done; return 1; }

if has tests; then
  MPCR_PARITY_LOG=$OUT/parity.jsonl run pytest_gpu 900 $PYT tests -m gpu
fi
if has quick; then  # round-6 changes: ABI v3 status word, the 30-tick C5 loop
  MPCR_PARITY_LOG=$OUT/parity_quick.jsonl run quick 900 $PYT -s tests/test_gpu_planner.py::test_dual_arm_c5_thirty_ticks "tests/test_gpu_parity.py::test_two_wave_variant_is_bitwise_one_wave" tests/test_gpu_parity.py::test_two_wave_dual_arm_flush_paths_bitwise tests/test_gpu_parity.py::test_dual_arm_c4_properties tests/test_gpu_parity.py::test_dual_arm_parity_to_conditioning tests/test_lib.py
fi
if has c5ticks; then  # BASELINE configs[4]: 30 closed-loop ticks
  run bench_c5_30 400 python bench.py --config c5 --no-cpu-baseline --ticks 30 --warmup 1
fi
if has c5share; then  # the C5 tick's stages at one rank's share on 8 GPUs
  run c5_share_stages 300 python tools/c5_share_stages.py
fi
if has c3precise; then  # C3 parity on the fast-math and the precise build, same batch
  MPCR_PARITY_LOG=$OUT/parity_c3_fast.jsonl run c3_fast 400 $PYT -s tests/test_gpu_parity.py -k test_parity_c3_full
  MPCR_LIB=build_variants/keep/precise.so MPCR_PARITY_LOG=$OUT/parity_c3_precise.jsonl \
    run c3_precise 400 $PYT -s tests/test_gpu_parity.py -k test_parity_c3_full
fi
if has mrank; then
  run mrank 400 $PYT tests/test_gpu_bench.py
fi
if has bench; then
  run bench_c3 300 python bench.py
fi
if has benchall; then
  run bench_c2 300 python bench.py --config c2
  run bench_c4 300 python bench.py --config c4 --no-cpu-baseline --steps 5 --warmup 1
  run bench_c5 300 python bench.py --config c5 --no-cpu-baseline --steps 5 --warmup 2
fi
if has phase; then  # needs libmpcr_prof.so (python tools/phase_profile.py --build, CPU container)
  N=1024 H=50 run phase_dual_1024x50 200 python tools/phase_profile.py dual_arm $OUT/phase_dual_1024x50.json
  N=4096 H=100 run phase_c4 300 python tools/phase_profile.py dual_arm $OUT/phase_c4.json
fi
if has share; then  # one rank's share of C3 / C5 at 1..8 GPUs, timed on one GPU
  for nh in "8192 50" "4096 50" "2048 50" "1024 50" "4096 100"; do
    set -- $nh
    MODEL=dual_arm N=$1 H=$2 R=5 run share_dual_${1}x$2 300 python tools/ab_time.py manipulator_mujoco_amd/libmpcr.so
  done
  for n in 4096 2048 1024 512; do
    N=$n R=20 run share_c3_$n 200 python tools/ab_time.py manipulator_mujoco_amd/libmpcr.so
  done
fi
if has ab; then  # interleaved A/B timing of build_variants/*.so (MODEL / N / H from the environment)
  for round in 1 2 3; do
    for so in build_variants/*.so; do
      run ab_${round}_$(basename $so .so) 200 python tools/ab_time.py "$so"
    done
  done
  grep -h "median" $OUT/ab_*.log | sort > $OUT/ab_summary.txt
fi
if has prof; then
  run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-sub --no-cpu-baseline --no-contact-report --steps 10 --warmup 2
fi
if has pmc; then
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    run pmc$i 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py --no-sub --no-cpu-baseline --no-contact-report --steps 3 --warmup 1
  done
fi
if has pmccfg; then  # the C2 / C4 lines' passes
  for cf in c2 c4; do
    for grp in FETCH_SIZE WRITE_SIZE; do
      run pmc_${cf}_$grp 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_${cf}_$grp -o run -- python3 bench.py --config $cf --no-cpu-baseline --no-contact-report --steps 2 --warmup 1
    done
    sfx=$([[ $cf == c2 ]] && echo c2_sq || echo c4)
    run pmc_$sfx 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_$sfx -o run -- python3 bench.py --config $cf --no-cpu-baseline --no-contact-report --steps 2 --warmup 1
  done
fi
echo "[session] done"
