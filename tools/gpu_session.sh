#!/bin/bash
# One gpurun session: GPU tests, bench, rocprofv3 kernel-trace stats.
# Stops at the first step that ends in a fault / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
TAG=${TAG:-r01}
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "[session] $name: $*"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[session] $name rc=$rc"; tail -5 "$OUT/$name.log"
  if fatal $rc; then echo "[session] fatal rc=$rc in $name, stopping"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-all}
if [[ $STEPS == all || $STEPS == *tests* ]]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
fi
if [[ $STEPS == all || $STEPS == *smoke* ]]; then
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
  run bench 600 python bench.py
  grep '^{' $OUT/bench.log > $OUT/bench_${TAG}.json || true
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
  export TMPDIR=/tmp
  run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG} -o run -- python bench.py --no-cpu-baseline --steps 10 --warmup 2
fi
if [[ $STEPS == *pmc* ]]; then
  export TMPDIR=/tmp
  run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_${TAG} -o run -- python bench.py --no-cpu-baseline --steps 3 --warmup 1
  run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_${TAG} -o run -- python bench.py --no-cpu-baseline --steps 3 --warmup 1
fi
echo "[session] done"
