#!/bin/bash
# Full GPU-box pass: parity tests, default bench (with the CPU baseline), rocprofv3 kernel
# trace + stats of the bench, PMC traffic passes.  Every GPU step has its own time limit;
# the script stops at the first step that faults, aborts or times out.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT
step() {   # step NAME TIMEOUT CMD...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -${TAIL:-4} $OUT/$name.log | cut -c1-600
  return $rc
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step bench 600 python bench.py || exit $?
step rocprof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python3 bench.py --no-cpu-baseline || exit $?
if [ -z "$SKIP_PMC" ]; then
  BENCH_ARGS=--no-cpu-baseline bash tools/gpu_pmc.sh || exit $?
fi
exit 0
