#!/bin/bash
# GPU-box check: parity tests, then a short bench.  Stops at the first abnormal exit
# (fault / abort / timeout); ordinary test failures (rc 1) still let the bench run.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "${BENCH_ARGS}" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
  rc=$?
  echo "bench rc=$rc"
  tail -5 gpurun_out/bench.log
  exit $rc
fi
