#!/bin/bash
# rocprofv3 kernel trace + stats of a bench command (kernel durations for profiles/).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 ${PROF_TIMEOUT:-900} rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python3 bench.py ${BENCH_ARGS} > gpurun_out/prof_bench.log 2>&1
rc=$?
echo "rocprof bench rc=$rc"
tail -3 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
