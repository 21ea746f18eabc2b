#!/bin/bash
# Round-2 closing measurement on one MI355X, part 1: the default bench line (CPU baseline plan +
# k_net_y secondary) and a rocprofv3 kernel-trace/stats run of the bench.  Part 2 = tools/gpu_pmc.sh.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r2end; mkdir -p $O
timeout -k 10 700 python bench.py ${BENCH_MAIN_ARGS} > $O/bench.log 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 $O/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --steps 2 --no-cpu-baseline --no-secondary > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
