#!/bin/bash
# Round-2 measurement pass on one MI355X: the default bench line (CPU baseline plan + k_net_y
# secondary), a rocprofv3 kernel-trace/stats run of the bench, and the PMC passes (traffic, MFMA
# busy, waits, LDS conflicts).  Each GPU step has its own time limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r2; mkdir -p $O
timeout -k 10 700 python bench.py ${BENCH_MAIN_ARGS} > $O/bench.log 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 $O/bench.log; tail -3 $O/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --steps 2 --no-cpu-baseline --no-secondary > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep '^{' $O/prof.log | cut -c1-200
if [ $rc -ne 0 ]; then exit $rc; fi
mkdir -p gpurun_out/pmc
bash tools/gpu_pmc.sh || exit $?
exit 0
