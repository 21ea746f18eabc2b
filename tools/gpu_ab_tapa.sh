#!/bin/bash
# In-process A/B of the tap-major K loop (variant 8388608) against the product k_net_z, then the
# network parity tests.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/tapa; mkdir -p $O
timeout -k 10 300 python tools/bench_net.py --variants 0,8388608,25165824,8192,8396800 --rounds 4 --iters 10 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc"; cat $O/ab.json | cut -c1-400
if [ $rc -ne 0 ]; then tail -5 $O/ab.err; exit $rc; fi
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_net.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_net.log
exit $rc
