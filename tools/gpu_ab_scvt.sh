#!/bin/bash
# The scaled-conversion probe, the in-process A/B of the scaled-conversion epilogue (33554432)
# against the product, then the full GPU parity suite.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/scvt; mkdir -p $O
timeout -k 10 60 ./tools/probes/cvt_scale_probe > $O/cvt_scale_probe.json 2>&1
rc=$?; echo "probe rc=$rc"; head -c 600 $O/cvt_scale_probe.json
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_net.py --variants 0,33554432,25165824 --rounds 4 --iters 10 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc"; python3 -c "
import json
for l in open('$O/ab.json'):
    d=json.loads(l); print(d['variant'], round(d['ms_median'],4), int(d['wg_cycles']), round(d['clock_ghz_stamped'],3), d['shares'], d['check'])"
if [ $rc -ne 0 ]; then tail -5 $O/ab.err; exit $rc; fi
if [ -n "$SKIP_SUITE" ]; then exit 0; fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
exit $rc
