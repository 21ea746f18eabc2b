#!/bin/bash
# In-process A/B: product k_net_z (tap-major loop, buffer-loaded weights, scaled-conversion
# epilogue) vs deeper Wh prefetch (67108864), the round-2 epilogue (33554432) and the round-2
# loop + epilogue (58720256), then the network parity tests and smoke().
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pd3; mkdir -p $O
timeout -k 10 300 python tools/bench_net.py --variants ${AB_VARIANTS:-0,67108864,33554432,58720256} --rounds 4 --iters 10 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc"; python3 -c "
import json
for l in open('$O/ab.json'):
    d=json.loads(l); print(d['variant'], round(d['ms_median'],4), int(d['wg_cycles']), round(d['clock_ghz_stamped'],3), d['shares'], d['check'])"
if [ $rc -ne 0 ]; then tail -5 $O/ab.err; exit $rc; fi
timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_net.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_net.log; grep -E "FAILED|ERROR" $O/pytest_net.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $O/smoke.log
exit $rc
