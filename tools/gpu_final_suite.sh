#!/bin/bash
# Final GPU pass on the committed tree: an in-process A/B of static issue priority for the second
# half of the waves (diagnostic library), the full parity suite, smoke().
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 300 python tools/bench_net.py --diag --variants 0,1048576 --rounds 4 --iters 10 > $O/ab_prio.json 2> $O/ab_prio.err
rc=$?; echo "ab rc=$rc"; python3 -c "
import json
for l in open('$O/ab_prio.json'):
    d=json.loads(l); print(d['variant'], round(d['ms_median'],4), int(d['wg_cycles']), round(d['clock_ghz_stamped'],3), d['check'])"
if [ $rc -ne 0 ]; then tail -5 $O/ab_prio.err; exit $rc; fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
exit $rc
