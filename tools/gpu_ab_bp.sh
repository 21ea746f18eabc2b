#!/bin/bash
# In-process A/B (diagnostic library): product vs a variant list (default: the board-pair wave layout 4194304) on the
# tap-major loop.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/bp; mkdir -p $O
timeout -k 10 300 python tools/bench_net.py --diag --variants ${AB_VARIANTS:-0,4194304} --rounds 4 --iters 10 > $O/ab.json 2> $O/ab.err
rc=$?; echo "ab rc=$rc"; python3 -c "
import json
for l in open('$O/ab.json'):
    d=json.loads(l); print(d['variant'], round(d['ms_median'],4), int(d['wg_cycles']), round(d['clock_ghz_stamped'],3), d['shares'], d['check'])"
if [ $rc -ne 0 ]; then tail -5 $O/ab.err; fi
exit $rc
