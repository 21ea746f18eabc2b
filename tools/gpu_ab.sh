#!/bin/bash
# GPU-box A/B of network builds: parity tests of the network kernels, then the in-process
# network timing harness (tools/bench_net.py) over VARIANTS, then optional bench lines.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_net.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_net.log 2>&1
rc=$?; echo "net tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" $O/pytest_net.log | cut -c1-160 | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/bench_net.py ${DIAG:+--diag} --n 4096 --iters 10 --rounds 3 --variants "${VARIANTS:-f16f8:0,f16f8:4194304}" > $O/bench_net.log 2>&1
rc=$?; echo "bench_net rc=$rc"; cut -c1-400 $O/bench_net.log | grep '^{'
if [ $rc -ne 0 ]; then exit $rc; fi
for v in ${BENCH_VARIANTS}; do
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --net-variant $v > $O/bench_$v.log 2>&1
  rc=$?; echo "bench $v rc=$rc"; grep '^{' $O/bench_$v.log | cut -c1-120; python -c "import json,sys; d=json.loads([l for l in open('$O/bench_$v.log') if l.startswith('{')][0]); print(d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
