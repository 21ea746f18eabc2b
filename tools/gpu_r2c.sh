cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r2c; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -5
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in 0 8192; do
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --net-variant $v > $O/bench_$v.log 2>$O/bench_$v.err
  rc=$?; echo "bench $v rc=$rc"; python -c "import json; d=json.loads([l for l in open('$O/bench_$v.log') if l.startswith('{')][0]); print(d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
