cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r02_b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_replay.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "drift or ring_equals" > $O/pytest_drift.log 2>&1; echo "drift rc=$?"; grep -E "PASSED|FAILED|drift|Error" $O/pytest_drift.log | cut -c1-300 | tail -8
timeout -k 10 300 python bench.py --gpus 2 --games 256 --device 0 --dist-backend gloo --no-cpu-baseline --no-secondary > $O/rehearse2.log 2>&1; echo "rehearse rc=$?"; grep '^{' $O/rehearse2.log | cut -c1-200
timeout -k 10 700 python bench.py > $O/bench_default.log 2>&1; echo "bench rc=$?"; tail -c 3000 $O/bench_default.log
