#!/bin/bash
# Round-2 closing pass on the final tree: bench line (CPU baseline plan + k_net_y secondary),
# rocprofv3 kernel stats, PMC passes, then the full parity suite and smoke().
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash tools/gpu_round2.sh || exit $?
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
exit $rc
