#!/bin/bash
# GPU-box pass of the parity suite: `pytest -m gpu` with a per-test time limit, log under
# gpurun_out/tests/ (the L3 identity summary lands in gpurun_out/l3_identity.json); K_EXPR = a -k filter.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tests
timeout -k 10 ${PYTEST_TIMEOUT:-1000} python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 \
  --timeout-method thread ${K_EXPR:+-k "$K_EXPR"} > gpurun_out/tests/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/tests/pytest_gpu.log | tail -60 | cut -c1-200
exit $rc
