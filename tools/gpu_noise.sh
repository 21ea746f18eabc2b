#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
K_EXPR="mcts or dropin or decisive or pipelined or multirank or wire or arena" bash tools/gpu_tests.sh || exit $?
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary > gpurun_out/bench_noise.log 2> gpurun_out/bench_noise.err || exit $?
python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_noise.log') if l.startswith('{')][0]); print(d['value'], d['roofline']['avg_launch_ms'], d['host_rng_s'], d['host_sync_s'])"
