#!/bin/bash
# does one GPU stay fed at the 8-rank host share?  The main bench line (4096 games x
# 64 sims) with the engine's per-move host work on N threads, for each N given (default 2 = 16 / 8,
# launch.rank_host_share at 8 ranks on the box's 16-CPU quota, and 16).  Usage:
#   bash tools/bench_host_threads.sh OUTDIR [N ...]
out=${1:?usage: bench_host_threads.sh OUTDIR [N ...]}
shift
mkdir -p "$out"
for n in "${@:-2 16}"; do
  for t in $n; do
    timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --default-sims 0 --host-threads "$t" \
      > "$out/bench_ht$t.json" 2> "$out/bench_ht$t.err" || exit $?
    cut -c1-300 "$out/bench_ht$t.json"
  done
done
