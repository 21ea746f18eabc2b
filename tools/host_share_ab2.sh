#!/bin/bash
# The 8-rank host share A/B (round 5): the 16-CPU line against one rank's share of an 8-rank node
# (bench.py --rank-share 8: 2 cores, 2 host threads, blocking-sync wait), alternated twice.
#   bash tools/host_share_ab2.sh OUTDIR [steps]
OUT=${1:?usage: host_share_ab2.sh OUTDIR [steps]}
STEPS=${2:-3}
mkdir -p "$OUT"
for i in 1 2; do
  for cfg in "full:" "share8:--rank-share 8"; do
    name=${cfg%%:*}$i
    args=${cfg#*:}
    timeout -k 10 300 python -u bench.py --steps "$STEPS" --warmup 1 --no-cpu-baseline --default-sims 0 $args \
      > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "[host_share_ab2] $name failed" >&2; exit 1; }
    cut -c1-160 "$OUT/$name.json" >&2
  done
done
