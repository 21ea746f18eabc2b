#!/bin/bash
# The 8-rank host share on the 1-GPU box: the main bench line at the full 16-CPU share
# and at one rank's share of an 8-rank node (bench.py --rank-share 8: 2 cores, 2 host threads), each
# with HIP's default stream wait and with a blocking-sync event (--sync-mode 1), alternated.
#   bash tools/host_share_ab.sh OUTDIR [steps]
# Every run under its own time limit; stops at the first failure.
OUT=${1:?usage: host_share_ab.sh OUTDIR [steps]}
STEPS=${2:-2}
mkdir -p "$OUT"
for cfg in "full:" "share8:--rank-share 8" "full_sync1:--sync-mode 1" "share8_sync1:--rank-share 8 --sync-mode 1"; do
  name=${cfg%%:*}
  args=${cfg#*:}
  echo "[host_share_ab] $name: $args" >&2
  timeout -k 10 300 python -u bench.py --steps "$STEPS" --warmup 1 --no-cpu-baseline --default-sims 0 $args \
    > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "[host_share_ab] $name failed rc=$?" >&2; exit 1; }
  cut -c1-200 "$OUT/$name.json" >&2
done
