#!/bin/bash
# In-process A/B of network variants in several experimental libraries (run through gpurun):
#   bash tools/ab_libs.sh OUT "VARIANTS" lib1 lib2 ...
# each lib is minitchess_alphazero_amd/libmtaz_<name>.so (tools/build_exp_libs.py: same sources, other -D flags on the
# network translation unit); results in gpurun_out/OUT/ab_<name>.json.  Stops at the first abnormal
# exit; never retries.
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/${1:?OUT}
VARS=${2:?variants}
shift 2
mkdir -p "$OUT"
for name in "$@"; do
  MTAZ_LIB=minitchess_alphazero_amd/libmtaz_$name.so timeout -k 10 300 python -u tools/bench_net.py --precision f16x3 \
    --variants "$VARS" --rounds "${AB_ROUNDS:-4}" --iters "${AB_ITERS:-10}" > "$OUT/ab_$name.json" 2> "$OUT/ab_$name.err"
  rc=$?
  echo "[ab_libs] $name rc=$rc"; cut -c1-330 "$OUT/ab_$name.json"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/ab_$name.err"; exit $rc; fi
done
