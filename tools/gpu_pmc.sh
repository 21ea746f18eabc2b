#!/bin/bash
# HBM traffic of the dominant kernel (k_net_z, product; k_net_y when selected) from PMC counters, one counter group per
# rocprofv3 pass (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), counters
# restricted to the k_net_* kernels.  No trace domains are combined with --pmc.
# Summaries: python tools/pmc_summary.py gpurun_out/pmc -> profiles/conv_traffic.json
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ARGS="${BENCH_ARGS:---no-cpu-baseline --no-secondary}"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -k 10 ${PMC_TIMEOUT:-420} rocprofv3 --pmc $grp --kernel-include-regex "k_net_[yz]" \
    -d gpurun_out/pmc/p$i -o pmc --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "pmc pass $i ($grp) rc=$rc"
  tail -2 gpurun_out/pmc/p$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
