#!/bin/bash
# SQ counters of the network kernel (tools/bench_net.py, 4096 boards) per variant: one rocprofv3
# --pmc pass per counter group (no trace domains beside --pmc), then the counter list.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pmcnet; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i + 1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-include-regex "k_net_" -d $O/p$i -o pmc --output-format csv -- \
    python3 tools/bench_net.py --n 4096 --iters 3 --rounds 1 --variants "${VARIANTS:-f16f8:0}" > $O/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; tail -2 $O/p$i.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
