#!/bin/bash
# Instruction-mix PMC pass for k_net_z (guides round 3): lists the device's counters, keeps those of
# the wanted set that exist (at most 7 SQ + GRBM_GUI_ACTIVE), one rocprofv3 --pmc pass of a short bench.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/pmci; mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || { echo "list failed"; tail -5 $O/counters.txt; exit 1; }
SEL=""
n=0
for c in SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_MFMA_MOPS_F16; do
  if grep -qw "$c" $O/counters.txt && [ $n -lt 7 ]; then SEL="$SEL $c"; n=$((n + 1)); fi
done
echo "counters:$SEL GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $SEL GRBM_GUI_ACTIVE --kernel-include-regex "k_net_z" -d $O/p -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --no-secondary > $O/run.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 $O/run.log
exit $rc
