#!/bin/bash
# One GPU-box driver for every measurement this repo takes (run through gpurun):
#
#   bash tools/gpu.sh OUT step [step ...]
#
# Results go to gpurun_out/OUT/.  Steps run in order, each under its own time limit; the script
# stops after a step that ends abnormally (fault, abort, time limit: rc >= 124, or any rc other
# than 0 / 1 from pytest) and never retries one.
#
#   tests            pytest -m gpu (K_EXPR: a -k filter, PYTEST_FILES: files instead of tests/)
#   smoke            __graft_entry__.smoke()
#   bench            python bench.py $BENCH_ARGS           -> bench.json (the JSON line), bench.err
#   prof             rocprofv3 --kernel-trace --stats of bench.py $PROF_ARGS (default: --no-cpu-baseline);
#                    per-evaluation main / tail / gap summary: python tools/trace_summary.py
#                    gpurun_out/OUT/prof/bench_kernel_trace.csv
#   pmc              rocprofv3 --pmc passes on the network kernel, one counter group per pass
#                    (FETCH_SIZE / WRITE_SIZE / TCC hit-miss / SQ busy group), of bench.py $PMC_ARGS;
#                    summarise with python tools/pmc_summary.py gpurun_out/OUT/pmc
#   pmcdiag          one PMC pass (MFMA busy, cycles, GRBM) over k_net_y's product + diagnostic forms
#   pmci             the instruction-mix PMC pass (SQ_INSTS_*) of bench.py $PMC_ARGS
#   ab               tools/bench_net.py A/B of network variants $AB_VARIANTS (AB_DIAG=1: diagnostic library)
#   netab            the same on the product library for the variants it accepts
#   stress           tools/train_stress.py $STRESS_ARGS
#   cmd              bash -c "$CMD" (one extra command, logged)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:?usage: gpu.sh OUT step...}
shift
mkdir -p "$OUT"

run() {   # name timeout command...
  local name=$1 lim=$2
  shift 2
  echo "[gpu.sh] $name: $*" >&2
  local t0=$(date +%s.%N)
  timeout -k 10 "$lim" "$@"
  local rc=$?
  local t1=$(date +%s.%N)
  echo "[gpu.sh] $name rc=$rc wall_s=$(awk "BEGIN{printf \"%.1f\", $t1 - $t0}")" >&2
  echo "$name rc=$rc wall_s=$(awk "BEGIN{printf \"%.1f\", $t1 - $t0}")" >> "$OUT/walls.txt"
  return $rc
}

abnormal() { [ "$1" -ge 124 ] || [ "$1" -lt 0 ]; }

for step in "$@"; do
  case $step in
    tests)
      run tests "${PYTEST_TIMEOUT:-1500}" python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -v -p no:cacheprovider \
        --timeout 300 --timeout-method thread ${K_EXPR:+-k "$K_EXPR"} > "$OUT/pytest_gpu.log" 2>&1
      rc=$?
      grep -E "passed|failed|FAILED|ERROR" "$OUT/pytest_gpu.log" | tail -30 | cut -c1-200
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ;;
    smoke)
      run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1
      rc=$?; tail -2 "$OUT/smoke.txt"; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    bench)
      run bench "${BENCH_TIMEOUT:-900}" python -u bench.py ${BENCH_ARGS} > "$OUT/bench.json" 2> "$OUT/bench.err"
      rc=$?; tail -3 "$OUT/bench.err"; cut -c1-600 "$OUT/bench.json"; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    prof)
      run prof "${PROF_TIMEOUT:-900}" rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv \
        -- python3 bench.py ${PROF_ARGS:---no-cpu-baseline} > "$OUT/prof_bench.log" 2>&1
      rc=$?; tail -3 "$OUT/prof_bench.log"; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    pmc)
      i=0
      for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
                 "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
        i=$((i + 1))
        run "pmc $i ($grp)" "${PMC_TIMEOUT:-420}" rocprofv3 --pmc $grp --kernel-include-regex "k_net_[yz]" \
          -d "$OUT/pmc/p$i" -o pmc --output-format csv -- python3 bench.py ${PMC_ARGS:---no-cpu-baseline --default-sims 0} \
          > "$OUT/pmc_p$i.log" 2>&1
        rc=$?; tail -1 "$OUT/pmc_p$i.log"; if [ $rc -ne 0 ]; then exit $rc; fi
      done ;;
    pmcnet)
      # the network kernel alone (tools/bench_net.py, 4096 boards): one counter group per pass
      i=0
      for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
                 "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
                 "FETCH_SIZE TCC_HIT_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
        i=$((i + 1))
        run "pmcnet $i" "${PMC_TIMEOUT:-300}" rocprofv3 --pmc $grp --kernel-include-regex "k_net_y" \
          -d "$OUT/pmcnet${PMCNET_TAG}/p$i" -o pmc --output-format csv -- python3 tools/bench_net.py --variants ${PMCNET_VARIANTS:-f16x3:0} \
          --rounds 1 --iters 5 > "$OUT/pmcnet${PMCNET_TAG}_p$i.log" 2>&1
        rc=$?; tail -1 "$OUT/pmcnet${PMCNET_TAG}_p$i.log"; if [ $rc -ne 0 ]; then exit $rc; fi
      done ;;
    pmcdiag)
      # one PMC pass (MFMA busy, wave and busy cycles, GPU-active clocks) over the network kernel's
      # product and diagnostic forms in one process (tools/bench_net.py --diag $PMCDIAG_VARIANTS)
      run pmcdiag "${PMC_TIMEOUT:-300}" rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "k_net_y" \
        -d "$OUT/pmcdiag" -o pmc --output-format csv -- python3 tools/bench_net.py --diag \
        --variants ${PMCDIAG_VARIANTS:-f16x3:0} --rounds 1 --iters 5 > "$OUT/pmcdiag.log" 2>&1
      rc=$?; tail -1 "$OUT/pmcdiag.log"; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    pmci)
      run pmci "${PMC_TIMEOUT:-420}" rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
        SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --kernel-include-regex "k_net_[yz]" \
        -d "$OUT/pmci" -o pmc --output-format csv -- python3 bench.py ${PMC_ARGS:---no-cpu-baseline --default-sims 0} \
        > "$OUT/pmci.log" 2>&1
      rc=$?; tail -1 "$OUT/pmci.log"; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    ab|netab)
      run ab "${AB_TIMEOUT:-400}" python -u tools/bench_net.py ${AB_DIAG:+--diag} --variants "${AB_VARIANTS:-0}" \
        --rounds "${AB_ROUNDS:-4}" --iters "${AB_ITERS:-10}" > "$OUT/ab.json" 2> "$OUT/ab.err"
      rc=$?; cut -c1-300 "$OUT/ab.json"; tail -3 "$OUT/ab.err"; if abnormal $rc; then exit $rc; fi ;;
    stress)
      run stress "${STRESS_TIMEOUT:-1000}" python -u tools/train_stress.py ${STRESS_ARGS} > "$OUT/train.jsonl" 2> "$OUT/train.err"
      rc=$?; tail -2 "$OUT/train.jsonl" | cut -c1-600; tail -3 "$OUT/train.err"; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    cmd)
      run cmd "${CMD_TIMEOUT:-600}" bash -c "$CMD" > "$OUT/cmd.log" 2>&1
      rc=$?; tail -5 "$OUT/cmd.log"; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    *)
      echo "[gpu.sh] unknown step $step"; exit 2 ;;
  esac
done
