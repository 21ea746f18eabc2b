cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r02_first; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.log 2>&1 || { echo bench failed; tail -20 $O/bench.log; exit 1; }
cut -c1-400 $O/bench.log | tail -2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --steps 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo prof failed; tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats*"
