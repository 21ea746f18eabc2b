#!/bin/bash
# Cross-library A/B (same box, alternating processes): the product library vs $ALT_LIB (the same
# sources built with other compiler options), each timed twice, plus a hash of the outputs.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/ablib; mkdir -p $O
for i in 1 2; do
  for L in minitchess_alphazero_amd/libmtaz.so $ALT_LIB; do
    MTAZ_LIB=$PWD/$L timeout -k 10 200 python tools/bench_net.py --variants 0 --rounds 4 --iters 10 > $O/ab_$(basename $L)_$i.json 2>> $O/ab.err
    rc=$?; if [ $rc -ne 0 ]; then tail -5 $O/ab.err; exit $rc; fi
    python3 -c "
import json; d=json.loads(open('$O/ab_$(basename $L)_$i.json').readline()); print('$L', $i, round(d['ms_median'],4), int(d['wg_cycles']), round(d['clock_ghz_stamped'],3), d['shares'])"
  done
done
for L in minitchess_alphazero_amd/libmtaz.so $ALT_LIB; do
  MTAZ_LIB=$PWD/$L timeout -k 10 200 python -c "
import sys, hashlib, numpy as np, torch
sys.path.insert(0, 'tests')
from minitchess_alphazero_amd.engine import Engine
from minitchess_alphazero_amd.environment import pos_from_fen
from minitchess_alphazero_amd.network import Network
from tests_positions import random_fens
eng = Engine(n_games=64, sims=4); eng.set_precision('f16f8'); torch.manual_seed(0); eng.set_weights(Network())
pos = np.stack([pos_from_fen(f) for f in random_fens(257, seed=3)])
l, v = eng.evaluate(pos)
print('$L', hashlib.sha256(l.tobytes() + v.tobytes()).hexdigest()[:16])
" || exit $?
done
