#!/bin/bash
# Rehearsal of bench.py's N-rank path on ONE GPU: 2 ranks under torch.distributed.run, both on
# cuda:0, gloo for the end-of-run reductions (RCCL needs one GPU per rank).  512 games per rank.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/multi
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 1 --games 512 --dist-backend gloo --device 0 \
  > gpurun_out/multi/rehearse2.log 2>&1
rc=$?; echo "[rehearse2] rc=$rc"; grep '^{' gpurun_out/multi/rehearse2.log | cut -c1-300; exit $rc
