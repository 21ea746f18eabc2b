"""One rank of the nccl (RCCL) code paths, started by tests/test_gpu_nccl.py with the launcher's
environment (WORLD_SIZE=1 on the one-GPU box): the process group of bench.py / loop.py, reduce_run
on CUDA tensors, the loop's flat weight broadcast and records gather, one C5 iteration."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from minitchess_alphazero_amd.loop import broadcast_weights, flat_weights, run_loop  # noqa: E402
from minitchess_alphazero_amd.network import Network  # noqa: E402
from minitchess_alphazero_amd.sharding import reduce_run  # noqa: E402


def main():
    local = int(os.environ['LOCAL_RANK'])
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', device_id=dev)          # bench.py:init / loop.main, RCCL
    out = {'backend': dist.get_backend(), 'world': dist.get_world_size()}
    dt, tot = reduce_run(1.25, {'games': 3.0, 'sims': 7.0}, dist, dev)
    out['reduce'] = [dt, tot]
    torch.manual_seed(0)
    net = Network()
    ref, _ = flat_weights(net, dev)
    got = broadcast_weights(net, dist, dev)
    out['broadcast_equal'] = bool(torch.equal(ref, got))
    hist, _net = run_loop(1, 8, 8, batch_size=32, lr=0.02, dist=dist, device=local, log=lambda s: None)
    out['loop_rows'] = hist[0]['rows'] if hist else None
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
