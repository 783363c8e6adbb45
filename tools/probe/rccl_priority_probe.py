"""Probe: a process group on the nccl (RCCL) backend with high-priority streams initialises
and all-reduces through this framework's distributed_init (run under torch.distributed.run,
one rank per GPU; on a 1-GPU box with one rank)."""
import argparse
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hetseq_9cme_amd.parallel import distributed as du  # noqa: E402

torch.cuda.set_device(int(os.environ.get('LOCAL_RANK', '0')))
args = argparse.Namespace(distributed_world_size=int(os.environ['WORLD_SIZE']), distributed_rank=int(os.environ['RANK']),
                          distributed_backend='nccl', distributed_init_method='env://', distributed_timeout=120, cpu=False)
if args.distributed_world_size == 1:
    # distributed_init refuses world 1 (as the reference does); exercise the same kwargs directly
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    dist.init_process_group('nccl', init_method='env://', world_size=1, rank=0, pg_options=opts,
                            device_id=torch.device('cuda', 0))
else:
    du.distributed_init(args)
t = torch.ones(1 << 20, device='cuda')
dist.all_reduce(t)
torch.cuda.synchronize()
pg = dist.group.WORLD
print('rank', dist.get_rank(), 'sum', t[0].item(), 'backend', dist.get_backend(), flush=True)
dist.destroy_process_group()
