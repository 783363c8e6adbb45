"""Probe: can two processes share one GPU in an RCCL (nccl backend) group?

Run under torch.distributed.run with 2 ranks on a 1-GPU box; each rank uses cuda:0.
Prints the all-reduced value on each rank, or the error RCCL raises."""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ['RANK'])
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', device_id=torch.device('cuda', 0))
    t = torch.full((1 << 20,), float(rank + 1), device='cuda')
    try:
        dist.all_reduce(t)
        torch.cuda.synchronize()
        print('rank {} all_reduce ok: {}'.format(rank, t[0].item()), flush=True)
    except Exception as e:  # noqa: BLE001
        print('rank {} all_reduce failed: {}'.format(rank, e), flush=True)
        sys.exit(3)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
