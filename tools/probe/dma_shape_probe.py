"""LDS-DMA throughput per CU by source segment shape (gemm_split.hip dma_probe_k): one
workgroup per CU streaming 42-KiB stages through a 3-stage ring (the piece GEMM's staging
without the MFMAs).  seg 1024 = each instruction reads one contiguous KiB; 64 = 16 rows x
64 B (natural layout, BK 32); 32 = 32 rows x 32 B (natural layout, BK 16)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from hetseq_9cme_amd.ops._ext import C
    src = torch.randint(0, 1000, (40 * 1024 * 1024 // 2,), dtype=torch.int16, device='cuda')   # 40 MiB
    iters = 400
    for ld in (6144, 24576):
        for seg in (1024, 128, 64, 32):
            for grid in (256,):
                for _ in range(2):
                    C().dma_probe(src, seg, ld, iters, grid)
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                C().dma_probe(src, seg, ld, iters, grid)
                b.record()
                b.synchronize()
                ms = a.elapsed_time(b)
                byt = grid * iters * 42 * 1024
                print('ld {:6d} seg {:5d} grid {:4d}: {:7.3f} ms  {:6.2f} TB/s chip  {:6.1f} GB/s per CU-workgroup'.format(
                    ld, seg, grid, ms, byt / ms / 1e9, byt / ms / 1e6 / min(grid, 256)), flush=True)


if __name__ == '__main__':
    main()
