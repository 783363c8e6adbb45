"""Probe: does PyTorch's TunableOp cover the split-GEMM bf16 x bf16 -> fp32 products
(torch.mm(..., out_dtype=torch.float32)), and what does tuning buy over the default?
Forward (NT) and data-gradient (NT, transposed weight planes) shapes of BERT-base, bf16x6."""
import os
import sys
import time

import torch


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(it):
            fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / it * 1e6)
    return best


T, n = 16384, 6
shapes = [('qkv fwd', T, 2304, 768), ('ao fwd', T, 768, 768), ('up fwd', T, 3072, 768), ('down fwd', T, 768, 3072),
          ('qkv dgrad', T, 768, 2304), ('ao dgrad', T, 768, 768), ('up dgrad', T, 768, 3072),
          ('down dgrad', T, 3072, 768)]
ops = []
for name, M, N, K in shapes:
    a = (torch.rand(M, n * K, device='cuda') * 2 - 1).bfloat16()
    b = (torch.rand(N, n * K, device='cuda') * 2 - 1).bfloat16()
    ops.append((name, a, b))
# prefix-form products of the deep, narrow shapes (split_gemm.prefix_mm): column prefixes of a
# 3-piece operand (row stride 3K) against piece-j weight blocks
for name, M, N, K in [('down/up-dgrad prefix', T, 768, 3072)]:
    a3 = (torch.rand(M, 3 * K, device='cuda') * 2 - 1).bfloat16()
    for j in range(3):
        m = (3 - j) * K
        b = (torch.rand(N, m, device='cuda') * 2 - 1).bfloat16()
        ops.append(('%s %d' % (name, j), a3[:, :m], b))
base = {name: timeit(lambda: torch.mm(a, b.t(), out_dtype=torch.float32)) for name, a, b in ops}
out = os.path.join(sys.argv[1] if len(sys.argv) > 1 else '.', 'tunable_bf16.csv')
torch.cuda.tunable.enable(True)
torch.cuda.tunable.tuning_enable(True)
torch.cuda.tunable.set_max_tuning_duration(200)
torch.cuda.tunable.set_filename(out, insert_device_ordinal=False)
for name, a, b in ops:
    torch.mm(a, b.t(), out_dtype=torch.float32)
torch.cuda.synchronize()
torch.cuda.tunable.tuning_enable(False)
tuned = {name: timeit(lambda: torch.mm(a, b.t(), out_dtype=torch.float32)) for name, a, b in ops}
for name, _, _ in ops:
    print('{:24s} default {:7.1f} us  tunable {:7.1f} us'.format(name, base[name], tuned[name]), flush=True)
print('results:', torch.cuda.tunable.get_results())
