"""Probe: nontemporal vs ordinary 16-B stores for the bias-GELU plane writer (bias_act_planes_k)
at BERT-base FFN shapes (T = 16384, N = 3072, bf16x6: 6 planes), interleaved in one process."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hetseq_9cme_amd.ops import split_gemm as sg  # noqa: E402


def timeit(fn, it=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e6


sg.set_fp32_gemm('bf16x6')
T, N = 16384, 3072
y = torch.randn(T, N, device='cuda')
b = torch.randn(N, device='cuda')
d = torch.randn(T, N, device='cuda')
db = torch.empty(N, device='cuda')
res = {'fwd': {0: [], 1: []}, 'bwd': {0: [], 1: []}}
# the kernel variant is chosen once per process (static): run as two child processes
mode = int(os.environ.get('HX_NT_STORES', '0'))
for r in range(5):
    res['fwd'][mode].append(timeit(lambda: sg.act_planes(y, b, 'gelu')))
    res['bwd'][mode].append(timeit(lambda: sg.act_grad_planes(d, y, b, 'gelu', db)))
fwd_b = T * N * (4 + 12)
bwd_b = T * N * (8 + 12)
f, g = min(res['fwd'][mode]), min(res['bwd'][mode])
print('nt={} fwd {:.1f} us ({:.2f} TB/s)  bwd {:.1f} us ({:.2f} TB/s)'.format(mode, f, fwd_b / f / 1e6, g,
                                                                            bwd_b / g / 1e6), flush=True)
