"""Probe: data-gradient GEMM layout for the split-plane path.

dgrad = dy' [T, nN] . W'' where W'' is either the stacked planes [nN, K] (NN form, what
ops/split_gemm.py uses) or the transposed-weight planes [K, nN] used as its transpose (NT
form, both operands contiguous along the reduction dimension, like the forward GEMMs).
Also times the beta = 1 (accumulate) variant.  BERT-base shapes, T = 16384, bf16x6."""
import json
import time

import torch


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = []
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(it):
            fn()
        torch.cuda.synchronize()
        best.append((time.perf_counter() - t) / it * 1e6)
    return min(best)


T = 16384
res = {}
for n in (6, 3):
    for name, n_in, n_out in (('qkv', 768, 2304), ('ao', 768, 768), ('up', 768, 3072), ('down', 3072, 768)):
        dys = (torch.rand(T, n * n_out, device='cuda') * 2 - 1).bfloat16()
        wb = (torch.rand(n * n_out, n_in, device='cuda') * 2 - 1).bfloat16()     # NN operand
        wt = wb.t().contiguous()                                                  # [K, nN]
        acc = torch.zeros(T, n_in, device='cuda')
        r = {
            'nn': timeit(lambda: torch.mm(dys, wb, out_dtype=torch.float32)),
            'nt': timeit(lambda: torch.mm(dys, wt.t(), out_dtype=torch.float32)),
            'nn_acc': timeit(lambda: torch.addmm(acc, dys, wb, out_dtype=torch.float32, out=acc)),
            'nt_acc': timeit(lambda: torch.addmm(acc, dys, wt.t(), out_dtype=torch.float32, out=acc)),
        }
        d = torch.mm(dys, wb, out_dtype=torch.float32) - torch.mm(dys, wt.t(), out_dtype=torch.float32)
        r['maxdiff'] = d.abs().max().item()
        gf = 2.0 * T * n * n_out * n_in / 1e9
        key = 'x{} {} dgrad'.format(n, name)
        res[key] = r
        print(key, ' '.join('{} {:.1f}us'.format(k, v) if k != 'maxdiff' else '{} {:.2e}'.format(k, v)
                            for k, v in r.items()),
              '| PF nn {:.2f} nt {:.2f}'.format(gf / r['nn'] / 1e3, gf / r['nt'] / 1e3), flush=True)
        del dys, wb, wt, acc
print(json.dumps(res))
