"""Per-shape library choice for the split-GEMM bf16 -> fp32 GEMMs (hipBLASLt vs rocBLAS):
the forward (x' [T, nK] . W'^T) and data-gradient (dy' [T, nN] . W'' [nN, K]) forms at
BERT-base shapes, T = 16384, for bf16x3 / bf16x6."""
import json
import time

import torch


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it * 1e6


T = 16384
res = {}
for n in (3, 6):
    for name, n_in, n_out in (('qkv', 768, 2304), ('ao', 768, 768), ('up', 768, 3072), ('down', 3072, 768)):
        xs = torch.randn(T, n * n_in, device='cuda').bfloat16()
        wq = torch.randn(n_out, n * n_in, device='cuda').bfloat16()
        dys = torch.randn(T, n * n_out, device='cuda').bfloat16()
        wb = torch.randn(n * n_out, n_in, device='cuda').bfloat16()
        for form, fn in (('fwd', lambda: torch.mm(xs, wq.t(), out_dtype=torch.float32)),
                         ('dgrad', lambda: torch.mm(dys, wb, out_dtype=torch.float32))):
            r = {}
            for lib in ('cublaslt', 'cublas'):
                torch.backends.cuda.preferred_blas_library(lib)
                r[lib] = timeit(fn)
            key = 'x{} {} {}'.format(n, name, form)
            res[key] = r
            print(key, ' '.join('{} {:.1f}'.format(k, v) for k, v in r.items()), flush=True)
        del xs, wq, dys, wb
print(json.dumps(res))
