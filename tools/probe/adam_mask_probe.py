"""Debug: where do the host-mask and device-mask Adam paths differ (test_optim_mask_gpu)?"""
import sys
import torch
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from test_optim_mask_gpu import _opt

dev = torch.device('cuda', 0)
for shadow in (False, True):
    a, b = _opt(dev, shadow), _opt(dev, shadow)
    print('shadow', shadow, 'init equal', torch.equal(a.flat.param_flat, b.flat.param_flat))
    n = len(a.flat.params)
    g = torch.Generator().manual_seed(3)
    live = torch.zeros(a.flat.numel, device=dev)
    for i in range(n):
        s, e = a.flat.param_range(i)
        live[s:e] = 1
    for step in range(4):
        grad = torch.randn(a.flat.numel, generator=g).to(dev) * live
        used = (torch.rand(n, generator=g) > 0.3).tolist()
        used[0] = used[-1] = bool(step % 2)
        for o in (a, b):
            o.flat.grad_flat.copy_(grad)
            o._gscale.fill_(0.5)
        a.used_mask = list(used)
        a.step()
        b.device_used = torch.tensor([2.0 * u for u in used], dtype=torch.float64, device=dev)
        b.step()
        torch.cuda.synchronize()
        d = (a.flat.param_flat != b.flat.param_flat).nonzero().flatten()
        hp = b._mask_hp.view(-1, 2).cpu()
        print(' step', step, 'ndiff', d.numel(), 'nan', bool(torch.isnan(a.flat.param_flat).any()),
              bool(torch.isnan(b.flat.param_flat).any()))
        if d.numel():
            pids = sorted({next(i for i in range(n) if a.flat.param_range(i)[0] <= int(x) < a.flat.param_range(i)[1] + 64)
                           for x in d[:2000].tolist()})
            print('  params', pids[:20], 'first idx', d[:8].tolist(), 'ranges', [a.flat.param_range(i) for i in pids[:5]])
            print('  a', a.flat.param_flat[d[:4]].tolist(), 'b', b.flat.param_flat[d[:4]].tolist())
            print('  used', [used[i] for i in pids[:10]], 'hp', [hp[i].tolist() for i in pids[:4]], 'steps', [a.steps[i] for i in pids[:4]])
