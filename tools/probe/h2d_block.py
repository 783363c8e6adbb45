"""Probe: does a kernel launched right after a pinned non_blocking H2D copy block the host
while the GPU is busy?  Prints host microseconds per operation."""
import time
import torch

dev = torch.device('cuda')
a = torch.randn(8192, 8192, device=dev)
host = [torch.randint(0, 2, (32, 48)).pin_memory() for _ in range(4)]
pageable = [torch.randint(0, 2, (32, 48)) for _ in range(4)]
dmask = torch.randint(0, 2, (32, 48), device=dev)


def busy():
    for _ in range(5):
        a @ a          # ~20 ms of queued GPU work


def t(label, fn, n=5):
    torch.cuda.synchronize()
    busy()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    dt = (time.perf_counter() - t0) / n * 1e6
    torch.cuda.synchronize()
    print('{:55s} {:9.1f} us/iter'.format(label, dt), flush=True)


cs = torch.cuda.Stream()


def _cs():
    with torch.cuda.stream(cs):
        ts = [h.to(dev, non_blocking=True) for h in host]
        ev = torch.cuda.Event()
        ev.record(cs)
    torch.cuda.current_stream().wait_event(ev)
    return ts[0].to(torch.float32)


for _ in range(2):   # first launches load code objects; measure warm
    dmask.to(torch.float32)
    _cs()
    (1.0 - dmask.to(torch.float32)) * -10000.0
    torch.cuda.synchronize()

t('cast of device tensor', lambda: dmask.to(torch.float32))
t('mask bias (rsub, mul) of device tensor', lambda: (1.0 - dmask.to(torch.float32)) * -10000.0)
t('pinned H2D non_blocking x4', lambda: [h.to(dev, non_blocking=True) for h in host])
t('pinned H2D x4 then cast', lambda: [h.to(dev, non_blocking=True) for h in host][0].to(torch.float32))
t('pageable .pin_memory() then H2D x4', lambda: [h.pin_memory().to(dev, non_blocking=True) for h in pageable])
t('pageable H2D blocking x1', lambda: pageable[0].to(dev))
t('copy-stream H2D x4 + wait_event + cast', _cs)
