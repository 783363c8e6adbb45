"""Time one kernel family from an explicit build of the extension (A/B of two builds on one box:
run this once per .so, alternating, each in its own process).

    python tools/probe/ext_ab.py path/to/_C.so attn_bwd|attn_fwd [reps]

Loads the given .so as ``hetseq_9cme_amd._C`` before anything imports the package's own build."""
import importlib.machinery
import importlib.util
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def load(path):
    import hetseq_9cme_amd  # noqa: F401  (the package, without its _C)
    loader = importlib.machinery.ExtensionFileLoader('hetseq_9cme_amd._C', path)
    spec = importlib.util.spec_from_file_location('hetseq_9cme_amd._C', path, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    sys.modules['hetseq_9cme_amd._C'] = mod
    return mod


def timed(fn, n=30):
    for _ in range(5):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ev)[n // 2] * 1e3


def main():
    C = load(sys.argv[1])
    what = sys.argv[2]
    dev = torch.device('cuda', 0)
    S = int(os.environ.get('S', '128'))
    B, nh, keep = 16384 // S, 12, 0.9
    H = 64 * nh
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B, S, 3 * H, device=dev, generator=g)
    bias = torch.randn(3 * H, device=dev, generator=g) * 0.1
    mb = torch.zeros(B, S, device=dev)
    mb[:, S - 9:] = -10000.0
    seed = torch.full((1,), 7, dtype=torch.int64, device=dev)
    out, lse, dm = C.attn_fwd_f16(qkv, mb, nh, keep, seed, 0, bias)[:3]
    dout = torch.randn(B, S, H, device=dev, generator=g)
    am = torch.empty(B * S, nh, device=dev)
    cm = torch.empty(B, 3 * H, device=dev) if S <= 128 else None
    if S > 128:
        am = None
    dbq, dbk, dbv = (torch.zeros(H, device=dev) for _ in range(3))
    if what == 'attn_bwd':
        fn = lambda: C.attn_bwd_f16(dout, qkv, mb, out, lse, dm, nh, keep, bias, dbq, dbk, dbv, am, cm)  # noqa: E731
    else:
        am2 = torch.empty(B * S, nh, device=dev)
        cm2 = torch.empty(B * ((S + 127) // 128), H, device=dev)
        nb = None if os.environ.get('NO_BIAS') else bias   # the step adds the bias in the QKV GEMM
        fn = lambda: C.attn_fwd_f16(qkv, mb, nh, keep, seed, 0, nb, am2, cm2)  # noqa: E731
    r = fn()
    ref = r[0] if isinstance(r, (list, tuple)) else r
    print('{} {} {:.1f} us  checksum {:.6e}'.format(os.path.basename(sys.argv[1]), what, timed(fn),
                                                     ref.double().abs().sum().item()), flush=True)


if __name__ == '__main__':
    main()
