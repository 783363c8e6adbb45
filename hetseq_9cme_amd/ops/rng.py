"""Counter-based dropout RNG state shared by all fused kernels.

Reference semantics (hetseq/controller.py:427-433): every update reseeds the RNG
with ``args.seed + num_updates`` on every rank (identical masks on all ranks,
SURVEY App. A14).  Here the per-update seed is the Philox key; each dropout call
site in forward order draws a fresh 64-bit *stream id*.  A kernel's mask is a pure
function of (seed, stream, element index), so backward regenerates it from the
(seed, stream) pair saved on the autograd context -- nothing is stored -- and the
same call order replays identically under HIP-graph capture.
"""


class DropoutRNG(object):
    def __init__(self, seed=0):
        self.seed = int(seed)
        self.counter = 0

    def set_seed(self, seed):
        self.seed = int(seed) & ((1 << 63) - 1)
        self.counter = 0

    def next(self):
        s = self.counter
        self.counter += 1
        return self.seed, s


_GLOBAL = DropoutRNG(0)


def get_rng():
    return _GLOBAL


def set_step_seed(seed):
    _GLOBAL.set_seed(seed)
