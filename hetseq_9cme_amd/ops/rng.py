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
    """The per-update key lives in a 1-element int64 tensor per device that the kernels
    read themselves (``const uint64_t* seed``): eager steps refresh it once per update
    (one tiny fill), a captured training step (utils/train_graph.py) writes it before each
    replay, so replays draw fresh masks while the stream ids stay baked into the graph."""

    def __init__(self, seed=0):
        self.seed = int(seed)
        self.counter = 0
        self._dev = {}       # device index -> (tensor, seed value it holds)
        self.external = False   # True while a graph replayer owns the device keys

    def set_seed(self, seed):
        self.seed = int(seed) & ((1 << 63) - 1)
        self.counter = 0

    def seed_tensor(self, device):
        """The device-resident key for ``device`` (refreshed to ``self.seed`` if stale)."""
        import torch
        idx = device.index if device.index is not None else torch.cuda.current_device()
        ent = self._dev.get(idx)
        if ent is None:
            t = torch.full((1,), self.seed, dtype=torch.int64, device=torch.device('cuda', idx))
            self._dev[idx] = [t, self.seed]
            return t
        if ent[1] != self.seed and not self.external and not torch.cuda.is_current_stream_capturing():
            ent[0].fill_(self.seed)
            ent[1] = self.seed
        return ent[0]

    def next(self, device=None):
        """(key, stream id) for the next dropout call site; the key is the device tensor
        when ``device`` is a GPU, else the integer seed."""
        s = self.counter
        self.counter += 1
        if device is not None and device.type == 'cuda':
            return self.seed_tensor(device), s
        return self.seed, s


_GLOBAL = DropoutRNG(0)


def get_rng():
    return _GLOBAL


def set_step_seed(seed):
    _GLOBAL.set_seed(seed)
