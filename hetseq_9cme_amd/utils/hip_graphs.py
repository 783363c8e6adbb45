"""HIP-graph replay for launch-bound inference loops.

A BERT-base forward at fine-tuning / evaluation sizes (batch 32, 10-60 tokens)
is ~100 kernel launches of a few microseconds each: the host's Python + launch
overhead, not the GPU, sets the pace (the NER evaluator of the reference,
hetseq/eval_ner.py, and this repo's ``eval_ner`` run exactly that loop).
``GraphedForward`` captures the forward once per input-shape key into a
``torch.cuda.CUDAGraph`` (a hipGraph on ROCm) and afterwards replays it: one
graph launch instead of ~100 kernel launches.

* Inputs are copied into static buffers owned by the graph, outputs come back
  as fresh tensors (cloned) unless ``clone_outputs=False``.
* Sequence lengths are padded up to a multiple of ``pad_multiple`` (masked
  positions, so real positions are unaffected) to bound the number of graphs;
  ``GraphedForward`` slices outputs back to the caller's length.
* Only for modules in eval mode under ``torch.no_grad()``: no dropout (the
  Philox seeds are launch arguments and would be frozen into the graph) and no
  autograd state.  Training steps stay eager.
* Shapes seen fewer than ``warmup`` times run eagerly (first-call library
  initialisation, GEMM-solution lookup) before being captured; at most
  ``max_graphs`` graphs are kept (oldest dropped).
"""
import collections

import torch


class GraphedForward(object):
    def __init__(self, fn, pad_multiple=16, warmup=1, max_graphs=32, clone_outputs=True):
        """``fn(input_ids, token_type_ids, attention_mask) -> Tensor [B, S, ...]``."""
        self.fn = fn
        self.pad = max(1, int(pad_multiple))
        self.warmup = warmup
        self.max_graphs = max_graphs
        self.clone = clone_outputs
        self.graphs = collections.OrderedDict()
        self.seen = collections.Counter()
        self.pool = None
        self.replays = 0

    def _padded(self, ids, tt, mask):
        B, S = ids.shape
        Sp = -(-S // self.pad) * self.pad
        if Sp == S:
            return ids, tt, mask
        z = lambda t: torch.nn.functional.pad(t, (0, Sp - S))   # noqa: E731  (pad ids/types/mask with 0)
        return z(ids), z(tt), z(mask)

    def __call__(self, input_ids, token_type_ids, attention_mask):
        if not input_ids.is_cuda:
            return self.fn(input_ids, token_type_ids, attention_mask)
        S = input_ids.shape[1]
        ids, tt, mask = self._padded(input_ids, token_type_ids, attention_mask)
        key = (tuple(ids.shape), ids.dtype, tt.dtype, mask.dtype, ids.device.index)
        entry = self.graphs.get(key)
        if entry is None:
            self.seen[key] += 1
            if self.seen[key] <= self.warmup:
                return self.fn(ids, tt, mask)[:, :S]
            entry = self._capture(key, ids, tt, mask)
        else:
            self.graphs.move_to_end(key)
        g, static_in, out = entry
        for s, t in zip(static_in, (ids, tt, mask)):
            s.copy_(t)
        g.replay()
        self.replays += 1
        out = out[:, :S]
        return out.clone() if self.clone else out

    def _capture(self, key, ids, tt, mask):
        static_in = [ids.clone(), tt.clone(), mask.clone()]
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):   # warm the exact call once more off the capture
            self.fn(*static_in)
        cur.wait_stream(side)
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self.pool):
            out = self.fn(*static_in)
        entry = (g, static_in, out)
        self.graphs[key] = entry
        while len(self.graphs) > self.max_graphs:
            self.graphs.popitem(last=False)
        return entry
