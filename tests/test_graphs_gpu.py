"""HIP-graph replay of the evaluation forward (hetseq_9cme_amd/utils/hip_graphs.py):
graphed logits == eager logits for several padded shapes, replays track new input
values, padding to the graph's length does not change real positions; prints the
eager vs graphed latency of a batch-32 BERT-base token-classification forward."""
import time

import pytest
import torch

from hetseq_9cme_amd.data.synthetic import BERT_BASE, BERT_TINY
from hetseq_9cme_amd.models.bert import BertConfig, BertForTokenClassification
from hetseq_9cme_amd.utils.hip_graphs import GraphedForward

pytestmark = pytest.mark.gpu


def _batch(B, S, V, dev, g):
    ids = torch.randint(1, V, (B, S), generator=g).to(dev)
    tt = torch.zeros(B, S, dtype=torch.long, device=dev)
    lens = torch.randint(max(1, S // 2), S + 1, (B,), generator=g)
    mask = (torch.arange(S)[None, :] < lens[:, None]).long().to(dev)
    return ids, tt, mask


def test_graphed_forward_matches_eager(dev):
    torch.manual_seed(0)
    cfg = BertConfig.from_dict(dict(BERT_TINY))
    model = BertForTokenClassification(cfg, 9).to(dev).eval()
    gf = GraphedForward(model, pad_multiple=16, warmup=1)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for S in (13, 16, 29, 13, 29, 40):
            for _ in range(3):
                ids, tt, mask = _batch(8, S, cfg.vocab_size, dev, g)
                ref = model(ids, tt, mask)
                out = gf(ids, tt, mask)
                assert out.shape == ref.shape
                keep = mask.bool()
                torch.testing.assert_close(out[keep], ref[keep], rtol=1e-4, atol=1e-5)
    assert gf.replays > 0 and len(gf.graphs) == 3   # padded lengths 16, 32, 48


def test_graphed_forward_latency_bert_base(dev):
    torch.manual_seed(0)
    cfg = BertConfig.from_dict(dict(BERT_BASE))
    model = BertForTokenClassification(cfg, 9).to(dev).eval()
    g = torch.Generator().manual_seed(2)

    def bench(fn, n=30):
        for _ in range(3):
            fn(ids, tt, mask)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn(ids, tt, mask)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    for B, S in ((1, 32), (8, 64), (32, 48)):
        gf = GraphedForward(model)
        ids, tt, mask = _batch(B, S, cfg.vocab_size, dev, g)
        with torch.no_grad():
            eager = bench(model)
            graphed = bench(gf)
            torch.testing.assert_close(gf(ids, tt, mask), model(ids, tt, mask), rtol=1e-4, atol=1e-4)
        print('BERT-base token-classification forward, batch {} x {}: eager {:.2f} ms, HIP graph {:.2f} ms'.format(
            B, S, eager, graphed))
