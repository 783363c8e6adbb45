"""Locate a --precision bf16 step that is not a function of its seed (tests/test_determinism_gpu.py
[128-True]): the same tiny BERT step twice with the hand-written bf16 GEMM on every site, on the
linears only, on the decoder only and on none; then each gemm_bf16 shape of that model run twice
(bitwise) and against an fp32 product of the same bf16 operands."""
import sys

import torch

sys.path.insert(0, '.')
from hetseq_9cme_amd import ops  # noqa: E402
from hetseq_9cme_amd.models.bert import BertConfig, BertForPreTraining  # noqa: E402
from hetseq_9cme_amd.ops import gemm16  # noqa: E402
from hetseq_9cme_amd.ops._ext import C  # noqa: E402
from hetseq_9cme_amd.parallel.flat_params import FlatParamSpace  # noqa: E402


def steps(dev, which, eval_mode=False):
    ok = gemm16.bf16_ok

    def patched(x2, n_out, n_in):
        dec = n_out == 64
        if which == 'none' or (which == 'linears' and dec) or (which == 'decoder' and not dec):
            return False
        return ok(x2, n_out, n_in)
    gemm16.bf16_ok = patched
    try:
        torch.manual_seed(0)
        cfg = BertConfig(1024, hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=512,
                         max_position_embeddings=256, hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.1)
        model = BertForPreTraining(cfg).to(dev)
        model.max_predictions_per_seq = 8
        flat = FlatParamSpace(model, dev, contiguous_groups=model.flat_contiguous_groups())
        flat.enable_bf16_shadow()
        model.set_compute_dtype(torch.bfloat16)
        model.eval() if eval_mode else model.train()
        B, S = 4, 128
        ids = torch.randint(5, 1024, (B, S), device=dev)
        seg = torch.zeros_like(ids)
        mask = torch.ones_like(ids)
        mask[1, S - 30:] = 0
        labels = torch.full_like(ids, -1)
        labels[:, 3:8] = ids[:, 3:8]
        nsp = torch.randint(0, 2, (B,), device=dev)
        out = []
        for seed in (11, 11, 11, 12):
            ops.set_step_seed(seed)
            flat.zero_grad()
            loss = model(ids, seg, mask, labels, nsp)
            fwd = loss.item()
            loss.backward()
            flat.adopt_all()
            torch.cuda.synchronize()
            out.append((fwd, flat.grad_flat.norm().item()))
        return out
    finally:
        gemm16.bf16_ok = ok


def kernel_repeats(dev):
    g = torch.Generator(device=dev).manual_seed(0)
    for (M, N, K, lda) in [(512, 384, 128, 128), (512, 128, 128, 128), (512, 512, 128, 128), (512, 128, 512, 512),
                           (32, 1536, 128, 128), (4, 128, 128, 16384), (300, 2304, 768, 768)]:
        a_full = torch.randn(M, lda, device=dev, generator=g).to(torch.bfloat16)
        a = a_full[:, :K]
        b = torch.randn(N, K, device=dev, generator=g).to(torch.bfloat16)
        bias = torch.randn(N, device=dev, generator=g)
        ref = a.float() @ b.float().t() + bias
        outs = [C().gemm_bf16(a, b, bias=bias) for _ in range(3)]
        torch.cuda.synchronize()
        same = all(torch.equal(outs[0], o) for o in outs[1:])
        err = ((outs[0].float() - ref).abs().max() / ref.abs().max()).item()
        print('gemm_bf16 M{} N{} K{} lda{}: repeat-identical {} max rel err {:.2e}'.format(M, N, K, lda, same, err),
              flush=True)


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    kernel_repeats(dev)
    for which in ('all', 'none', 'linears', 'decoder'):
        r = steps(dev, which)
        print('{:8s} (loss, |g|) seed11 x3 / seed12: {}'.format(which, r), flush=True)
    print('all eval {}'.format(steps(dev, 'all', eval_mode=True)), flush=True)


if __name__ == '__main__':
    main()
