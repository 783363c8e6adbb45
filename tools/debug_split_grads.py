"""Debug: per-parameter gradient difference, native fp32 vs split-GEMM modes, BERT-tiny."""
import sys
import torch
sys.path.insert(0, '.')
from hetseq_9cme_amd import ops
from hetseq_9cme_amd.models.bert import BertConfig, BertForPreTraining
from hetseq_9cme_amd.parallel.flat_params import FlatParamSpace

dev = torch.device('cuda', 0)
cfg = BertConfig(1024, hidden_size=128, num_hidden_layers=2, num_attention_heads=2, intermediate_size=512,
                 max_position_embeddings=128, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
B, S = 8, 128
g = torch.Generator().manual_seed(0)
ids = torch.randint(5, 1024, (B, S), generator=g).to(dev)
seg = torch.zeros_like(ids)
mask = torch.ones_like(ids)
labels = torch.full_like(ids, -1)
labels[:, 3:23] = ids[:, 3:23]
nsp = torch.randint(0, 2, (B,), generator=g).to(dev)
grads = {}
for mode in sys.argv[1:] or ['native', 'bf16x6', 'bf16x3']:
    torch.manual_seed(0)
    model = BertForPreTraining(cfg).to(dev)
    model.max_predictions_per_seq = 20
    flat = FlatParamSpace(model, dev, contiguous_groups=model.flat_contiguous_groups())
    ops.set_fp32_gemm(mode)
    ops.set_step_seed(1)
    model.train()
    flat.zero_grad()
    loss = model(ids, seg, mask, labels, nsp)
    loss.backward()
    flat.adopt_all()
    torch.cuda.synchronize()
    grads[mode] = {n: p.grad.detach().double().clone() for n, p in zip(flat.names, flat.params)}
    print(mode, 'loss', loss.item())
ops.set_fp32_gemm('native')
for mode in grads:
    if mode == 'native':
        continue
    for n, gn in grads['native'].items():
        gm = grads[mode][n]
        e = (gm - gn).abs().max().item() / (gn.abs().max().item() + 1e-30)
        flag = '  <<<' if e > 1e-3 else ''
        print('{:8s} {:60s} {:.3e}{}'.format(mode, n, e, flag))
