"""Optimizer state is indexed by position in ``model.parameters()`` -- the order a
torch optimizer (and therefore a reference checkpoint's ``last_optimizer_state``)
uses -- not by the flat buffer's internal order."""
import argparse

import torch

from hetseq_9cme_amd.models.bert import BertConfig, BertForPreTraining
from hetseq_9cme_amd.optim.optimizers import _Adam
from hetseq_9cme_amd.parallel.flat_params import FlatParamSpace


def _args():
    return argparse.Namespace(lr=[1e-4], adam_betas='(0.9, 0.999)', adam_eps=1e-8, weight_decay=0.01,
                              fused_kernels=False)


def _model():
    torch.manual_seed(0)
    cfg = BertConfig(200, hidden_size=64, num_hidden_layers=2, num_attention_heads=2, intermediate_size=128,
                     max_position_embeddings=64)
    return BertForPreTraining(cfg)


def test_flat_order_differs_from_model_order():
    model = _model()
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    flat = FlatParamSpace(model, contiguous_groups=model.flat_contiguous_groups())
    assert flat.names != names                       # the case the mapping exists for
    assert [flat.names[i] for i in flat.model_order] == names


def test_load_reference_ordered_state():
    """A torch.optim.Adam state over model.parameters() loads onto the right tensors."""
    model = _model()
    params = [p for p in model.parameters() if p.requires_grad]
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    ref = torch.optim.Adam(params, lr=1e-4)
    g = torch.Generator().manual_seed(1)
    for p in params:
        ref.state[p] = {'step': torch.tensor(7.0),
                        'exp_avg': torch.randn(p.shape, generator=g),
                        'exp_avg_sq': torch.rand(p.shape, generator=g)}
    sd = ref.state_dict()
    expect = {n: (sd['state'][k]['exp_avg'].clone(), sd['state'][k]['exp_avg_sq'].clone())
              for k, n in enumerate(names)}

    flat = FlatParamSpace(model, contiguous_groups=model.flat_contiguous_groups())
    opt = _Adam(_args(), flat)
    opt.load_state_dict(sd)
    for i, n in enumerate(flat.names):
        s, e = flat.param_range(i)
        assert torch.equal(opt.exp_avg[s:e], expect[n][0].reshape(-1)), n
        assert torch.equal(opt.exp_avg_sq[s:e], expect[n][1].reshape(-1)), n
        assert opt.steps[i] == 7

    # and what we write loads back into a torch optimizer over model.parameters()
    out = opt.state_dict()
    ref2 = torch.optim.Adam(params, lr=1e-4)
    ref2.load_state_dict(out)
    for k, p in enumerate(params):
        st = ref2.state[p]
        assert st['exp_avg'].shape == p.shape
        assert torch.equal(st['exp_avg'], expect[names[k]][0])


def test_mismatched_shapes_raise():
    model = _model()
    flat = FlatParamSpace(model, contiguous_groups=model.flat_contiguous_groups())
    opt = _Adam(_args(), flat)
    sd = opt.state_dict()
    n = len(flat.params)
    # a state whose tensors are in FLAT order (the old, wrong indexing) is rejected loudly
    bad = {'state': {}, 'param_groups': sd['param_groups']}
    for pos in range(n):
        i = flat.model_order[pos]
        j = flat.model_order[(pos + 1) % n]
        shape = flat.params[j].shape
        bad['state'][pos] = {'step': 1, 'exp_avg': torch.zeros(shape), 'exp_avg_sq': torch.zeros(shape)}
        if flat.params[i].shape.numel() != shape.numel():
            break
    try:
        opt.load_state_dict(bad)
    except ValueError as e:
        assert 'shape' in str(e)
    else:
        raise AssertionError('mis-shaped optimizer state must not load')


def _flat_ordered_state(opt):
    """What this framework wrote before the state-order tag: state numbered by FLAT index."""
    sd = opt.state_dict()
    state = {}
    for pos, i in enumerate(opt.flat.model_order):
        if pos in sd['state']:
            state[i] = sd['state'][pos]
    return {'state': state, 'param_groups': sd['param_groups']}


def test_state_order_tag_and_legacy_flat_files():
    """state_dict() carries param_order='model'; an untagged flat-order state of this framework
    (legacy_flat_order) is remapped onto the right tensors -- same-shaped Q/K/V weights and
    LayerNorm vectors included -- instead of silently permuting Adam moments."""
    model = _model()
    flat = FlatParamSpace(model, contiguous_groups=model.flat_contiguous_groups())
    opt = _Adam(_args(), flat)
    g = torch.Generator().manual_seed(3)
    opt.exp_avg.copy_(torch.randn(opt.exp_avg.shape, generator=g))
    opt.exp_avg_sq.copy_(torch.rand(opt.exp_avg_sq.shape, generator=g))
    opt.steps = [5] * len(flat.params)
    sd = opt.state_dict()
    assert sd['param_order'] == 'model'
    legacy = _flat_ordered_state(opt)

    def same(o):
        for i in range(len(flat.params)):
            s, e = flat.param_range(i)
            if not (torch.equal(o.exp_avg[s:e], opt.exp_avg[s:e]) and torch.equal(o.exp_avg_sq[s:e], opt.exp_avg_sq[s:e])):
                return False
        return True
    for state, kw in ((sd, {}), (legacy, {'legacy_flat_order': True})):
        opt2 = _Adam(_args(), flat)
        opt2.load_state_dict(state, **kw)
        assert same(opt2)
    # the untagged flat-order file read as model order scrambles same-shaped tensors
    opt3 = _Adam(_args(), flat)
    try:
        opt3.load_state_dict(legacy)
        assert not same(opt3)
    except ValueError:
        pass   # or a shape mismatch is caught


def _cpu_controller(tmp_path):
    from hetseq_9cme_amd import options, tasks
    from hetseq_9cme_amd.controller import Controller
    from hetseq_9cme_amd.data.synthetic import BERT_TINY, write_bert_config, write_synthetic_bert_shards, write_vocab
    d = tmp_path / 'data'
    if not d.exists():
        d.mkdir()
        write_synthetic_bert_shards(str(d), n_files=1, samples_per_file=16, seq_len=32, max_pred=5, vocab_size=1024,
                                    split='train', seed=1)
        write_bert_config(str(d / 'tiny.json'), **BERT_TINY)
        write_vocab(str(d / 'vocab.txt'), 1024)
    args = options.parse_training_args(
        ['--task', 'bert', '--data', str(d), '--dict', str(d / 'vocab.txt'), '--config_file', str(d / 'tiny.json'),
         '--max-sentences', '4', '--fast-stat-sync', '--num-workers', '1', '--lr', '1e-3', '--weight-decay', '0.01',
         '--save-dir', str(tmp_path / 'ck'), '--cpu'])
    args.device_id, args.distributed_rank = 0, 0
    torch.manual_seed(args.seed)
    task = tasks.setup_task(args)
    ctl = Controller(args, task, task.build_model(args))
    itr = ctl.get_train_iterator(epoch=0)
    return ctl, itr


def test_controller_resumes_untagged_model_order_state(tmp_path):
    """an untagged state written by this framework after --fp32-gemm existed is in
    model order and must come back bit for bit through Controller.load_checkpoint; an untagged
    state of the earliest builds (own flags, no fp32_gemm) is refused, never silently permuted."""
    import os
    from hetseq_9cme_amd import checkpoint_utils
    from hetseq_9cme_amd.data import iterators
    ctl, itr = _cpu_controller(tmp_path)
    batches = iterators.GroupedIterator(itr.next_epoch_itr(shuffle=False), 1)
    for _ in range(2):
        ctl.train_step(next(batches))
    os.makedirs(str(tmp_path / 'ck'), exist_ok=True)
    path = str(tmp_path / 'ck' / 'untagged.pt')
    ctl.save_checkpoint(path, {})
    st = checkpoint_utils.load_checkpoint_to_cpu(path)
    assert hasattr(st['args'], 'fp32_gemm')
    del st['last_optimizer_state']['param_order']        # what round-2 builds wrote
    torch.save(st, path)
    ctl2, _ = _cpu_controller(tmp_path)
    ctl2.load_checkpoint(path)
    o1, o2 = ctl.optimizer, ctl2.optimizer
    assert torch.equal(o1.exp_avg, o2.exp_avg) and torch.equal(o1.exp_avg_sq, o2.exp_avg_sq)
    # the earliest builds' files: refused with a pointer to --reset-optimizer
    delattr(st['args'], 'fp32_gemm')
    torch.save(st, path)
    ctl3, _ = _cpu_controller(tmp_path)
    try:
        ctl3.load_checkpoint(path)
    except RuntimeError as e:
        assert '--reset-optimizer' in str(e)
    else:
        raise AssertionError('an order-ambiguous optimizer state must not load')
    ctl3.load_checkpoint(path, reset_optimizer=True)      # the documented way out
