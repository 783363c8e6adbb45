"""Command-line flag system.

Flag names, defaults and the two-phase (task / optimizer / lr-scheduler
pre-parse, then conditional groups) structure follow the reference
(hetseq/options.py:5-382, train.py:204-212; full list in SURVEY App. B) so a
reference launch line works unchanged.  Additions are MI355X-specific knobs
(``--precision``, ``--fused-kernels``, ``--gemm-tuning``, ``--profile-phases``,
``--distributed-timeout``, ``--user-module``)
that default to the reference behaviour.

Deliberate fixes: ``--num-workers -1`` means "auto" (A7);
``--log-format json`` exists (A11).
"""
import argparse

import torch


def _visible_gpus():
    try:
        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return 0


def _registries():
    from .optim import LR_SCHEDULER_REGISTRY, OPTIMIZER_REGISTRY
    from .tasks import TASK_REGISTRY
    return TASK_REGISTRY, OPTIMIZER_REGISTRY, LR_SCHEDULER_REGISTRY


def get_task_preparser():
    tasks, optims, scheds = _registries()
    p = argparse.ArgumentParser(allow_abbrev=False, add_help=False)
    p.add_argument('--task', type=str, default='bert', choices=list(tasks))
    p.add_argument('--optimizer', type=str, default='adam', choices=list(optims))
    p.add_argument('--lr-scheduler', type=str, default='PolynomialDecayScheduler', choices=list(scheds))
    return p


def get_training_parser(task='bert', optimizer='adam', lr_scheduler='PolynomialDecayScheduler'):
    parser = argparse.ArgumentParser(allow_abbrev=False)
    parser.add_argument('--no-progress-bar', action='store_true', help='disable progress bar')
    parser.add_argument('--seed', default=19940802, type=int, metavar='N',
                        help='pseudo random number generator seed')
    parser.add_argument('--cpu', action='store_true', help='use CPU instead of the GPU')
    parser.add_argument('--log-interval', type=int, default=1, metavar='N',
                        help='log progress every N updates')
    parser.add_argument('--log-format', default='simple', choices=['none', 'simple', 'json', 'tqdm'],
                        help='log format to use')
    # --- MI355X-native execution knobs (not in the reference) ---
    parser.add_argument('--precision', default='fp32', choices=['fp32', 'bf16'],
                        help='compute precision: fp32 (the reference\'s precision: fp32 tensors end to end; '
                             'the GEMMs and attention products run as --fp32-gemm says -- by default fp16x3, '
                             'fp32 class on the fp16 matrix cores; --fp32-gemm native gives plain f32 MFMA, '
                             'bitwise the reference\'s fp32 FMA chain) or bf16 (bf16 MFMA, fp32 master weights '
                             'and optimizer state)')
    parser.add_argument('--fp32-gemm', default='fp16x3', choices=['fp16x3', 'native'],
                        help='how fp32 (--precision fp32) runs use the matrix cores: fp16x3 (default: every '
                             'linear-layer GEMM on the hand-written kernels with operands scaled by a power of two '
                             'from their max |x| and split into two fp16 pieces -- 22 bits each, three exact piece '
                             'products; measured GEMM error 0.6-0.7x native fp32\'s; the attention products as three '
                             'fp16 passes as well) or native (f32 MFMA, 157 TF/s peak, '
                             'through the libraries: the numerics oracle); see ops/fp32_mode.py')
    parser.add_argument('--graph-train-step', dest='graph_train_step', action='store_const', const='on',
                        default='auto',
                        help='one micro-batch per update: capture each input shape\'s whole update (forward, '
                             'backward, clip, optimizer; with an RCCL group the bucket all-reduces too) in a HIP '
                             'graph after two eager warm-up steps and replay it -- removes the host launch '
                             'overhead of small-batch fine-tuning (see utils/train_graph.py).  Default (auto): on '
                             'for GPU token-classification fine-tuning (BertForTokenClassification), off otherwise; '
                             'updates the graph cannot hold run eagerly either way')
    parser.add_argument('--no-graph-train-step', dest='graph_train_step', action='store_const', const='off')
    parser.add_argument('--pad-to-multiple-of', type=int, default=None, metavar='N',
                        help='token-classification batches: pad sequence length to a multiple of N '
                             '(default 16 when graph-captured updates are on, else the batch maximum)')
    parser.add_argument('--fused-kernels', default=True, type=eval_bool_arg,
                        help='use the hand-written HIP kernels on GPU (True) or plain torch ops')
    parser.add_argument('--user-module', default=None, metavar='PATH',
                        help='python file / package imported before parsing (registers custom '
                             'tasks, optimizers, LR schedulers)')
    parser.add_argument('--gemm-tuning', default='table', choices=['off', 'table', 'online', 'retune'],
                        help='library-GEMM solution selection: shipped per-shape table (default), '
                             'online benchmarking of unseen shapes, or library defaults')
    parser.add_argument('--gemm-tuning-file', default=None, metavar='PATH',
                        help='where --gemm-tuning online writes its table (device ordinal appended)')
    parser.add_argument('--overlap-wgrad', dest='overlap_wgrad', action='store_const', const='on', default='auto',
                        help='run every weight-gradient GEMM / bias column sum on a side HIP stream, '
                             'concurrent with the data-gradient chain (default, auto: the side stream for '
                             'products of >= 8192 token rows -- BERT-base phase 1 at 128 sequences per GPU, phase '
                             '2 -- the compute stream for smaller ones; measured, profiles/r6e_overlap_ab.txt)')
    parser.add_argument('--no-overlap-wgrad', dest='overlap_wgrad', action='store_const', const='off',
                        help='weight gradients on the compute stream always')
    parser.add_argument('--debug-kernels', action='store_true',
                        help='debug mode: serialised kernel launches (AMD_SERIALIZE_KERNEL=3, '
                             'HIP_LAUNCH_BLOCKING=1), range checks on token/type ids and labels and finite '
                             'checks on every fused kernel output (host syncs: slow)')
    parser.add_argument('--profile-phases', action='store_true',
                        help='log host wall time per step phase (prep/sample/fwd_bwd/stats/optimizer/'
                             'meters); a phase that waits on the GPU shows up as long')

    add_dataset_args(parser, train=True, task=task)
    add_distributed_training_args(parser)
    add_optimization_args(parser, optimizer=optimizer, lr_scheduler=lr_scheduler)
    add_checkpoint_args(parser)
    return parser


def add_dataset_args(parser, train=False, gen=False, task='bert'):
    group = parser.add_argument_group('Dataset and data loading')
    group.add_argument('--num-workers', default=-1, type=int, metavar='N',
                       help='data loading worker threads (-1 = auto)')
    group.add_argument('--max-tokens', type=int, metavar='N',
                       help='maximum number of tokens in a batch')
    group.add_argument('--max-sentences', '--batch-size', type=int, metavar='N',
                       help='maximum number of sentences in a batch')
    group.add_argument('--required-batch-size-multiple', default=1, type=int, metavar='N',
                       help='batch size will be a multiple of this value')
    if train:
        group.add_argument('--train-subset', default='train', metavar='SPLIT',
                           choices=['train', 'valid', 'test'])
        group.add_argument('--valid-subset', default='valid', metavar='SPLIT')
        group.add_argument('--validate-interval', type=int, default=1, metavar='N')
        group.add_argument('--disable-validation', action='store_true')
        group.add_argument('--max-tokens-valid', type=int, metavar='N')
        group.add_argument('--max-sentences-valid', type=int, metavar='N')
        group.add_argument('--curriculum', default=0, type=int, metavar='N',
                           help="don't shuffle batches for first N epochs")

        parser.add_argument('--task', type=str, default=task)
        parser.add_argument('--data', type=str, help='path including data')
        if task == 'bert':
            group.add_argument('--dict', type=str, metavar='PATH', help='PATH to dictionary')
            group.add_argument('--config_file', type=str, metavar='PATH',
                               help='PATH to bert model configuration', required=True)
            group.add_argument('--max_pred_length', type=int, default=512,
                               help='max number of tokens in a sentence')
            group.add_argument('--num_file', type=int, default=0,
                               help='number of file to run, 0 for all')
        elif task == 'mnist':
            pass
        elif task in ('BertForTokenClassification', 'BertForELClassification'):
            group.add_argument('--dict', type=str, metavar='PATH', help='PATH to dictionary')
            group.add_argument('--config_file', type=str, metavar='PATH',
                               help='PATH to bert model configuration', required=True)
            group.add_argument('--max_pred_length', type=int, default=512)
            group.add_argument('--hetseq_state_dict', type=str, default=None,
                               help='PATH to a hetseq checkpoint whose ["model"] is loaded')
            group.add_argument('--transformers_state_dict', type=str, default=None,
                               help='PATH to a transformers-format BERT state dict')
            group.add_argument('--train_file', type=str, default=None)
            group.add_argument('--validation_file', type=str, default=None)
            group.add_argument('--test_file', type=str, default=None)
            group.add_argument('--extension_file', type=str, default=None,
                               help='dataset format/extension (json/csv/conll) used to read NER files')
            group.add_argument('--load_state_dict_strict', type=eval, default="False",
                               help='whether strictly load state_dict')
            if task == 'BertForELClassification':
                parser.add_argument('--root_data_dir', type=str, default='./deep_ed_data/')
                parser.add_argument('--entities', type=str, default='RLTD',
                                    choices=['RLTD', '4EX', 'ALL'])
                parser.add_argument('--ent_vecs_filename', type=str, default=None,
                                    help='entity embedding matrix (.pt/.npy/.safetensors)')
                parser.add_argument('--ent_name_id_file', type=str, default=None,
                                    help='tab separated "entity_name<TAB>thid" dictionary '
                                         '(replaces deep_ed_PyTorch.EntNameID)')
        else:
            tasks = _registries()[0]
            if task not in tasks:
                raise ValueError('unsupported task: {}'.format(task))
            if hasattr(tasks[task], 'add_args'):
                tasks[task].add_args(group)


def add_distributed_training_args(parser):
    group = parser.add_argument_group('Distributed training')
    group.add_argument('--distributed-world-size', type=int, metavar='N',
                       default=max(1, _visible_gpus()),
                       help='total number of GPUs across all nodes (default: all visible GPUs)')
    group.add_argument('--distributed-rank', default=0, type=int,
                       help='rank of the first GPU of this node')
    group.add_argument('--distributed-gpus', default=4, type=int,
                       help='number of GPUs used on the current node')
    group.add_argument('--distributed-backend', default='nccl', type=str,
                       help='distributed backend (nccl == RCCL on ROCm; gloo for CPU)')
    group.add_argument('--distributed-init-method', default=None, type=str,
                       help='tcp://host:port or file:///shared/path rendezvous')
    group.add_argument('--device-id', '--local_rank', default=0, type=int,
                       help='which GPU to use (usually configured automatically)')
    group.add_argument('--distributed-no-spawn', action='store_true',
                       help='do not spawn multiple processes even if multiple GPUs are visible')
    group.add_argument('--device-offset', default=0, type=int,
                       help='MI355X: first local GPU of this launcher -- spawned rank i runs on GPU '
                            'device-offset + i, with every GPU of the host visible (several "node" '
                            'launchers sharing one host keep peer access / IPC for the xGMI transport)')
    group.add_argument('--distributed-timeout', default=1800, type=int,
                       help='collective / rendezvous timeout in seconds')
    group.add_argument('--ddp-backend', default='c10d', type=str, choices=['c10d'],
                       help='gradient reducer backend (kept for flag compatibility)')
    group.add_argument('--bucket-cap-mb', default=25, type=int, metavar='MB',
                       help='gradient all-reduce bucket size (upper bound; see --bucket-peer-mb)')
    group.add_argument('--bucket-peer-mb', default=3.0, type=float, metavar='MB',
                       help='MI355X: target bytes per peer chunk of a bucket -- buckets are sized '
                            'min(--bucket-cap-mb, max(2, W) x this), so every one of the W ranks\' '
                            'chunks keeps the 7 xGMI links busy while small worlds still overlap early '
                            '(0 = --bucket-cap-mb alone)')
    group.add_argument('--allreduce-impl', default='rccl', choices=['rccl', 'xgmi'],
                       help='gradient all-reduce transport: RCCL, or the hand-written intra-node two-shot '
                            'xGMI kernel over IPC-mapped peer buffers (single host only; falls back to RCCL)')
    group.add_argument('--rccl-normal-priority', action='store_true',
                       help='run RCCL collectives on normal-priority HIP streams (default: high priority, so '
                            'bucket all-reduces are scheduled ahead of queued backward kernels)')
    group.add_argument('--xgmi-blocks', default=64, type=int, metavar='N',
                       help='workgroups per xGMI all-reduce launch (CUs taken from backward while it runs)')
    group.add_argument('--comm-cus', default=0, type=_comm_cus_arg, metavar='N',
                       help='MI355X: CUs left to the gradient all-reduce while it overlaps the backward (world > 1): '
                            'from the first bucket collective to the end of backward the one-round GEMM / '
                            'weight-gradient plans are sized for the other CUs, RCCL is capped at N channels '
                            '(NCCL_MAX_NCHANNELS, one workgroup each) and the xGMI kernel runs on N CUs -- see '
                            'csrc/kernels/cu_reserve.hip and profiles/r3_comm_contention.md (a 16-CU comm load: '
                            '+15 %% step time unplanned, +6 %% with the plans sized around it).  0 (default) = off '
                            'until a multi-GPU measurement justifies a reservation; auto = 16 on GPU runs with '
                            'world > 1, else off')
    group.add_argument('--force-reducer', action='store_true',
                       help='MI355X: run the bucketed gradient reducer even in a one-rank process group, so a '
                            'one-GPU run exercises the RCCL stream path (buckets, side-stream ordering, '
                            'end-of-backward waits); the one-rank sum leaves gradients unchanged')
    group.add_argument('--fix-batches-to-gpus', action='store_true')
    group.add_argument('--find-unused-parameters', default=False, action='store_true')
    group.add_argument('--fast-stat-sync', default=False, action='store_true')
    group.add_argument('--check-params-every', default=0, type=int,
                       help='debug / race check, NOT a fast path: every N updates a host-synchronising '
                            'parameter checksum (.item()) is all-gathered (pickled) and compared across ranks')
    return group


def add_optimization_args(parser, optimizer='adam', lr_scheduler='PolynomialDecayScheduler'):
    group = parser.add_argument_group('Optimization')
    group.add_argument('--max-epoch', '--me', default=0, type=int, metavar='N')
    group.add_argument('--max-update', '--mu', default=0, type=int, metavar='N')
    group.add_argument('--clip-norm', default=25, type=float, metavar='NORM')
    group.add_argument('--update-freq', default='1', metavar='N1,N2,...,N_K',
                       type=lambda uf: eval_str_list(uf, type=int))
    group.add_argument('--lr', '--learning-rate', default='0.25', type=eval_str_list,
                       metavar='LR_1,LR_2,...,LR_N')
    group.add_argument('--min-lr', default=-1, type=float, metavar='LR')
    group.add_argument('--use-bmuf', default=False, action='store_true')
    if optimizer == 'adam':
        group.add_argument('--optimizer', default='adam', type=str)
        group.add_argument('--adam-betas', default='(0.9, 0.999)', metavar='B')
        group.add_argument('--adam-eps', type=float, default=1e-8, metavar='D')
        group.add_argument('--weight-decay', '--wd', default=0.0, type=float, metavar='WD')
    elif optimizer == 'adadelta':
        group.add_argument('--optimizer', default='adadelta', type=str)
        group.add_argument('--adadelta_rho', default='0.9', type=float)
        group.add_argument('--adadelta_eps', default='1e-6', type=float)
        group.add_argument('--dadelta_weight_decay', default='0', type=float)
    else:
        optims = _registries()[1]
        if optimizer not in optims:
            raise ValueError('unsupported optimizer: {}'.format(optimizer))
        group.add_argument('--optimizer', default=optimizer, type=str)
        if hasattr(optims[optimizer], 'add_args'):
            optims[optimizer].add_args(group)
    if lr_scheduler == 'PolynomialDecayScheduler':
        group.add_argument('--lr_scheduler', default='PolynomialDecayScheduler', type=str)
        group.add_argument('--force-anneal', '--fa', type=int, metavar='N')
        group.add_argument('--warmup-updates', default=0, type=int, metavar='N')
        group.add_argument('--end-learning-rate', default=0.0, type=float)
        group.add_argument('--power', default=1.0, type=float)
        group.add_argument('--total-num-update', default=1000000, type=int)
    else:
        scheds = _registries()[2]
        if lr_scheduler not in scheds:
            raise ValueError('unsupported lr_scheduler: {}'.format(lr_scheduler))
        group.add_argument('--lr_scheduler', default=lr_scheduler, type=str)
        if hasattr(scheds[lr_scheduler], 'add_args'):
            scheds[lr_scheduler].add_args(group)
    return group


def add_checkpoint_args(parser):
    group = parser.add_argument_group('Checkpointing')
    group.add_argument('--save-dir', metavar='DIR', default='checkpoints')
    group.add_argument('--restore-file', default='checkpoint_last.pt')
    group.add_argument('--reset-dataloader', action='store_true')
    group.add_argument('--reset-lr-scheduler', action='store_true')
    group.add_argument('--reset-meters', action='store_true')
    group.add_argument('--reset-optimizer', action='store_true')
    group.add_argument('--optimizer-overrides', default="{}", type=str, metavar='DICT')
    group.add_argument('--save-interval', type=int, default=1, metavar='N')
    group.add_argument('--save-interval-updates', type=int, default=0, metavar='N')
    group.add_argument('--keep-interval-updates', type=int, default=-1, metavar='N')
    group.add_argument('--keep-last-epochs', type=int, default=-1, metavar='N')
    group.add_argument('--no-save', action='store_true')
    group.add_argument('--no-epoch-checkpoints', action='store_true')
    group.add_argument('--no-last-checkpoints', action='store_true')
    group.add_argument('--no-save-optimizer-state', action='store_true')
    group.add_argument('--best-checkpoint-metric', type=str, default='loss')
    group.add_argument('--maximize-best-checkpoint-metric', action='store_true')
    group.add_argument('--async-save', action='store_true',
                       help='write checkpoints from a background thread (state snapshotted first)')
    return group


def eval_str_list(x, type=float):
    if x is None:
        return None
    if isinstance(x, str):
        x = eval(x)
    try:
        return list(map(type, x))
    except TypeError:
        return [type(x)]


def eval_bool(x, default=False):
    if x is None:
        return default
    try:
        return bool(eval(x))
    except TypeError:
        return default


def eval_bool_arg(x):
    if isinstance(x, bool):
        return x
    return str(x).lower() in ('1', 'true', 'yes', 'on')


AUTO_COMM_CUS = 16


def _comm_cus_arg(v):
    return 'auto' if str(v) == 'auto' else int(v)


def comm_cus(args):
    """--comm-cus resolved: 'auto' = AUTO_COMM_CUS on GPU runs with world > 1 (channel cap of the
    RCCL communicator + the plans' reservation), else 0."""
    v = getattr(args, 'comm_cus', 0)
    if v == 'auto':
        gpu = not getattr(args, 'cpu', False) and getattr(args, 'distributed_backend', 'nccl') == 'nccl'
        return AUTO_COMM_CUS if gpu and getattr(args, 'distributed_world_size', 1) > 1 else 0
    return max(0, int(v))


def parse_args_and_arch(parser, s=None):
    args = parser.parse_args(s)
    if hasattr(args, 'max_sentences_valid') and args.max_sentences_valid is None:
        args.max_sentences_valid = args.max_sentences
    if hasattr(args, 'max_tokens_valid') and args.max_tokens_valid is None:
        args.max_tokens_valid = args.max_tokens
    return args


def import_user_module(path):
    """Import a user file / package that registers tasks, optimizers or LR
    schedulers (``--user-module``) before the real parse."""
    import importlib
    import importlib.util
    import os
    import sys
    if path is None:
        return None
    if os.path.exists(path):
        path = os.path.abspath(path)
        name = os.path.splitext(os.path.basename(path.rstrip('/')))[0]
        if os.path.isdir(path):
            sys.path.insert(0, os.path.dirname(path))
            return importlib.import_module(name)
        spec = importlib.util.spec_from_file_location(name, path)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod
        spec.loader.exec_module(mod)
        return mod
    return importlib.import_module(path)


def parse_training_args(argv=None):
    """Two-phase parse: pre-parse task/optimizer/scheduler, then the full parser
    (reference train.py:204-213).  ``--user-module`` is imported first so that
    the registries it extends are visible to the choices."""
    um = argparse.ArgumentParser(add_help=False)
    um.add_argument('--user-module', default=None)
    um_args, _ = um.parse_known_args(argv)
    import_user_module(um_args.user_module)
    pre, rest = get_task_preparser().parse_known_args(argv)
    parser = get_training_parser(task=pre.task, optimizer=pre.optimizer,
                                 lr_scheduler=pre.lr_scheduler)
    # the task/optimizer groups re-declare --task/--optimizer with the pre-parsed
    # values as defaults, exactly like the reference
    args = parse_args_and_arch(parser, rest)
    args.lr_scheduler = pre.lr_scheduler
    return args


# tasks whose GPU updates default to HIP-graph replay (--graph-train-step auto): small-batch
# fine-tuning, host-bound when eager (docs/performance.md, NER)
GRAPH_STEP_TASKS = ('BertForTokenClassification',)


def graph_train_step_enabled(args):
    """--graph-train-step on / off / auto (auto: on for GPU runs of GRAPH_STEP_TASKS)."""
    v = getattr(args, 'graph_train_step', 'auto')
    if v in (True, 'on'):
        return True
    if v in (False, None, 'off'):
        return False
    return getattr(args, 'task', None) in GRAPH_STEP_TASKS and not getattr(args, 'cpu', False)
