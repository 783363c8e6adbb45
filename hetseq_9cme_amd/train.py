"""Training entry point: ``python -m hetseq_9cme_amd.train --task bert ...``.

Launch modes (reference hetseq/train.py:196-246):
  (a) ``--distributed-init-method tcp://HOST:PORT | file:///shared/file`` with
      ``--distributed-gpus g > 1``: this *node* spawns g processes, process i
      gets ``device_id = i`` and global rank ``--distributed-rank + i``.  Nodes
      may have different GPU counts (the heterogeneous-cluster feature: e.g. a
      5-GPU node with ``--distributed-rank 0`` and a 3-GPU node with
      ``--distributed-rank 5`` form one world of 8).
  (b) init method with one GPU or ``--distributed-no-spawn``: run one process.
  (c) no init method, ``--distributed-world-size > 1``: single node, a free
      localhost port, spawn world-size processes.
  (d) otherwise single process.
  (e) launched by torchrun (RANK / WORLD_SIZE / LOCAL_RANK in the environment):
      one process per GPU, ``env://`` rendezvous.
"""
import collections
import math
import os

import numpy as np
import torch

from . import checkpoint_utils, options, tasks
from .controller import Controller
from .data import iterators
from .parallel import distributed as dist_utils
from .utils import progress_bar
from .utils.meters import AverageMeter, StopwatchMeter
from .utils.misc import get_perplexity


def main(args, init_distributed=False):
    assert args.max_tokens is not None or args.max_sentences is not None, \
        'Must specify batch size either with --max-tokens or --max-sentences'
    if torch.cuda.is_available() and not args.cpu:
        # more ranks than local GPUs is allowed for rehearsals with the gloo backend
        torch.cuda.set_device(args.device_id % torch.cuda.device_count())
    np.random.seed(args.seed)
    torch.manual_seed(args.seed)
    if init_distributed:
        args.distributed_rank = dist_utils.distributed_init(args)
    if dist_utils.is_master(args):
        checkpoint_utils.verify_checkpoint_directory(args.save_dir)
    print(args, flush=True)

    task = tasks.setup_task(args)
    if not args.disable_validation:
        for valid_sub_split in args.valid_subset.split(','):
            task.load_dataset(valid_sub_split, combine=False, epoch=0)
    model = task.build_model(args)
    print('| num. model params: {} (num. trained: {})'.format(
        sum(p.numel() for p in model.parameters()),
        sum(p.numel() for p in model.parameters() if p.requires_grad)))

    controller = Controller(args, task, model)
    print('| training on {} GPUs'.format(args.distributed_world_size))
    print('| max tokens per GPU = {} and max sentences per GPU = {}'.format(args.max_tokens, args.max_sentences))

    extra_state, epoch_itr = checkpoint_utils.load_checkpoint(args, controller)

    max_epoch = args.max_epoch or math.inf
    max_update = args.max_update or math.inf
    lr = controller.get_lr()
    train_meter = StopwatchMeter()
    train_meter.start()
    while (lr > args.min_lr
           and (epoch_itr.epoch < max_epoch or (epoch_itr.epoch == max_epoch and epoch_itr._next_epoch_itr is not None))
           and controller.get_num_updates() < max_update):
        train(args, controller, task, epoch_itr)
        valid_losses = [None]   # reference: validation is never run (App. A13)
        lr = controller.lr_step(epoch_itr.epoch, valid_losses[0])
        if epoch_itr.epoch % args.save_interval == 0:
            checkpoint_utils.save_checkpoint(args, controller, epoch_itr, valid_losses[0])
        reload_dataset = getattr(args, 'data', None) is not None and ':' in getattr(args, 'data', '')
        epoch_itr = controller.get_train_iterator(epoch_itr.epoch, load_dataset=reload_dataset)
    train_meter.stop()
    controller.check_transport_all()   # the last updates' xGMI words (lagged check), on every rank
    controller.wait_for_save()
    print('| done training in {:.1f} seconds'.format(train_meter.sum))
    return controller


def train(args, controller, task, epoch_itr):
    """Train for one epoch."""
    update_freq = args.update_freq[epoch_itr.epoch - 1] \
        if epoch_itr.epoch <= len(args.update_freq) else args.update_freq[-1]
    itr = epoch_itr.next_epoch_itr(fix_batches_to_gpus=args.fix_batches_to_gpus,
                                   shuffle=(epoch_itr.epoch >= args.curriculum))
    itr = iterators.GroupedIterator(itr, update_freq)
    progress = progress_bar.build_progress_bar(args, itr, epoch_itr.epoch, no_progress_bar='simple')
    extra_meters = collections.defaultdict(lambda: AverageMeter())
    max_update = args.max_update or math.inf
    fail_at = int(os.environ.get('HETSEQ_FAIL_AT_UPDATE', '0'))
    for i, samples in enumerate(progress, start=epoch_itr.iterations_in_epoch):
        log_output = controller.train_step(samples)
        if log_output is None:
            continue
        stats = get_training_stats(controller)
        for k, v in log_output.items():
            if k in ['loss', 'nll_loss', 'ntokens', 'nsentences', 'sample_size', 'ooms']:
                continue
            if 'loss' in k or k == 'accuracy':
                extra_meters[k].update(v, log_output['sample_size'])
            else:
                extra_meters[k].update(v)
            stats[k] = extra_meters[k].avg
        progress.log(stats, tag='train', step=stats['num_updates'])
        if i == 0:
            controller.get_meter('wps').reset()
            controller.get_meter('ups').reset()
        num_updates = controller.get_num_updates()
        if args.check_params_every > 0 and num_updates % args.check_params_every == 0 \
                and args.distributed_world_size > 1:
            sums = dist_utils.all_gather_list(controller.param_checksum())
            assert all(abs(s - sums[0]) <= 1e-6 * max(1.0, abs(sums[0])) for s in sums), \
                'parameter replicas diverged across ranks: {}'.format(sums)
            controller.check_transport_all()
        if (args.save_interval_updates > 0 and num_updates % args.save_interval_updates == 0
                and not epoch_itr.end_of_epoch()):
            checkpoint_utils.save_checkpoint(args, controller, epoch_itr, None)
        if fail_at and num_updates == fail_at:
            raise SystemExit('HETSEQ_FAIL_AT_UPDATE={} reached (fault injection)'.format(fail_at))
        if num_updates >= max_update:
            break


def get_training_stats(controller):
    stats = collections.OrderedDict()
    stats['loss'] = controller.get_meter('train_loss')
    if controller.get_meter('train_nll_loss').count > 0:
        nll_loss = controller.get_meter('train_nll_loss')
        stats['nll_loss'] = nll_loss
    else:
        nll_loss = controller.get_meter('train_loss')
    stats['ppl'] = _LazyPPL(nll_loss)
    stats['wps'] = controller.get_meter('wps')
    stats['ups'] = controller.get_meter('ups')
    stats['wpb'] = controller.get_meter('wpb')
    stats['bsz'] = controller.get_meter('bsz')
    stats['num_updates'] = controller.get_num_updates()
    stats['lr'] = controller.get_lr()
    stats['gnorm'] = controller.get_meter('gnorm')
    stats['clip'] = controller.get_meter('clip')
    stats['oom'] = controller.get_meter('oom')
    if controller.get_meter('loss_scale') is not None:
        stats['loss_scale'] = controller.get_meter('loss_scale')
    stats['wall'] = round(controller.get_meter('wall').elapsed_time)
    stats['train_wall'] = controller.get_meter('train_wall')
    if getattr(controller, '_profile_phases', False) and controller.phases.steps > 0:
        # per-update ms in each phase of the step since the last log line:
        # t_* host wall time, d_* device (HIP event) time
        rep = controller.phase_report(reset=True)
        for k, v in rep['host'].items():
            stats['t_' + k] = round(v * 1e3 / rep['steps'], 2)
        for k, v in rep['device'].items():
            stats['d_' + k] = round(v * 1e3 / rep['steps'], 2)
    return stats


class _LazyPPL(object):
    """2**avg_loss, evaluated only when the log line is formatted."""

    def __init__(self, meter):
        self.meter = meter

    def __str__(self):
        return '{:g}'.format(get_perplexity(self.meter.avg))

    def strip(self):
        return str(self)


def distributed_main(i, args, start_rank=0):
    args.device_id = i + getattr(args, 'device_offset', 0)
    if args.distributed_rank is None:
        args.distributed_rank = start_rank + i
    main(args, init_distributed=True)
    _teardown()


def _teardown():
    """An orderly process-group teardown: a group left to the interpreter's exit can abort a rank
    ("terminate called without an active exception") while its gloo / RCCL threads still run."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def _from_torchrun(args):
    env = os.environ
    if 'RANK' in env and 'WORLD_SIZE' in env and int(env['WORLD_SIZE']) > 1 and args.distributed_init_method is None:
        args.distributed_init_method = 'env://'
        args.distributed_world_size = int(env['WORLD_SIZE'])
        args.distributed_rank = int(env['RANK'])
        args.device_id = int(env.get('LOCAL_RANK', 0))
        return True
    return False


def cli_main(argv=None):
    args = options.parse_training_args(argv)
    if getattr(args, 'debug_kernels', False):
        # must be in the environment before the HIP runtime initialises (also
        # inherited by spawned ranks)
        os.environ['AMD_SERIALIZE_KERNEL'] = '3'
        os.environ['HIP_LAUNCH_BLOCKING'] = '1'
    if _from_torchrun(args):
        main(args, init_distributed=True)
        _teardown()
    elif args.distributed_init_method is not None:
        if not args.cpu and args.distributed_backend == 'nccl':
            assert args.distributed_gpus <= max(1, torch.cuda.device_count())
        if args.distributed_gpus > 1 and not args.distributed_no_spawn:
            start_rank = args.distributed_rank
            args.distributed_rank = None
            torch.multiprocessing.spawn(fn=distributed_main, args=(args, start_rank), nprocs=args.distributed_gpus)
        else:
            distributed_main(args.device_id, args)
    elif args.distributed_world_size > 1:
        if not args.cpu and args.distributed_backend == 'nccl':
            assert args.distributed_world_size <= torch.cuda.device_count()
        # a port the OS reports free (the reference draws random.randint(10000, 20000), which
        # collides now and then when several jobs share a host)
        import socket
        with socket.socket() as sk:
            sk.bind(('127.0.0.1', 0))
            port = sk.getsockname()[1]
        args.distributed_init_method = 'tcp://127.0.0.1:{port}'.format(port=port)
        args.distributed_rank = None
        torch.multiprocessing.spawn(fn=distributed_main, args=(args,), nprocs=args.distributed_world_size)
    else:
        main(args)


if __name__ == '__main__':
    cli_main()
