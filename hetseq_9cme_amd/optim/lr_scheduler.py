"""Learning-rate schedulers (reference: hetseq/lr_scheduler.py:6-104).

``PolynomialDecayScheduler``: linear warmup ``lr * n / warmup`` for
``n <= warmup``; afterwards ``(lr - end) * (1 - (n - w)/(T - w))**power + end``;
``end_learning_rate`` from ``total_num_update`` on.  Per-epoch ``step`` picks
``lr[min(epoch, len-1)]`` unless ``--force-anneal`` kicked in.  State dict is
``{'best': ...}`` (checkpoint compatible).

The LR is a host scalar; the fused optimizer receives it (already folded into
the bias-corrected step size) as a kernel argument each update.
"""


class _LRScheduler(object):
    def __init__(self, args, optimizer):
        self.args = args
        self.optimizer = optimizer
        self.best = None

    def state_dict(self):
        return {'best': self.best}

    def load_state_dict(self, state_dict):
        self.best = state_dict['best']

    def step(self, epoch, val_loss=None):
        if val_loss is not None:
            self.best = val_loss if self.best is None else min(self.best, val_loss)

    def step_update(self, num_updates):
        return self.optimizer.get_lr()


class PolynomialDecayScheduler(_LRScheduler):
    def __init__(self, args, optimizer):
        super().__init__(args, optimizer)
        args.warmup_updates = getattr(args, 'warmup_updates', 0) or 0
        self.lr = args.lr[0]
        self.warmup_factor = 1. / args.warmup_updates if args.warmup_updates > 0 else 1
        self.end_learning_rate = args.end_learning_rate
        self.total_num_update = args.total_num_update
        self.power = args.power
        self.optimizer.set_lr(self.warmup_factor * self.lr)

    def get_next_lr(self, epoch):
        lrs = self.args.lr
        if getattr(self.args, 'force_anneal', None) is None or epoch < self.args.force_anneal:
            return lrs[min(epoch, len(lrs) - 1)]
        return self.optimizer.get_lr()

    def step(self, epoch, val_loss=None):
        super().step(epoch, val_loss)
        self.lr = self.get_next_lr(epoch)
        self.optimizer.set_lr(self.warmup_factor * self.lr)
        return self.optimizer.get_lr()

    def lr_at(self, num_updates):
        w = self.args.warmup_updates
        if w > 0 and num_updates <= w:
            self.warmup_factor = num_updates / float(w)
            return self.warmup_factor * self.lr
        if num_updates >= self.total_num_update:
            return self.end_learning_rate
        lr_range = self.lr - self.end_learning_rate
        pct_remaining = 1 - (num_updates - w) / (self.total_num_update - w)
        return lr_range * pct_remaining ** self.power + self.end_learning_rate

    def step_update(self, num_updates):
        self.optimizer.set_lr(self.lr_at(num_updates))
        return self.optimizer.get_lr()


LR_SCHEDULER_REGISTRY = {'PolynomialDecayScheduler': PolynomialDecayScheduler}


def register_lr_scheduler(name):
    """Class decorator adding an ``_LRScheduler`` subclass to ``--lr-scheduler``
    choices.  Optional ``add_args(group)`` static method declares its flags."""
    def deco(cls):
        if name in LR_SCHEDULER_REGISTRY and LR_SCHEDULER_REGISTRY[name] is not cls:
            raise ValueError('lr scheduler {} already registered'.format(name))
        LR_SCHEDULER_REGISTRY[name] = cls
        return cls
    return deco


def build_lr_scheduler(args, optimizer):
    name = getattr(args, 'lr_scheduler', 'PolynomialDecayScheduler')
    if name not in LR_SCHEDULER_REGISTRY:
        raise ValueError('unsupported lr_scheduler - {}'.format(name))
    return LR_SCHEDULER_REGISTRY[name](args, optimizer)
