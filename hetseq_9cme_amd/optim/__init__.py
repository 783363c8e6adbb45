from .optimizers import (_Optimizer, _Adam, _Adadelta, build_optimizer, OPTIMIZER_REGISTRY,  # noqa: F401
                         register_optimizer)
from .lr_scheduler import (_LRScheduler, PolynomialDecayScheduler, build_lr_scheduler,  # noqa: F401
                           LR_SCHEDULER_REGISTRY, register_lr_scheduler)
