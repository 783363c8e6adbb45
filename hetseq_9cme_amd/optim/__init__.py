from .optimizers import _Optimizer, _Adam, _Adadelta, build_optimizer  # noqa: F401
from .lr_scheduler import PolynomialDecayScheduler, build_lr_scheduler  # noqa: F401
