from .meters import AverageMeter, TimeMeter, StopwatchMeter  # noqa: F401
from .misc import apply_to_sample, move_to_device, move_to_cuda, item, get_perplexity  # noqa: F401
