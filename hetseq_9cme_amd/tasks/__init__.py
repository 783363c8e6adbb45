"""Task registry.  Unlike the reference (hetseq/tasks/__init__.py:2-3, SURVEY
App. A2) the fine-tuning tasks ARE exported, so every ``--task`` choice works,
and new tasks plug in without editing this package::

    from hetseq_9cme_amd.tasks import Task, register_task

    @register_task('my_task')
    class MyTask(Task):
        @staticmethod
        def add_args(parser):          # optional: task-specific flags
            parser.add_argument('--my-flag', type=int, default=0)
        ...

(the module defining the task must be imported before the command line is
parsed, e.g. via ``--user-module`` or by importing it in a launcher script).
"""
from .base import Task  # noqa: F401
from .language_modeling import LanguageModelingTask  # noqa: F401
from .mnist import MNISTTask  # noqa: F401
from .token_classification import BertForTokenClassificationTask  # noqa: F401
from .el_classification import BertForELClassificationTask  # noqa: F401

TASK_REGISTRY = {
    'bert': LanguageModelingTask,
    'mnist': MNISTTask,
    'BertForTokenClassification': BertForTokenClassificationTask,
    'BertForELClassification': BertForELClassificationTask,
}
BUILTIN_TASKS = tuple(TASK_REGISTRY)


def register_task(name):
    """Class decorator adding a ``Task`` subclass to ``--task`` choices."""
    def deco(cls):
        if name in TASK_REGISTRY and TASK_REGISTRY[name] is not cls:
            raise ValueError('task {} already registered'.format(name))
        if not issubclass(cls, Task):
            raise TypeError('task {} must subclass Task'.format(name))
        TASK_REGISTRY[name] = cls
        return cls
    return deco


def setup_task(args):
    if args.task not in TASK_REGISTRY:
        raise ValueError('unsupported task: {}'.format(args.task))
    return TASK_REGISTRY[args.task].setup_task(args)
