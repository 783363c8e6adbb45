"""Task registry.  Unlike the reference (hetseq/tasks/__init__.py:2-3, SURVEY
App. A2) the fine-tuning tasks ARE exported, so every ``--task`` choice works."""
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


def setup_task(args):
    if args.task not in TASK_REGISTRY:
        raise ValueError('unsupported task: {}'.format(args.task))
    return TASK_REGISTRY[args.task].setup_task(args)
