"""MNIST task (reference hetseq/tasks/tasks.py:269-316)."""
import os

from ..data import MNISTDataset
from ..models.mnist import MNISTNet
from .base import Task


class MNISTTask(Task):
    @classmethod
    def setup_task(cls, args, **kwargs):
        return cls(args)

    def build_model(self, args):
        return MNISTNet()

    def load_dataset(self, split, **kwargs):
        path = self.args.data
        if path is None or not os.path.exists(path):
            raise FileNotFoundError('Dataset not found: ({}) -- offline environment: create it with '
                                    'hetseq_9cme_amd.data.synthetic.write_synthetic_mnist'.format(path))
        dataset = MNISTDataset.from_path(path, split)
        print('| loaded {} sentences from: {}'.format(len(dataset), path), flush=True)
        self.datasets[split] = dataset
        print('| loading finished')
