"""BERT pre-training task (MLM + NSP) over HDF5 shards (reference
hetseq/tasks/tasks.py:195-267)."""
import os

from ..data import BertH5pyData, ConBertH5pyData
from .base import Task


class LanguageModelingTask(Task):
    def __init__(self, args, dictionary):
        super().__init__(args)
        self.dictionary = dictionary
        self.max_pred = None

    @classmethod
    def setup_task(cls, args, **kwargs):
        dictionary = cls.load_dictionary(getattr(args, 'dict', None))
        return cls(args, dictionary)

    def build_model(self, args):
        if args.task != 'bert':
            raise ValueError('Unsupported language modeling task: {}'.format(args.task))
        from ..models.bert import BertConfig, BertForPreTraining
        config = BertConfig.from_json_file(args.config_file)
        model = BertForPreTraining(config)
        self.configure_model(model)
        return model

    def configure_model(self, model):
        if self.max_pred and hasattr(model, 'max_predictions_per_seq'):
            model.max_predictions_per_seq = self.max_pred

    def load_dataset(self, split, **kwargs):
        path = self.args.data
        if path is None or not os.path.exists(path):
            raise FileNotFoundError('Dataset not found: ({})'.format(path))
        files = [os.path.join(path, f) for f in os.listdir(path)] if os.path.isdir(path) else [path]
        files = sorted([f for f in files if split in os.path.basename(f)])
        if getattr(self.args, 'num_file', 0) > 0:
            files = files[0:self.args.num_file]
        assert len(files) > 0, 'no suitable file in split ***{}***'.format(split)
        datasets = [BertH5pyData(f) for f in files]
        dataset = ConBertH5pyData(datasets)
        self.max_pred = max(self.max_pred or 0, dataset.max_pred)
        print('| loaded {} sentences from: {}'.format(len(dataset), path), flush=True)
        self.datasets[split] = dataset
        print('| loading finished')
