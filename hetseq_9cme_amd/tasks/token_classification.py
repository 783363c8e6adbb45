"""BERT token-classification (NER, CoNLL-2003) fine-tuning task
(reference hetseq/tasks/bert_for_token_classification_task.py:16-228).

Setup: WordPiece tokenizer from ``--dict`` (``transformers.BertTokenizerFast``),
splits from ``--train_file/--validation_file/--test_file`` (CoNLL columns, JSON
or CSV; ``--extension_file`` names the format), label list from the data
(sorted, or the CoNLL-2003 order when the tags are CoNLL-2003's), first
word-piece labelled / others -100.  ``build_model`` loads ``--hetseq_state_dict``
(a hetseq checkpoint's ``['model']``) or ``--transformers_state_dict`` (keys
remapped: SURVEY App. A16) strictly or not.  ``train_step`` is
``model(**sample)`` with ``sample_size = len(labels)`` (= batch size).

Deliberate fix (App. A2): the task is registered, so ``--task
BertForTokenClassification`` works from the CLI.
"""
import argparse

import torch

from ..data.collators import DataCollatorForTokenClassification
from ..data.ner_dataset import BertNerDataset, get_label_list, load_split, tokenize_and_align
from .base import Task
from ..utils.misc import ensure_train

SPLIT_ALIASES = {'train': 'train', 'valid': 'validation', 'validation': 'validation', 'test': 'test'}


def safe_load_checkpoint(path):
    """torch.load that never executes code from the file: weights_only, with
    argparse.Namespace (stored by hetseq checkpoints under 'args') allow-listed."""
    with torch.serialization.safe_globals([argparse.Namespace]):
        return torch.load(path, map_location='cpu', weights_only=True)


def build_tokenizer(vocab_file):
    """Uncased WordPiece tokenizer over a BERT ``vocab.txt``.

    The vocabulary is passed positionally: transformers 5.x ignores the
    ``vocab_file=`` keyword of ``BertTokenizerFast`` and silently builds a
    5-token (special tokens only) vocabulary, which maps every word to [UNK].
    """
    from transformers import BertTokenizerFast
    tok = BertTokenizerFast(vocab_file, do_lower_case=True)
    with open(vocab_file, encoding='utf-8') as f:
        n = sum(1 for line in f if line.strip())
    if len(tok.vocab) < n:
        raise RuntimeError('tokenizer loaded {} of the {} entries of {}'.format(len(tok.vocab), n, vocab_file))
    return tok


class BertForTokenClassificationTask(Task):
    collator_cls = DataCollatorForTokenClassification
    entity_key = None

    @classmethod
    def setup_task(cls, args, **kwargs):
        tokenizer = build_tokenizer(args.dict)
        # --graph-train-step captures one graph per batch shape: pad lengths to a multiple of 16
        # so a handful of shapes cover the corpus (attention masks make padding exact)
        from .. import options
        mult = getattr(args, 'pad_to_multiple_of', None) or (16 if options.graph_train_step_enabled(args) else None)
        collator = cls.collator_cls(tokenizer, max_length=args.max_pred_length, padding=True,
                                    pad_to_multiple_of=mult)
        files = {'train': args.train_file, 'validation': args.validation_file, 'test': args.test_file}
        ext = args.extension_file if args.extension_file in ('json', 'jsonl', 'csv', 'conll') else None
        raw = {k: cls.read_split(v, ext) for k, v in files.items() if v is not None}
        if not raw:
            raise ValueError('dataset must contain "train"/"validation"/"test"')
        label_list = get_label_list(raw.values())
        label_to_id = {l: i for i, l in enumerate(label_list)}
        extra = cls.extra_setup(args, raw)
        tokenized = {k: tokenize_and_align(v, tokenizer, label_to_id, max_length=args.max_pred_length,
                                           entity_key=cls.entity_key, entity_to_id=extra.get('entity_to_id'))
                     for k, v in raw.items()}
        args.tokenized_datasets = tokenized
        args.num_labels = len(label_list)
        args.label_list = label_list
        args.tokenizer = tokenizer
        args.data_collator = collator
        task = cls(args)
        task.label_list = label_list
        return task

    @classmethod
    def read_split(cls, path, extension=None):
        return load_split(path, extension)

    @classmethod
    def extra_setup(cls, args, raw):
        return {}

    def _new_model(self, args, config):
        from ..models.bert import BertForTokenClassification
        return BertForTokenClassification(config, args.num_labels)

    def build_model(self, args):
        from ..models.bert import BertConfig, remap_state_dict_keys
        config = BertConfig.from_json_file(args.config_file)
        model = self._new_model(args, config)
        state_dict = None
        if getattr(args, 'hetseq_state_dict', None):
            state_dict = safe_load_checkpoint(args.hetseq_state_dict)['model']
        elif getattr(args, 'transformers_state_dict', None):
            state_dict = safe_load_checkpoint(args.transformers_state_dict)
            state_dict = remap_state_dict_keys(state_dict, set(model.state_dict().keys()))
        if state_dict is not None:
            strict = bool(args.load_state_dict_strict)
            res = model.load_state_dict(state_dict, strict=strict)
            if not strict:
                print('| loaded state dict (non-strict): {} missing, {} unexpected keys'.format(
                    len(res.missing_keys), len(res.unexpected_keys)))
        return model

    def load_dataset(self, split, **kwargs):
        if split in self.datasets:
            return
        name = SPLIT_ALIASES.get(split, split)
        tok = self.args.tokenized_datasets
        if name not in tok:
            # reference behaviour: fall back to whatever split exists
            name = 'train' if 'train' in tok else next(iter(tok))
        self.datasets[split] = BertNerDataset(tok[name], self.args)
        print('| loaded {} sentences for split {}'.format(len(tok[name]), split))
        print('| loading finished')

    def train_step(self, sample, model, optimizer, ignore_grad=False):
        ensure_train(model)
        loss = model(**sample)
        if ignore_grad:
            loss = loss * 0
        sample_size = 0 if sample is None or len(sample['labels']) == 0 else len(sample['labels'])
        logging_output = {'nsentences': sample_size, 'loss': loss.detach(), 'nll_loss': loss.detach(),
                          'ntokens': 0, 'sample_size': sample_size}
        optimizer.backward(loss)
        return loss, sample_size, logging_output
