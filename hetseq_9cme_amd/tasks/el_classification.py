"""BERT entity-linking fine-tuning task (reference
hetseq/tasks/bert_for_el_classification_task.py:1-304).

The reference depends on the external ``deep_ed_PyTorch`` package for its entity
name -> id dictionary (:13) and a frozen entity-embedding file.  Here the
dictionary is a plain TSV (``--ent_name_id_file``: ``name<TAB>id`` per line) and
the embedding matrix is read from ``--ent_vecs_filename`` (.pt tensor via
weights_only, .npy, or .safetensors 'ent_vecs').  Alignment: the first word-piece
of a 'B' mention carries the entity id, out-of-dictionary entities get -1,
everything else -100 (:112-183).  Data files are CoNLL columns whose last column
holds the entity name of 'B' tokens.
"""

import numpy as np
import torch

from ..data.collators import DataCollatorForELClassification
from ..data.ner_dataset import read_conll
from .token_classification import BertForTokenClassificationTask


def load_entity_vectors(path):
    if path is None:
        raise ValueError('--ent_vecs_filename is required for BertForELClassification')
    if path.endswith('.npy'):
        return torch.from_numpy(np.load(path, allow_pickle=False)).float()
    if path.endswith('.safetensors'):
        from safetensors.torch import load_file
        d = load_file(path)
        return (d.get('ent_vecs') or next(iter(d.values()))).float()
    obj = torch.load(path, map_location='cpu', weights_only=True)
    if isinstance(obj, dict):
        obj = obj.get('ent_vecs', next(iter(obj.values())))
    return obj.float()


def load_entity_dict(path):
    d = {}
    if path is None:
        return d
    with open(path, 'r', encoding='utf-8') as f:
        for line in f:
            parts = line.rstrip('\n').split('\t')
            if len(parts) >= 2:
                d[parts[0]] = int(parts[1])
    return d


class BertForELClassificationTask(BertForTokenClassificationTask):
    collator_cls = DataCollatorForELClassification
    entity_key = 'entities'

    @classmethod
    def extra_setup(cls, args, raw):
        vecs = load_entity_vectors(args.ent_vecs_filename)
        args.EntityEmbedding = vecs
        args.num_entity_labels = vecs.shape[0]
        args.dim_entity_emb = vecs.shape[1]
        ent_to_id = load_entity_dict(getattr(args, 'ent_name_id_file', None))
        return {'entity_to_id': ent_to_id}

    @classmethod
    def read_split(cls, path, extension=None):
        # EL files carry the entity name of 'B' tokens in the 5th column
        return read_conll(path, token_col=0, label_col=3, entity_col=4)

    def _new_model(self, args, config):
        from ..models.el import BertForELClassification
        return BertForELClassification(config, args)
