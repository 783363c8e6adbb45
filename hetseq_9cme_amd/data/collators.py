"""Padding collators for token-level fine-tuning (reference
hetseq/data_collator/data_collator.py:9-310).

Pads every field to the batch's longest example (right padding by default, left
when the tokenizer pads left) with the reference pad values: input_ids 0,
labels -100, token_type_ids 0, attention_mask 0, entity_labels -100.  Returns a
dict of int64 tensors.  No tokenizer object is needed beyond its padding side.
"""
import numpy as np
import torch

PADS = {'input_ids': 0, 'labels': -100, 'token_type_ids': 0, 'attention_mask': 0, 'entity_labels': -100}


def _as_list(x):
    if torch.is_tensor(x):
        return x.tolist()
    if isinstance(x, np.ndarray):
        return x.tolist()
    return list(x)


class DataCollatorForTokenClassification(object):
    fields = ('input_ids', 'labels', 'token_type_ids', 'attention_mask')

    def __init__(self, tokenizer=None, padding=True, max_length=None, pad_to_multiple_of=None,
                 label_pad_token_id=-100, padding_side=None):
        self.tokenizer = tokenizer
        self.padding = padding
        self.max_length = max_length
        self.pad_to_multiple_of = pad_to_multiple_of
        self.label_pad_token_id = label_pad_token_id
        side = padding_side or getattr(tokenizer, 'padding_side', 'right')
        self.padding_side = side

    def __call__(self, features):
        label_name = 'label' if 'label' in features[0] else 'labels'
        max_len = max(len(f[label_name]) for f in features)
        if self.pad_to_multiple_of:
            m = self.pad_to_multiple_of
            max_len = (max_len + m - 1) // m * m
        batch = {}
        for k in self.fields:
            if k not in features[0]:
                continue
            pad = PADS.get(k, 0) if k != 'labels' else self.label_pad_token_id
            rows = []
            for f in features:
                v = _as_list(f[k])
                padding = [pad] * (max_len - len(v))
                rows.append(v + padding if self.padding_side == 'right' else padding + v)
            batch[k] = torch.from_numpy(np.asarray(rows, dtype=np.int64))
        return batch


class DataCollatorForELClassification(DataCollatorForTokenClassification):
    fields = ('input_ids', 'labels', 'token_type_ids', 'attention_mask', 'entity_labels')


# reference class names
YD_DataCollatorForTokenClassification = DataCollatorForTokenClassification
YD_DataCollatorForELClassification = DataCollatorForELClassification
