"""Token-classification (NER) and entity-linking datasets.

Reference: hetseq/data/bert_ner_dataset.py, bert_el_dataset.py (wrappers over an
HF arrow dataset) and the tokenise-and-align step of
hetseq/tasks/bert_for_token_classification_task.py:81-113 /
bert_for_el_classification_task.py:112-183.

The reference builds its splits with a ``datasets`` loading script; modern
``datasets`` (5.x, installed here) no longer runs scripts, so CoNLL-format files
are parsed directly (``read_conll``); ``.json``/``.jsonl``/``.csv`` files go through
``datasets``.  Alignment: the first word-piece of every word gets the word's label,
other pieces and special tokens get -100.
"""
import json
import os

import numpy as np
import torch
import torch.utils.data

CONLL2003_NER = ['O', 'B-PER', 'I-PER', 'B-ORG', 'I-ORG', 'B-LOC', 'I-LOC', 'B-MISC', 'I-MISC']


def read_conll(path, token_col=0, label_col=-1, entity_col=None):
    """CoNLL column format: one token per line, blank line between sentences,
    ``-DOCSTART-`` lines skipped.  Returns a list of dicts with ``tokens`` and
    ``ner_tags`` (strings) and optionally ``entities``."""
    sents, toks, tags, ents = [], [], [], []

    def flush():
        if toks:
            d = {'tokens': list(toks), 'ner_tags': list(tags)}
            if entity_col is not None:
                d['entities'] = list(ents)
            sents.append(d)
        toks.clear(), tags.clear(), ents.clear()

    with open(path, 'r', encoding='utf-8') as f:
        for line in f:
            line = line.rstrip('\n')
            if not line.strip() or line.startswith('-DOCSTART-'):
                flush()
                continue
            cols = line.split('\t') if '\t' in line else line.split()
            toks.append(cols[token_col])
            tags.append(cols[label_col])
            if entity_col is not None:
                ents.append(cols[entity_col] if len(cols) > entity_col else '')
    flush()
    return sents


def load_split(path, extension=None):
    ext = (extension or os.path.splitext(path)[1].lstrip('.')).lower()
    if ext in ('json', 'jsonl'):
        with open(path, 'r', encoding='utf-8') as f:
            txt = f.read().strip()
        if txt.startswith('['):
            return json.loads(txt)
        return [json.loads(l) for l in txt.splitlines() if l.strip()]
    if ext == 'csv':
        import datasets
        return list(datasets.load_dataset('csv', data_files=path)['train'])
    return read_conll(path)


def get_label_list(splits, label_key='ner_tags'):
    labels = set()
    for s in splits:
        for ex in s:
            labels.update(ex[label_key])
    labels = sorted(labels)
    if set(labels) <= set(CONLL2003_NER) and len(labels) > 3:
        return list(CONLL2003_NER)
    return labels


def tokenize_and_align(examples, tokenizer, label_to_id, max_length=512, label_all_tokens=False,
                       entity_key=None, entity_to_id=None):
    texts = [ex['tokens'] for ex in examples]
    enc = tokenizer(texts, padding=False, truncation=True, max_length=max_length, is_split_into_words=True,
                    return_offsets_mapping=True)
    feats = []
    for i, ex in enumerate(examples):
        offsets = enc['offset_mapping'][i]
        label_ids, ent_ids = [], []
        widx = 0
        cur = -100
        cur_ent = -100
        tags = ex['ner_tags']
        for off in offsets:
            if off[0] == 0 and off[1] != 0:
                tag = tags[widx]
                cur = label_to_id[tag] if not isinstance(tag, int) else tag
                label_ids.append(cur)
                if entity_key is not None:
                    e = ex[entity_key][widx]
                    # only the first piece of a 'B' mention carries an entity id; unknown -> -1
                    if str(tag).startswith('B'):
                        cur_ent = entity_to_id.get(e, -1) if entity_to_id else -1
                    else:
                        cur_ent = -100
                    ent_ids.append(cur_ent)
                widx += 1
            elif off[0] == 0 and off[1] == 0:
                label_ids.append(-100)
                if entity_key is not None:
                    ent_ids.append(-100)
            else:
                label_ids.append(cur if label_all_tokens else -100)
                if entity_key is not None:
                    ent_ids.append(-100)
        f = {'input_ids': enc['input_ids'][i], 'token_type_ids': enc['token_type_ids'][i],
             'attention_mask': enc['attention_mask'][i], 'labels': label_ids}
        if entity_key is not None:
            f['entity_labels'] = ent_ids
        feats.append(f)
    return feats


class BertNerDataset(torch.utils.data.Dataset):
    """Dataset protocol over a list of tokenised feature dicts."""

    def __init__(self, dataset, args=None, collator=None):
        self.args = args
        self.dataset = dataset
        self.collator = collator if collator is not None else getattr(args, 'data_collator', None)

    def __getitem__(self, index):
        return self.dataset[index]

    def __len__(self):
        return len(self.dataset)

    def ordered_indices(self):
        return np.arange(len(self.dataset))

    def num_tokens(self, index):
        return len(self.dataset[index]['labels'])

    def num_tokens_vec(self, indices):
        return np.asarray([len(self.dataset[int(i)]['labels']) for i in indices], dtype=np.int64)

    def collater(self, samples):
        if len(samples) == 0:
            return None
        return self.collator(samples)

    def set_epoch(self, epoch):
        pass


class BertELDataset(BertNerDataset):
    pass
