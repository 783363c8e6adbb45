"""NER evaluation of a fine-tuned BertForTokenClassification checkpoint
(reference: test/test_eval_bert_fine_tuning.py:39-169 -- the reference's
hetseq/eval_bert_fine_tuning_ner.py is a broken stub).

Predicts on a CoNLL-format file, keeps the first word-piece of every word, and
reports token accuracy and entity-level (IOB2 chunk) precision / recall / F1,
computed here exactly like ``seqeval``'s default mode (``seqeval`` is not
installed; parity against it is unpinned).

``python -m hetseq_9cme_amd.eval_ner --model_ckpt CKPT --config_file C --dict VOCAB
--test_file test.txt [--train_file train.txt]`` (train file only for the label list).
"""
import argparse

import torch

from .checkpoint_utils import load_checkpoint_to_cpu
from .data.collators import DataCollatorForTokenClassification
from .data.ner_dataset import get_label_list, load_split, tokenize_and_align
from .models.bert import BertConfig, BertForTokenClassification
from .tasks.token_classification import build_tokenizer
from .utils.hip_graphs import GraphedForward


def get_entities(seq):
    """IOB2/IOB1 chunks as (type, start, end) -- seqeval's default semantics."""
    chunks = []
    prev_tag, prev_type, begin = 'O', '', 0
    for i, chunk in enumerate(list(seq) + ['O']):
        tag = chunk[0] if chunk != 'O' else 'O'
        typ = chunk.split('-', 1)[-1] if chunk != 'O' else ''
        end_chunk = (prev_tag in ('B', 'I') and (tag in ('B', 'O') or (tag == 'I' and typ != prev_type)))
        start_chunk = (tag == 'B' or (tag == 'I' and (prev_tag == 'O' or typ != prev_type)))
        if end_chunk:
            chunks.append((prev_type, begin, i - 1))
        if start_chunk:
            begin = i
        prev_tag, prev_type = tag, typ
    return chunks


def ner_scores(true_seqs, pred_seqs):
    tp = n_pred = n_true = 0
    correct = total = 0
    for t, p in zip(true_seqs, pred_seqs):
        te, pe = set(get_entities(t)), set(get_entities(p))
        tp += len(te & pe)
        n_pred += len(pe)
        n_true += len(te)
        correct += sum(a == b for a, b in zip(t, p))
        total += len(t)
    prec = tp / n_pred if n_pred else 0.0
    rec = tp / n_true if n_true else 0.0
    f1 = 2 * prec * rec / (prec + rec) if prec + rec > 0 else 0.0
    return {'accuracy': correct / max(total, 1), 'precision': prec, 'recall': rec, 'f1': f1}


def evaluate(model_ckpt, config_file, vocab, test_file, label_list=None, train_file=None, device=None,
             batch_size=32, max_length=512, graphs=True):
    device = torch.device(device or ('cuda' if torch.cuda.is_available() else 'cpu'))
    test = load_split(test_file)
    if label_list is None:
        label_list = get_label_list([test] + ([load_split(train_file)] if train_file else []))
    label_to_id = {l: i for i, l in enumerate(label_list)}
    tok = build_tokenizer(vocab)
    feats = tokenize_and_align(test, tok, label_to_id, max_length=max_length)
    model = BertForTokenClassification(BertConfig.from_json_file(config_file), len(label_list))
    model.load_state_dict(load_checkpoint_to_cpu(model_ckpt)['model'], strict=True)
    model.to(device).eval()
    coll = DataCollatorForTokenClassification(tok)
    # launch-bound loop (~100 short kernels per batch): replay one HIP graph per padded shape
    fwd = GraphedForward(model) if (graphs and device.type == 'cuda') else model
    trues, preds = [], []
    with torch.no_grad():
        for i in range(0, len(feats), batch_size):
            batch = coll(feats[i:i + batch_size])
            logits = fwd(batch['input_ids'].to(device), batch['token_type_ids'].to(device),
                         batch['attention_mask'].to(device))
            pred = logits.argmax(-1).cpu()
            for row_p, row_l in zip(pred, batch['labels']):
                keep = row_l != -100
                trues.append([label_list[x] for x in row_l[keep].tolist()])
                preds.append([label_list[x] for x in row_p[keep].tolist()])
    return ner_scores(trues, preds)


def main(argv=None):
    p = argparse.ArgumentParser(description='evaluate a fine-tuned NER checkpoint')
    p.add_argument('--model_ckpt', required=True)
    p.add_argument('--config_file', required=True)
    p.add_argument('--dict', required=True)
    p.add_argument('--test_file', required=True)
    p.add_argument('--train_file', default=None)
    p.add_argument('--cpu', action='store_true')
    p.add_argument('--no-graphs', action='store_true', help='eager forward (no HIP-graph replay)')
    a = p.parse_args(argv)
    res = evaluate(a.model_ckpt, a.config_file, a.dict, a.test_file, train_file=a.train_file,
                   device='cpu' if a.cpu else None, graphs=not a.no_graphs)
    print('accuracy={accuracy:.4f} precision={precision:.4f} recall={recall:.4f} f1={f1:.4f}'.format(**res))


if __name__ == '__main__':
    main()
