"""NER evaluation of a fine-tuned BertForTokenClassification checkpoint
(reference: test/test_eval_bert_fine_tuning.py:39-169 -- the reference's
hetseq/eval_bert_fine_tuning_ner.py is a broken stub).

Predicts on a CoNLL-format file, keeps the first word-piece of every word, and
reports token accuracy and entity-level (IOB2 chunk) precision / recall / F1,
computed by conlleval's chunk rules as ``seqeval``'s default mode does (IOB1 / IOB2 / IOE /
IOBES).  ``seqeval`` is not installed, so parity is pinned only against its documented README
example (``tests/test_finetune_cpu.py``), not against the library itself.

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


def _end_of_chunk(prev_tag, tag, prev_type, typ):
    """conlleval's chunk-end rule (IOB1 / IOB2 / IOE / IOBES tags), as seqeval's default mode."""
    if prev_tag in ('E', 'S'):
        return True
    if prev_tag in ('B', 'I') and tag in ('B', 'S', 'O'):
        return True
    return prev_tag not in ('O', '.') and prev_type != typ


def _start_of_chunk(prev_tag, tag, prev_type, typ):
    """conlleval's chunk-start rule."""
    if tag in ('B', 'S'):
        return True
    if tag in ('E', 'I') and prev_tag in ('E', 'S', 'O'):
        return True
    return tag not in ('O', '.') and prev_type != typ


def get_entities(seq):
    """Chunks of one tag sequence as (type, start, end) -- seqeval's default (conlleval)
    semantics, for IOB1 / IOB2 / IOE / IOBES tags."""
    chunks = []
    prev_tag, prev_type, begin = 'O', '', 0
    for i, chunk in enumerate(list(seq) + ['O']):
        tag = chunk[0] if chunk != 'O' else 'O'
        typ = chunk.split('-', 1)[-1] if chunk != 'O' else ''
        if _end_of_chunk(prev_tag, tag, prev_type, typ):
            chunks.append((prev_type, begin, i - 1))
        if _start_of_chunk(prev_tag, tag, prev_type, typ):
            begin = i
        prev_tag, prev_type = tag, typ
    return chunks


def ner_scores(true_seqs, pred_seqs, per_type=False):
    """Token accuracy and micro entity precision / recall / F1 (``per_type``: also a
    {type: {precision, recall, f1, support}} report, seqeval's classification_report numbers)."""
    tp = n_pred = n_true = 0
    correct = total = 0
    by = {}
    for t, p in zip(true_seqs, pred_seqs):
        te, pe = set(get_entities(t)), set(get_entities(p))
        tp += len(te & pe)
        n_pred += len(pe)
        n_true += len(te)
        correct += sum(a == b for a, b in zip(t, p))
        total += len(t)
        if per_type:
            for key, ents in (('t', te), ('p', pe), ('tp', te & pe)):
                for e in ents:
                    d = by.setdefault(e[0], {'t': 0, 'p': 0, 'tp': 0})
                    d[key] += 1

    def prf(tp_, np_, nt_):
        pr = tp_ / np_ if np_ else 0.0
        rc = tp_ / nt_ if nt_ else 0.0
        return pr, rc, (2 * pr * rc / (pr + rc) if pr + rc > 0 else 0.0)
    prec, rec, f1 = prf(tp, n_pred, n_true)
    out = {'accuracy': correct / max(total, 1), 'precision': prec, 'recall': rec, 'f1': f1}
    if per_type:
        out['per_type'] = {k: dict(zip(('precision', 'recall', 'f1'), prf(d['tp'], d['p'], d['t'])), support=d['t'])
                           for k, d in sorted(by.items())}
    return out


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
