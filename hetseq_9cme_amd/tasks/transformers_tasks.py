"""Alternative tasks backed by HuggingFace ``transformers`` model classes
(reference hetseq/transformers_tasks.py:1-568, which is not imported anywhere in
the reference either).  ``TransformersBertForTokenClassificationTask`` trains the
stock ``transformers.BertForTokenClassification`` (its own module names:
``intermediate.dense`` etc.) through this engine; loss is ``model(**sample)['loss']``
with ``sample_size = 1`` (reference :470-477).  The model runs on torch ops (no
fused HIP kernels); use ``BertForTokenClassificationTask`` for the fast path.
"""

from .token_classification import BertForTokenClassificationTask, safe_load_checkpoint
from ..utils.misc import ensure_train


class TransformersBertForTokenClassificationTask(BertForTokenClassificationTask):
    def build_model(self, args):
        import json
        from transformers import BertConfig as HFConfig
        from transformers import BertForTokenClassification as HFModel
        with open(args.config_file) as f:
            cfg = json.load(f)
        cfg['num_labels'] = args.num_labels
        model = HFModel(HFConfig(**cfg))
        if getattr(args, 'transformers_state_dict', None):
            sd = safe_load_checkpoint(args.transformers_state_dict)
            model.load_state_dict(sd, strict=bool(args.load_state_dict_strict))
        return model

    def train_step(self, sample, model, optimizer, ignore_grad=False):
        ensure_train(model)
        loss = model(**sample)['loss']
        if ignore_grad:
            loss = loss * 0
        sample_size = 1
        logging_output = {'nsentences': sample_size, 'loss': loss.detach(), 'nll_loss': loss.detach(),
                          'ntokens': 0, 'sample_size': sample_size}
        optimizer.backward(loss)
        return loss, sample_size, logging_output
