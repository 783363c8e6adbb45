"""BERT entity-linking model (reference hetseq/model/bert_for_EL_classification.py:22-113).

BertModel -> dropout -> two heads:
  * mention tagging: Linear(H, num_labels), CE over attention-masked tokens
    (inactive tokens -> ignore_index -100);
  * entity: tanh(Linear(H, dim_entity_emb)) scored with CosineEmbeddingLoss(target=1)
    against a FROZEN entity-embedding table for tokens with entity_labels > 0.
The reference selects entity rows with a boolean index (host sync) and drops the
entity loss when it is NaN (no entity in the batch); here the cosine loss is a
masked mean with static shapes and contributes 0 when the batch has no entity.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .bert import BertModel, BertPreTrainedModel

_OUT_DICT_ENTITY_ID = -1
_IGNORE_CLASSIFICATION_LABEL = -100
NER_LABEL_DICT = {'B': 0, 'I': 1, 'O': 2}


class BertForELClassification(BertPreTrainedModel):
    def __init__(self, config, args):
        super().__init__(config)
        self.config = config
        self.num_labels = args.num_labels
        self.bert = BertModel(config)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)
        self.classifier = nn.Linear(config.hidden_size, self.num_labels)
        self.num_entity_labels = args.num_entity_labels
        self.dim_entity_emb = args.dim_entity_emb
        self.entity_classifier = nn.Linear(config.hidden_size, self.dim_entity_emb)
        self.apply(self.init_bert_weights)
        self.entity_emb = nn.Embedding.from_pretrained(args.EntityEmbedding, freeze=True)
        assert self.entity_emb.weight.shape == (self.num_entity_labels, self.dim_entity_emb)
        self.verbose = getattr(args, 'el_verbose', False)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, labels=None, entity_labels=None,
                checkpoint_activations=False):
        sequence_output, _ = self.bert(input_ids, token_type_ids, attention_mask, output_all_encoded_layers=False,
                                       checkpoint_activations=checkpoint_activations)
        sequence_output = ops.dropout(sequence_output, self.dropout.p, self.training)
        seq = sequence_output.to(self.classifier.weight.dtype)
        logits = self.classifier(seq)
        entity_logits = torch.tanh(self.entity_classifier(seq))
        if labels is None:
            return logits, entity_logits
        if attention_mask is None:
            raise ValueError('mask has to not None ')
        active = attention_mask.view(-1) == 1
        active_labels = torch.where(active, labels.view(-1), torch.full_like(labels.view(-1), -100))
        ner_loss = F.cross_entropy(logits.view(-1, self.num_labels).float(), active_labels, ignore_index=-100)

        ent = entity_labels.view(-1)
        m = (ent > 0).to(torch.float32)
        emb = self.entity_emb.weight[ent.clamp(min=0)]
        cos = F.cosine_similarity(entity_logits.view(-1, self.dim_entity_emb).float(), emb.float(), dim=-1,
                                  eps=1e-8)
        count = m.sum()
        entity_loss = ((1.0 - cos) * m).sum() / count.clamp(min=1.0)
        loss = ner_loss + torch.where(count > 0, entity_loss, torch.zeros_like(entity_loss))
        if self.verbose:
            print('ner_loss', ner_loss.item(), 'entity_loss', entity_loss.item())
        return loss
