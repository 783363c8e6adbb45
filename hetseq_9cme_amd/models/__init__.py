from .bert import (  # noqa: F401
    BertConfig, BertModel, BertForPreTraining, BertForMaskedLM, BertForNextSentencePrediction,
    BertForSequenceClassification, BertForMultipleChoice, BertForTokenClassification,
    BertForQuestionAnswering, BertPreTrainedModel, LinearActivation, BertLayerNorm,
    remap_state_dict_keys,
)
from .mnist import MNISTNet  # noqa: F401
from .el import BertForELClassification  # noqa: F401
