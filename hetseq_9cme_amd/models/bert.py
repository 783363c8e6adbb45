"""BERT model family, MI355X-native.

Module tree and parameter names reproduce the reference exactly so checkpoints
are interchangeable (hetseq/bert_modeling.py:132-1329, key schema in SURVEY
App. C), including its quirks:
  * post-LN BERT, TF-style LayerNorm (eps inside sqrt, 1e-12),
  * GELU = x*0.5*(1+erf(x/1.41421)),
  * additive attention mask (1-m)*-10000,
  * ``LinearActivation`` is NOT an nn.Linear, so it keeps kaiming-uniform init
    (SURVEY App. A5), while nn.Linear/nn.Embedding get N(0, initializer_range).

The compute path is different: every hot op goes through ``hetseq_9cme_amd.ops``
(gfx950 HIP kernels on GPU):
  * Q/K/V projections run as ONE N=3H GEMM over adjacent weight storage,
  * attention is the fused flash-style kernel (no [B,nh,S,S] tensors),
  * dense -> bias -> dropout -> +residual -> LayerNorm is one kernel after the GEMM,
  * the residual branch's gradient is accumulated by the QKV / FFN-up dgrad GEMM
    (beta = 1, ``ops.ResidualGrad``) instead of a separate add kernel,
  * GEMM -> bias+GELU / bias+tanh is one epilogue kernel,
  * embedding gathers + sum + LN + dropout is one kernel,
  * the MLM head only runs on the masked rows (gathered without host sync) and the
    decoder bias + softmax-cross-entropy (+ its gradient) is one kernel.
"""
import copy
import json
import logging
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn import init
from torch.nn.parameter import Parameter

from .. import ops
from ..ops.rng import get_rng

logger = logging.getLogger(__name__)

CONFIG_NAME = 'bert_config.json'
WEIGHTS_NAME = 'pytorch_model.bin'
# short names -> the archive URLs the reference downloads (bert_modeling.py:30-38), fetched into
# the ETag-keyed download cache by utils.file_utils.cached_path (a cached copy is used offline)
_S3 = 'https://s3.amazonaws.com/models.huggingface.co/bert/{}.tar.gz'
PRETRAINED_MODEL_ARCHIVE_MAP = {n: _S3.format(n) for n in (
    'bert-base-uncased', 'bert-large-uncased', 'bert-base-cased', 'bert-large-cased',
    'bert-base-multilingual-uncased', 'bert-base-multilingual-cased', 'bert-base-chinese')}


def gelu(x):
    return ops.gelu_ref(x)


def swish(x):
    return x * torch.sigmoid(x)


ACT2FN = {'gelu': gelu, 'relu': F.relu, 'swish': swish, 'tanh': torch.tanh}

class BertConfig(object):
    """Configuration of a BERT model (reference bert_modeling.py:180-266)."""

    def __init__(self, vocab_size_or_config_json_file, hidden_size=768, num_hidden_layers=12,
                 num_attention_heads=12, intermediate_size=3072, hidden_act='gelu',
                 hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.1,
                 max_position_embeddings=512, type_vocab_size=2, initializer_range=0.02):
        if isinstance(vocab_size_or_config_json_file, str):
            with open(vocab_size_or_config_json_file, 'r', encoding='utf-8') as reader:
                json_config = json.loads(reader.read())
            for key, value in json_config.items():
                self.__dict__[key] = value
        elif isinstance(vocab_size_or_config_json_file, int):
            self.vocab_size = vocab_size_or_config_json_file
            self.hidden_size = hidden_size
            self.num_hidden_layers = num_hidden_layers
            self.num_attention_heads = num_attention_heads
            self.hidden_act = hidden_act
            self.intermediate_size = intermediate_size
            self.hidden_dropout_prob = hidden_dropout_prob
            self.attention_probs_dropout_prob = attention_probs_dropout_prob
            self.max_position_embeddings = max_position_embeddings
            self.type_vocab_size = type_vocab_size
            self.initializer_range = initializer_range
        else:
            raise ValueError('First argument must be either a vocabulary size (int) '
                             'or the path to a pretrained model config file (str)')

    @classmethod
    def from_dict(cls, json_object):
        config = BertConfig(vocab_size_or_config_json_file=-1)
        for key, value in json_object.items():
            config.__dict__[key] = value
        return config

    @classmethod
    def from_json_file(cls, json_file):
        with open(json_file, 'r', encoding='utf-8') as reader:
            return cls.from_dict(json.loads(reader.read()))

    def __repr__(self):
        return str(self.to_json_string())

    def to_dict(self):
        return copy.deepcopy(self.__dict__)

    def to_json_string(self):
        return json.dumps(self.to_dict(), indent=2, sort_keys=True) + '\n'


class LinearActivation(nn.Module):
    """Linear + activation; GELU/tanh with bias run as one fused epilogue kernel."""
    __constants__ = ['bias']

    def __init__(self, in_features, out_features, act='gelu', bias=True):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.act = act if isinstance(act, str) else None
        self.act_fn = None if isinstance(act, str) else act
        self.weight = Parameter(torch.Tensor(out_features, in_features))
        if bias:
            self.bias = Parameter(torch.Tensor(out_features))
        else:
            self.register_parameter('bias', None)
        self.reset_parameters()

    def reset_parameters(self):
        init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            fan_in, _ = init._calculate_fan_in_and_fan_out(self.weight)
            bound = 1 / math.sqrt(fan_in)
            init.uniform_(self.bias, -bound, bound)

    def forward(self, x, res_grad=None):
        y = ops.linear(x, self.weight, res_grad=res_grad)
        if self.act in ('gelu', 'tanh', 'relu'):
            return ops.bias_act(y, self.bias, self.act)
        if self.bias is not None:
            y = y + self.bias
        fn = self.act_fn or ACT2FN[self.act]
        return fn(y)

    def extra_repr(self):
        return 'in_features={}, out_features={}, bias={}'.format(
            self.in_features, self.out_features, self.bias is not None)


class BertLayerNorm(nn.Module):
    """TF-style LayerNorm (epsilon inside the square root)."""

    def __init__(self, hidden_size, eps=1e-12):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden_size))
        self.bias = nn.Parameter(torch.zeros(hidden_size))
        self.variance_epsilon = eps

    def forward(self, x):
        return ops.layer_norm(x, self.weight, self.bias, self.variance_epsilon)


class BertEmbeddings(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.word_embeddings = nn.Embedding(config.vocab_size, config.hidden_size)
        self.position_embeddings = nn.Embedding(config.max_position_embeddings, config.hidden_size)
        self.token_type_embeddings = nn.Embedding(config.type_vocab_size, config.hidden_size)
        self.LayerNorm = BertLayerNorm(config.hidden_size, eps=1e-12)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)
        self.compute_dtype = torch.float32

    def forward(self, input_ids, token_type_ids=None):
        return ops.embed_ln(input_ids, token_type_ids, self.word_embeddings.weight,
                            self.position_embeddings.weight, self.token_type_embeddings.weight,
                            self.LayerNorm.weight, self.LayerNorm.bias, self.LayerNorm.variance_epsilon,
                            self.dropout.p, self.training, self.compute_dtype)


# where the Q/K/V biases are added: the projection GEMM's epilogue (default; the attention kernels
# then skip the adds and only produce the bias gradient) or the attention kernels
# (HX_QKV_BIAS_EPILOGUE=0, the round-2..5 layout)
_QKV_BIAS_EPILOGUE = os.environ.get('HX_QKV_BIAS_EPILOGUE', '1') != '0'


class BertSelfAttention(nn.Module):
    def __init__(self, config):
        super().__init__()
        if config.hidden_size % config.num_attention_heads != 0:
            raise ValueError('The hidden size (%d) is not a multiple of the number of attention heads (%d)'
                             % (config.hidden_size, config.num_attention_heads))
        self.num_attention_heads = config.num_attention_heads
        self.attention_head_size = int(config.hidden_size / config.num_attention_heads)
        self.all_head_size = self.num_attention_heads * self.attention_head_size
        self.query = nn.Linear(config.hidden_size, self.all_head_size)
        self.key = nn.Linear(config.hidden_size, self.all_head_size)
        self.value = nn.Linear(config.hidden_size, self.all_head_size)
        self.dropout = nn.Dropout(config.attention_probs_dropout_prob)

    def forward(self, hidden_states, attention_mask_bias, res_grad=None):
        bias = (self.query.bias, self.key.bias, self.value.bias)
        if _QKV_BIAS_EPILOGUE:
            # one N=3H projection GEMM with the Q/K/V biases in its epilogue; their gradients (the
            # column sums of dQKV) come out of the fused attention backward's registers
            qkv = ops.linear3(hidden_states, self.query.weight, self.key.weight, self.value.weight, *bias,
                              res_grad=res_grad, bias_grad=False)
            return ops.attention(qkv, attention_mask_bias, self.num_attention_heads, self.dropout.p, self.training,
                                 bias_grad=bias)
        # bias-less projection; the biases are added (and their gradients produced) in the attention
        qkv = ops.linear3(hidden_states, self.query.weight, self.key.weight, self.value.weight,
                          None, None, None, res_grad=res_grad)
        return ops.attention(qkv, attention_mask_bias, self.num_attention_heads, self.dropout.p, self.training,
                             bias=bias)


class BertSelfOutput(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.dense = nn.Linear(config.hidden_size, config.hidden_size)
        self.LayerNorm = BertLayerNorm(config.hidden_size, eps=1e-12)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)

    def forward(self, hidden_states, input_tensor, res_grad=None):
        y = ops.linear(hidden_states, self.dense.weight)
        return ops.bias_dropout_residual_ln(y, self.dense.bias, input_tensor, self.LayerNorm.weight,
                                            self.LayerNorm.bias, self.LayerNorm.variance_epsilon,
                                            self.dropout.p, self.training, res_grad=res_grad)


class BertAttention(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.self = BertSelfAttention(config)
        self.output = BertSelfOutput(config)

    def forward(self, input_tensor, attention_mask_bias):
        # the residual gradient of input_tensor is fused into the QKV dgrad GEMM
        rg = ops.ResidualGrad()
        ctx = self.self(input_tensor, attention_mask_bias, rg)
        return self.output(ctx, input_tensor, rg)


class BertIntermediate(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.dense_act = LinearActivation(config.hidden_size, config.intermediate_size, act=config.hidden_act)

    def forward(self, hidden_states, res_grad=None):
        return self.dense_act(hidden_states, res_grad)


class BertOutput(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.dense = nn.Linear(config.intermediate_size, config.hidden_size)
        self.LayerNorm = BertLayerNorm(config.hidden_size, eps=1e-12)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)

    def forward(self, hidden_states, input_tensor, res_grad=None):
        return self.finish(ops.linear(hidden_states, self.dense.weight), input_tensor, res_grad)

    def finish(self, y, input_tensor, res_grad=None):
        """dense bias -> dropout -> + residual -> LayerNorm on the bias-less projection ``y``."""
        return ops.bias_dropout_residual_ln(y, self.dense.bias, input_tensor, self.LayerNorm.weight,
                                            self.LayerNorm.bias, self.LayerNorm.variance_epsilon,
                                            self.dropout.p, self.training, res_grad=res_grad)


class BertLayer(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.attention = BertAttention(config)
        self.intermediate = BertIntermediate(config)
        self.output = BertOutput(config)

    def forward(self, hidden_states, attention_mask_bias):
        attention_output = self.attention(hidden_states, attention_mask_bias)
        rg = ops.ResidualGrad()     # residual grad of attention_output -> FFN-up dgrad GEMM
        up = self.intermediate.dense_act
        if up.act == 'gelu' and ops.ffn_fusable(attention_output, up.weight, up.bias, self.output.dense.weight):
            # fp32 runs: bias + GELU in the FFN-up GEMM's epilogue, the GELU backward in the
            # FFN-down data gradient's (ops.ffn)
            y = ops.ffn(attention_output, up.weight, up.bias, self.output.dense.weight, rg)
            return self.output.finish(y, attention_output, rg)
        return self.output(self.intermediate(attention_output, rg), attention_output, rg)


def _rng_replaying(fn):
    """Wrap a checkpointed segment so its recomputation replays the same dropout
    streams (our RNG is counter-based; torch's checkpoint only restores torch RNG)."""
    rng = get_rng()
    start = rng.counter

    def run(*inputs):
        cur = rng.counter
        rng.counter = start
        out = fn(*inputs)
        if cur != start:
            rng.counter = cur
        return out
    return run


class BertEncoder(nn.Module):
    def __init__(self, config):
        super().__init__()
        layer = BertLayer(config)
        self.layer = nn.ModuleList([copy.deepcopy(layer) for _ in range(config.num_hidden_layers)])

    def forward(self, hidden_states, attention_mask_bias, output_all_encoded_layers=True,
                checkpoint_activations=False):
        with ops.weight_pieces_scope(self._piece_weights(), hidden_states):
            return self._forward(hidden_states, attention_mask_bias, output_all_encoded_layers,
                                 checkpoint_activations)

    def _piece_weights(self):
        """The encoder's linear weights (the fused QKV view, attention output, FFN up / down):
        prepared for the hand-written GEMMs in one launch per forward (ops.weight_pieces_scope).
        The Parameter objects are collected once (module attribute walks cost ~0.25 ms of host
        time per update); their storage is read at each call, so re-pointed ``.data`` is seen."""
        ps = self.__dict__.get('_pw_params')
        if ps is None or len(ps) != 4 * len(self.layer):
            ps = []
            for layer in self.layer:
                sa = layer.attention.self
                ps += [(sa.query.weight, sa.key.weight, sa.value.weight), layer.attention.output.dense.weight,
                       layer.intermediate.dense_act.weight, layer.output.dense.weight]
            self.__dict__['_pw_params'] = ps
        return [ops.qkv_weight_view(*p) if isinstance(p, tuple) else p for p in ps]

    def _forward(self, hidden_states, attention_mask_bias, output_all_encoded_layers, checkpoint_activations):
        all_encoder_layers = []
        if checkpoint_activations:
            from torch.utils.checkpoint import checkpoint

            def custom(start, end):
                def custom_forward(x, m):
                    for layer in self.layer[start:end]:
                        x = layer(x, m)
                    return x
                return custom_forward

            num_layers = len(self.layer)
            chunk = math.ceil(math.sqrt(num_layers))
            l = 0
            while l < num_layers:
                hidden_states = checkpoint(_rng_replaying(custom(l, l + chunk)), hidden_states,
                                           attention_mask_bias, use_reentrant=False)
                l += chunk
        else:
            for layer_module in self.layer:
                hidden_states = layer_module(hidden_states, attention_mask_bias)
                if output_all_encoded_layers:
                    all_encoder_layers.append(hidden_states)
        if not output_all_encoded_layers or checkpoint_activations:
            all_encoder_layers.append(hidden_states)
        return all_encoder_layers


class BertPooler(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.dense_act = LinearActivation(config.hidden_size, config.hidden_size, act='tanh')

    def forward(self, hidden_states):
        return self.dense_act(hidden_states[:, 0].contiguous())


class BertPredictionHeadTransform(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.dense_act = LinearActivation(config.hidden_size, config.hidden_size, act=config.hidden_act)
        self.LayerNorm = BertLayerNorm(config.hidden_size, eps=1e-12)

    def forward(self, hidden_states):
        return self.LayerNorm(self.dense_act(hidden_states))


class BertLMPredictionHead(nn.Module):
    def __init__(self, config, bert_model_embedding_weights):
        super().__init__()
        self.transform = BertPredictionHeadTransform(config)
        self.decoder = nn.Linear(bert_model_embedding_weights.size(1), bert_model_embedding_weights.size(0),
                                 bias=False)
        self.decoder.weight = bert_model_embedding_weights
        self.bias = nn.Parameter(torch.zeros(bert_model_embedding_weights.size(0)))

    def forward(self, hidden_states):
        hidden_states = self.transform(hidden_states)
        with torch.autograd.profiler.record_function('mlm_decoder'):
            return F.linear(hidden_states, self.decoder.weight.to(hidden_states.dtype)) + self.bias

    def loss(self, hidden_states, labels_flat):
        """Masked-LM CE over rows of ``hidden_states`` [M, H] (labels -1 ignored)."""
        h = self.transform(hidden_states)
        with torch.autograd.profiler.record_function('mlm_decoder_xent'):
            return ops.decoder_xent(h, self.decoder.weight, self.bias, labels_flat)


class BertOnlyMLMHead(nn.Module):
    def __init__(self, config, bert_model_embedding_weights):
        super().__init__()
        self.predictions = BertLMPredictionHead(config, bert_model_embedding_weights)

    def forward(self, sequence_output):
        return self.predictions(sequence_output)


class BertOnlyNSPHead(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.seq_relationship = nn.Linear(config.hidden_size, 2)

    def forward(self, pooled_output):
        return self.seq_relationship(pooled_output)


class BertPreTrainingHeads(nn.Module):
    def __init__(self, config, bert_model_embedding_weights):
        super().__init__()
        self.predictions = BertLMPredictionHead(config, bert_model_embedding_weights)
        self.seq_relationship = nn.Linear(config.hidden_size, 2)

    def forward(self, sequence_output, pooled_output):
        return self.predictions(sequence_output), self.seq_relationship(pooled_output)


# HF/transformers names -> reference names (SURVEY App. A16 fix)
_KEY_RENAMES = [
    ('.intermediate.dense.', '.intermediate.dense_act.'),
    ('pooler.dense.', 'pooler.dense_act.'),
    ('cls.predictions.transform.dense.', 'cls.predictions.transform.dense_act.'),
    ('.gamma', '.weight'),
    ('.beta', '.bias'),
]


TF_WEIGHTS_NAME = 'model.ckpt'
_TF_SKIP = ('adam_v', 'adam_m', 'AdamWeightDecayOptimizer', 'AdamWeightDecayOptimizer_1', 'global_step',
            'bad_steps', 'good_steps', 'loss_scale')


def _tf_resolve(model, name):
    """Walk a TF variable name (``bert/encoder/layer_3/attention/self/query/kernel``)
    down the module tree with the reference's rules (bert_modeling.py:66-93):
    ``kernel``/``gamma``/``output_weights`` -> weight, ``beta``/``output_bias`` ->
    bias, ``name_N`` -> ``name[N]``, ``*_embeddings`` -> its ``.weight``, and a
    ``kernel`` is transposed.  One fix: TF's ``dense`` resolves to this schema's
    ``dense_act`` (``LinearActivation``) where a module has no ``dense`` -- the
    reference raises AttributeError on the intermediate / pooler / MLM-transform
    layers of Google's checkpoints because of that rename."""
    import re
    pointer, transpose = model, False
    parts = name.split('/')
    for m_name in parts:
        if re.fullmatch(r'[A-Za-z]+_\d+', m_name):
            l = re.split(r'_(\d+)', m_name)
        else:
            l = [m_name]
        if l[0] in ('kernel', 'gamma', 'output_weights'):
            pointer = getattr(pointer, 'weight')
        elif l[0] in ('output_bias', 'beta'):
            pointer = getattr(pointer, 'bias')
        elif l[0] == 'dense' and not hasattr(pointer, 'dense') and hasattr(pointer, 'dense_act'):
            pointer = getattr(pointer, 'dense_act')
        elif l[0] == 'squad' and not hasattr(pointer, 'squad') and hasattr(pointer, 'classifier'):
            pointer = getattr(pointer, 'classifier')
        else:
            pointer = getattr(pointer, l[0])
        if len(l) >= 2:
            pointer = pointer[int(l[1])]
    if parts[-1].endswith('_embeddings'):
        pointer = getattr(pointer, 'weight')
    elif parts[-1] == 'kernel':
        transpose = True
    return pointer, transpose


def load_tf_weights_in_bert(model, tf_checkpoint_path):
    """Load a TensorFlow BERT checkpoint into ``model`` (reference
    bert_modeling.py:43-101) without tensorflow: the bundle is decoded by
    ``utils.tf_checkpoint``.  Values are copied into the existing parameter
    storage (flat-buffer views stay valid); optimizer slots and step counters are
    skipped."""
    from ..utils.tf_checkpoint import TFCheckpointReader
    reader = TFCheckpointReader(tf_checkpoint_path)
    logger.info('Converting TensorFlow checkpoint from %s', reader.prefix)
    loaded = []
    for name, shape in reader.list_variables():
        if any(n in _TF_SKIP for n in name.split('/')):
            logger.info('Skipping %s', name)
            continue
        pointer, transpose = _tf_resolve(model, name)
        array = reader.get_tensor(name)
        if transpose:
            array = array.T
        if tuple(pointer.shape) != tuple(array.shape):
            raise ValueError('TF variable {} has shape {}, model parameter {}'.format(
                name, tuple(array.shape), tuple(pointer.shape)))
        with torch.no_grad():
            pointer.data.copy_(torch.from_numpy(array.copy()).to(pointer.dtype))
        loaded.append(name)
    logger.info('Initialized %d PyTorch weights from TF', len(loaded))
    return model


def bert_state_to_tf_names(model):
    """Inverse of :func:`load_tf_weights_in_bert`: ``{tf_name: ndarray}`` in Google's
    naming (``kernel`` transposed, LayerNorm ``gamma/beta``, ``layer_N``,
    ``cls/predictions/output_bias``, ``cls/seq_relationship/output_weights``).
    The tied decoder weight is the word embedding and is not emitted twice."""
    import re
    out = {}
    lin_weights = {n for n, m in model.named_modules() if isinstance(m, (nn.Linear, LinearActivation))}
    for key, t in model.state_dict().items():
        if key == 'cls.predictions.decoder.weight':
            continue
        mod, _, leaf = key.rpartition('.')
        parts = mod.split('.') if mod else []
        tf_parts = []
        i = 0
        while i < len(parts):
            if i + 1 < len(parts) and parts[i + 1].isdigit():
                tf_parts.append('{}_{}'.format(parts[i], parts[i + 1]))
                i += 2
                continue
            tf_parts.append('dense' if parts[i] == 'dense_act' else parts[i])
            i += 1
        arr = t.detach().float().cpu().numpy()
        if mod.endswith('LayerNorm'):
            tf_parts.append('gamma' if leaf == 'weight' else 'beta')
        elif re.search(r'_embeddings$', mod):
            pass                                   # '<name>_embeddings' holds the table itself
        elif mod == 'cls.seq_relationship':
            tf_parts.append('output_weights' if leaf == 'weight' else 'output_bias')
        elif mod == 'cls.predictions' and leaf == 'bias':
            tf_parts.append('output_bias')
        elif mod in lin_weights and leaf == 'weight':
            tf_parts.append('kernel')
            arr = arr.T
        else:
            tf_parts.append(leaf)
        out['/'.join(tf_parts)] = arr
    return out


def remap_state_dict_keys(state_dict, model_keys=None):
    """Map transformers-style keys (``intermediate.dense``, ``pooler.dense``,
    LayerNorm ``gamma/beta``) onto this schema.  Returns a new dict."""
    out = {}
    for k, v in state_dict.items():
        nk = k
        for a, b in _KEY_RENAMES:
            if a in nk and (model_keys is None or nk.replace(a, b) in model_keys or a.startswith('.g')
                            or a.startswith('.b')):
                nk = nk.replace(a, b)
        out[nk] = v
    return out


class BertPreTrainedModel(nn.Module):
    def __init__(self, config, *inputs, **kwargs):
        super().__init__()
        if not isinstance(config, BertConfig):
            raise ValueError('Parameter config in `{}(config)` should be an instance of class `BertConfig`.'
                             .format(self.__class__.__name__))
        self.config = config

    def init_bert_weights(self, module):
        if isinstance(module, (nn.Linear, nn.Embedding)):
            module.weight.data.normal_(mean=0.0, std=self.config.initializer_range)
        elif isinstance(module, BertLayerNorm):
            module.bias.data.zero_()
            module.weight.data.fill_(1.0)
        if isinstance(module, nn.Linear) and module.bias is not None:
            module.bias.data.zero_()

    def set_compute_dtype(self, dtype):
        for m in self.modules():
            if isinstance(m, BertEmbeddings):
                m.compute_dtype = dtype

    def flat_contiguous_groups(self):
        """Parameter-name groups that must be adjacent in the flat buffer so the
        fused kernels can view them as one tensor (Q/K/V weights and biases)."""
        groups = []
        for name, m in self.named_modules():
            if isinstance(m, BertSelfAttention):
                p = name + '.' if name else ''
                groups.append([p + 'query.weight', p + 'key.weight', p + 'value.weight'])
                groups.append([p + 'query.bias', p + 'key.bias', p + 'value.bias'])
        return groups

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path, state_dict=None, cache_dir=None, from_tf=False,
                        *inputs, **kwargs):
        """Instantiate from pretrained weights (reference bert_modeling.py:612-752).

        ``pretrained_model_name_or_path`` is a local directory holding
        ``bert_config.json`` + ``pytorch_model.bin`` (or ``model.safetensors``), a
        ``.tar.gz`` archive of such a directory (extracted to a temp dir with the
        reference's path-traversal guard), or a URL / short name that ``utils.file_utils.cached_path``
        downloads into its cache (or finds there when offline).  ``from_tf=True`` reads
        ``model.ckpt`` (TF V2 bundle) from the directory through the native-format
        reader -- no tensorflow needed.  Weights load with ``weights_only=True``."""
        import shutil
        import tarfile
        import tempfile
        from ..utils.file_utils import cached_path
        archive = PRETRAINED_MODEL_ARCHIVE_MAP.get(pretrained_model_name_or_path, pretrained_model_name_or_path)
        try:
            resolved = cached_path(archive, cache_dir=cache_dir)
        except EnvironmentError:
            raise EnvironmentError('pretrained model not found (neither a local path, a reachable URL nor a '
                                   'cached download): {}'.format(pretrained_model_name_or_path))
        tempdir = None
        if os.path.isdir(resolved) or from_tf:
            serialization_dir = resolved
        else:
            tempdir = tempfile.mkdtemp()
            with tarfile.open(resolved, 'r:*') as tar:
                root = os.path.abspath(tempdir)
                for member in tar.getmembers():
                    target = os.path.abspath(os.path.join(tempdir, member.name))
                    if os.path.commonpath([root, target]) != root or member.issym() or member.islnk():
                        raise EnvironmentError('unsafe member in archive {}: {}'.format(resolved, member.name))
                tar.extractall(tempdir)
            serialization_dir = tempdir
            # archives may wrap the files in one top-level directory
            if not os.path.exists(os.path.join(tempdir, CONFIG_NAME)):
                subs = [d for d in os.listdir(tempdir) if os.path.isdir(os.path.join(tempdir, d))]
                if len(subs) == 1:
                    serialization_dir = os.path.join(tempdir, subs[0])
        try:
            config = BertConfig.from_json_file(os.path.join(serialization_dir, CONFIG_NAME))
            model = cls(config, *inputs, **kwargs)
            if from_tf:
                return load_tf_weights_in_bert(model, os.path.join(serialization_dir, TF_WEIGHTS_NAME))
            if state_dict is None:
                st = os.path.join(serialization_dir, 'model.safetensors')
                if os.path.exists(st):
                    from safetensors.torch import load_file
                    state_dict = load_file(st)
                else:
                    state_dict = torch.load(os.path.join(serialization_dir, WEIGHTS_NAME), map_location='cpu',
                                            weights_only=True)
        finally:
            if tempdir:
                shutil.rmtree(tempdir, ignore_errors=True)
        keys = set(model.state_dict().keys())
        state_dict = remap_state_dict_keys(state_dict, keys)
        if not any(k.startswith('bert.') for k in keys) or any(k.startswith('bert.') for k in state_dict):
            pass
        elif any(k.startswith('bert.') for k in keys):
            state_dict = {('bert.' + k if not k.startswith('cls.') else k): v for k, v in state_dict.items()}
        missing, unexpected = model.load_state_dict(state_dict, strict=False)
        if missing:
            logger.info('Weights of %s not initialized from pretrained model: %s', cls.__name__, missing)
        if unexpected:
            logger.info('Weights from pretrained model not used in %s: %s', cls.__name__, unexpected)
        return model


def _mask_bias(attention_mask, input_ids):
    if attention_mask is None:
        attention_mask = torch.ones_like(input_ids)
    return (1.0 - attention_mask.to(torch.float32)) * -10000.0


class BertModel(BertPreTrainedModel):
    def __init__(self, config):
        super().__init__(config)
        self.embeddings = BertEmbeddings(config)
        self.encoder = BertEncoder(config)
        self.pooler = BertPooler(config)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, output_all_encoded_layers=True,
                checkpoint_activations=False):
        mask_bias = _mask_bias(attention_mask, input_ids)
        embedding_output = self.embeddings(input_ids, token_type_ids)
        encoded_layers = self.encoder(embedding_output, mask_bias,
                                      output_all_encoded_layers=output_all_encoded_layers,
                                      checkpoint_activations=checkpoint_activations)
        sequence_output = encoded_layers[-1]
        pooled_output = self.pooler(sequence_output)
        if not output_all_encoded_layers:
            encoded_layers = encoded_layers[-1]
        return encoded_layers, pooled_output


class BertForPreTraining(BertPreTrainedModel):
    """BERT + MLM + NSP heads; ``forward(ids, seg, mask, mlm_labels, nsp_label)`` returns
    the summed loss (reference :838-907).

    ``max_predictions_per_seq`` (set by the LM task from the shard's
    ``masked_lm_positions`` width) bounds the number of masked rows per sequence;
    the MLM head then runs on at most B * max_predictions_per_seq gathered rows,
    which is mathematically identical to the reference's all-rows CE (ignored rows
    contribute exactly zero to loss and gradients)."""

    def __init__(self, config):
        super().__init__(config)
        self.bert = BertModel(config)
        self.cls = BertPreTrainingHeads(config, self.bert.embeddings.word_embeddings.weight)
        self.apply(self.init_bert_weights)
        self.max_predictions_per_seq = getattr(config, 'max_predictions_per_seq', None)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, masked_lm_labels=None,
                next_sentence_label=None, checkpoint_activations=False):
        sequence_output, pooled_output = self.bert(input_ids, token_type_ids, attention_mask,
                                                   output_all_encoded_layers=False,
                                                   checkpoint_activations=checkpoint_activations)
        if masked_lm_labels is not None and next_sentence_label is not None:
            H = sequence_output.shape[-1]
            seq_flat = sequence_output.reshape(-1, H)
            labels_flat = masked_lm_labels.reshape(-1)
            cap = None
            if self.max_predictions_per_seq:
                cap = input_ids.shape[0] * int(self.max_predictions_per_seq)
            rows = ops.masked_rows(labels_flat, cap)
            if rows is not None:
                seq_flat = seq_flat.index_select(0, rows)
                labels_flat = labels_flat.index_select(0, rows)
            masked_lm_loss = self.cls.predictions.loss(seq_flat, labels_flat)
            nsp_logits = self.cls.seq_relationship(pooled_output.to(self.cls.seq_relationship.weight.dtype))
            next_sentence_loss = F.cross_entropy(nsp_logits.view(-1, 2).float(), next_sentence_label.view(-1),
                                                 ignore_index=-1)
            return masked_lm_loss + next_sentence_loss
        return self.cls(sequence_output, pooled_output)


class BertForMaskedLM(BertPreTrainedModel):
    def __init__(self, config):
        super().__init__(config)
        self.bert = BertModel(config)
        self.cls = BertOnlyMLMHead(config, self.bert.embeddings.word_embeddings.weight)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, masked_lm_labels=None,
                checkpoint_activations=False):
        sequence_output, _ = self.bert(input_ids, token_type_ids, attention_mask, output_all_encoded_layers=False)
        if masked_lm_labels is not None:
            H = sequence_output.shape[-1]
            return self.cls.predictions.loss(sequence_output.reshape(-1, H), masked_lm_labels.reshape(-1))
        return self.cls(sequence_output)


class BertForNextSentencePrediction(BertPreTrainedModel):
    def __init__(self, config):
        super().__init__(config)
        self.bert = BertModel(config)
        self.cls = BertOnlyNSPHead(config)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, next_sentence_label=None,
                checkpoint_activations=False):
        _, pooled_output = self.bert(input_ids, token_type_ids, attention_mask, output_all_encoded_layers=False)
        seq_relationship_score = self.cls(pooled_output)
        if next_sentence_label is not None:
            return F.cross_entropy(seq_relationship_score.view(-1, 2).float(), next_sentence_label.view(-1),
                                   ignore_index=-1)
        return seq_relationship_score


class BertForSequenceClassification(BertPreTrainedModel):
    def __init__(self, config, num_labels):
        super().__init__(config)
        self.num_labels = num_labels
        self.bert = BertModel(config)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)
        self.classifier = nn.Linear(config.hidden_size, num_labels)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, labels=None,
                checkpoint_activations=False):
        _, pooled_output = self.bert(input_ids, token_type_ids, attention_mask, output_all_encoded_layers=False)
        pooled_output = ops.dropout(pooled_output, self.dropout.p, self.training)
        logits = self.classifier(pooled_output.to(self.classifier.weight.dtype))
        if labels is not None:
            return F.cross_entropy(logits.view(-1, self.num_labels).float(), labels.view(-1))
        return logits


class BertForMultipleChoice(BertPreTrainedModel):
    def __init__(self, config, num_choices):
        super().__init__(config)
        self.num_choices = num_choices
        self.bert = BertModel(config)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)
        self.classifier = nn.Linear(config.hidden_size, 1)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, labels=None,
                checkpoint_activations=False):
        flat_input_ids = input_ids.view(-1, input_ids.size(-1))
        flat_token_type_ids = token_type_ids.view(-1, token_type_ids.size(-1)) if token_type_ids is not None else None
        flat_attention_mask = attention_mask.view(-1, attention_mask.size(-1)) if attention_mask is not None else None
        _, pooled_output = self.bert(flat_input_ids, flat_token_type_ids, flat_attention_mask,
                                     output_all_encoded_layers=False)
        pooled_output = ops.dropout(pooled_output, self.dropout.p, self.training)
        logits = self.classifier(pooled_output.to(self.classifier.weight.dtype))
        reshaped_logits = logits.view(-1, self.num_choices)
        if labels is not None:
            return F.cross_entropy(reshaped_logits.float(), labels)
        return reshaped_logits


class BertForTokenClassification(BertPreTrainedModel):
    """Token classification (NER).  The reference selects active tokens with a
    boolean index (host sync, dynamic shape, :1228-1232); here inactive tokens get
    label -100 (CrossEntropyLoss's ignore_index) -- the same mean over active,
    non-ignored tokens, computed with static shapes."""

    def __init__(self, config, num_labels):
        super().__init__(config)
        self.num_labels = num_labels
        self.bert = BertModel(config)
        self.dropout = nn.Dropout(config.hidden_dropout_prob)
        self.classifier = nn.Linear(config.hidden_size, num_labels)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, labels=None,
                checkpoint_activations=False):
        sequence_output, _ = self.bert(input_ids, token_type_ids, attention_mask, output_all_encoded_layers=False,
                                       checkpoint_activations=checkpoint_activations)
        sequence_output = ops.dropout(sequence_output, self.dropout.p, self.training)
        logits = self.classifier(sequence_output.to(self.classifier.weight.dtype))
        if labels is not None:
            flat_labels = labels.view(-1)
            if attention_mask is not None:
                active = attention_mask.view(-1) == 1
                flat_labels = torch.where(active, flat_labels, torch.full_like(flat_labels, -100))
            return F.cross_entropy(logits.view(-1, self.num_labels).float(), flat_labels, ignore_index=-100)
        return logits


class BertForQuestionAnswering(BertPreTrainedModel):
    def __init__(self, config):
        super().__init__(config)
        self.bert = BertModel(config)
        self.qa_outputs = nn.Linear(config.hidden_size, 2)
        self.apply(self.init_bert_weights)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, start_positions=None,
                end_positions=None, checkpoint_activations=False):
        sequence_output, _ = self.bert(input_ids, token_type_ids, attention_mask, output_all_encoded_layers=False)
        logits = self.qa_outputs(sequence_output.to(self.qa_outputs.weight.dtype))
        start_logits, end_logits = logits.split(1, dim=-1)
        start_logits = start_logits.squeeze(-1)
        end_logits = end_logits.squeeze(-1)
        if start_positions is not None and end_positions is not None:
            if start_positions.dim() > 1:
                start_positions = start_positions.squeeze(-1)
            if end_positions.dim() > 1:
                end_positions = end_positions.squeeze(-1)
            ignored_index = start_logits.size(1)
            start_positions = start_positions.clamp(0, ignored_index)
            end_positions = end_positions.clamp(0, ignored_index)
            start_loss = F.cross_entropy(start_logits.float(), start_positions, ignore_index=ignored_index)
            end_loss = F.cross_entropy(end_logits.float(), end_positions, ignore_index=ignored_index)
            return (start_loss + end_loss) / 2
        return start_logits, end_logits
