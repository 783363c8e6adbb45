from . import data_utils, iterators  # noqa: F401
from .h5_dataset import BertH5pyData, ConBertH5pyData  # noqa: F401
from .mnist_dataset import MNISTDataset  # noqa: F401
from .ner_dataset import BertNerDataset, BertELDataset  # noqa: F401
from .collators import (  # noqa: F401
    DataCollatorForTokenClassification, DataCollatorForELClassification,
    YD_DataCollatorForTokenClassification, YD_DataCollatorForELClassification,
)
from .prefetch import DevicePrefetcher  # noqa: F401
