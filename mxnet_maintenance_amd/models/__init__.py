"""Reference model families beyond the vision zoo, and training harnesses.

* ``classification`` -- flagship ResNet training step (bench.py, smoke test)
* ``bert``           -- BERT base/large encoder with MLM/NSP heads
* ``language_model`` -- word-level LSTM/GRU language model
* ``ssd``            -- SSD detector on a ResNet-50 backbone (MultiBoxTarget/Detection)

``get_model(name)`` resolves these names and every ``gluon.model_zoo.vision`` model.
"""
from . import bert, language_model, classification, ssd
from .ssd import SSD, SSDMultiBoxLoss, SSDTrainStep, ssd_512_resnet50_v1, ssd_300_resnet50_v1
from .bert import BERTModel, BERTEncoder, BERTEncoderCell, get_bert_model, bert_12_768_12, bert_24_1024_16
from .language_model import RNNModel, standard_lstm_lm_200, standard_lstm_lm_650, standard_lstm_lm_1500
from .classification import ClassificationTrainer

_MODELS = {
    'bert_12_768_12': bert_12_768_12, 'bert_24_1024_16': bert_24_1024_16,
    'standard_lstm_lm_200': standard_lstm_lm_200, 'standard_lstm_lm_650': standard_lstm_lm_650,
    'standard_lstm_lm_1500': standard_lstm_lm_1500,
    'ssd_512_resnet50_v1': ssd_512_resnet50_v1, 'ssd_300_resnet50_v1': ssd_300_resnet50_v1,
}


def get_model(name, **kwargs):
    if name in _MODELS:
        return _MODELS[name](**kwargs)
    from ..gluon.model_zoo import vision
    return vision.get_model(name, **kwargs)


def list_models():
    from ..gluon.model_zoo import vision
    return sorted(_MODELS)
