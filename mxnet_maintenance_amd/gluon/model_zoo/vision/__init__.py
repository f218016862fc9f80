"""Vision models (mx.gluon.model_zoo.vision).  Parity: python/mxnet/gluon/model_zoo/vision/__init__.py."""
from .resnet import *  # noqa: F401,F403
from .others import *  # noqa: F401,F403
from . import resnet, others


def get_model(name, **kwargs):
    """Return a model by name, e.g. ``get_model('resnet50_v1b', layout='NHWC')``."""
    models = {k: v for k, v in list(resnet.__dict__.items()) + list(others.__dict__.items())
              if callable(v) and k[0].islower() and not k.startswith('get_') and not k.startswith('_')}
    models.update({'inceptionv3': others.inception_v3, 'squeezenet1.0': others.squeezenet1_0,
                   'squeezenet1.1': others.squeezenet1_1, 'mobilenet1.0': others.mobilenet1_0,
                   'mobilenet0.75': others.mobilenet0_75, 'mobilenet0.5': others.mobilenet0_5,
                   'mobilenet0.25': others.mobilenet0_25, 'mobilenetv2_1.0': others.mobilenet_v2_1_0,
                   'mobilenetv2_0.75': others.mobilenet_v2_0_75, 'mobilenetv2_0.5': others.mobilenet_v2_0_5,
                   'mobilenetv2_0.25': others.mobilenet_v2_0_25})
    name = name.lower()
    if name not in models:
        raise ValueError('Model %s is not supported. Available options are\n\t%s' % (
            name, '\n\t'.join(sorted(models.keys()))))
    return models[name](**kwargs)
