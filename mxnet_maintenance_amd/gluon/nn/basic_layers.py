"""Basic Gluon layers.

Parity: python/mxnet/gluon/nn/basic_layers.py (Sequential, HybridSequential,
Dense, Dropout, BatchNorm, BatchNormReLU, Embedding, Flatten, InstanceNorm,
LayerNorm, GroupNorm, Lambda, HybridLambda).
"""
import warnings

import numpy as np

from ... import initializer
from ...base import numeric_types
from ..block import Block, HybridBlock
from ..utils import _indent

__all__ = ['Sequential', 'HybridSequential', 'Dense', 'Dropout', 'Embedding', 'BatchNorm', 'BatchNormReLU',
           'InstanceNorm', 'LayerNorm', 'GroupNorm', 'Flatten', 'Lambda', 'HybridLambda']


class Sequential(Block):
    """Stacks Blocks sequentially."""

    def __init__(self, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)

    def add(self, *blocks):
        for block in blocks:
            self.register_child(block)

    def forward(self, x, *args):
        for block in self._children.values():
            x = block(x, *args)
            args = []
            if isinstance(x, (tuple, list)):
                args = x[1:]
                x = x[0]
        if args:
            x = tuple([x] + list(args))
        return x

    def __repr__(self):
        s = '{name}(\n{modstr}\n)'
        modstr = '\n'.join(['  ({key}): {block}'.format(key=key, block=_indent(block.__repr__(), 2))
                            for key, block in self._children.items()])
        return s.format(name=self.__class__.__name__, modstr=modstr)

    def __getitem__(self, key):
        layers = list(self._children.values())[key]
        if isinstance(layers, list):
            net = type(self)(prefix=self._prefix)
            with net.name_scope():
                net.add(*layers)
            return net
        return layers

    def __len__(self):
        return len(self._children)

    def hybridize(self, active=True, **kwargs):
        if self._children and all(isinstance(c, HybridBlock) for c in self._children.values()):
            warnings.warn("All children of this Sequential layer '%s' are HybridBlocks. Consider using "
                          "HybridSequential for the best performance." % self.prefix, stacklevel=2)
        super().hybridize(active, **kwargs)


class HybridSequential(HybridBlock):
    """Stacks HybridBlocks sequentially."""

    def __init__(self, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)

    def add(self, *blocks):
        for block in blocks:
            self.register_child(block)

    def hybrid_forward(self, F, x, *args):
        for block in self._children.values():
            x = block(x, *args)
            args = []
            if isinstance(x, (tuple, list)):
                args = x[1:]
                x = x[0]
        if args:
            x = tuple([x] + list(args))
        return x

    def __repr__(self):
        s = '{name}(\n{modstr}\n)'
        modstr = '\n'.join(['  ({key}): {block}'.format(key=key, block=_indent(block.__repr__(), 2))
                            for key, block in self._children.items()])
        return s.format(name=self.__class__.__name__, modstr=modstr)

    def __getitem__(self, key):
        layers = list(self._children.values())[key]
        if isinstance(layers, list):
            net = type(self)(prefix=self._prefix)
            with net.name_scope():
                net.add(*layers)
            return net
        return layers

    def __len__(self):
        return len(self._children)


class Dense(HybridBlock):
    """Fully-connected layer: ``activation(dot(input, weight.T) + bias)``."""

    def __init__(self, units, activation=None, use_bias=True, flatten=True, dtype='float32',
                 weight_initializer=None, bias_initializer='zeros', in_units=0, **kwargs):
        super().__init__(**kwargs)
        self._flatten = flatten
        with self.name_scope():
            self._units = units
            self._in_units = in_units
            self.weight = self.params.get('weight', shape=(units, in_units), init=weight_initializer,
                                          dtype=dtype, allow_deferred_init=True)
            if use_bias:
                self.bias = self.params.get('bias', shape=(units,), init=bias_initializer, dtype=dtype,
                                            allow_deferred_init=True)
            else:
                self.bias = None
            if activation is not None:
                from .activations import Activation
                self.act = Activation(activation, prefix=activation + '_')
            else:
                self.act = None

    def hybrid_forward(self, F, x, weight, bias=None):
        act = F.FullyConnected(x, weight, bias, no_bias=bias is None, num_hidden=self._units,
                               flatten=self._flatten, name='fwd')
        if self.act is not None:
            act = self.act(act)
        return act

    def __repr__(self):
        s = '{name}({layout}, {act})'
        shape = self.weight.shape
        return s.format(name=self.__class__.__name__, act=self.act if self.act else 'linear',
                        layout='{0} -> {1}'.format(shape[1] if shape[1] else None, shape[0]))


class Dropout(HybridBlock):
    def __init__(self, rate, axes=(), **kwargs):
        super().__init__(**kwargs)
        self._rate = rate
        self._axes = axes

    def hybrid_forward(self, F, x):
        if self._rate > 0:
            return F.Dropout(x, p=self._rate, axes=self._axes, name='fwd', cudnn_off=False)
        return F.identity(x)

    def __repr__(self):
        s = '{name}(p = {_rate}, axes={_axes})'
        return s.format(name=self.__class__.__name__, **self.__dict__)


class _BatchNorm(HybridBlock):
    def __init__(self, axis=1, momentum=0.9, epsilon=1e-5, center=True, scale=True, use_global_stats=False,
                 fuse_relu=False, beta_initializer='zeros', gamma_initializer='ones',
                 running_mean_initializer='zeros', running_variance_initializer='ones', in_channels=0, **kwargs):
        super().__init__(**kwargs)
        self._kwargs = {'axis': axis, 'eps': epsilon, 'momentum': momentum, 'fix_gamma': not scale,
                        'use_global_stats': use_global_stats}
        self.fuse_relu = fuse_relu
        if in_channels != 0:
            self.in_channels = in_channels
        self.gamma = self.params.get('gamma', grad_req='write' if scale else 'null', shape=(in_channels,),
                                     init=gamma_initializer, allow_deferred_init=True, differentiable=scale)
        self.beta = self.params.get('beta', grad_req='write' if center else 'null', shape=(in_channels,),
                                    init=beta_initializer, allow_deferred_init=True, differentiable=center)
        self.running_mean = self.params.get('running_mean', grad_req='null', shape=(in_channels,),
                                            init=running_mean_initializer, allow_deferred_init=True,
                                            differentiable=False)
        self.running_var = self.params.get('running_var', grad_req='null', shape=(in_channels,),
                                           init=running_variance_initializer, allow_deferred_init=True,
                                           differentiable=False)

    def cast(self, dtype):
        from ...base import dtype_name
        if dtype_name(dtype) in ('float16', 'bfloat16'):
            dtype = 'float32'   # BatchNorm statistics and affine params stay fp32
        super().cast(dtype)

    def hybrid_forward(self, F, x, gamma, beta, running_mean, running_var):
        if self.fuse_relu:
            return F.contrib.BatchNormWithReLU(x, gamma, beta, running_mean, running_var, name='fwd',
                                               **self._kwargs)
        return F.BatchNorm(x, gamma, beta, running_mean, running_var, name='fwd', **self._kwargs)

    def __repr__(self):
        s = '{name}({content}'
        in_channels = self.gamma.shape[0]
        s += ', in_channels={0}'.format(in_channels if in_channels else None)
        s += ')'
        return s.format(name=self.__class__.__name__,
                        content=', '.join(['='.join([k, v.__repr__()]) for k, v in self._kwargs.items()]))


class BatchNorm(_BatchNorm):
    """Batch normalization (Ioffe & Szegedy, 2015)."""

    def __init__(self, axis=1, momentum=0.9, epsilon=1e-5, center=True, scale=True, use_global_stats=False,
                 beta_initializer='zeros', gamma_initializer='ones', running_mean_initializer='zeros',
                 running_variance_initializer='ones', in_channels=0, **kwargs):
        super().__init__(axis=axis, momentum=momentum, epsilon=epsilon, center=center, scale=scale,
                         use_global_stats=use_global_stats, fuse_relu=False, beta_initializer=beta_initializer,
                         gamma_initializer=gamma_initializer, running_mean_initializer=running_mean_initializer,
                         running_variance_initializer=running_variance_initializer, in_channels=in_channels,
                         **kwargs)


class BatchNormReLU(_BatchNorm):
    """Batch normalization fused with ReLU (one HIP kernel on gfx950)."""

    def __init__(self, axis=1, momentum=0.9, epsilon=1e-5, center=True, scale=True, use_global_stats=False,
                 beta_initializer='zeros', gamma_initializer='ones', running_mean_initializer='zeros',
                 running_variance_initializer='ones', in_channels=0, **kwargs):
        super().__init__(axis=axis, momentum=momentum, epsilon=epsilon, center=center, scale=scale,
                         use_global_stats=use_global_stats, fuse_relu=True, beta_initializer=beta_initializer,
                         gamma_initializer=gamma_initializer, running_mean_initializer=running_mean_initializer,
                         running_variance_initializer=running_variance_initializer, in_channels=in_channels,
                         **kwargs)


class Embedding(HybridBlock):
    def __init__(self, input_dim, output_dim, dtype='float32', weight_initializer=None, sparse_grad=False,
                 **kwargs):
        super().__init__(**kwargs)
        grad_stype = 'row_sparse' if sparse_grad else 'default'
        self._kwargs = {'input_dim': input_dim, 'output_dim': output_dim, 'dtype': dtype,
                        'sparse_grad': sparse_grad}
        self.weight = self.params.get('weight', shape=(input_dim, output_dim), init=weight_initializer,
                                      dtype=dtype, allow_deferred_init=True, grad_stype=grad_stype)

    def hybrid_forward(self, F, x, weight):
        return F.Embedding(x, weight, name='fwd', **self._kwargs)

    def __repr__(self):
        s = '{block_name}({input_dim} -> {output_dim}, {dtype})'
        return s.format(block_name=self.__class__.__name__, **self._kwargs)


class Flatten(HybridBlock):
    def __init__(self, **kwargs):
        super().__init__(**kwargs)

    def hybrid_forward(self, F, x):
        return F.Flatten(x)

    def __repr__(self):
        return self.__class__.__name__


class InstanceNorm(HybridBlock):
    def __init__(self, axis=1, epsilon=1e-5, center=True, scale=False, beta_initializer='zeros',
                 gamma_initializer='ones', in_channels=0, **kwargs):
        super().__init__(**kwargs)
        self._kwargs = {'eps': epsilon, 'axis': axis, 'center': center, 'scale': scale}
        self._axis = axis
        self._epsilon = epsilon
        self.gamma = self.params.get('gamma', grad_req='write' if scale else 'null', shape=(in_channels,),
                                     init=gamma_initializer, allow_deferred_init=True)
        self.beta = self.params.get('beta', grad_req='write' if center else 'null', shape=(in_channels,),
                                    init=beta_initializer, allow_deferred_init=True)

    def hybrid_forward(self, F, x, gamma, beta):
        if self._axis == 1:
            return F.InstanceNorm(x, gamma, beta, name='fwd', eps=self._epsilon)
        x = x.swapaxes(1, self._axis)
        return F.InstanceNorm(x, gamma, beta, name='fwd', eps=self._epsilon).swapaxes(1, self._axis)

    def __repr__(self):
        s = '{name}({content}'
        in_channels = self.gamma.shape[0]
        s += ', in_channels={0}'.format(in_channels)
        s += ')'
        return s.format(name=self.__class__.__name__,
                        content=', '.join(['='.join([k, v.__repr__()]) for k, v in self._kwargs.items()]))


class LayerNorm(HybridBlock):
    def __init__(self, axis=-1, epsilon=1e-5, center=True, scale=True, beta_initializer='zeros',
                 gamma_initializer='ones', in_channels=0, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)
        self._kwargs = {'eps': epsilon, 'axis': axis, 'center': center, 'scale': scale}
        self._axis = axis
        self._epsilon = epsilon
        self._center = center
        self._scale = scale
        self.gamma = self.params.get('gamma', grad_req='write' if scale else 'null', shape=(in_channels,),
                                     init=gamma_initializer, allow_deferred_init=True)
        self.beta = self.params.get('beta', grad_req='write' if center else 'null', shape=(in_channels,),
                                    init=beta_initializer, allow_deferred_init=True)

    def hybrid_forward(self, F, data, gamma, beta):
        return F.LayerNorm(data, gamma=gamma, beta=beta, axis=self._axis, eps=self._epsilon)

    def __repr__(self):
        s = '{name}({content}'
        in_channels = self.gamma.shape[0]
        s += ', in_channels={0}'.format(in_channels)
        s += ')'
        return s.format(name=self.__class__.__name__,
                        content=', '.join(['='.join([k, v.__repr__()]) for k, v in self._kwargs.items()]))


class GroupNorm(HybridBlock):
    def __init__(self, num_groups=1, epsilon=1e-5, center=True, scale=True, beta_initializer='zeros',
                 gamma_initializer='ones', prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)
        self._kwargs = {'eps': epsilon, 'num_groups': num_groups, 'center': center, 'scale': scale}
        self._num_groups = num_groups
        self._epsilon = epsilon
        self._center = center
        self._scale = scale
        self.gamma = self.params.get('gamma', grad_req='write' if scale else 'null', shape=(num_groups,),
                                     init=gamma_initializer, allow_deferred_init=True)
        self.beta = self.params.get('beta', grad_req='write' if center else 'null', shape=(num_groups,),
                                    init=beta_initializer, allow_deferred_init=True)

    def hybrid_forward(self, F, data, gamma, beta):
        return F.GroupNorm(data, gamma=gamma, beta=beta, num_groups=self._num_groups, eps=self._epsilon)

    def __repr__(self):
        s = '{name}({content})'
        return s.format(name=self.__class__.__name__,
                        content=', '.join(['='.join([k, v.__repr__()]) for k, v in self._kwargs.items()]))


class Lambda(Block):
    def __init__(self, function, prefix=None):
        super().__init__(prefix=prefix)
        if isinstance(function, str):
            from ... import ndarray as nd
            assert hasattr(nd, function), 'Function name %s is not found in ndarray.' % function
            self._func_impl = getattr(nd, function)
        elif callable(function):
            self._func_impl = function
        else:
            raise ValueError('Unrecognized function in lambda: {} of type {}'.format(function, type(function)))

    def forward(self, *args):
        return self._func_impl(*args)

    def __repr__(self):
        return '{name}({function})'.format(name=self.__class__.__name__, function=self._func_impl.__name__)


class HybridLambda(HybridBlock):
    def __init__(self, function, prefix=None):
        super().__init__(prefix=prefix)
        if isinstance(function, str):
            from ... import ndarray as nd, symbol as sym
            assert hasattr(nd, function) and hasattr(sym, function), \
                'Function name %s is not found in symbol/ndarray.' % function
            func_dict = {sym: getattr(sym, function), nd: getattr(nd, function)}
            self._func = lambda F, *args: func_dict[F](*args)
            self._func_name = function
        elif callable(function):
            self._func = function
            self._func_name = function.__name__
        else:
            raise ValueError('Unrecognized function in lambda: {} of type {}'.format(function, type(function)))

    def hybrid_forward(self, F, x, *args):
        return self._func(F, x, *args)

    def __repr__(self):
        return '{name}({function})'.format(name=self.__class__.__name__, function=self._func_name)
