"""gluon.contrib.nn layers (parity: python/mxnet/gluon/contrib/nn/basic_layers.py)."""
from ... import nn
from ...block import Block, HybridBlock
from ....context import cpu

__all__ = ['Concurrent', 'HybridConcurrent', 'Identity', 'SparseEmbedding', 'SyncBatchNorm', 'PixelShuffle1D',
           'PixelShuffle2D', 'PixelShuffle3D']


class Concurrent(nn.Sequential):
    """Run children on the same input and concatenate their outputs along ``axis``."""

    def __init__(self, axis=-1, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)
        self.axis = axis

    def forward(self, x):
        from .... import ndarray as nd
        out = [block(x) for block in self._children.values()]
        return nd.concat(*out, dim=self.axis)


class HybridConcurrent(nn.HybridSequential):
    def __init__(self, axis=-1, prefix=None, params=None):
        super().__init__(prefix=prefix, params=params)
        self.axis = axis

    def hybrid_forward(self, F, x):
        out = [block(x) for block in self._children.values()]
        return F.concat(*out, dim=self.axis)


class Identity(HybridBlock):
    def hybrid_forward(self, F, x):
        return x


class SparseEmbedding(Block):
    """Embedding whose weight gradient is row_sparse (only looked-up rows are updated)."""

    def __init__(self, input_dim, output_dim, dtype='float32', weight_initializer=None, **kwargs):
        super().__init__(**kwargs)
        self._kwargs = {'input_dim': input_dim, 'output_dim': output_dim, 'dtype': dtype, 'sparse_grad': True}
        self.weight = self.params.get('weight', shape=(input_dim, output_dim), init=weight_initializer, dtype=dtype,
                                      grad_stype='row_sparse', stype='row_sparse')

    def forward(self, x):
        from .... import ndarray as nd
        weight = self.weight.row_sparse_data(x) if hasattr(self.weight, 'row_sparse_data') else self.weight.data()
        return nd.Embedding(x, weight, name='fwd', **self._kwargs)

    def __repr__(self):
        return '{block_name}({input_dim} -> {output_dim}, {dtype})'.format(block_name=self.__class__.__name__,
                                                                           **self._kwargs)


class SyncBatchNorm(nn.BatchNorm):
    """BatchNorm whose batch statistics are all-reduced across the data-parallel process group (RCCL)."""

    def __init__(self, in_channels=0, num_devices=None, momentum=0.9, epsilon=1e-5, center=True, scale=True,
                 use_global_stats=False, beta_initializer='zeros', gamma_initializer='ones',
                 running_mean_initializer='zeros', running_variance_initializer='ones', axis=1, **kwargs):
        super().__init__(axis=axis, momentum=momentum, epsilon=epsilon, center=center, scale=scale,
                         use_global_stats=use_global_stats, beta_initializer=beta_initializer,
                         gamma_initializer=gamma_initializer, running_mean_initializer=running_mean_initializer,
                         running_variance_initializer=running_variance_initializer, in_channels=in_channels,
                         **kwargs)
        num_devices = self._get_num_devices() if num_devices is None else num_devices
        self._kwargs = {'eps': epsilon, 'momentum': momentum, 'fix_gamma': not scale,
                        'use_global_stats': use_global_stats, 'ndev': num_devices, 'key': self.prefix, 'axis': axis}

    def _get_num_devices(self):
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_world_size()
        return 1

    def hybrid_forward(self, F, x, gamma, beta, running_mean, running_var):
        return F.contrib.SyncBatchNorm(x, gamma, beta, running_mean, running_var, name='fwd', **self._kwargs)


class PixelShuffle1D(HybridBlock):
    """(N, C*f, W) -> (N, C, W*f)."""

    def __init__(self, factor):
        super().__init__()
        self._factor = int(factor)

    def hybrid_forward(self, F, x):
        f = self._factor
        x = F.reshape(x, (0, -4, -1, f, 0))
        x = F.transpose(x, (0, 1, 3, 2))
        return F.reshape(x, (0, 0, -3))

    def __repr__(self):
        return '{}({})'.format(self.__class__.__name__, self._factor)


class PixelShuffle2D(HybridBlock):
    """(N, C*f1*f2, H, W) -> (N, C, H*f1, W*f2)."""

    def __init__(self, factor):
        super().__init__()
        try:
            self._factors = (int(factor),) * 2
        except TypeError:
            self._factors = tuple(int(fac) for fac in factor)
            assert len(self._factors) == 2, 'wrong length {}'.format(len(self._factors))

    def hybrid_forward(self, F, x):
        f1, f2 = self._factors
        x = F.reshape(x, (0, -4, -1, f1 * f2, 0, 0))
        x = F.reshape(x, (0, 0, -4, f1, f2, 0, 0))
        x = F.transpose(x, (0, 1, 4, 2, 5, 3))
        x = F.reshape(x, (0, 0, -3, -3))
        return x

    def __repr__(self):
        return '{}({})'.format(self.__class__.__name__, self._factors)


class PixelShuffle3D(HybridBlock):
    """(N, C*f1*f2*f3, D, H, W) -> (N, C, D*f1, H*f2, W*f3)."""

    def __init__(self, factor):
        super().__init__()
        try:
            self._factors = (int(factor),) * 3
        except TypeError:
            self._factors = tuple(int(fac) for fac in factor)
            assert len(self._factors) == 3, 'wrong length {}'.format(len(self._factors))

    def hybrid_forward(self, F, x):
        f1, f2, f3 = self._factors
        x = F.reshape(x, (0, -4, -1, f1 * f2 * f3, 0, 0, 0))
        x = F.swapaxes(x, 2, 3)
        x = F.reshape(x, (0, 0, 0, -4, f1, f2 * f3, 0, 0))
        x = F.reshape(x, (0, 0, -3, 0, 0, 0))
        x = F.swapaxes(x, 3, 4)
        x = F.reshape(x, (0, 0, 0, 0, -4, f2, f3, 0))
        x = F.reshape(x, (0, 0, 0, -3, 0, 0))
        x = F.swapaxes(x, 4, 5)
        x = F.reshape(x, (0, 0, 0, 0, -3))
        return x

    def __repr__(self):
        return '{}({})'.format(self.__class__.__name__, self._factors)
