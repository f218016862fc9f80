"""Operator precision classes for AMP on MI355X.

* ``LP16``: GEMM-shaped ops that run on the MFMA matrix cores — fp16/bf16
  inputs, fp32 accumulation (2.5 PF dense bf16 vs 157 TF fp32 vector).
* ``FP32``: numerically sensitive ops (exponentials, logs, reductions of
  many terms, normalisations computed from scratch, losses).
* ``WIDEST``: multi-input elementwise ops whose inputs must share a dtype;
  they run in the widest input type.
* ``CONDITIONAL_FP32``: (op, param, values) that need fp32 only for some
  parameter values.
Everything else is dtype-neutral and runs in whatever dtype arrives.
Parity: python/mxnet/contrib/amp/lists/symbol_{fp16,bf16}.py (same classes).
"""

LP16 = ['Convolution', 'Deconvolution', 'FullyConnected', 'RNN', 'dot', 'batch_dot', '_linalg_gemm', '_linalg_gemm2',
        'linalg_gemm', 'linalg_gemm2', '_contrib_interleaved_matmul_selfatt_qk',
        '_contrib_interleaved_matmul_selfatt_valatt', '_contrib_interleaved_matmul_encdec_qk',
        '_contrib_interleaved_matmul_encdec_valatt']

FP32 = ['exp', 'expm1', 'log', 'log10', 'log2', 'log1p', 'pow', '_power', 'power', 'broadcast_power', 'rsqrt',
        'rcbrt', 'reciprocal', 'square', 'sqrt', 'cbrt', 'arccos', 'arcsin', 'arctanh', 'arccosh', 'cosh', 'sinh',
        'tan', 'erfinv', 'gamma', 'gammaln', 'digamma',
        'softmax', 'log_softmax', 'softmin', 'SoftmaxActivation', 'softmax_cross_entropy', 'SoftmaxOutput',
        'LinearRegressionOutput', 'LogisticRegressionOutput', 'MAERegressionOutput', 'CTCLoss', 'ctc_loss',
        'MakeLoss', 'make_loss', 'SVMOutput',
        'norm', 'L2Normalization', 'LayerNorm', 'GroupNorm', 'InstanceNorm', 'LRN', 'moments',
        'sum', 'sum_axis', 'nansum', 'prod', 'nanprod', 'mean', 'topk', 'sort', 'argsort', 'cumsum',
        '_contrib_MultiBoxDetection', '_contrib_MultiBoxPrior', '_contrib_MultiBoxTarget', '_contrib_box_nms',
        '_contrib_ROIAlign', 'ROIPooling', 'Correlation', 'BilinearSampler', 'GridGenerator', 'SpatialTransformer']

WIDEST = ['elemwise_add', 'elemwise_sub', 'elemwise_mul', 'elemwise_div', '_plus', '_Plus', '_add', '_minus',
          '_Minus', '_sub', '_mul', '_Mul', '_div', '_Div', '_mod', '_Mod', '_maximum', '_minimum', '_hypot',
          '_equal', '_not_equal', '_greater', '_greater_equal', '_lesser', '_lesser_equal',
          'broadcast_add', 'broadcast_plus', 'broadcast_sub', 'broadcast_minus', 'broadcast_mul', 'broadcast_div',
          'broadcast_mod', 'broadcast_maximum', 'broadcast_minimum', 'broadcast_hypot', 'broadcast_equal',
          'broadcast_not_equal', 'broadcast_greater', 'broadcast_greater_equal', 'broadcast_lesser',
          'broadcast_lesser_equal', 'Concat', 'concat', 'stack', 'add_n', 'ElementWiseSum', 'where',
          '_contrib_BatchNormAddReLU', 'BatchNormAddReLU']

CONDITIONAL_FP32 = [('Activation', 'act_type', ['softrelu']), ('LeakyReLU', 'act_type', ['elu', 'selu'])]

LOSS_OUTPUT = ['SoftmaxOutput', 'LinearRegressionOutput', 'LogisticRegressionOutput', 'MAERegressionOutput']
