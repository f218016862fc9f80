"""Post-training INT8 quantization (parity: python/mxnet/contrib/quantization.py).

``quantize_model(sym, arg_params, aux_params, ...)`` rewrites an fp32 graph:
Convolution / FullyConnected become ``_contrib_quantized_*`` fed by
``quantize_v2`` nodes; ReLU / Pooling / Flatten between quantized ops stay in
int8; ``requantize`` narrows int32 results back to int8 using calibrated
ranges; ``dequantize`` returns to fp32 wherever an fp32 consumer (or a graph
output) needs it.  Calibration modes: ``none`` (ranges computed on the fly),
``naive`` (min/max over the calibration data) and ``entropy`` (KL-divergence
optimal thresholds over 8001-bin histograms).  ``quantize_net`` does the same
for a Gluon HybridBlock and returns a SymbolBlock.
"""
import logging

import numpy as np

from .. import ndarray as nd
from .. import symbol as sym_mod
from ..base import MXNetError
from ..context import cpu

__all__ = ['quantize_model', 'quantize_graph', 'quantize_net', 'quantize_net_v2', 'calib_graph',
           'combine_histogram', 'get_optimal_threshold']

_QUANTIZABLE = ('Convolution', 'FullyConnected')
_INT8_PASSTHROUGH = {'Activation': '_contrib_quantized_act', 'Pooling': '_contrib_quantized_pooling',
                     'Flatten': '_contrib_quantized_flatten', 'flatten': '_contrib_quantized_flatten'}


def _entry_name(node, idx):
    if node.op is None:
        return node.name
    return '%s_output' % node.name if node.num_outputs() == 1 else '%s_output%d' % (node.name, idx)


def quantize_graph(sym, excluded_sym_names=None, excluded_op_names=None, calib_ranges=None,
                   quantized_dtype='int8', quantize_mode='full'):
    """Return the quantized symbol.  ``calib_ranges``: {fp32 entry name: (min, max)}."""
    from ..symbol.symbol import _Node, Symbol
    excluded = set(excluded_sym_names or [])
    excluded_ops = set(excluded_op_names or [])
    calib_ranges = calib_ranges or {}
    src = sym_mod.load_json(sym.tojson())
    order = src._topo()
    qmap = {}        # (id(node), idx) of the fp32 graph -> (q entry, min entry, max entry)
    fmap = {}        # (id(node), idx) -> fp32 entry in the new graph
    deq_cache = {}
    counter = [0]

    def uniq(base):
        counter[0] += 1
        return '%s%d' % (base, counter[0]) if False else base

    def fp32_of(entry):
        """fp32 version of an old-graph entry (dequantizing if it only exists quantized)."""
        key = (id(entry[0]), entry[1])
        if key in fmap:
            return fmap[key]
        q, mn, mx = qmap[key]
        if key not in deq_cache:
            d = _Node('_contrib_dequantize', '%s_dequantize' % entry[0].name, {'out_type': 'float32'}, [q, mn, mx])
            deq_cache[key] = (d, 0)
        fmap[key] = deq_cache[key]
        return fmap[key]

    def quant_of(entry, name):
        key = (id(entry[0]), entry[1])
        if key in qmap:
            return qmap[key]
        attrs = {'out_type': 'int8'}
        rng = calib_ranges.get(_entry_name(entry[0], entry[1]))
        if rng is not None:
            attrs['min_calib_range'] = repr(float(rng[0]))
            attrs['max_calib_range'] = repr(float(rng[1]))
        qn = _Node('_contrib_quantize_v2', '%s_quantize' % name, attrs, [fp32_of(entry)])
        qmap[key] = ((qn, 0), (qn, 1), (qn, 2))
        return qmap[key]

    for n in order:
        if n.op is None:
            fmap[(id(n), 0)] = (n, 0)
            continue
        ins_fp = n.inputs
        quantizable = (n.op in _QUANTIZABLE and n.name not in excluded and n.op not in excluded_ops)
        passthrough = (n.op in _INT8_PASSTHROUGH and n.name not in excluded
                       and (id(ins_fp[0][0]), ins_fp[0][1]) in qmap and (id(ins_fp[0][0]), ins_fp[0][1]) not in fmap
                       and (n.op != 'Activation' or n.attrs.get('act_type') == 'relu')
                       and (n.op != 'Pooling' or n.attrs.get('pool_type', 'max') in ('max', 'avg')))
        if quantizable:
            p = n.parsed()
            no_bias = bool(p.get('no_bias', False))
            data_q = quant_of(ins_fp[0], n.name + '_data')
            w_q = quant_of(ins_fp[1], ins_fp[1][0].name)
            inputs = [data_q[0], w_q[0]]
            rng_inputs = [data_q[1], data_q[2], w_q[1], w_q[2]]
            if not no_bias and len(ins_fp) > 2:
                b_q = quant_of(ins_fp[2], ins_fp[2][0].name)
                inputs.append(b_q[0])
                rng_inputs += [b_q[1], b_q[2]]
            attrs = {k: v for k, v in n.attrs.items() if not (k.startswith('__') and k.endswith('__'))}
            qop = '_contrib_quantized_conv' if n.op == 'Convolution' else '_contrib_quantized_fully_connected'
            qn = _Node(qop, 'quantized_' + n.name, attrs, inputs + rng_inputs)
            rattrs = {'out_type': 'int8'}
            rng = calib_ranges.get(_entry_name(n, 0))
            if rng is not None:
                rattrs['min_calib_range'] = repr(float(rng[0]))
                rattrs['max_calib_range'] = repr(float(rng[1]))
            rq = _Node('_contrib_requantize', n.name + '_requantize', rattrs, [(qn, 0), (qn, 1), (qn, 2)])
            qmap[(id(n), 0)] = ((rq, 0), (rq, 1), (rq, 2))
            continue
        if (n.op == 'BatchNorm' and quantize_mode == 'full' and n.name not in excluded
                and n.op not in excluded_ops and n.num_visible_outputs() == 1):
            # int8 BatchNorm (inference): quantized input, fp32 statistics, calibrated int8 output
            data_q = quant_of(ins_fp[0], n.name + '_data')
            attrs = {k: v for k, v in n.attrs.items() if not (k.startswith('__') and k.endswith('__'))}
            rng = calib_ranges.get(_entry_name(n, 0))
            if rng is not None:
                attrs['min_calib_range'] = repr(float(rng[0]))
                attrs['max_calib_range'] = repr(float(rng[1]))
            qn = _Node('_contrib_quantized_batch_norm', 'quantized_' + n.name, attrs,
                       [data_q[0]] + [fp32_of(e) for e in ins_fp[1:5]] + [data_q[1], data_q[2]])
            qmap[(id(n), 0)] = ((qn, 0), (qn, 1), (qn, 2))
            continue
        if passthrough:
            q, mn, mx = qmap[(id(ins_fp[0][0]), ins_fp[0][1])]
            attrs = {k: v for k, v in n.attrs.items() if not (k.startswith('__') and k.endswith('__'))}
            if n.op in ('Flatten', 'flatten'):
                attrs = {}
            qn = _Node(_INT8_PASSTHROUGH[n.op], 'quantized_' + n.name, attrs, [q, mn, mx])
            qmap[(id(n), 0)] = ((qn, 0), (qn, 1), (qn, 2))
            continue
        new_inputs = [fp32_of(e) for e in ins_fp]
        nn_ = _Node(n.op, n.name, dict(n.attrs), new_inputs)
        for i in range(n.num_outputs()):
            fmap[(id(n), i)] = (nn_, i)
    outs = [fp32_of(e) for e in src._outputs]
    return Symbol(outs)


def _collect_ranges(sym, arg_params, aux_params, calib_data, num_calib_examples, ctx, data_names, label_names,
                    mode):
    from ..module import Module
    internals = sym.get_internals()
    mod = Module(sym, data_names=data_names, label_names=label_names or None, context=ctx)
    mod.bind(calib_data.provide_data, calib_data.provide_label if label_names else None, for_training=False)
    mod.set_params(arg_params, aux_params, allow_missing=False)
    stats = {}
    hists = {}

    def cb(name, arr):
        a = nd.NDArray(arr).asnumpy()
        if not np.issubdtype(a.dtype, np.floating):
            return
        mn, mx = float(a.min()), float(a.max())
        if name in stats:
            stats[name] = (min(stats[name][0], mn), max(stats[name][1], mx))
        else:
            stats[name] = (mn, mx)
        if mode == 'entropy':
            th = max(abs(mn), abs(mx))
            if name in hists:
                hists[name] = combine_histogram(hists[name], a, mn, mx, th)
            else:
                hist, edges = np.histogram(a, bins=8001, range=(-th, th))
                hists[name] = (hist, edges, mn, mx, th)
    for exe in mod._exec_group.execs:
        exe.set_monitor_callback(cb)
    seen = 0
    calib_data.reset()
    for batch in calib_data:
        mod.forward(batch, is_train=False)
        seen += batch.data[0].shape[0]
        if num_calib_examples is not None and seen >= num_calib_examples:
            break
    # inputs (data variables) ranges too
    if mode == 'entropy':
        ranges = {}
        for name, (hist, edges, mn, mx, th) in hists.items():
            t = get_optimal_threshold((hist, edges, mn, mx, th))
            ranges[name] = (-t, t)
        return ranges
    return stats


def combine_histogram(old_hist, arr, new_min, new_max, new_th):
    """Merge ``arr`` into an existing (hist, edges, min, max, th) histogram, widening the range if needed."""
    (old_hist, old_edges, old_min, old_max, old_th) = old_hist
    if new_th <= old_th:
        hist, _ = np.histogram(arr, bins=len(old_hist), range=(-old_th, old_th))
        return (old_hist + hist, old_edges, min(old_min, new_min), max(old_max, new_max), old_th)
    old_num_bins = len(old_hist)
    old_step = 2 * old_th / old_num_bins
    half_increased_bins = int((new_th - old_th) // old_step + 1)
    new_num_bins = half_increased_bins * 2 + old_num_bins
    new_th = half_increased_bins * old_step + old_th
    hist, hist_edges = np.histogram(arr, bins=new_num_bins, range=(-new_th, new_th))
    hist[half_increased_bins:new_num_bins - half_increased_bins] += old_hist
    return (hist, hist_edges, min(old_min, new_min), max(old_max, new_max), new_th)


def _smooth(p, eps=0.0001):
    is_zeros = (p == 0).astype(np.float64)
    is_nonzeros = (p != 0).astype(np.float64)
    n_zeros = is_zeros.sum()
    n_nonzeros = p.size - n_zeros
    if not n_nonzeros:
        raise ValueError('The discrete probability distribution is malformed. All entries are 0.')
    eps1 = eps * float(n_zeros) / float(n_nonzeros)
    hist = p.astype(np.float64)
    hist += eps * is_zeros + (-eps1) * is_nonzeros
    return hist


def get_optimal_threshold(hist_data, quantized_dtype='int8', num_quantized_bins=255):
    """Threshold minimising KL(P || Q) between the clipped fp32 histogram P and its int8 quantisation Q."""
    hist, hist_edges, min_val, max_val, _ = hist_data
    hist, hist_edges = np.asarray(hist), np.asarray(hist_edges)
    num_bins = len(hist)
    assert num_bins % 2 == 1
    if min_val >= 0 and quantized_dtype in ('auto', 'uint8'):
        num_quantized_bins = num_quantized_bins * 2 + 1
    zero_bin_idx = num_bins // 2
    num_half_quantized_bins = num_quantized_bins // 2
    best_div, best_th = np.inf, hist_edges[-1]
    for i in range(num_quantized_bins // 2, num_bins // 2 + 1, max(1, (num_bins // 2) // 200)):
        p_bin_idx_start = zero_bin_idx - i
        p_bin_idx_stop = zero_bin_idx + i + 1
        sliced = hist[p_bin_idx_start:p_bin_idx_stop].astype(np.float64)
        p = sliced.copy()
        p[0] += hist[:p_bin_idx_start].sum()
        p[-1] += hist[p_bin_idx_stop:].sum()
        is_nonzeros = (p != 0).astype(np.int64)
        num_merged_bins = sliced.size // num_quantized_bins
        quantized_bins = np.zeros(num_quantized_bins, dtype=np.float64)
        for j in range(num_quantized_bins):
            start = j * num_merged_bins
            stop = start + num_merged_bins
            quantized_bins[j] = sliced[start:stop].sum()
        quantized_bins[-1] += sliced[num_quantized_bins * num_merged_bins:].sum()
        q = np.zeros(sliced.size, dtype=np.float64)
        for j in range(num_quantized_bins):
            start = j * num_merged_bins
            stop = -1 if j == num_quantized_bins - 1 else start + num_merged_bins
            norm = is_nonzeros[start:stop].sum()
            if norm != 0:
                q[start:stop] = float(quantized_bins[j]) / float(norm)
        q[p == 0] = 0
        try:
            ps, qs = _smooth(p), _smooth(q)
        except ValueError:
            continue
        ps /= ps.sum()
        qs /= qs.sum()
        div = float(np.sum(ps * np.log(ps / qs)))
        if div < best_div:
            best_div = div
            best_th = hist_edges[p_bin_idx_stop]
    return float(best_th)


def _smooth_distribution(p, eps=0.0001):
    """Reference-named helper: move ``eps`` of mass onto the zero bins of a histogram (ValueError when
    every bin is zero)."""
    return _smooth(np.asarray(p), eps)


def _get_optimal_threshold(hist_data, quantized_dtype, num_quantized_bins=255):
    """(min, max, threshold, divergence) of the KL-optimal threshold (reference return layout)."""
    th = get_optimal_threshold(hist_data, quantized_dtype, num_quantized_bins)
    return hist_data[2], hist_data[3], th, None


def _get_optimal_thresholds(hist_dict, quantized_dtype, num_quantized_bins=255, logger=None):
    """{name: (-th, th)} for a dict of (hist, edges, min, max, th) histograms."""
    out = {}
    for name, hist in hist_dict.items():
        th = get_optimal_threshold(hist, quantized_dtype, num_quantized_bins)
        out[name] = (-th, th)
        if logger is not None:
            logger.debug('layer=%s, min_val=%f, max_val=%f, th=%f', name, hist[2], hist[3], th)
    return out


def calib_graph(qsym, arg_params, aux_params, collector=None, calib_mode='entropy', quantized_dtype='int8',
                logger=logging):
    return qsym, arg_params, aux_params


def quantize_model(sym, arg_params, aux_params, data_names=('data',), label_names=('softmax_label',), ctx=cpu(),
                   excluded_sym_names=None, excluded_op_names=None, calib_mode='entropy', calib_data=None,
                   num_calib_examples=None, quantized_dtype='int8', quantize_mode='smart', logger=logging):
    """Quantize an fp32 model; returns (qsym, qarg_params, aux_params)."""
    if quantized_dtype not in ('int8', 'auto', 'uint8'):
        raise ValueError('unknown quantized_dtype %s' % quantized_dtype)
    ranges = None
    if calib_mode != 'none':
        if calib_data is None:
            raise ValueError('calib_data must be provided when calib_mode=%s' % calib_mode)
        if calib_mode not in ('naive', 'entropy'):
            raise ValueError('unknown calibration mode %s' % calib_mode)
        ranges = _collect_ranges(sym, arg_params, aux_params, calib_data, num_calib_examples, ctx,
                                 list(data_names), list(label_names or []), calib_mode)
        logger.info('Collected calibration ranges for %d tensors (%s)', len(ranges), calib_mode)
    qsym = quantize_graph(sym, excluded_sym_names, excluded_op_names, ranges, quantized_dtype,
                          quantize_mode=quantize_mode)
    return qsym, dict(arg_params), dict(aux_params)


def quantize_net_v2(network, quantized_dtype='auto', quantize_mode='full', exclude_layers=None,
                    exclude_layers_match=None, exclude_operators=None, calib_data=None, data_shapes=None,
                    calib_mode='none', num_calib_examples=None, ctx=cpu(), logger=logging):
    """Quantize a Gluon HybridBlock; returns a SymbolBlock running the int8 graph."""
    from ..gluon.block import SymbolBlock
    from .. import io as mxio
    network.hybridize()
    if calib_data is not None and not isinstance(calib_data, mxio.DataIter):
        from ..gluon.data import DataLoader
        if isinstance(calib_data, DataLoader):
            calib_data = _DataLoaderIter(calib_data, data_shapes)
    if data_shapes is None:
        if calib_data is None:
            raise ValueError('data_shapes required when no calib_data is given')
        data_shapes = calib_data.provide_data
    shapes = [d[1] if isinstance(d, tuple) else d.shape for d in data_shapes]
    network(*[nd.zeros(s, ctx=ctx) for s in shapes])
    inputs, out = network._cached_graph
    params = network.collect_params()
    arg_params = {k: v.data() for k, v in params.items() if k in out.list_arguments()}
    aux_params = {k: v.data() for k, v in params.items() if k in out.list_auxiliary_states()}
    excluded = list(exclude_layers or [])
    if exclude_layers_match:
        import re
        for n in out._topo():
            if n.op is not None and any(re.match(p, n.name) for p in exclude_layers_match):
                excluded.append(n.name)
    data_names = [i.name for i in inputs]
    qsym, qarg, qaux = quantize_model(out, arg_params, aux_params, data_names=data_names, label_names=None,
                                      ctx=ctx, excluded_sym_names=excluded, excluded_op_names=exclude_operators,
                                      calib_mode=calib_mode, calib_data=calib_data,
                                      num_calib_examples=num_calib_examples, quantized_dtype=quantized_dtype,
                                      logger=logger)
    net = SymbolBlock(qsym, inputs)
    rp = net.collect_params()
    for name, p in rp.items():
        src = qarg.get(name, qaux.get(name))
        if src is not None:
            p._load_init(src, ctx)
    return net


def quantize_net(network, quantized_dtype='auto', quantize_mode='full', exclude_layers=None,
                 exclude_layers_match=None, exclude_operators=None, calib_data=None, data_shapes=None,
                 calib_mode='none', num_calib_examples=None, ctx=cpu(), logger=logging):
    return quantize_net_v2(network, quantized_dtype, quantize_mode, exclude_layers, exclude_layers_match,
                           exclude_operators, calib_data, data_shapes, calib_mode, num_calib_examples, ctx, logger)


class _DataLoaderIter:
    """Adapt a gluon DataLoader to the DataIter interface used by calibration."""

    def __init__(self, loader, data_shapes):
        from .. import io as mxio
        self.loader = loader
        first = next(iter(loader))
        x = first[0] if isinstance(first, (list, tuple)) else first
        self.provide_data = data_shapes or [mxio.DataDesc('data', x.shape)]
        self.provide_label = None
        self.batch_size = x.shape[0]

    def reset(self):
        pass

    def __iter__(self):
        from .. import io as mxio
        for b in self.loader:
            x = b[0] if isinstance(b, (list, tuple)) else b
            yield mxio.DataBatch([x], None)
