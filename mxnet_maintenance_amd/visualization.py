"""Network visualisation (parity: python/mxnet/visualization.py).

``print_summary`` prints the layer table (output shapes, parameter counts,
inputs) of a Symbol; ``plot_network`` builds a Graphviz DOT description.
The ``graphviz`` Python package is used when importable; otherwise a small
stand-in object exposes ``source`` / ``save`` / ``render`` (writes the .dot).
"""
import copy
import json
import re

from .base import MXNetError
from .symbol import Symbol

__all__ = ['print_summary', 'plot_network']


def _str2tuple(string):
    return re.findall(r'\d+', string)


def print_summary(symbol, shape=None, line_length=120, positions=(.44, .64, .74, 1.)):
    """Print a summary of the network: layer (type), output shape, #params, previous layer."""
    if not isinstance(symbol, Symbol):
        raise TypeError('symbol must be Symbol')
    show_shape = False
    shape_dict = {}
    if shape is not None:
        show_shape = True
        interals = symbol.get_internals()
        _, out_shapes, _ = interals.infer_shape(**shape)
        if out_shapes is None:
            raise ValueError('Input shape is incomplete')
        shape_dict = dict(zip(interals.list_outputs(), out_shapes))
    conf = json.loads(symbol.tojson())
    nodes = conf['nodes']
    heads = set(conf['heads'][0])
    if positions[-1] <= 1:
        positions = [int(line_length * p) for p in positions]
    to_display = ['Layer (type)', 'Output Shape', 'Param #', 'Previous Layer']
    lines = []

    def print_row(fields, positions):
        line = ''
        for i, field in enumerate(fields):
            line += str(field)
            line = line[:positions[i]]
            line += ' ' * (positions[i] - len(line))
        lines.append(line)
    lines.append('_' * line_length)
    print_row(to_display, positions)
    lines.append('=' * line_length)

    def print_layer_summary(node, out_shape):
        op = node['op']
        pre_node = []
        pre_filter = 0
        if op != 'null':
            inputs = node['inputs']
            for item in inputs:
                input_node = nodes[item[0]]
                input_name = input_node['name']
                if input_node['op'] != 'null' or item[0] in heads:
                    pre_node.append(input_name)
                    if show_shape:
                        key = input_name + '_output' if input_node['op'] != 'null' else input_name
                        if key in shape_dict:
                            shp = shape_dict[key][1:]
                            pre_filter = pre_filter + int(shp[0]) if shp else pre_filter
        cur_param = 0
        attrs = node.get('attrs', node.get('param', {})) or {}
        if op == 'Convolution':
            num_group = int(attrs.get('num_group', '1'))
            cur_param = pre_filter * int(attrs['num_filter']) // num_group
            for k in _str2tuple(attrs['kernel']):
                cur_param *= int(k)
            if attrs.get('no_bias', 'False') not in ('True', 'true', '1'):
                cur_param += int(attrs['num_filter'])
        elif op == 'FullyConnected':
            if attrs.get('no_bias', 'False') in ('True', 'true', '1'):
                cur_param = pre_filter * int(attrs['num_hidden'])
            else:
                cur_param = (pre_filter + 1) * int(attrs['num_hidden'])
        elif op == 'BatchNorm':
            key = node['name'] + '_output'
            if show_shape and key in shape_dict:
                num_filter = shape_dict[key][1]
                cur_param = int(num_filter) * 2
        elif op == 'Embedding':
            cur_param = int(attrs['input_dim']) * int(attrs['output_dim'])
        if not pre_node:
            first_connection = ''
        else:
            first_connection = pre_node[0]
        fields = [node['name'] + '(' + op + ')', 'x'.join([str(x) for x in out_shape]), cur_param,
                  first_connection]
        print_row(fields, positions)
        for i in range(1, len(pre_node)):
            print_row(['', '', '', pre_node[i]], positions)
        return cur_param

    total_params = 0
    for i, node in enumerate(nodes):
        out_shape = []
        op = node['op']
        if op == 'null' and i > 0:
            continue
        if op != 'null' or i in heads:
            if show_shape:
                key = node['name'] + '_output' if op != 'null' else node['name']
                if key in shape_dict:
                    out_shape = shape_dict[key][1:]
        total_params += print_layer_summary(nodes[i], out_shape)
        if i == len(nodes) - 1:
            lines.append('=' * line_length)
        else:
            lines.append('_' * line_length)
    lines.append('Total params: %s' % total_params)
    lines.append('_' * line_length)
    print('\n'.join(lines))


class _Dot:
    """Minimal stand-in for graphviz.Digraph."""

    def __init__(self, name, fmt='pdf', node_attr=None):
        self.name = name
        self.format = fmt
        self.node_attr = node_attr or {}
        self.body = []

    @staticmethod
    def _attrs(kw):
        return ', '.join('%s="%s"' % (k, v) for k, v in kw.items())

    def node(self, name, label=None, **kw):
        if label is not None:
            kw['label'] = label
        self.body.append('  "%s" [%s]' % (name, self._attrs(kw)))

    def edge(self, tail, head, label=None, **kw):
        if label is not None:
            kw['label'] = label
        self.body.append('  "%s" -> "%s" [%s]' % (tail, head, self._attrs(kw)))

    @property
    def source(self):
        return 'digraph %s {\n  node [%s]\n%s\n}\n' % (self.name, self._attrs(self.node_attr), '\n'.join(self.body))

    def save(self, filename=None, directory=None):
        fn = filename or (self.name + '.gv')
        with open(fn, 'w') as f:
            f.write(self.source)
        return fn

    def render(self, filename=None, directory=None, view=False, cleanup=False, format=None):  # noqa: A002
        return self.save(filename)


def plot_network(symbol, title='plot', save_format='pdf', shape=None, dtype=None, node_attrs=None,
                 hide_weights=True):
    """Graph of the network (Digraph); parameter inputs hidden unless ``hide_weights=False``."""
    try:
        from graphviz import Digraph
    except ImportError:
        Digraph = None
    if not isinstance(symbol, Symbol):
        raise TypeError('symbol must be a Symbol')
    internals = symbol.get_internals()
    draw_shape = shape is not None
    shape_dict = {}
    if draw_shape:
        _, out_shapes, _ = internals.infer_shape(**shape)
        if out_shapes is None:
            raise ValueError('Input shape is incomplete')
        shape_dict = dict(zip(internals.list_outputs(), out_shapes))
    conf = json.loads(symbol.tojson())
    nodes = conf['nodes']
    node_attr = {'shape': 'box', 'fixedsize': 'true', 'width': '1.3', 'height': '0.8034', 'style': 'filled'}
    node_attr.update(node_attrs or {})
    dot = Digraph(name=title, format=save_format) if Digraph is not None else _Dot(title, save_format)
    if Digraph is not None:
        dot.attr('node', **node_attr)
    else:
        dot.node_attr = node_attr
    cm = ('#8dd3c7', '#fb8072', '#ffffb3', '#bebada', '#80b1d3', '#fdb462', '#b3de69', '#fccde5')

    def looks_like_weight(name):
        weight_like = ('_weight', '_bias', '_beta', '_gamma', '_moving_var', '_moving_mean', '_running_var',
                       '_running_mean')
        return name.endswith(weight_like)

    hidden_nodes = set()
    for node in nodes:
        op = node['op']
        name = node['name']
        attrs = {'label': name}
        attr = node.get('attrs', node.get('param', {})) or {}
        if op == 'null':
            if looks_like_weight(node['name']):
                if hide_weights:
                    hidden_nodes.add(node['name'])
                continue
            attrs['shape'] = 'oval'
            attrs['fillcolor'] = cm[0]
        elif op == 'Convolution':
            label = 'Convolution\n%s/%s, %s' % ('x'.join(_str2tuple(attr['kernel'])),
                                                'x'.join(_str2tuple(attr.get('stride', '1'))) or '1',
                                                attr['num_filter'])
            attrs['label'] = label
            attrs['fillcolor'] = cm[1]
        elif op == 'FullyConnected':
            attrs['label'] = 'FullyConnected\n%s' % attr['num_hidden']
            attrs['fillcolor'] = cm[1]
        elif op == 'BatchNorm':
            attrs['fillcolor'] = cm[3]
        elif op in ('Activation', 'LeakyReLU'):
            attrs['label'] = '%s\n%s' % (op, attr.get('act_type', ''))
            attrs['fillcolor'] = cm[2]
        elif op == 'Pooling':
            attrs['label'] = 'Pooling\n%s, %s/%s' % (attr.get('pool_type', 'max'),
                                                     'x'.join(_str2tuple(attr.get('kernel', '1'))),
                                                     'x'.join(_str2tuple(attr.get('stride', '1'))))
            attrs['fillcolor'] = cm[4]
        elif op in ('Concat', 'Flatten', 'Reshape'):
            attrs['fillcolor'] = cm[5]
        elif op == 'Softmax':
            attrs['fillcolor'] = cm[6]
        else:
            attrs['fillcolor'] = cm[7]
            if op == 'Custom':
                attrs['label'] = attr.get('op_type', op)
        dot.node(name=name, **attrs)
    for node in nodes:
        op = node['op']
        name = node['name']
        if op == 'null':
            continue
        for item in node['inputs']:
            input_node = nodes[item[0]]
            input_name = input_node['name']
            if input_name not in hidden_nodes:
                attrs = {'dir': 'back', 'arrowtail': 'open'}
                if draw_shape:
                    key = input_name + '_output' if input_node['op'] != 'null' else input_name
                    if key in shape_dict:
                        attrs['label'] = 'x'.join(str(x) for x in shape_dict[key][1:])
                dot.edge(tail=name, head=input_name, **attrs)
    return dot
