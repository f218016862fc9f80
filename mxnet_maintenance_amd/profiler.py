"""Profiler: operator spans, user domains/tasks/frames/events/counters/markers,
Chrome-trace dump and aggregate statistics.

Parity: python/mxnet/profiler.py + src/profiler (set_config, set_state,
pause/resume, dump, dumps(format='table'|'json', sort_by, ascending),
Domain/Task/Frame/Event/Counter/Marker).

Operator spans come from the two dispatch points of the framework: the
imperative ``invoke`` path (``profile_imperative``) and the graph program
that runs symbols / hybridized blocks (``profile_symbolic``).  With
``gpu_sync=True`` (or MXAMD_PROFILER_SYNC=1) each span waits for the HIP
stream so the duration is device time; otherwise it is host dispatch time
(kernel-level device timing comes from ``rocprofv3``; see profiles/).
"""
import json
import os
import threading
import time

__all__ = ['set_config', 'profiler_set_config', 'set_state', 'profiler_set_state', 'dump', 'dump_profile', 'dumps',
           'pause', 'resume', 'Domain', 'Task', 'Frame', 'Event', 'Counter', 'Marker', 'scope']

_lock = threading.Lock()
_config = {'filename': 'profile.json', 'profile_all': False, 'profile_symbolic': True,
           'profile_imperative': True, 'profile_memory': False, 'profile_api': False, 'aggregate_stats': False,
           'continuous_dump': False, 'dump_period': 1.0, 'gpu_sync': os.environ.get('MXAMD_PROFILER_SYNC') == '1'}
_state = {'running': False, 'paused': False}
_events = []
_agg = {}
_agg_kind = {}          # (cat, name) -> 'counter' for memory counters (duration otherwise)
_mem_live = {}          # device -> live bytes of profiled NDArrays
_t0 = time.perf_counter()
_pid = os.getpid()
_scope = threading.local()

# fast flags read by the dispatchers
active_imperative = False
active_symbolic = False
active_memory = False
_MEMORY_DOMAINS = ('Device Storage', 'Pool Memory')


def _now_us():
    return (time.perf_counter() - _t0) * 1e6


def _refresh_flags():
    global active_imperative, active_symbolic, active_memory
    on = _state['running'] and not _state['paused']
    active_imperative = on and (_config['profile_imperative'] or _config['profile_all'])
    active_symbolic = on and (_config['profile_symbolic'] or _config['profile_all'])
    active_memory = on and (_config['profile_memory'] or _config['profile_all'])


def set_config(**kwargs):
    """Configure the profiler (filename, profile_all, profile_symbolic, profile_imperative, profile_memory,
    profile_api, aggregate_stats, continuous_dump, dump_period, gpu_sync)."""
    for k, v in kwargs.items():
        if k not in _config:
            raise ValueError('unknown profiler config key %s' % k)
        _config[k] = v
    _refresh_flags()


def profiler_set_config(mode='symbolic', filename='profile.json'):
    set_config(profile_symbolic=mode in ('symbolic', 'all'), profile_all=mode == 'all', filename=filename)


def set_state(state='stop', profile_process='worker'):
    if state not in ('run', 'stop'):
        raise ValueError('state must be run or stop')
    _state['running'] = state == 'run'
    _state['paused'] = False        # a state change ends a pause (pause/resume only act while running)
    _refresh_flags()
    if state == 'stop' and _config['continuous_dump']:
        dump(finished=False)


def profiler_set_state(state='stop'):
    set_state(state)


def pause(profile_process='worker'):
    _state['paused'] = True
    _refresh_flags()


def resume(profile_process='worker'):
    _state['paused'] = False
    _refresh_flags()


def _sync():
    if _config['gpu_sync']:
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize()
        except Exception:
            pass


def record_span(name, cat, start_us, end_us, args=None):
    ev = {'name': name, 'cat': cat, 'ph': 'X', 'ts': start_us, 'dur': max(end_us - start_us, 0.0), 'pid': _pid,
          'tid': threading.get_ident() % 100000}
    if args:
        ev['args'] = args
    with _lock:
        _events.append(ev)
        if _config['aggregate_stats'] or True:
            st = _agg.setdefault((cat, name), [0, 0.0, float('inf'), 0.0])
            d = ev['dur']
            st[0] += 1
            st[1] += d
            st[2] = min(st[2], d)
            st[3] = max(st[3], d)


def _counter_sample(cat, name, value):
    """One sample of a memory counter (aggregated as Count / Min / Max, reference kCounter)."""
    key = (cat, name)
    st = _agg.setdefault(key, [0, 0.0, float('inf'), float('-inf')])
    _agg_kind[key] = 'counter'
    st[0] += 1
    st[1] = value
    st[2] = min(st[2], value)
    st[3] = max(st[3], value)
    _events.append({'name': name, 'cat': cat, 'ph': 'C', 'ts': _now_us(), 'pid': _pid, 'args': {name: value}})


def _device_of(t):
    return 'gpu/%d' % t.device.index if t.device.type == 'cuda' else 'cpu/0'


def memory_alloc(arr):
    """Storage profiler (reference storage_profiler.h, domain 'Device Storage'): count the bytes of a new
    NDArray against its device until it is garbage collected."""
    import weakref
    t = getattr(arr, '_data', None)
    if t is None:
        return
    nbytes = t.numel() * t.element_size()
    dev = _device_of(t)
    with _lock:
        live = _mem_live[dev] = _mem_live.get(dev, 0) + nbytes
        _counter_sample('Device Storage', 'Memory: %s' % dev, live)
    try:
        weakref.finalize(arr, _memory_free, dev, nbytes)
    except TypeError:
        pass


def _memory_free(dev, nbytes):
    with _lock:
        live = _mem_live[dev] = _mem_live.get(dev, 0) - nbytes
        if _state['running']:
            _counter_sample('Device Storage', 'Memory: %s' % dev, live)


# custom operators (reference custom.cc profiling): the Python body of a Custom op is a span
# '<op_type>::pure_python' in the 'Custom Operator' domain, and operators it invokes are recorded
# there as '<op_type>::<op>'
_custom = threading.local()


class custom_op_scope:  # noqa: N801
    def __init__(self, op_type, backward=False):
        self.op_type = op_type
        self.name = ('_backward_%s' if backward else '%s') % op_type + '::pure_python'

    def __enter__(self):
        self.prev = getattr(_custom, 'op', None)
        _custom.op = self.op_type
        self.t = _now_us()
        return self

    def __exit__(self, *a):
        _custom.op = self.prev
        if active_imperative or active_symbolic:
            record_span(self.name, 'Custom Operator', self.t, _now_us())


class _OpSpan:
    """Context helper used by the dispatchers."""
    __slots__ = ('name', 'cat', 't')

    def __init__(self, name, cat):
        custom = getattr(_custom, 'op', None)
        if custom is not None:
            name, cat = '%s::%s' % (custom, name), 'Custom Operator'
        self.name = name
        self.cat = cat

    def __enter__(self):
        _sync()
        self.t = _now_us()
        return self

    def __exit__(self, *a):
        _sync()
        record_span(self.name, self.cat, self.t, _now_us())


def op_span(name, symbolic=False):
    return _OpSpan(name, 'operator' if not symbolic else 'symbolic')


def dump(finished=True, profile_process='worker'):
    """Write the Chrome trace (chrome://tracing / Perfetto) to the configured filename."""
    with _lock:
        evs = list(_events)
        if finished:
            _events.clear()
    with open(_config['filename'], 'w') as f:
        json.dump({'traceEvents': evs, 'displayTimeUnit': 'ms'}, f)


def dump_profile():
    dump(True)


def dumps(reset=False, format='table', sort_by='total', ascending=False):  # noqa: A002
    """Aggregate statistics: operator / user-span durations per (domain, name) -- Count, Total, Min,
    Max, Avg ms -- and memory counters ('Device Storage': Count, Min, Max, Avg kB)."""
    keys = ('total', 'avg', 'min', 'max', 'count')
    if sort_by not in keys:
        raise ValueError('sort_by must be one of %s' % list(keys))
    with _lock:
        rows = [(cat, name, v[0], v[1], v[2], v[3], _agg_kind.get((cat, name), 'duration'))
                for (cat, name), v in _agg.items()]
        if reset:
            _agg.clear()
            _agg_kind.clear()

    def stats(r):
        cat, name, cnt, tot, mn, mx_, kind = r
        if kind == 'counter':
            return {'Count': cnt, 'Min': mn / 1024.0, 'Max': mx_ / 1024.0, 'Avg': (mx_ - mn) / 2 / 1024.0}
        return {'Count': cnt, 'Total': tot / 1e3, 'Min': mn / 1e3, 'Max': mx_ / 1e3, 'Avg': tot / max(cnt, 1) / 1e3}

    field = {'total': 'Total', 'avg': 'Avg', 'min': 'Min', 'max': 'Max', 'count': 'Count'}[sort_by]

    def key(r):
        st = stats(r)
        return st.get(field, st['Count'])
    rows.sort(key=key, reverse=not ascending)
    if format == 'json':
        time_out, mem_out = {}, {}
        for r in rows:
            (mem_out if r[0] in _MEMORY_DOMAINS else time_out).setdefault(r[0], {})[r[1]] = stats(r)
        return json.dumps({'Time': time_out, 'Memory': mem_out, 'Unit': {'Time': 'ms', 'Memory': 'kB'}})
    lines = ['Profile Statistics:', '\tNote the difference in units for different entries.']
    cur = None
    for r in sorted(rows, key=lambda r: r[0]):
        cat, name = r[0], r[1]
        st = stats(r)
        mem = cat in _MEMORY_DOMAINS
        if cat != cur:
            cur = cat
            lines.append('%s' % cat)
            lines.append('=' * 80)
            if mem:
                lines.append('%-40s %12s %14s %14s %14s' % ('Name', 'Total Count', 'Min Use  (kB)', 'Max Use  (kB)',
                                                            'Avg Use  (kB)'))
            else:
                lines.append('%-40s %12s %14s %12s %12s %12s' % ('Name', 'Total Count', 'Time (ms)', 'Min Time (ms)',
                                                                 'Max Time (ms)', 'Avg Time (ms)'))
        if mem:
            lines.append('%-40s %12d %14.4f %14.4f %14.4f' % (name[:40], st['Count'], st['Min'], st['Max'], st['Avg']))
        else:
            lines.append('%-40s %12d %14.4f %12.4f %12.4f %12.4f' % (name[:40], st['Count'], st['Total'], st['Min'],
                                                                     st['Max'], st['Avg']))
    return '\n'.join(lines)


class Domain:
    """A named group of user-defined profiling objects."""

    def __init__(self, name):
        self.name = name

    def __str__(self):
        return self.name

    def new_task(self, name):
        return Task(self, name)

    def new_frame(self, name):
        return Frame(self, name)

    def new_counter(self, name, value=None):
        return Counter(self, name, value)

    def new_marker(self, name):
        return Marker(self, name)


class _Span:
    _cat = 'span'

    def __init__(self, domain, name):
        self.domain = domain
        self.name = name
        self._t = None

    def start(self):
        self._t = _now_us()

    def stop(self):
        if self._t is not None and _state['running']:
            record_span(self.name, '%s:%s' % (self._cat, self.domain), self._t, _now_us())
        self._t = None

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, *a):
        self.stop()

    def __str__(self):
        return self.name


class Task(_Span):
    _cat = 'task'


class Frame(_Span):
    _cat = 'frame'


class Event(_Span):
    _cat = 'event'

    def __init__(self, name):
        super().__init__('event', name)


class Counter:
    def __init__(self, domain, name, value=None):
        self.domain = domain
        self.name = name
        self.value = 0
        if value is not None:
            self.set_value(value)

    def _emit(self):
        if _state['running']:
            with _lock:
                _events.append({'name': self.name, 'cat': 'counter:%s' % self.domain, 'ph': 'C', 'ts': _now_us(),
                                'pid': _pid, 'args': {self.name: self.value}})

    def set_value(self, value):
        self.value = value
        self._emit()

    def increment(self, delta=1):
        self.set_value(self.value + delta)

    def decrement(self, delta=1):
        self.set_value(self.value - delta)

    def __iadd__(self, delta):
        self.increment(delta)
        return self

    def __isub__(self, delta):
        self.decrement(delta)
        return self

    def __str__(self):
        return self.name


class Marker:
    def __init__(self, domain, name):
        self.domain = domain
        self.name = name

    def mark(self, scope='process'):
        if _state['running']:
            with _lock:
                _events.append({'name': self.name, 'cat': 'marker:%s' % self.domain, 'ph': 'i', 'ts': _now_us(),
                                'pid': _pid, 's': {'global': 'g', 'process': 'p', 'thread': 't'}.get(scope, 'p')})


class scope:  # noqa: N801  (reference spells it as a lowercase context manager)
    """``with profiler.scope('name'):`` prefixes operator spans recorded inside it."""

    def __init__(self, name='<unk>:', append_mode=False):
        self.name = name
        self.append = append_mode

    def __enter__(self):
        self.prev = getattr(_scope, 'name', '')
        _scope.name = (self.prev + self.name) if self.append else self.name
        return self

    def __exit__(self, *a):
        _scope.name = self.prev


def current_scope():
    return getattr(_scope, 'name', '')
