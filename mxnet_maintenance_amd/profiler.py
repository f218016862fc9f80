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
_t0 = time.perf_counter()
_pid = os.getpid()
_scope = threading.local()

# fast flags read by the dispatchers
active_imperative = False
active_symbolic = False


def _now_us():
    return (time.perf_counter() - _t0) * 1e6


def _refresh_flags():
    global active_imperative, active_symbolic
    on = _state['running'] and not _state['paused']
    active_imperative = on and (_config['profile_imperative'] or _config['profile_all'])
    active_symbolic = on and (_config['profile_symbolic'] or _config['profile_all'])


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


class _OpSpan:
    """Context helper used by the dispatchers."""
    __slots__ = ('name', 'cat', 't')

    def __init__(self, name, cat):
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
    """Aggregate statistics per (category, name): count, total/min/max/avg microseconds."""
    keys = {'total': 1, 'avg': None, 'min': 2, 'max': 3, 'count': 0}
    if sort_by not in keys:
        raise ValueError('sort_by must be one of %s' % list(keys))
    with _lock:
        rows = [(cat, name, v[0], v[1], v[2], v[3]) for (cat, name), v in _agg.items()]
        if reset:
            _agg.clear()

    def key(r):
        if sort_by == 'avg':
            return r[3] / max(r[2], 1)
        return {'total': r[3], 'min': r[4], 'max': r[5], 'count': r[2]}[sort_by]
    rows.sort(key=key, reverse=not ascending)
    if format == 'json':
        out = {}
        for cat, name, cnt, tot, mn, mx_ in rows:
            out.setdefault(cat, {})[name] = {'Count': cnt, 'Total': tot / 1e3, 'Min': mn / 1e3, 'Max': mx_ / 1e3,
                                             'Avg': tot / max(cnt, 1) / 1e3}
        return json.dumps({'Time': out, 'Unit': {'Time': 'ms'}})
    lines = ['Profile Statistics:', '\tNote the difference in units for different entries.']
    cur = None
    for cat, name, cnt, tot, mn, mx_ in sorted(rows, key=lambda r: r[0]):
        if cat != cur:
            cur = cat
            lines.append('%s' % cat)
            lines.append('=' * 80)
            lines.append('%-40s %12s %14s %12s %12s %12s' % ('Name', 'Total Count', 'Time (ms)', 'Min Time (ms)',
                                                             'Max Time (ms)', 'Avg Time (ms)'))
            lines.append('%-40s %12s %14s %12s %12s %12s' % ('----', '-----------', '---------', '-------------',
                                                             '-------------', '-------------'))
        lines.append('%-40s %12d %14.4f %12.4f %12.4f %12.4f' % (name[:40], cnt, tot / 1e3, mn / 1e3, mx_ / 1e3,
                                                                 tot / max(cnt, 1) / 1e3))
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
