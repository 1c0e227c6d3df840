"""hpx::future for GPU completion.

Reference: completion of a CUDA target becomes an ``hpx::future<void>``
through a stream callback that sets the shared state
(src/compute/cuda/cuda_target.cpp:97-142).  Here the shared state holds a
HIP event recorded on the target's stream behind the work: ``is_ready`` is
``hipEventQuery``, ``get``/``wait`` is ``hipEventSynchronize``, and the
value (if any) is produced by a thunk run once the event has completed
(e.g. the D2H read of a reduction result).  Continuations (``then``),
``when_all`` and ``dataflow`` compose the way hpx/lcos/future.hpp:852 and
dataflow.hpp:532 do, run on the thread that asks for the value.
"""
from __future__ import annotations

import ctypes
import threading

from . import _lib as L


class _Event:
    __slots__ = ("handle",)

    def __init__(self):
        h = ctypes.c_void_p()
        L.call("hpxhip_event_create", ctypes.byref(h))
        self.handle = h

    def record(self, stream):
        L.call("hpxhip_event_record", self.handle, stream)

    def query(self) -> bool:
        rc = L.load().hpxhip_event_query(self.handle)
        if rc == L.ERROR_NOT_READY:
            return False
        L.check(rc, "hpxhip_event_query")
        return True

    def synchronize(self):
        L.call("hpxhip_event_synchronize", self.handle)

    def __del__(self):
        try:
            if self.handle:
                L.load().hpxhip_event_destroy(self.handle)
        except Exception:
            pass


class future:
    """Single-assignment result of an asynchronous GPU operation."""

    def __init__(self, event: _Event | None = None, thunk=None, value=None, ready=False, deps=()):
        self._event = event
        self._thunk = thunk
        self._value = value
        self._exc = None
        self._done = ready
        self._deps = tuple(deps)
        self._lock = threading.Lock()
        self._error_map = None  # set on an algorithm's future: failures -> exception_list

    # -- construction helpers ------------------------------------------
    @classmethod
    def on_stream(cls, stream, thunk=None):
        ev = _Event()
        ev.record(stream)
        return cls(event=ev, thunk=thunk)

    # -- hpx::future interface ---------------------------------------------
    def valid(self) -> bool:
        return True

    def is_ready(self) -> bool:
        if self._done:
            return True
        if any(not d.is_ready() for d in self._deps):
            return False
        return self._event.query() if self._event is not None else True

    def wait(self):
        self._resolve()

    def get(self):
        self._resolve()
        if self._exc is not None:
            raise self._exc
        return self._value

    def has_exception(self) -> bool:
        self._resolve()
        return self._exc is not None

    def then(self, fn):
        """Continuation: fn(self) once ready (hpx::future::then)."""
        parent = self
        return future(thunk=lambda: fn(parent), deps=(parent,))

    def share(self):
        return self

    def _resolve(self):
        with self._lock:
            if self._done:
                return
            try:
                for d in self._deps:
                    d.wait()
                if self._event is not None:
                    self._event.synchronize()
                if self._thunk is not None:
                    self._value = self._thunk()
            except BaseException as e:  # exceptional future, like set_exception
                self._exc = self._error_map(e) if self._error_map is not None else e
            self._done = True
            self._thunk = None


shared_future = future


def make_ready_future(value=None) -> future:
    return future(value=value, ready=True)


def make_exceptional_future(exc: BaseException) -> future:
    f = future(ready=True)
    f._exc = exc
    return f


def when_all(*futures) -> future:
    """hpx::when_all: ready when every input is; value = list of inputs."""
    if len(futures) == 1 and isinstance(futures[0], (list, tuple)):
        futures = tuple(futures[0])
    fs = tuple(futures)
    return future(thunk=lambda: list(fs), deps=fs)


def wait_all(*futures):
    if len(futures) == 1 and isinstance(futures[0], (list, tuple)):
        futures = tuple(futures[0])
    for f in futures:
        f.wait()


def dataflow(fn, *args) -> future:
    """hpx::dataflow: fn(*values) once every future argument is ready."""
    deps = tuple(a for a in args if isinstance(a, future))

    def run():
        vals = [a.get() if isinstance(a, future) else a for a in args]
        return fn(*vals)

    return future(thunk=run, deps=deps)
