"""siddhi_amd — MI355X-native Siddhi pattern/sequence matching, Python host mirror of the reference API.

Mirrors the reference's user-facing classes (modules/siddhi-core/src/main/java/org/wso2/siddhi/core/):
  SiddhiManager.createSiddhiAppRuntime (SiddhiManager.java:73)
  SiddhiAppRuntime.getInputHandler / addCallback / start / shutdown (SiddhiAppRuntime.java:243-396)
  InputHandler.send(Object[]) / send(long, Object[]) / send(Event) / send(Event[]) (InputHandler.java:47-65)
  StreamCallback.receive(Event[]) (StreamCallback.java:101), QueryCallback.receive(long, Event[], Event[])
  (QueryCallback.java:105), Event(timestamp, data) (core/event/Event.java)
over the C ABI of libsiddhi_amd.so. Differences from the reference: events are processed on the GPU when the
runtime flushes (flush(), shutdown(), or when the staging buffer fills), so callbacks fire at those points —
in the reference's order, one call per output chunk (the events one trigger made one query emit) — instead of
inside send(). Callbacks run with the runtime unlocked: they may send into the same runtime.
"""
import ctypes
import time

from . import _lib
from ._lib import (OperationNotSupportedException, SiddhiAppCreationException, SiddhiAppValidationException,
                   SiddhiDeviceError, SiddhiError, SiddhiParserException, SiddhiTypeError, check, lib)

__all__ = ["SiddhiManager", "SiddhiAppRuntime", "InputHandler", "Event", "StreamCallback", "QueryCallback",
           "SiddhiError", "SiddhiParserException", "SiddhiAppValidationException", "SiddhiAppCreationException",
           "OperationNotSupportedException", "SiddhiTypeError", "SiddhiDeviceError"]


class Event:
    """core/event/Event.java"""

    def __init__(self, timestamp=-1, data=None, is_expired=False):
        self.timestamp = timestamp
        self.data = list(data) if data is not None else []
        self.is_expired = is_expired

    def getData(self):
        return self.data

    def getTimestamp(self):
        return self.timestamp

    def isExpired(self):
        return self.is_expired

    def __repr__(self):
        return f"Event{{timestamp={self.timestamp}, data={self.data}, isExpired={self.is_expired}}}"


class StreamCallback:
    """Subclass and override receive(events)."""

    def receive(self, events):
        raise NotImplementedError


class ColumnsStreamCallback(StreamCallback):
    """A StreamCallback taking each chunk as columns (sm_app_add_stream_columns_callback): override
    receive_columns(timestamps, values, null_bits), values[k][a] the 8-byte word of attribute a of event k (FLOAT /
    DOUBLE as the double's bits)."""

    def receive_columns(self, timestamps, values, null_bits):
        raise NotImplementedError


class QueryCallback:
    """Subclass and override receive(timestamp, in_events, remove_events)."""

    def receive(self, timestamp, in_events, remove_events):
        raise NotImplementedError


def _py_value(v):
    if v.is_null:
        return None
    t = v.type
    if t in (2, 3):
        return v.d
    if t == 4:
        return v.s.decode() if v.s is not None else None
    if t == 5:
        return bool(v.i)
    return v.i


def _events(ptr, n):
    out = []
    for k in range(n):
        e = ptr[k]
        out.append(Event(e.timestamp, [_py_value(e.data[j]) for j in range(e.n)]))
    return out


class InputHandler:
    def __init__(self, runtime, stream_id, handle, types):
        self._rt = runtime
        self.stream_id = stream_id
        self._h = handle
        self._types = types

    def _row(self, data):
        if len(data) != len(self._types):
            raise SiddhiTypeError(f"stream {self.stream_id} expects {len(self._types)} attributes")
        arr = (_lib.SmValue * max(len(data), 1))()
        keep = []
        for k, (v, t) in enumerate(zip(data, self._types)):
            arr[k].type = t
            if v is None:
                arr[k].is_null = 1
            elif t == 4:
                b = str(v).encode()
                keep.append(b)
                arr[k].s = b
            elif t in (2, 3):
                arr[k].d = float(v)
            elif t == 5:
                arr[k].i = 1 if v else 0
            else:
                arr[k].i = int(v)
        return arr, keep

    def send(self, *args):
        """send(data) | send(timestamp, data) | send(Event) | send([Event, ...])"""
        if len(args) == 2:
            ts, data = args
            self._send(int(ts), data)
        elif isinstance(args[0], Event):
            self._send(args[0].timestamp, args[0].data)
        elif args[0] and isinstance(args[0][0], Event):
            for e in args[0]:
                self._send(e.timestamp, e.data)
        else:
            self._send(int(time.time() * 1000), args[0])

    def _send(self, ts, data):
        arr, keep = self._row(data)
        check(lib().sm_input_send(self._h, ts, arr, len(data)))

    def send_columns(self, timestamps, columns, null_flags=None):
        """send(Event[]) in columnar form: numpy arrays, int64 timestamps and one column per attribute at its native
        width (INT int32, LONG int64, FLOAT float32, DOUBLE float64, BOOL uint8; STRING an object array of str),
        null_flags an optional list of per-attribute uint8 arrays (or None entries). A large batch without nulls or
        STRING attributes goes to the device in chunks and is processed inside this call (sm_input_send_columns)."""
        import numpy as np
        ts = np.ascontiguousarray(timestamps, dtype=np.int64)
        n = ts.shape[0]
        if len(columns) != len(self._types):
            raise SiddhiTypeError(f"stream {self.stream_id} expects {len(self._types)} attributes")
        want = {0: np.int32, 1: np.int64, 2: np.float32, 3: np.float64, 5: np.uint8}
        keep, ptrs = [ts], []
        for c, t in zip(columns, self._types):
            if len(c) != n:
                raise ValueError("every column must hold one value per timestamp")
            if t == 4:
                enc = [None if v is None else str(v).encode() for v in c]
                arr = (ctypes.c_char_p * max(n, 1))(*enc)
                keep.append((enc, arr))
                ptrs.append(ctypes.cast(arr, ctypes.c_void_p).value)
            else:
                a = np.ascontiguousarray(c, dtype=want[t])
                keep.append(a)
                ptrs.append(a.ctypes.data)
        cp = (ctypes.c_void_p * max(len(ptrs), 1))(*ptrs)
        nf = None
        if null_flags is not None and any(f is not None for f in null_flags):
            fl = [None if f is None else np.ascontiguousarray(f, dtype=np.uint8) for f in null_flags]
            keep.append(fl)
            nf = (ctypes.c_void_p * len(fl))(*[None if f is None else f.ctypes.data for f in fl])
        check(lib().sm_input_send_columns(self._h, n, ts.ctypes.data, cp, nf))


class SiddhiAppRuntime:
    def __init__(self, handle):
        self._h = handle
        self._cbs = []  # keep ctypes trampolines alive
        self._inputs = {}

    def getInputHandler(self, stream_id):
        if stream_id not in self._inputs:
            h = ctypes.c_void_p()
            check(lib().sm_app_input_handler(self._h, stream_id.encode(), ctypes.byref(h)))
            self._inputs[stream_id] = InputHandler(self, stream_id, h, self.stream_schema(stream_id))
        return self._inputs[stream_id]

    def stream_schema(self, stream_id):
        types = (ctypes.c_int32 * 64)()
        n = ctypes.c_size_t()
        check(lib().sm_app_stream_schema(self._h, stream_id.encode(), types, 64, ctypes.byref(n)))
        return [types[k] for k in range(n.value)]

    def addCallback(self, name, callback):
        if isinstance(callback, ColumnsStreamCallback):
            def tramp(user, n, ts, vals, nb, ns, cb=callback):
                cb.receive_columns([ts[k] for k in range(n)], [[vals[k * ns + a] for a in range(ns)] for k in range(n)],
                                   [nb[k] for k in range(n)])
            f = _lib.COLUMNS_CB(tramp)
            check(lib().sm_app_add_stream_columns_callback(self._h, name.encode(), f, None))
        elif isinstance(callback, StreamCallback):
            def tramp(user, evs, n, cb=callback):
                cb.receive(_events(evs, n))
            f = _lib.STREAM_CB(tramp)
            check(lib().sm_app_add_stream_callback(self._h, name.encode(), f, None))
        elif isinstance(callback, QueryCallback):
            def tramp(user, ts, ins, nin, rm, nrm, cb=callback):
                cb.receive(ts, _events(ins, nin) if nin else None, _events(rm, nrm) if nrm else None)
            f = _lib.QUERY_CB(tramp)
            check(lib().sm_app_add_query_callback(self._h, name.encode(), f, None))
        else:
            raise TypeError("callback must be a StreamCallback or QueryCallback")
        self._cbs.append(f)

    def start(self):
        check(lib().sm_app_start(self._h))

    def sendDeviceBatch(self, stream_id, ts, cols, ordinals=None, ordinal_base=0, hip_stream=None):
        """Bulk ingest of one stream's columns already in device memory (torch tensors: int64 event times, one
        tensor per attribute at its native width): the device form of a sequence of InputHandler.send(ts, row)
        calls (InputHandler.java:53 → StreamJunction.sendData :232). Filter queries and `every e1 -> e2 within T`
        patterns on the stream run on the GPU; their outputs reach the registered callbacks in the reference's
        order, one call per input event that produced output (sm_app_process_device_batch)."""
        import torch
        n = ts.numel()
        for name, t in [("ts", ts), ("ordinals", ordinals)] + [(f"column {k}", c) for k, c in enumerate(cols)]:
            if t is None:
                continue
            if not isinstance(t, torch.Tensor) or not t.is_cuda or not t.is_contiguous() or t.dim() != 1:
                raise ValueError(f"sendDeviceBatch: {name} must be a contiguous 1-D tensor on the GPU")
            if t.numel() != n:
                raise ValueError(f"sendDeviceBatch: {name} holds {t.numel()} values for {n} events")
        if ts.dtype != torch.int64 or (ordinals is not None and ordinals.dtype != torch.int64):
            raise ValueError("sendDeviceBatch: event times and ordinals are int64 tensors")
        schema = self.stream_schema(stream_id)
        if len(cols) != len(schema):
            raise ValueError(f"sendDeviceBatch: stream {stream_id} has {len(schema)} attributes, got {len(cols)}")
        width = {0: 4, 1: 8, 2: 4, 3: 8, 4: 4, 5: 1}
        for k, (c, t) in enumerate(zip(cols, schema)):
            if c.element_size() != width[t]:
                raise ValueError(f"sendDeviceBatch: column {k} has {c.element_size()}-byte elements, attribute type "
                                 f"{_lib.TYPE_NAMES[t]} needs {width[t]}")
        ptrs = (ctypes.c_void_p * len(cols))(*[c.data_ptr() for c in cols])
        check(lib().sm_app_process_device_batch(self._h, stream_id.encode(), ts.numel(), ts.data_ptr(), ptrs,
                                                ordinals.data_ptr() if ordinals is not None else None,
                                                int(ordinal_base), hip_stream))

    def flush(self):
        check(lib().sm_app_flush(self._h))

    def shutdown(self):
        if self._h:
            check(lib().sm_app_shutdown(self._h))
            lib().sm_app_destroy(self._h)
            self._h = None

    def advance_time(self, ts):
        check(lib().sm_app_advance_time(self._h, int(ts)))

    def advance_wallclock(self, ts):
        """Wall-clock scheduler emulation: fire every due timer at its scheduled time up to ts."""
        check(lib().sm_app_advance_wallclock(self._h, int(ts)))

    def __del__(self):
        try:
            if self._h:
                lib().sm_app_destroy(self._h)
        except Exception:
            pass


def compile_dump(siddhi_app):
    """SiddhiCompiler.parse: the app's query tree (dict), without a device. Raises the reference's exceptions."""
    import json
    n = ctypes.c_size_t()
    check(lib().sm_compile_dump(siddhi_app.encode(), None, 0, ctypes.byref(n)))
    buf = ctypes.create_string_buffer(n.value + 1)
    check(lib().sm_compile_dump(siddhi_app.encode(), buf, n.value + 1, ctypes.byref(n)))
    return json.loads(buf.value.decode())


class SiddhiManager:
    def __init__(self):
        h = ctypes.c_void_p()
        check(lib().sm_manager_create(ctypes.byref(h)))
        self._h = h

    def createSiddhiAppRuntime(self, siddhi_app):
        h = ctypes.c_void_p()
        check(lib().sm_app_create(self._h, siddhi_app.encode(), ctypes.byref(h)))
        return SiddhiAppRuntime(h)

    def shutdown(self):
        if self._h:
            lib().sm_manager_destroy(self._h)
            self._h = None
