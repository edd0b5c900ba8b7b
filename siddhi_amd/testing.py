"""Adapters used by the parity tests: drive the product through the C ABI with the same surface as the
oracle's OracleApp (start / send / advance_time / advance_wallclock / flush / outputs)."""
import ctypes
import json

from . import _lib
from ._lib import check, lib


class EngineError(Exception):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def _call(rc):
    if rc != _lib.SM_OK:
        raise EngineError(rc, lib().sm_last_error().decode(errors="replace"))


class ProductApp:
    _mgr = None

    def __init__(self, siddhiql, **options):
        L = lib()
        if ProductApp._mgr is None:
            m = ctypes.c_void_p()
            _call(L.sm_manager_create(ctypes.byref(m)))
            ProductApp._mgr = m
        h = ctypes.c_void_p()
        _call(L.sm_app_create(ProductApp._mgr, siddhiql.encode(), ctypes.byref(h)))
        self.h = h
        for k, v in options.items():
            _call(L.sm_app_set_option(self.h, k.encode(), int(v)))
        _call(L.sm_app_set_collect(self.h, 1))
        self._collect = True
        self._inputs = {}

    def close(self):
        if self.h:
            lib().sm_app_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def start(self):
        _call(lib().sm_app_start(self.h))

    def _input(self, sid):
        if sid not in self._inputs:
            h = ctypes.c_void_p()
            _call(lib().sm_app_input_handler(self.h, sid.encode(), ctypes.byref(h)))
            self._inputs[sid] = h
        return self._inputs[sid]

    def send(self, sid, ts, row, types):
        arr = (_lib.SmValue * max(len(row), 1))()
        keep = []
        for k, (v, t) in enumerate(zip(row, types)):
            arr[k].type = _lib.TYPE_CODES[t]
            if v is None:
                arr[k].is_null = 1
            elif t == "STRING":
                b = str(v).encode()
                keep.append(b)
                arr[k].s = b
            elif t in ("FLOAT", "DOUBLE"):
                arr[k].d = float(v)
            elif t == "BOOL":
                arr[k].i = 1 if v else 0
            else:
                arr[k].i = int(v)
        _call(lib().sm_input_send(self._input(sid), int(ts), arr, len(row)))

    def send_columns(self, sid, ts, cols):
        """ts: int64 numpy array; cols: list of numpy arrays (native widths)."""
        n = len(ts)
        ptrs = (ctypes.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
        _call(lib().sm_input_send_columns(self._input(sid), n, ts.ctypes.data, ptrs, None))

    def advance_time(self, ts):
        _call(lib().sm_app_advance_time(self.h, int(ts)))

    def advance_wallclock(self, ts):
        _call(lib().sm_app_advance_wallclock(self.h, int(ts)))

    def flush(self):
        _call(lib().sm_app_flush(self.h))

    def outputs(self):
        L = lib()
        n = L.sm_app_dump_outputs(self.h, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        L.sm_app_dump_outputs(self.h, buf, n + 1)
        return json.loads(buf.value.decode())

    def set_collect(self, on):
        """Keep (on) or drop (off) the JSON dump of delivered outputs; output counts are kept either way."""
        _call(lib().sm_app_set_collect(self.h, 1 if on else 0))
        self._collect = bool(on)

    def set_option(self, key, value):
        _call(lib().sm_app_set_option(self.h, key.encode(), int(value)))

    def process_device_batch(self, stream, ts_tensor, col_tensors, ordinals=None, ordinal_base=0, hip_stream=None,
                             collect=False):
        """collect=False keeps the batch's outputs out of the JSON dump (the parity tests read the device tuples;
        the dump would cost a host round trip per output)."""
        ptrs = (ctypes.c_void_p * len(col_tensors))(*[t.data_ptr() for t in col_tensors])
        quiet = self._collect and not collect
        if quiet:
            _call(lib().sm_app_set_collect(self.h, 0))
        try:
            _call(lib().sm_app_process_device_batch(self.h, stream.encode(), ts_tensor.numel(), ts_tensor.data_ptr(),
                                                    ptrs, ordinals.data_ptr() if ordinals is not None else None,
                                                    int(ordinal_base), hip_stream))
        finally:
            if quiet:
                _call(lib().sm_app_set_collect(self.h, 1))

    def process_device_events(self, stream_idx, ts_tensor, col_tensors, ordinals=None, ordinal_base=0,
                              hip_stream=None):
        """Interleaved batch over streams of one schema (event i -> stream stream_idx[i], int32 tensor)."""
        ptrs = (ctypes.c_void_p * len(col_tensors))(*[t.data_ptr() for t in col_tensors])
        _call(lib().sm_app_process_device_events(self.h, ts_tensor.numel(), stream_idx.data_ptr(), ts_tensor.data_ptr(),
                                                 ptrs, ordinals.data_ptr() if ordinals is not None else None,
                                                 int(ordinal_base), hip_stream))

    def snapshot(self):
        """SiddhiAppRuntime.snapshot(): bytes"""
        n = ctypes.c_size_t()
        _call(lib().sm_app_snapshot(self.h, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value)
        _call(lib().sm_app_snapshot(self.h, buf, n.value, ctypes.byref(n)))
        return buf.raw[:n.value]

    def restore(self, data):
        """SiddhiAppRuntime.restore(byte[])"""
        _call(lib().sm_app_restore(self.h, data, len(data)))

    def device_matches(self, query):
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        _call(lib().sm_app_device_matches(self.h, query.encode(), ctypes.byref(p), ctypes.byref(n)))
        return p.value, n.value

    def copy_device_matches(self, query, dst):
        """The last device batch's tuples into the device tensor `dst` (int64 per tuple = (e2 << 32) | e1, or int32
        kept rows of a filter) on the current stream; returns the tuple count."""
        import torch
        n = ctypes.c_size_t()
        s = ctypes.c_void_p(torch.cuda.current_stream(dst.device).cuda_stream)
        _call(lib().sm_app_copy_device_matches(self.h, query.encode(), ctypes.c_void_p(dst.data_ptr()),
                                               dst.numel() * dst.element_size(), ctypes.byref(n), s))
        return n.value

    def copy_device_outputs(self, query):
        """The last interleaved device batch's output records (option keep_outputs) as an int64 device tensor
        (n, stride / 8) in delivery order: sm_out_rec (pos = trigger ordinal) + select values + ordinals."""
        import torch
        n = ctypes.c_size_t()
        st = ctypes.c_size_t()
        _call(lib().sm_app_copy_device_outputs(self.h, query.encode(), None, 0, ctypes.byref(n), ctypes.byref(st),
                                               None))
        dev = torch.device("cuda", torch.cuda.current_device())
        out = torch.empty((max(n.value, 1), st.value // 8), dtype=torch.int64, device=dev)
        s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        _call(lib().sm_app_copy_device_outputs(self.h, query.encode(), ctypes.c_void_p(out.data_ptr()),
                                               out.numel() * 8, ctypes.byref(n), ctypes.byref(st), s))
        torch.cuda.synchronize()
        return out[:n.value]

    def get_stat(self, key):
        v = ctypes.c_double()
        _call(lib().sm_app_get_stat(self.h, key.encode(), ctypes.byref(v)))
        return v.value

    def device_project(self, query):
        """sm_app_device_project: the last closed-form batch's outputs projected on the device. Returns (values,
        nulls, ts) as torch tensors on the current device: values (n, nsel) int64 (the raw 64-bit word: integers,
        dictionary ids, or double bits for FLOAT / DOUBLE), nulls (n, nsel) bool, ts (n,) int64."""
        import torch
        n = ctypes.c_size_t()
        ns = ctypes.c_int32()
        _call(lib().sm_app_device_project(self.h, query.encode(), None, 0, None, ctypes.byref(n), ctypes.byref(ns),
                                          None))
        dev = torch.device("cuda", torch.cuda.current_device())
        raw = torch.empty((max(n.value, 1), max(ns.value, 1), 2), dtype=torch.int64, device=dev)  # 16-B sm_dval
        ts = torch.empty(max(n.value, 1), dtype=torch.int64, device=dev)
        s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        _call(lib().sm_app_device_project(self.h, query.encode(), ctypes.c_void_p(raw.data_ptr()),
                                          n.value * ns.value, ctypes.c_void_p(ts.data_ptr()), ctypes.byref(n),
                                          ctypes.byref(ns), s))
        m, k = n.value, ns.value
        vals = raw[:m, :k, 0]
        nulls = (raw[:m, :k, 1] & 0xFFFFFFFF) != 0
        return vals, nulls, ts[:m]

    def device_matches_host(self, query):
        """Copy the last device batch's match tuples to the host: numpy uint32 array of shape (n, 2) = (e1, e2)."""
        import numpy as np
        p, n = self.device_matches(query)
        out = np.empty((n, 2), dtype=np.uint32)
        if n:
            _hip_memcpy_d2h(out.ctypes.data, p, n * 8)
        return out

    def device_rows_host(self, query):
        """Kept rows of the last device batch for a filter query: numpy uint32 array (ordinal - base)."""
        import numpy as np
        p, n = self.device_matches(query)
        out = np.empty(n, dtype=np.uint32)
        if n:
            _hip_memcpy_d2h(out.ctypes.data, p, n * 4)
        return out


_hip = None


def _hip_memcpy_d2h(dst, src, nbytes):
    global _hip
    if _hip is None:
        _hip = ctypes.CDLL("libamdhip64.so")
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipDeviceSynchronize.argtypes = []
    _hip.hipDeviceSynchronize()
    rc = _hip.hipMemcpy(dst, src, nbytes, 2)  # hipMemcpyDeviceToHost
    if rc != 0:
        raise RuntimeError(f"hipMemcpy failed ({rc})")
