"""ctypes binding of the CPU oracle (oracle/build/libcpu_ref.so) — test infrastructure only."""
import ctypes
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "build", "libcpu_ref.so")

TYPE_CODES = {"INT": 0, "LONG": 1, "FLOAT": 2, "DOUBLE": 3, "STRING": 4, "BOOL": 5}


class CValue(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("is_null", ctypes.c_int32), ("i", ctypes.c_int64),
                ("d", ctypes.c_double), ("s", ctypes.c_char_p)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle not built: {LIB_PATH} (run __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        L.cr_app_create.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p, ctypes.c_size_t]
        L.cr_app_destroy.argtypes = [ctypes.c_void_p]
        L.cr_app_start.argtypes = [ctypes.c_void_p]
        L.cr_stream_index.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.cr_send.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.POINTER(CValue), ctypes.c_char_p,
                              ctypes.c_size_t]
        L.cr_send_columns.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p,
                                      ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p, ctypes.c_size_t]
        L.cr_send_interleaved.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p, ctypes.c_size_t]
        L.cr_send_interleaved_ord.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p,
                                              ctypes.c_size_t]
        L.cr_output_order.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t]
        L.cr_output_order.restype = ctypes.c_size_t
        L.cr_advance_time.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_size_t]
        L.cr_advance_wallclock.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_char_p, ctypes.c_size_t]
        L.cr_dump_outputs.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        L.cr_dump_outputs.restype = ctypes.c_size_t
        L.cr_output_count.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        L.cr_output_count.restype = ctypes.c_int64
        L.cr_clear_outputs.argtypes = [ctypes.c_void_p]
        L.cr_set_collect.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _lib = L
    return _lib


class EngineError(Exception):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class OracleApp:
    """Oracle app handle with the same surface the KAT runner drives on the product."""

    def __init__(self, siddhiql):
        L = lib()
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(2048)
        rc = L.cr_app_create(siddhiql.encode(), ctypes.byref(h), err, 2048)
        if rc != 0:
            raise EngineError(rc, err.value.decode())
        self.h = h
        self._streams = {}

    def close(self):
        if self.h:
            lib().cr_app_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def start(self):
        lib().cr_app_start(self.h)

    def stream_index(self, sid):
        if sid not in self._streams:
            self._streams[sid] = lib().cr_stream_index(self.h, sid.encode())
        return self._streams[sid]

    def send(self, sid, ts, row, types):
        n = len(row)
        arr = (CValue * max(n, 1))()
        keep = []
        for k, (v, t) in enumerate(zip(row, types)):
            arr[k].type = TYPE_CODES[t]
            if v is None:
                arr[k].is_null = 1
                continue
            if t == "STRING":
                b = str(v).encode()
                keep.append(b)
                arr[k].s = b
            elif t in ("FLOAT", "DOUBLE"):
                arr[k].d = float(v)
            elif t == "BOOL":
                arr[k].i = 1 if v else 0
            else:
                arr[k].i = int(v)
        err = ctypes.create_string_buffer(2048)
        rc = lib().cr_send(self.h, self.stream_index(sid), int(ts), arr, err, 2048)
        if rc != 0:
            raise EngineError(rc, err.value.decode())

    def send_interleaved(self, stream_idx, ts, cols):
        """numpy arrays: int32 stream index per event, int64 event time, one column per schema attribute."""
        import numpy as np
        sidx = np.ascontiguousarray(stream_idx, dtype=np.int32)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        cols = [np.ascontiguousarray(c) for c in cols]
        ptrs = (ctypes.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
        err = ctypes.create_string_buffer(512)
        rc = lib().cr_send_interleaved(self.h, len(ts), sidx.ctypes.data, ts.ctypes.data, ptrs, err, 512)
        if rc != 0:
            raise EngineError(rc, err.value.decode())

    def send_interleaved_ord(self, stream_idx, ts, ords, cols):
        """send_interleaved with given arrival ordinals (a heartbeat's entry: its trigger's ordinal)."""
        import numpy as np
        sidx = np.ascontiguousarray(stream_idx, dtype=np.int32)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        ords = np.ascontiguousarray(ords, dtype=np.int64)
        cols = [np.ascontiguousarray(c) for c in cols]
        ptrs = (ctypes.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
        err = ctypes.create_string_buffer(512)
        rc = lib().cr_send_interleaved_ord(self.h, len(ts), sidx.ctypes.data, ts.ctypes.data, ords.ctypes.data, ptrs,
                                           err, 512)
        if rc != 0:
            raise EngineError(rc, err.value.decode())

    def output_order(self, sid):
        """(n, 4) int64: trigger ordinal, phase, clock step, instance creation ordinal of each collected output."""
        import numpy as np
        n = lib().cr_output_order(self.h, sid.encode(), None, 0)
        out = np.zeros((n, 4), dtype=np.int64)
        if n:
            lib().cr_output_order(self.h, sid.encode(), out.ctypes.data, n)
        return out

    def advance_time(self, ts):
        err = ctypes.create_string_buffer(2048)
        rc = lib().cr_advance_time(self.h, int(ts), err, 2048)
        if rc != 0:
            raise EngineError(rc, err.value.decode())

    def advance_wallclock(self, ts):
        err = ctypes.create_string_buffer(2048)
        rc = lib().cr_advance_wallclock(self.h, int(ts), err, 2048)
        if rc != 0:
            raise EngineError(rc, err.value.decode())

    def flush(self):
        pass

    def outputs(self):
        L = lib()
        n = L.cr_dump_outputs(self.h, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        L.cr_dump_outputs(self.h, buf, n + 1)
        return json.loads(buf.value.decode())

    def output_count(self, sid):
        return lib().cr_output_count(self.h, sid.encode())

    def set_collect(self, on):
        lib().cr_set_collect(self.h, 1 if on else 0)
