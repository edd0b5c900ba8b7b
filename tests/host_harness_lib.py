"""ctypes adapter for the CPU debug build of the device NFA code (tests/native) — test infrastructure."""
import ctypes
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


class HV(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("is_null", ctypes.c_int32), ("i", ctypes.c_int64),
                ("d", ctypes.c_double), ("s", ctypes.c_char_p)]


_L = {}


def lib(asan=False):
    key = "asan" if asan else "plain"
    if key not in _L:
        p = os.path.join(HERE, "native", "build", "libnfa_host_asan.so" if asan else "libnfa_host.so")
        L = ctypes.CDLL(p)
        L.h_create.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p, ctypes.c_size_t]
        L.h_destroy.argtypes = [ctypes.c_void_p]
        L.h_start.argtypes = [ctypes.c_void_p]
        L.h_send.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64, ctypes.POINTER(HV)]
        L.h_advance.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
        L.h_flush.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        L.h_dump.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
        L.h_dump.restype = ctypes.c_size_t
        _L[key] = L
    return _L[key]


class HarnessError(Exception):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class HostHarnessApp:
    asan = False
    TYPES = {"INT": 0, "LONG": 1, "FLOAT": 2, "DOUBLE": 3, "STRING": 4, "BOOL": 5}

    def __init__(self, text):
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(1024)
        rc = lib(self.asan).h_create(text.encode(), ctypes.byref(h), err, 1024)
        if rc:
            raise HarnessError(rc, err.value.decode())
        self.h = h

    def close(self):
        if self.h:
            lib(self.asan).h_destroy(self.h)
            self.h = None

    def start(self):
        lib(self.asan).h_start(self.h)

    def send(self, sid, ts, row, types):
        arr = (HV * max(len(row), 1))()
        keep = []
        for k, (v, t) in enumerate(zip(row, types)):
            arr[k].type = self.TYPES[t]
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
        lib(self.asan).h_send(self.h, sid.encode(), int(ts), arr)

    def advance_time(self, ts):
        lib(self.asan).h_advance(self.h, int(ts), 0)

    def advance_wallclock(self, ts):
        lib(self.asan).h_advance(self.h, int(ts), 1)

    def flush(self):
        err = ctypes.create_string_buffer(1024)
        rc = lib(self.asan).h_flush(self.h, err, 1024)
        if rc:
            raise HarnessError(rc, err.value.decode())

    def outputs(self):
        n = lib(self.asan).h_dump(self.h, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        lib(self.asan).h_dump(self.h, buf, n + 1)
        return json.loads(buf.value.decode())
