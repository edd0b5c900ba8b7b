"""ctypes binding of the C ABI (include/siddhi_amd.h) in siddhi_amd/lib/libsiddhi_amd.so.

The product has no CPU fallback: importing works without a GPU (the library loads), but creating an app
fails loudly with SM_E_DEVICE when no MI355X is visible."""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# SM_LIB_VARIANT=<dir> loads siddhi_amd/<dir>/libsiddhi_amd.so instead (A/B builds of the same sources)
LIB_PATH = os.path.join(HERE, os.environ.get("SM_LIB_VARIANT", "lib"), "libsiddhi_amd.so")

SM_OK, SM_E_PARSE, SM_E_VALIDATION, SM_E_UNSUPPORTED, SM_E_TYPE, SM_E_DEVICE, SM_E_RUNTIME, SM_E_ARG = range(8)
TYPE_CODES = {"INT": 0, "LONG": 1, "FLOAT": 2, "DOUBLE": 3, "STRING": 4, "BOOL": 5}
TYPE_NAMES = {v: k for k, v in TYPE_CODES.items()}

# Every symbol include/siddhi_amd.h declares (checked by tests/test_boundary.py).
EXPORTS = [
    "sm_last_error", "sm_version", "sm_build_id", "sm_manager_create", "sm_manager_destroy", "sm_app_create", "sm_app_destroy",
    "sm_app_start", "sm_app_flush", "sm_app_shutdown", "sm_app_input_handler", "sm_input_send",
    "sm_input_send_columns", "sm_app_stream_schema", "sm_app_advance_time", "sm_app_advance_wallclock",
    "sm_app_add_stream_callback", "sm_app_add_query_callback", "sm_app_set_collect", "sm_app_dump_outputs",
    "sm_app_set_option", "sm_app_process_device_batch", "sm_app_process_device_events", "sm_app_device_matches",
    "sm_app_snapshot", "sm_app_restore", "sm_partition_by_owner", "sm_order_matches", "sm_app_copy_device_matches",
    "sm_app_get_stat", "sm_compile_dump", "sm_nfa_jit_compile", "sm_app_device_project", "sm_merge_heartbeats",
    "sm_unpack_records", "sm_count_events_callback", "sm_app_copy_device_outputs", "sm_order_outputs",
    "sm_app_add_stream_columns_callback", "sm_count_columns_callback",
]


class SmValue(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("is_null", ctypes.c_int32), ("i", ctypes.c_int64),
                ("d", ctypes.c_double), ("s", ctypes.c_char_p)]


class SmEvent(ctypes.Structure):
    _fields_ = [("timestamp", ctypes.c_int64), ("data", ctypes.POINTER(SmValue)), ("n", ctypes.c_int32)]


STREAM_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.POINTER(SmEvent), ctypes.c_size_t)
COLUMNS_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int64),
                              ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_uint8), ctypes.c_int32)
QUERY_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(SmEvent), ctypes.c_size_t,
                            ctypes.POINTER(SmEvent), ctypes.c_size_t)

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"siddhi_amd native library missing: {LIB_PATH} — run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        vp, cp, i64, sz = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64, ctypes.c_size_t
        L.sm_last_error.restype = cp
        L.sm_version.restype = cp
        L.sm_build_id.restype = cp
        L.sm_manager_create.argtypes = [ctypes.POINTER(vp)]
        L.sm_manager_destroy.argtypes = [vp]
        L.sm_app_create.argtypes = [vp, cp, ctypes.POINTER(vp)]
        L.sm_app_destroy.argtypes = [vp]
        for f in ("sm_app_start", "sm_app_flush", "sm_app_shutdown"):
            getattr(L, f).argtypes = [vp]
        L.sm_app_input_handler.argtypes = [vp, cp, ctypes.POINTER(vp)]
        L.sm_input_send.argtypes = [vp, i64, ctypes.POINTER(SmValue), sz]
        L.sm_input_send_columns.argtypes = [vp, sz, vp, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        L.sm_app_stream_schema.argtypes = [vp, cp, ctypes.POINTER(ctypes.c_int32), sz, ctypes.POINTER(sz)]
        L.sm_app_advance_time.argtypes = [vp, i64]
        L.sm_app_advance_wallclock.argtypes = [vp, i64]
        L.sm_app_add_stream_callback.argtypes = [vp, cp, STREAM_CB, vp]
        L.sm_app_add_query_callback.argtypes = [vp, cp, QUERY_CB, vp]
        L.sm_app_add_stream_columns_callback.argtypes = [vp, cp, COLUMNS_CB, vp]
        L.sm_app_set_collect.argtypes = [vp, ctypes.c_int]
        L.sm_app_dump_outputs.argtypes = [vp, ctypes.c_char_p, sz]
        L.sm_app_dump_outputs.restype = sz
        L.sm_app_set_option.argtypes = [vp, cp, i64]
        L.sm_app_process_device_batch.argtypes = [vp, cp, sz, vp, ctypes.POINTER(vp), vp, i64, vp]
        L.sm_app_process_device_events.argtypes = [vp, sz, vp, vp, ctypes.POINTER(vp), vp, i64, vp]
        L.sm_partition_by_owner.argtypes = [vp, ctypes.c_int, sz, ctypes.c_uint32, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                            ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_uint64), vp]
        L.sm_order_matches.argtypes = [vp, sz, i64, i64, vp, vp]
        L.sm_unpack_records.argtypes = [vp, sz, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int32),
                                        ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(vp), ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64), vp, vp]
        L.sm_merge_heartbeats.argtypes = [sz, vp, vp, vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int32),
                                          ctypes.POINTER(vp), sz, vp, vp, vp, vp, vp, ctypes.POINTER(vp),
                                          ctypes.POINTER(sz), vp]
        L.sm_app_copy_device_matches.argtypes = [vp, cp, vp, sz, ctypes.POINTER(sz), vp]
        L.sm_app_copy_device_outputs.argtypes = [vp, cp, vp, sz, ctypes.POINTER(sz), ctypes.POINTER(sz), vp]
        L.sm_order_outputs.argtypes = [vp, sz, sz, vp, vp]
        L.sm_app_snapshot.argtypes = [vp, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
        L.sm_app_restore.argtypes = [vp, ctypes.c_char_p, sz]
        L.sm_app_device_matches.argtypes = [vp, cp, ctypes.POINTER(vp), ctypes.POINTER(sz)]
        L.sm_app_device_project.argtypes = [vp, cp, vp, sz, vp, ctypes.POINTER(sz), ctypes.POINTER(ctypes.c_int32), vp]
        L.sm_app_get_stat.argtypes = [vp, cp, ctypes.POINTER(ctypes.c_double)]
        L.sm_compile_dump.argtypes = [cp, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
        L.sm_nfa_jit_compile.argtypes = [cp, ctypes.c_int, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
        _lib = L
    return _lib


class SiddhiError(Exception):
    code = SM_E_RUNTIME


class SiddhiParserException(SiddhiError):
    code = SM_E_PARSE


class SiddhiAppValidationException(SiddhiError):
    code = SM_E_VALIDATION


class SiddhiAppCreationException(SiddhiError):
    code = SM_E_VALIDATION


class OperationNotSupportedException(SiddhiError):
    code = SM_E_UNSUPPORTED


class SiddhiTypeError(SiddhiError):
    code = SM_E_TYPE


class SiddhiDeviceError(SiddhiError):
    code = SM_E_DEVICE


_ERRORS = {SM_E_PARSE: SiddhiParserException, SM_E_VALIDATION: SiddhiAppValidationException,
           SM_E_UNSUPPORTED: OperationNotSupportedException, SM_E_TYPE: SiddhiTypeError,
           SM_E_DEVICE: SiddhiDeviceError}


def check(rc):
    if rc != SM_OK:
        msg = lib().sm_last_error().decode(errors="replace")
        raise _ERRORS.get(rc, SiddhiError)(f"[{rc}] {msg}")
