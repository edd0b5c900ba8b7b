"""The drop-in boundary: the C-ABI library loads and exports every symbol include/siddhi_amd.h declares;
errors map to the reference's exception classes; no CPU fallback exists (app creation needs the GPU)."""
import ctypes
import os
import re

import pytest

import siddhi_amd
from siddhi_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    header = open(os.path.join(ROOT, "include", "siddhi_amd.h")).read()
    declared = set(re.findall(r"^\s*(?:int|void|size_t|const char\*)\s+(sm_\w+)\(", header, re.M))
    assert declared == set(_lib.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name


def test_version():
    assert b"gfx950" in _lib.lib().sm_version()


def test_parse_error_reported_before_device():
    m = siddhi_amd.SiddhiManager()
    with pytest.raises(siddhi_amd.SiddhiParserException):
        m.createSiddhiAppRuntime("define stream S (a int); from S[a >] select a insert into O;")


def test_unsupported_construct():
    m = siddhi_amd.SiddhiManager()
    with pytest.raises(siddhi_amd.OperationNotSupportedException):
        m.createSiddhiAppRuntime("define stream S (a int); from S#window.time(1 sec) select a insert into O;")


def test_validation_error():
    m = siddhi_amd.SiddhiManager()
    with pytest.raises(siddhi_amd.SiddhiAppValidationException):
        m.createSiddhiAppRuntime("define stream S (a int); from e1=S -> e2=S[b > e1.a] select e1.a as a insert into O;")


def test_no_cpu_fallback_without_gpu():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    m = siddhi_amd.SiddhiManager()
    with pytest.raises(siddhi_amd.SiddhiDeviceError):
        m.createSiddhiAppRuntime("define stream S (a int); from S[a > 1] select a insert into O;")


def test_build_id_names_the_sources_in_tree():
    """sm_build_id() is the hash gen_build_id.py computes over this tree's library sources: the loaded library was
    built from them (a profile recorded with this id measured this kernel build)."""
    import hashlib
    import glob
    import re
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "siddhi_amd", "csrc")
    mk = open(os.path.join(csrc, "Makefile")).read()
    srcs = re.search(r"^SRCS = (.*)$", mk, re.M).group(1).split()
    hdrs = [os.path.relpath(p, csrc) for pat in ("*.h", "siddhiql/*.h", "kernels/*.h") for p in
            glob.glob(os.path.join(csrc, pat))] + ["../../include/siddhi_amd.h"]
    files = sorted(set(srcs + hdrs + ["Makefile", "embed_jit.py", "gen_build_id.py"]))
    h = hashlib.sha256()
    h.update(b"")
    for f in files:
        h.update(b"\0" + os.path.basename(f).encode() + b"\0")
        h.update(open(os.path.join(csrc, f), "rb").read())
    got = _lib.lib().sm_build_id().decode()
    assert re.fullmatch(r"[0-9a-f]{16}", got)
    if os.environ.get("SM_LIB_VARIANT"):
        pytest.skip("an A/B library variant is loaded")
    assert got == h.hexdigest()[:16]
