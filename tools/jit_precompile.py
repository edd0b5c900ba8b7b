"""Fill the query-specialised NFA kernels' code-object cache (siddhi_amd/jit_cache, nfa_jit.cpp) on the build host for
the plans the GPU tests and bench.py run, so that a GPU box loads them instead of compiling each for minutes. CPU only;
one process per plan. Usage: python tools/jit_precompile.py [-j N]"""
import argparse
import ctypes
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def plans():
    import bench
    import synth
    from test_device_events import VARIANTS
    apps = {"bench_config5": bench.APP5}
    for k, v in VARIANTS.items():
        apps[f"device_events_{k}"] = synth.app5(v)
    for k, v in bench.VARIANTS5.items():
        apps[f"bench_{k}"] = bench.app5_variant(v)
    return apps


def one(name):
    # torch first, as in every test and bench process: the library then compiles with the hiprtc and comgr torch
    # bundles, which make faster code for this kernel than /opt/rocm's (nfa_jit.cpp; the cache key has the version)
    import torch  # noqa: F401
    from siddhi_amd import _lib
    app = plans()[name]
    L = _lib.lib()
    log = ctypes.create_string_buffer(8192)
    size = ctypes.c_size_t()
    t = time.time()
    rc = L.sm_nfa_jit_compile(app.encode(), 0, log, 8192, ctypes.byref(size))
    print(f"{name}: rc {rc}, {size.value} bytes, {time.time() - t:.0f} s {log.value.decode()[:200]}", flush=True)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=4)
    ap.add_argument("--one")
    ap.add_argument("--only", help="comma-separated plan names")
    a = ap.parse_args()
    if a.one:
        sys.exit(one(a.one))
    env = dict(os.environ, SM_NFA_JIT_COMPACT="1")
    names = a.only.split(",") if a.only else list(plans())
    procs, rc = [], 0
    while names or procs:
        while names and len(procs) < a.j:
            name = names.pop(0)
            procs.append(subprocess.Popen([sys.executable, __file__, "--one", name], env=env))
        p = procs.pop(0)
        rc |= p.wait()
    sys.exit(rc)


if __name__ == "__main__":
    main()
