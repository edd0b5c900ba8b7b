"""Runs a transcribed reference KAT (tests/golden/kats.json) against an engine.

An engine factory takes SiddhiQL text and returns an app object with start / send / advance_time /
flush / outputs (the oracle: tests/oracle_lib.OracleApp; the product: siddhi_amd.testing.ProductApp).
Wall-clock sleeps of the reference test become timestamp deltas; for absent ("not … for") tests that
ran on the wall clock the app is run in playback mode and the clock is advanced at every sleep
(the reference's playback heartbeat), which is where the wall-clock scheduler would have fired.
"""
import json
import os
import re

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BASE_TS = 1_000_000


def load_kats():
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        return json.load(f)


def stream_schemas(app):
    out = {}
    for m in re.finditer(r"define\s+stream\s+(\w+)\s*\(([^)]*)\)", app, re.I):
        cols = []
        for part in m.group(2).split(","):
            name, typ = part.split()
            cols.append(typ.upper())
        out[m.group(1)] = cols
    return out


def coerce(v, t):
    if v is None:
        return None
    if isinstance(v, dict):
        if "bool" in v:
            return bool(v["bool"])
        v = v["v"]
    if t in ("INT", "LONG"):
        return int(v)
    if t in ("FLOAT", "DOUBLE"):
        return float(v)
    if t == "BOOL":
        return bool(v)
    return v


def expected_value(v):
    if isinstance(v, dict):
        if "bool" in v:
            return v["bool"]
        return v["v"]
    return v


def values_equal(exp, act):
    e = expected_value(exp)
    if e is None or act is None:
        return e is None and act is None
    if isinstance(e, bool) or isinstance(act, bool):
        return e == act
    if isinstance(e, (int, float)) and isinstance(act, (int, float)):
        return float(e) == float(act)
    return e == act


class KatFailure(AssertionError):
    pass


def run_kat(factory, kat):
    app_text = kat["app"]
    wallclock_absent = kat.get("absent_wallclock", False)
    if wallclock_absent:
        app_text = "@app:playback " + app_text
    schemas = stream_schemas(app_text)
    try:
        app = factory(app_text)
    except Exception as e:  # creation-time error
        code = getattr(e, "code", None)
        if kat.get("expect_error"):
            return "error-as-expected"
        if code == 3:
            return "unsupported: " + str(e)
        raise
    try:
        return _drive(app, kat, schemas, wallclock_absent)
    finally:
        close = getattr(app, "close", None)
        if close:
            close()


def _outputs_for(outs, cb):
    if cb["kind"] == "query":
        calls = outs["queries"].get(cb["target"], [])
        return [ev for call in calls for ev in call[1]]
    return [e[1] for e in outs["streams"].get(cb["target"], [])]


def _drive(app, kat, schemas, wallclock_absent):
    wall = BASE_TS
    counters = {cb.get("counter"): cb for cb in kat["callbacks"]}
    checked = set()
    try:
        for ev in kat["events"]:
            tag = ev[0]
            if tag == "__start__":
                if wallclock_absent:
                    app.advance_time(wall)
                app.start()
            elif tag == "__sleep__":
                wall += ev[1]
                if wallclock_absent:
                    app.advance_wallclock(wall)
            elif tag == "__assert__":
                _, counter, n = ev
                cb = counters.get(counter)
                if cb is not None:
                    app.flush()
                    got = len(_outputs_for(app.outputs(), cb))
                    if got != n:
                        raise KatFailure(f"{cb['target']}: expected {n} events at this point, got {got}")
                    checked.add(counter)
            elif tag == "__wait__":
                _, sleep, count, counter, timeout = ev
                cb = counters.get(counter) or counters.get(counter + ".in")
                elapsed = 0
                while True:
                    app.flush()
                    have = len(_outputs_for(app.outputs(), cb)) if cb else count
                    if have >= count or elapsed > timeout:
                        break
                    wall += sleep
                    elapsed += sleep
                    if wallclock_absent:
                        app.advance_wallclock(wall)
            else:
                sid, ts, vals = ev
                types = schemas[sid]
                row = [coerce(v, t) for v, t in zip(vals, types)]
                if wallclock_absent and ts is None:
                    app.advance_wallclock(wall)
                app.send(sid, wall if ts is None else ts, row, types)
        app.flush()
    except Exception as e:
        if kat.get("expect_error"):
            return "error-as-expected"
        raise
    if kat.get("expect_error"):
        raise KatFailure("expected an error, none raised")
    outs = app.outputs()
    for cb in kat["callbacks"]:
        got = _outputs_for(outs, cb)
        if "count" in cb and cb.get("counter") not in checked and len(got) != cb["count"]:
            raise KatFailure(f"{cb['target']}: expected {cb['count']} events, got {len(got)}: {got[:6]}")
        for k, exp in cb.get("expect_by_index", {}).items():
            i = int(k) - 1
            if i < len(got):
                if len(exp) != len(got[i]) or not all(values_equal(a, b) for a, b in zip(exp, got[i])):
                    raise KatFailure(f"{cb['target']} event {k}: expected {exp}, got {got[i]}")
        if "expect_all" in cb:
            exp = cb["expect_all"]
            for i, g in enumerate(got):
                if len(exp) != len(g) or not all(values_equal(a, b) for a, b in zip(exp, g)):
                    raise KatFailure(f"{cb['target']} event {i + 1}: expected {exp}, got {g}")
    return "pass"


def drive_only(factory, kat):
    """Drive a KAT's event sequence (no expectation checks); returns the outputs dict or an error code."""
    app_text = kat["app"]
    wallclock_absent = kat.get("absent_wallclock", False)
    if wallclock_absent:
        app_text = "@app:playback " + app_text
    schemas = stream_schemas(app_text)
    try:
        app = factory(app_text)
    except Exception as e:
        return ("create-error", getattr(e, "code", None))
    wall = BASE_TS
    try:
        for ev in kat["events"]:
            tag = ev[0]
            if tag == "__start__":
                if wallclock_absent:
                    app.advance_time(wall)
                app.start()
            elif tag == "__sleep__":
                wall += ev[1]
                if wallclock_absent:
                    app.advance_wallclock(wall)
            elif tag in ("__assert__", "__wait__"):
                if tag == "__wait__":
                    # waits end immediately in synchronous processing when the count is reached; emulate by
                    # advancing `sleep` once (both engines see the same sequence)
                    pass
                continue
            else:
                sid, ts, vals = ev
                types = schemas[sid]
                row = [coerce(v, t) for v, t in zip(vals, types)]
                if wallclock_absent and ts is None:
                    app.advance_wallclock(wall)
                app.send(sid, wall if ts is None else ts, row, types)
        app.flush()
        return app.outputs()
    except Exception as e:
        return ("runtime-error", getattr(e, "code", None))
    finally:
        close = getattr(app, "close", None)
        if close:
            close()
