"""Generate tests/golden/kats.json from the reference's TestNG suites (run HERE only, where
/root/reference exists; the JSON it writes is committed and travels to the GPU box).

Each reference test builds a SiddhiQL app, sends events (with wall-clock timestamps separated by
Thread.sleep, or explicit timestamps in playback tests) and asserts on the callback outputs. This script
re-expresses each test as data: the app text, the event sequence with explicit
timestamps (cumulative sleeps → timestamp deltas), and the expected outputs (ordered data arrays where
the test pins them, plus the final counts). Only literal test data is emitted — no reference source text.

Tests whose structure this extractor cannot reduce to data (loops, persistence, custom extensions,
Thread-based sends, ...) are listed with a reason and skipped.
"""
import json
import os
import re

import java_builder  # noqa: E402 (same directory)
import struct
import sys

REF = "/root/reference/modules/siddhi-core/src/test/java/org/wso2/siddhi/core/query"
SUITES = [
    "pattern/EveryPatternTestCase.java",
    "pattern/WithinPatternTestCase.java",
    "pattern/CountPatternTestCase.java",
    "pattern/LogicalPatternTestCase.java",
    "pattern/ComplexPatternTestCase.java",
    "sequence/SequenceTestCase.java",
    "partition/PatternPartitionTestCase.java",
    "partition/SequencePartitionTestCase.java",
    "FilterTestCase1.java",
    "FilterTestCase2.java",
    "pattern/absent/AbsentPatternTestCase.java",
    "pattern/absent/EveryAbsentPatternTestCase.java",
    "pattern/absent/LogicalAbsentPatternTestCase.java",
    "pattern/absent/AbsentWithEveryPatternTestCase.java",
    "sequence/absent/AbsentSequenceTestCase.java",
    "sequence/absent/EveryAbsentSequenceTestCase.java",
    "sequence/absent/LogicalAbsentSequenceTestCase.java",
    "sequence/absent/AbsentWithEverySequenceTestCase.java",
]
BASE_TS = 1_000_000  # arbitrary wall-clock origin for sleep-based tests


def f32(x):
    return struct.unpack("f", struct.pack("f", float(x)))[0]


def split_methods(src):
    """Yield (name, annotation, body, start_line) for each @Test method."""
    for m in re.finditer(r"@Test(\([^)]*\))?\s*public void (\w+)\(\)[^{]*\{", src):
        start = m.end()
        depth, i = 1, start
        while depth and i < len(src):
            c = src[i]
            if c == '"':
                j = i + 1
                while src[j] != '"':
                    j += 2 if src[j] == "\\" else 1
                i = j
            elif c == "{":
                depth += 1
            elif c == "}":
                depth -= 1
            i += 1
        line = src.count("\n", 0, m.start()) + 1
        yield m.group(2), m.group(1) or "", src[start:i - 1], line


STR_LIT = r'"(?:[^"\\]|\\.)*"'


def java_str(lit):
    return bytes(lit[1:-1], "utf-8").decode("unicode_escape")


def eval_concat(expr, env):
    """Evaluate a Java string concatenation of literals / known variables."""
    out = []
    for tok in re.finditer(STR_LIT + r"|\w+", expr):
        t = tok.group(0)
        if t.startswith('"'):
            out.append(java_str(t))
        elif t in env:
            out.append(env[t])
        else:
            raise ValueError("unknown symbol in concat: " + t)
    return "".join(out)


def parse_value(v):
    v = v.strip()
    if v == "null":
        return None
    if v in ("true", "false"):
        return {"bool": v == "true"}
    if v.startswith('"'):
        return java_str(v)
    m = re.fullmatch(r"\(\s*(int|long|float|double|Integer|Long|Float|Double)\s*\)\s*(.+)", v)
    if m:
        t, rest = m.groups()
        inner = parse_value(rest)
        num = inner["v"] if isinstance(inner, dict) else inner
        t = t.lower()[:1]
        return {"t": {"i": "int", "l": "long", "f": "float", "d": "double"}[t], "v": float(num) if t in "fd" else int(num)}
    m = re.fullmatch(r"([-+]?\d+(?:\.\d*)?(?:[eE][-+]?\d+)?|[-+]?\.\d+(?:[eE][-+]?\d+)?)([fFdDlL]?)", v)
    if not m:
        raise ValueError("unsupported literal: " + v)
    num, suf = m.groups()
    if suf in ("f", "F"):
        return {"t": "float", "v": f32(num)}
    if suf in ("l", "L"):
        return {"t": "long", "v": int(num)}
    if suf in ("d", "D") or "." in num or "e" in num.lower():
        return {"t": "double", "v": float(num)}
    return {"t": "int", "v": int(num)}


def split_args(s):
    out, depth, cur, i = [], 0, "", 0
    while i < len(s):
        c = s[i]
        if c == '"':
            m = re.match(STR_LIT, s[i:])
            cur += m.group(0)
            i += len(m.group(0))
            continue
        if c in "({[":
            depth += 1
        elif c in ")}]":
            depth -= 1
        if c == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += c
        i += 1
    if cur.strip():
        out.append(cur)
    return out


def extract(path, name, ann, body, line):
    rel = "modules/siddhi-core/src/test/java/org/wso2/siddhi/core/query/" + path
    kat = {"name": f"{os.path.basename(path)[:-5]}.{name}", "source": f"{rel}:{line}"}
    if "expectedExceptions" in ann:
        kat["expect_error"] = True
    for bad, why in [("persist", "persistence"), ("restoreRevision", "persistence"), ("for (", "loop"),
                     ("while (", "loop"), ("new Thread", "threads"), ("setExtension", "extension"),
                     ("getSiddhiAppRuntime(", "multiple runtimes"), ("debug()", "debugger"),
                     ("removeCallback", "callbacks"), ("ExecutorService", "threads"),
                     ("addCallback(\"#", "inner stream callback")]:
        if bad in body:
            # loops inside callbacks (for (Event event : inEvents)) are fine
            if bad == "for (" and all("Event " in m or "Event event" in m
                                      for m in re.findall(r"for \(([^)]*)\)", body)):
                continue
            kat["skip"] = why
            return kat
    env = {}
    for m in re.finditer(r"String (\w+)\s*=\s*((?:" + STR_LIT + r"|\w+|\s|\+)+);", body):
        try:
            env[m.group(1)] = eval_concat(m.group(2), env)
        except ValueError as e:
            kat["skip"] = str(e)
            return kat
    if "new SiddhiApp(" in body or "SiddhiApp.siddhiApp(" in body:
        try:  # programmatic query API (FilterTestCase1/2): transcribe the builders into SiddhiQL text
            env.update(java_builder.builder_apps(body))
        except java_builder.Unsupported as e:
            kat["skip"] = str(e)
            return kat
    m = re.search(r"createSiddhiAppRuntime\(([^;]*)\);", body)
    if not m:
        kat["skip"] = "no app"
        return kat
    try:
        kat["app"] = eval_concat(m.group(1), env)
    except ValueError as e:
        kat["skip"] = str(e)
        return kat
    handlers = dict(re.findall(r"InputHandler (\w+)\s*=\s*\w+\.getInputHandler\(\"(\w+)\"\)", body))
    # callbacks
    cbs = []
    for m in re.finditer(r"addCallback\(\"(\w+)\",\s*new (QueryCallback|StreamCallback)\(\)\s*\{", body):
        start = m.end()
        depth, i = 1, start
        while depth:
            depth += {"{": 1, "}": -1}.get(body[i], 0)
            i += 1
        cb_body = body[start:i - 1]
        cb = {"target": m.group(1), "kind": "query" if m.group(2) == "QueryCallback" else "stream"}
        cands = [m2.group(1) for pat in (r"(\w+)\s*=\s*\1\s*\+\s*(?:inEvents|events)\.length",
                                          r"(\w+)\s*\+=\s*(?:inEvents|events)\.length", r"(\w+)\+\+",
                                          r"(\w+)\.incrementAndGet\(\)", r"(\w+)\.addAndGet\((?:inEvents|events)")
                 for m2 in re.finditer(pat, cb_body)]
        cands = [c for c in cands if "remove" not in c.lower()]
        cb["counter"] = cands[0] if cands else None
        exp = {}
        uncond = []
        sw = re.search(r"switch\s*\((\w+)(?:\.get\(\))?\)\s*\{(.*)\}", cb_body, re.S)
        arrays = list(re.finditer(r"assertArrayEquals\(\s*new\s+Object\[\]\s*\{(.*?)\}\s*,\s*(\w+)(\[\d+\])?\.getData\(\)\)",
                                  cb_body, re.S))
        try:
            if sw:
                for cm2 in re.finditer(r"case\s+(\d+):(.*?)(?=case\s+\d+:|default:|$)", sw.group(2), re.S):
                    am = re.search(r"assertArrayEquals\(\s*new\s+Object\[\]\s*\{(.*?)\}\s*,", cm2.group(2), re.S)
                    if am:
                        exp[int(cm2.group(1))] = [parse_value(x) for x in split_args(am.group(1))]
                if exp and min(exp) == 0:
                    exp = {k + 1: v for k, v in exp.items()}
            elif len(arrays) == 1 and not re.search(r"\bif\s*\((?!inEvents|events|removeEvents)", cb_body):
                uncond = [parse_value(x) for x in split_args(arrays[0].group(1))]
            elif arrays:
                cb["unpinned_data"] = True
        except ValueError as e:
            kat["skip"] = str(e)
            return kat
        if exp:
            cb["expect_by_index"] = {str(k): v for k, v in sorted(exp.items())}
        if uncond:
            cb["expect_all"] = uncond
        cbs.append(cb)
    for m in re.finditer(r"TestUtil\.TestCallback (\w+)\s*=\s*TestUtil\.add(Query|Stream)Callback\(\s*\w+\s*,\s*\"(\w+)\"\s*,?(.*?)\);",
                         body, re.S):
        cb = {"target": m.group(3), "kind": m.group(2).lower(), "counter": m.group(1) + ".in"}
        try:
            seq = [[parse_value(x) for x in split_args(a.group(1))]
                   for a in re.finditer(r"new\s+Object\[\]\s*\{(.*?)\}(?=\s*[,)]|\s*$)", m.group(4), re.S)]
        except ValueError as e:
            kat["skip"] = str(e)
            return kat
        if seq:
            cb["expect_by_index"] = {str(i + 1): v for i, v in enumerate(seq)}
        cbs.append(cb)
    kat["callbacks"] = cbs
    # sends and sleeps in program order (outside callbacks)
    main = body
    for m in re.finditer(r"addCallback\(.*?\n\s*\}\);", body, re.S):
        main = main.replace(m.group(0), "")
    events, ts = [], BASE_TS
    # local event-time variables: `long t = System.currentTimeMillis();` then `t += 1000;` (explicit timestamps
    # relative to the run's base time, e.g. EveryAbsentPatternTestCase.testQueryAbsent3's playback clock)
    tvars = {}
    for m in re.finditer(r"long\s+(\w+)\s*=\s*System\.currentTimeMillis\(\)\s*;|(\w+)\s*\+=\s*(\d+)L?\s*;|"
                         r"(\w+)\.send\((.*?)\);\s*$|Thread\.sleep\((\d+)\)|siddhiAppRuntime\.start\(\)|"
                         r"waitForEvents\(\s*(\d+)\s*,\s*(\d+)\s*,\s*(\w+)\s*,\s*(\d+)\s*\)|"
                         r"assertEquals\((?:\"[^\"]*\",\s*)?(\d+),\s*(\w+)(\.get\(\)|\.getInEventCount\(\))?\)|"
                         r"siddhiAppRuntime\.shutdown\(\)",
                         main, re.S | re.M):
        if m.group(0).startswith("siddhiAppRuntime.shutdown"):
            break
        if m.group(1):
            tvars[m.group(1)] = BASE_TS
            continue
        if m.group(2):
            if m.group(2) in tvars:
                tvars[m.group(2)] += int(m.group(3))
            continue
        if m.group(11):
            name = m.group(12) + (".in" if m.group(13) == ".getInEventCount()" else "")
            events.append(["__assert__", name, int(m.group(11))])
            continue
        if m.group(6):
            ts += int(m.group(6))
            events.append(["__sleep__", int(m.group(6))])
            continue
        if m.group(7):
            events.append(["__wait__", int(m.group(7)), int(m.group(8)), m.group(9), int(m.group(10))])
            continue
        if m.group(0).startswith("siddhiAppRuntime.start"):
            events.append(["__start__"])
            continue
        h, args = m.group(4), m.group(5).strip()
        if h not in handlers:
            kat["skip"] = "send on unknown handler " + h
            return kat
        try:
            am = re.fullmatch(r"new\s+Object\[\]\s*\{(.*)\}", args, re.S)
            if am:
                events.append([handlers[h], None, [parse_value(x) for x in split_args(am.group(1))]])
                continue
            am = re.fullmatch(r"(\d+)L?\s*,\s*new\s+Object\[\]\s*\{(.*)\}", args, re.S)
            if am:
                events.append([handlers[h], int(am.group(1)), [parse_value(x) for x in split_args(am.group(2))]])
                continue
            am = re.fullmatch(r"(\w+)\s*,\s*new\s+Object\[\]\s*\{(.*)\}", args, re.S)
            if am and am.group(1) in tvars:
                events.append([handlers[h], tvars[am.group(1)], [parse_value(x) for x in split_args(am.group(2))]])
                continue
            am = re.fullmatch(r"new Event\((\d+)L?\s*,\s*new\s+Object\[\]\s*\{(.*)\}\)", args, re.S)
            if am:
                events.append([handlers[h], int(am.group(1)), [parse_value(x) for x in split_args(am.group(2))]])
                continue
            am = re.fullmatch(r"new Event\[\]\s*\{(.*)\}", args, re.S)
            if am:
                for ev in re.finditer(r"new Event\((\d+)L?\s*,\s*new\s+Object\[\]\s*\{(.*?)\}\)", am.group(1), re.S):
                    events.append([handlers[h], int(ev.group(1)), [parse_value(x) for x in split_args(ev.group(2))]])
                continue
        except ValueError as e:
            kat["skip"] = str(e)
            return kat
        kat["skip"] = "unsupported send form"
        return kat
    if "siddhiAppRuntime.start()" not in main:
        events.insert(0, ["__start__"])
    kat["events"] = events
    # final count assertions
    counts = {}
    for m in re.finditer(r"assertEquals\((?:\"[^\"]*\",\s*)?(\d+),\s*(\w+)(?:\.get\(\))?\)", main):
        counts[m.group(2)] = int(m.group(1))
    for m in re.finditer(r"assertEquals\((?:\"[^\"]*\",\s*)?(\w+)(?:\.get\(\))?,\s*(\d+)\)", main):
        counts.setdefault(m.group(1), int(m.group(2)))
    for m in re.finditer(r"waitForEvents\(\s*\d+\s*,\s*(\d+)\s*,\s*(\w+)\s*,", main):
        counts.setdefault(m.group(2), int(m.group(1)))
    for m in re.finditer(r"assertEquals\((?:\"[^\"]*\",\s*)?(\d+),\s*(\w+)\.getInEventCount\(\)\)", main):
        counts[m.group(2) + ".in"] = int(m.group(1))
    for cb in cbs:
        if cb["counter"] in counts:
            cb["count"] = counts[cb["counter"]]
    if "@app:playback" not in kat["app"] and re.search(r"\bnot\s+\w+", kat["app"]):
        kat["absent_wallclock"] = True
    if not any("count" in cb or "expect_by_index" in cb or "expect_all" in cb for cb in cbs) and \
            not kat.get("expect_error"):
        kat["skip"] = "no pinned expectation"
    return kat


def main():
    kats, skipped = [], 0
    for suite in SUITES:
        src = open(os.path.join(REF, suite)).read()
        for name, ann, body, line in split_methods(src):
            k = extract(suite, name, ann, body, line)
            if "skip" in k:
                skipped += 1
            kats.append(k)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kats.json")
    with open(out, "w") as f:
        json.dump(kats, f, indent=0)
    print(f"{len(kats)} tests, {len(kats) - skipped} extracted, {skipped} skipped -> {out}", file=sys.stderr)


if __name__ == "__main__":
    main()
