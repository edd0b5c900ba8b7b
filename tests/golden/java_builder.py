"""Transcribe the reference tests' programmatic Siddhi API (siddhi-query-api builders: StreamDefinition.id(..)
.attribute(..), new Query().from(InputStream.stream(..).filter(Expression..)).select(Selector.selector()..)
.insertInto(..), new SiddhiApp(..).defineStream(..).addQuery(..)) into the equivalent SiddhiQL text, so that
make_kats.py can turn those tests (FilterTestCase1/2) into known-answer fixtures like the text-based ones.

Test infrastructure (fixture generation only): reads the reference's Java test bodies as text, emits SiddhiQL."""
import re

TOK = re.compile(r'\s*(?:(?P<str>"(?:[^"\\]|\\.)*")|(?P<num>-?\d+(?:\.\d+)?(?:[eE][+-]?\d+)?[LlFfDd]?)|'
                 r'(?P<id>[A-Za-z_]\w*)|(?P<sym>[().,=]))')

OPS = {"EQUAL": "==", "NOT_EQUAL": "!=", "GREATER_THAN": ">", "GREATER_THAN_EQUAL": ">=", "LESS_THAN": "<",
       "LESS_THAN_EQUAL": "<="}
MATH = {"add": "+", "subtract": "-", "multiply": "*", "divide": "/", "mod": "%"}
TYPES = {"STRING": "string", "INT": "int", "LONG": "long", "FLOAT": "float", "DOUBLE": "double", "BOOL": "bool"}


class Unsupported(ValueError):
    pass


def tokens(s):
    out, i = [], 0
    while i < len(s):
        if s[i].isspace():
            i += 1
            continue
        m = TOK.match(s, i)
        if not m or m.end() == i:
            raise Unsupported(f"java builder: cannot tokenise {s[i:i + 20]!r}")
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
        i = m.end()
    return out


class Parser:
    """expr := primary ('.' IDENT ['(' args ')'])* ; primary := STR | NUM | 'new' IDENT '(' args ')' | IDENT"""

    def __init__(self, toks):
        self.t, self.i = toks, 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def eat(self, val=None):
        tok = self.peek()
        if val is not None and tok[1] != val:
            raise Unsupported(f"java builder: expected {val!r}, got {tok[1]!r}")
        self.i += 1
        return tok

    def args(self):
        self.eat("(")
        out = []
        if self.peek()[1] != ")":
            out.append(self.expr())
            while self.peek()[1] == ",":
                self.eat(",")
                out.append(self.expr())
        self.eat(")")
        return out

    def primary(self):
        kind, val = self.eat()
        if kind == "str":
            return ("str", bytes(val[1:-1], "utf-8").decode("unicode_escape"))
        if kind == "num":
            return ("num", val)
        if kind == "id" and val == "new":
            cls = self.eat()[1]
            return ("new", cls, self.args())
        if kind == "id":
            return ("name", val)
        raise Unsupported(f"java builder: unexpected {val!r}")

    def expr(self):
        node = self.primary()
        while self.peek()[1] == ".":
            self.eat(".")
            name = self.eat()[1]
            if self.peek()[1] == "(":
                node = ("call", node, name, self.args())
            else:
                node = ("field", node, name)
        return node


def parse(s):
    p = Parser(tokens(s))
    e = p.expr()
    if p.i != len(p.t):
        raise Unsupported("java builder: trailing tokens in " + s[:60])
    return e


def chain(node):
    """Flatten a call chain: (root, [(name, args), ...])"""
    calls = []
    while node[0] in ("call", "field"):
        calls.append((node[2], node[3] if node[0] == "call" else None))
        node = node[1]
    return node, calls[::-1]


def literal(node):
    if node[0] == "str":
        return "'" + node[1].replace("'", "\\'") + "'"
    if node[0] == "num":
        v = node[1]
        if v[-1] in "dD":
            v = v[:-1] + ("" if "." in v[:-1] else ".0")
        elif v[-1] in "fF":
            v = v[:-1] + "f"
        elif v[-1] in "lL":
            v = v[:-1] + "L"
        return v
    if node == ("name", "true") or node == ("name", "false"):
        return node[1]
    if node == ("name", "null"):
        return "null"
    raise Unsupported(f"java builder: literal {node!r}")


def expr(node):
    root, calls = chain(node)
    if root == ("name", "Expression") and calls:
        name, args = calls[0]
        rest = calls[1:]
        if name == "variable":
            text = args[0][1]
            for n2, a2 in rest:
                if n2 == "ofStream":
                    text = a2[0][1] + "." + text
                else:
                    raise Unsupported("java builder: variable." + n2)
            return text
        if rest:
            raise Unsupported("java builder: chained " + name)
        if name == "value":
            return literal(args[0])
        if name == "compare":
            op = chain(args[1])[1][-1][0]
            return f"({expr(args[0])} {OPS[op]} {expr(args[2])})"
        if name in MATH:
            return f"({expr(args[0])} {MATH[name]} {expr(args[1])})"
        if name in ("and", "or"):
            return f"({expr(args[0])} {name} {expr(args[1])})"
        if name == "not":
            return f"(not {expr(args[0])})"
        if name == "isNull":
            return f"({expr(args[0])} is null)"
    raise Unsupported(f"java builder: expression {node!r}"[:120])


def stream_def(node):
    root, calls = chain(node)
    if root != ("name", "StreamDefinition") or calls[0][0] != "id":
        raise Unsupported("java builder: stream definition")
    sid = calls[0][1][0][1]
    attrs = []
    for name, args in calls[1:]:
        if name != "attribute":
            raise Unsupported("java builder: StreamDefinition." + name)
        t = chain(args[1])[1][-1][0]
        attrs.append(f"{args[0][1]} {TYPES[t]}")
    return f"define stream {sid} ({', '.join(attrs)});"


def query_text(calls):
    ann, src, sel, out = "", None, "", None
    for name, args in calls:
        if name == "annotation":
            r, cs = chain(args[0])
            aname = cs[0][1][0][1]
            elems = ", ".join(f"{a[0][1]}='{a[1][1]}'" for n, a in cs[1:] if n == "element")
            ann = f"@{aname}({elems}) "
        elif name == "from":
            r, cs = chain(args[0])
            if r != ("name", "InputStream") or cs[0][0] != "stream":
                raise Unsupported("java builder: input stream")
            src = cs[0][1][0][1]
            for n, a in cs[1:]:
                if n != "filter":
                    raise Unsupported("java builder: InputStream." + n)
                src += f"[{expr(a[0])}]"
        elif name == "select":
            r, cs = chain(args[0])
            items = []
            for n, a in cs:
                if n == "selector":
                    continue
                if n != "select":
                    raise Unsupported("java builder: Selector." + n)
                items.append(a[0][1] if len(a) == 1 else f"{expr(a[1])} as {a[0][1]}")
            sel = "select " + ", ".join(items) + " " if items else ""
        elif name == "insertInto":
            if len(args) != 1:
                raise Unsupported("java builder: insertInto with an output event type")
            out = args[0][1]
        elif name == "query":
            continue
        else:
            raise Unsupported("java builder: Query." + name)
    if src is None or out is None:
        raise Unsupported("java builder: incomplete query")
    return f"{ann}from {src} {sel}insert into {out};"


def statements(body):
    body = re.sub(r"//[^\n]*", "", body)
    out, depth, cur, instr = [], 0, [], False
    i = 0
    while i < len(body):
        c = body[i]
        if c == '"':
            j = i + 1
            while body[j] != '"':
                j += 2 if body[j] == "\\" else 1
            cur.append(body[i:j + 1])
            i = j + 1
            continue
        if c in "({":
            depth += 1
        elif c in ")}":
            depth -= 1
        if c == ";" and depth == 0:
            out.append("".join(cur).strip())
            cur = []
        else:
            cur.append(c)
        i += 1
    return out


def builder_apps(body):
    """SiddhiQL text of every SiddhiApp variable the test body builds with the query API: {var: text}."""
    defs, queries, apps = {}, {}, {}
    for st in statements(body):
        st = " ".join(st.split())
        m = re.match(r"(?:final )?(StreamDefinition|Query|SiddhiApp) (\w+) = (.+)$", st)
        if m:
            kind, var, rhs = m.groups()
            node = parse(rhs)
            if kind == "StreamDefinition":
                defs[var] = stream_def(node)
            elif kind == "Query":
                root, calls = chain(node)
                queries[var] = calls if root != ("new", "Query", []) else calls
            else:
                root, calls = chain(node)
                apps[var] = {"streams": [], "queries": []}
                for name, args in calls:
                    (apps[var]["streams"] if name == "defineStream" else apps[var]["queries"]).append(args[0])
            continue
        m = re.match(r"(\w+)\.(\w+)\((.*)\)$", st)
        if not m:
            continue
        var, meth, arg = m.groups()
        if var in queries:
            queries[var].append((meth, parse(f"x.f({arg})")[3]))
        elif var in apps and meth in ("defineStream", "addQuery"):
            apps[var]["streams" if meth == "defineStream" else "queries"].append(parse(arg))
    texts = {}
    for var, a in apps.items():
        parts = []
        for s in a["streams"]:
            parts.append(defs[s[1]] if s[0] == "name" else stream_def(s))
        for q in a["queries"]:
            parts.append(query_text(queries[q[1]] if q[0] == "name" else chain(q)[1]))
        texts[var] = " ".join(parts)
    return texts
