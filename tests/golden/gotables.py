"""Minimal Go composite-literal reader used to transcribe the reference's
table-driven tests into JSON fixtures (tests/golden/*.json).

Run only in the development container, where /root/reference exists:
    python tests/golden/make_golden.py
The emitted JSON files are the committed golden vectors; the GPU box and the
test suite never read /root/reference.
"""
import re

TOKEN = re.compile(r'''
    (?P<ws>\s+|//[^\n]*|/\*.*?\*/) |
    (?P<str>"(?:\\.|[^"\\])*"|`[^`]*`) |
    (?P<num>-?\d+(?:\.\d+)?) |
    (?P<id>[A-Za-z_][A-Za-z0-9_]*(?:\.[A-Za-z_][A-Za-z0-9_]*)*) |
    (?P<p>[{}\[\]():,&*.])
''', re.S | re.X)


def tokenize(s):
    out = []
    for m in TOKEN.finditer(s):
        k = m.lastgroup
        if k == "ws":
            continue
        v = m.group(k)
        if k == "str":
            v = bytes(v[1:-1], "utf-8").decode("unicode_escape") if v[0] == '"' else v[1:-1]
        out.append((k, v))
    return out


class Comp:
    """A composite literal: type name + (key, value) items (key None for positional)."""

    def __init__(self, typ, items):
        self.typ, self.items = typ, items

    def get(self, key, default=None):
        for k, v in self.items:
            if k == key:
                return v
        return default

    def values(self):
        return [v for _, v in self.items]

    def __repr__(self):
        return "Comp(%s,%r)" % (self.typ, self.items)


class Call:
    def __init__(self, fn, args):
        self.fn, self.args = fn, args

    def __repr__(self):
        return "Call(%s,%r)" % (self.fn, self.args)


class Ref:
    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return "Ref(%s)" % self.name


class Parser:
    def __init__(self, toks):
        self.t, self.i = toks, 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def eat(self, v=None):
        tok = self.t[self.i]
        if v is not None and tok[1] != v:
            raise SyntaxError("expected %r got %r at %d" % (v, tok, self.i))
        self.i += 1
        return tok

    def parse_type(self):
        s = ""
        while True:
            k, v = self.peek()
            if v == "[":
                self.eat("[")
                if self.peek()[1] == "]":
                    self.eat("]")
                    s += "[]"
                else:
                    s += "[" + self.parse_type() + "]"
                    self.eat("]")
            elif v == "*":
                self.eat()
                s += "*"
            elif v == "map":
                self.eat()
                s += "map"
            elif v == "struct":
                self.eat()
                self.skip_braces()
                return s + "struct"
            elif k == "id":
                self.eat()
                return s + v
            else:
                return s

    def skip_braces(self):
        depth = 0
        while True:
            _, v = self.eat()
            if v == "{":
                depth += 1
            elif v == "}":
                depth -= 1
                if depth == 0:
                    return

    def parse_value(self):
        k, v = self.peek()
        if v == "&":
            self.eat()
            return self.parse_value()
        if v == "{":
            return self.parse_body(None)
        if v in ("[", "map", "*"):
            typ = self.parse_type()
            return self.parse_body(typ)
        if k == "str":
            self.eat()
            return v
        if k == "num":
            self.eat()
            return float(v) if "." in v else int(v)
        if v == "-":
            self.eat()
            return -self.parse_value()
        if k == "id":
            self.eat()
            nk, nv = self.peek()
            if nv == "{":
                return self.parse_body(v)
            if nv == "(":
                self.eat("(")
                args = []
                while self.peek()[1] != ")":
                    args.append(self.parse_value())
                    if self.peek()[1] == ",":
                        self.eat(",")
                self.eat(")")
                val = Call(v, args)
                while self.peek()[1] == ".":  # method chain: f(x).Method(y)
                    self.eat(".")
                    _, name = self.eat()
                    margs = []
                    if self.peek()[1] == "(":
                        self.eat("(")
                        while self.peek()[1] != ")":
                            margs.append(self.parse_value())
                            if self.peek()[1] == ",":
                                self.eat(",")
                        self.eat(")")
                    val = Call(name, [val] + margs)
                return val
            if v == "true":
                return True
            if v == "false":
                return False
            if v == "nil":
                return None
            return Ref(v)
        raise SyntaxError("unexpected %r" % (self.peek(),))

    def parse_body(self, typ):
        self.eat("{")
        items = []
        while self.peek()[1] != "}":
            val = self.parse_value()
            if self.peek()[1] == ":":
                self.eat(":")
                key = val.name if isinstance(val, Ref) else val
                val = self.parse_value()
                items.append((key, val))
            else:
                items.append((None, val))
            if self.peek()[1] == ",":
                self.eat(",")
        self.eat("}")
        return Comp(typ, items)


def func_body(src, name):
    i = src.index("func %s(" % name)
    j = src.index("{", src.index(")", i))
    depth, k = 0, j
    while True:
        c = src[k]
        if c == "{":
            depth += 1
        elif c == "}":
            depth -= 1
            if depth == 0:
                return src[j:k + 1], src[:j].count("\n") + 1
        elif c == '"':
            k += 1
            while src[k] != '"':
                k += 2 if src[k] == "\\" else 1
        elif c == "`":
            k = src.index("`", k + 1)
        k += 1


def table(src, func, var="tests"):
    """Parses `var := []struct{...}{...}` inside func; returns (list of Comp, line)."""
    body, line0 = func_body(src, func)
    m = re.search(r"\b%s\s*:?=\s*\[\]struct\s*\{" % var, body)
    if not m:
        m = re.search(r"\b%s\s*:?=\s*\[\]\w+\s*\{" % var, body)
    toks = tokenize(body[m.start():])
    p = Parser(toks)
    p.eat()  # var
    p.eat()  # := or =  (tokenized as ':' then '='?)
    while p.peek()[1] != "[":
        p.eat()
    p.parse_type()
    comp = p.parse_body("table")
    return comp.values(), line0 + body[:m.start()].count("\n")
