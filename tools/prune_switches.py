"""Resolve compile-time experiment switches to their defaults (a small unifdef).

    python tools/prune_switches.py FILE... --keep NAME,NAME,...

Every `SHIPENV_*` macro that a file gives a default with the form

    #ifndef SHIPENV_X
    #define SHIPENV_X <value>
    #endif

and that is not listed in --keep is resolved: the default block is dropped and every
`#if` / `#elif` whose expression mentions only resolved macros and integer constants is
evaluated, keeping the taken branch's text and dropping the rest. Expressions that mention
any other identifier are left as they are (their branches are still processed). Remaining
textual uses of a resolved macro (in code, not in a directive) are reported, not rewritten.

Used once in round 6 to delete the variants measured slower or even;
`tools/isa_diff.sh` checks that the product kernels' ISA did not change.
"""
from __future__ import annotations

import re
import sys

DIRECTIVE = re.compile(r"^\s*#\s*(if|ifdef|ifndef|elif|else|endif|define|undef)\b(.*)$")
IDENT = re.compile(r"[A-Za-z_]\w*")


def strip_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s)
    return s.split("//", 1)[0]


class Expr:
    """C preprocessor integer expressions: || && | ^ & == != < <= > >= << >> + - * / % ! ~ ( )."""

    TOK = re.compile(r"\s*(\d+|[A-Za-z_]\w*|\|\||&&|==|!=|<=|>=|<<|>>|[()!~<>|^&+\-*/%])")

    def __init__(self, text, env):
        self.toks = []
        pos = 0
        text = text.strip()
        while pos < len(text):
            m = self.TOK.match(text, pos)
            if not m:
                raise ValueError(f"cannot tokenise {text!r}")
            self.toks.append(m.group(1))
            pos = m.end()
            while pos < len(text) and text[pos].isspace():
                pos += 1
        self.i = 0
        self.env = env

    def peek(self):
        return self.toks[self.i] if self.i < len(self.toks) else None

    def take(self):
        t = self.peek()
        self.i += 1
        return t

    def parse(self):
        v = self.binary(0)
        if self.peek() is not None:
            raise ValueError("trailing tokens")
        return v

    LEVELS = [["||"], ["&&"], ["|"], ["^"], ["&"], ["==", "!="], ["<", "<=", ">", ">="],
              ["<<", ">>"], ["+", "-"], ["*", "/", "%"]]

    def binary(self, lvl):
        if lvl == len(self.LEVELS):
            return self.unary()
        v = self.binary(lvl + 1)
        while self.peek() in self.LEVELS[lvl]:
            op = self.take()
            w = self.binary(lvl + 1)
            v = {"||": lambda a, b: int(bool(a) or bool(b)), "&&": lambda a, b: int(bool(a) and bool(b)),
                 "|": lambda a, b: a | b, "^": lambda a, b: a ^ b, "&": lambda a, b: a & b,
                 "==": lambda a, b: int(a == b), "!=": lambda a, b: int(a != b),
                 "<": lambda a, b: int(a < b), "<=": lambda a, b: int(a <= b),
                 ">": lambda a, b: int(a > b), ">=": lambda a, b: int(a >= b),
                 "<<": lambda a, b: a << b, ">>": lambda a, b: a >> b,
                 "+": lambda a, b: a + b, "-": lambda a, b: a - b, "*": lambda a, b: a * b,
                 "/": lambda a, b: int(a / b), "%": lambda a, b: a % b}[op](v, w)
        return v

    def unary(self):
        t = self.take()
        if t == "!":
            return int(not self.unary())
        if t == "~":
            return ~self.unary()
        if t == "-":
            return -self.unary()
        if t == "(":
            v = self.binary(0)
            if self.take() != ")":
                raise ValueError("unbalanced")
            return v
        if t == "defined":
            paren = self.peek() == "("
            if paren:
                self.take()
            name = self.take()
            if paren:
                self.take()
            return int(name in self.env)
        if t is not None and t.isdigit():
            return int(t)
        if t in self.env:
            return self.env[t]
        raise KeyError(t)


def resolve(expr, env):
    """The expression's value if every identifier in it is resolved, else None."""
    expr = strip_comments(expr)
    names = set(IDENT.findall(expr)) - {"defined"}
    if not names or not names <= set(env):
        return None
    return Expr(expr, env).parse()


def collect_defaults(lines, keep):
    """SHIPENV_* defaults given as #ifndef X / #define X v / #endif."""
    raw = {}
    for i in range(len(lines)):
        m = re.match(r"^\s*#\s*ifndef\s+(SHIPENV_\w+)\s*$", lines[i])
        if not m or m.group(1) in keep:
            continue
        j = i + 1
        while j < len(lines) and lines[j].strip().startswith("//"):
            j += 1
        d = re.match(r"^\s*#\s*define\s+(SHIPENV_\w+)\s*(.*)$", lines[j])
        k = j + 1
        while k < len(lines) and lines[k].strip().startswith("//"):
            k += 1
        if d and d.group(1) == m.group(1) and re.match(r"^\s*#\s*endif\b", lines[k]):
            raw[m.group(1)] = strip_comments(d.group(2)).strip()
    return raw


def evaluate_defaults(raw):
    env = {}
    pending = dict(raw)
    for _ in range(10):
        for k, v in list(pending.items()):
            try:
                val = resolve(v, env) if IDENT.search(v) else int(v)
            except (KeyError, ValueError):
                val = None
            if val is not None:
                env[k] = val
                del pending[k]
    if pending:
        raise SystemExit(f"unresolvable defaults: {pending}")
    return env


def prune(lines, env):
    out = []
    stack = []  # each: dict(kind='keep'|'res', active, taken, emitted)

    def emitting():
        return all(s["active"] for s in stack)

    i = 0
    n = len(lines)
    while i < n:
        line = lines[i]
        m = DIRECTIVE.match(line)
        if not m:
            if emitting():
                out.append(line)
            i += 1
            continue
        kw, rest = m.group(1), m.group(2)
        parent = emitting()
        if kw in ("if", "ifdef", "ifndef"):
            if kw == "if":
                r = resolve(rest, env)
            else:
                name = strip_comments(rest).strip()
                if name in env:
                    r = int(kw == "ifdef")
                    if kw == "ifndef":
                        r = 1  # the default block: taken, its #define dropped below
                else:
                    r = None
            if r is None:
                stack.append(dict(kind="keep", active=True, taken=False, emitted=True, parent=parent))
                if parent:
                    out.append(line)
            else:
                stack.append(dict(kind="res", active=bool(r), taken=bool(r), emitted=False, parent=parent))
        elif kw == "elif":
            s = stack[-1]
            r = resolve(rest, env)
            if s["kind"] == "res":
                if s["taken"]:
                    s["active"] = False
                elif r is None:
                    s["kind"] = "keep"
                    s["emitted"] = True
                    s["active"] = True
                    if s["parent"]:
                        out.append(re.sub(r"#\s*elif", "#if", line, count=1))
                else:
                    s["active"] = bool(r)
                    s["taken"] = bool(r)
            else:  # keep
                if s["taken"]:
                    s["active"] = False
                elif r is None:
                    s["active"] = True
                    if s["parent"]:
                        out.append(line)
                elif r:
                    s["active"] = True
                    s["taken"] = True
                    if s["parent"]:
                        out.append(re.sub(r"#\s*elif.*", "#else", line, count=1))
                else:
                    s["active"] = False
        elif kw == "else":
            s = stack[-1]
            if s["kind"] == "res":
                s["active"] = not s["taken"]
            else:
                if s["taken"]:
                    s["active"] = False
                else:
                    s["active"] = True
                    if s["parent"]:
                        out.append(line)
        elif kw == "endif":
            s = stack.pop()
            if s["kind"] == "keep" and s["parent"]:
                out.append(line)
        elif kw in ("define", "undef"):
            name = IDENT.match(rest.strip()).group(0) if rest.strip() else ""
            if name in env:
                pass  # the resolved macro's default definition
            elif parent:
                out.append(line)
        i += 1
    assert not stack, "unbalanced conditionals"
    return out


def main(argv):
    keep = set()
    files = []
    it = iter(argv)
    for a in it:
        if a == "--keep":
            keep |= {k for k in next(it).split(",") if k}
        else:
            files.append(a)
    texts = {f: open(f).read().split("\n") for f in files}
    raw = {}
    for f, lines in texts.items():
        raw.update(collect_defaults(lines, keep))
    env = evaluate_defaults(raw)
    print("resolved:", ", ".join(f"{k}={v}" for k, v in sorted(env.items())))
    for f, lines in texts.items():
        out = prune(lines, env)
        with open(f, "w") as fh:
            fh.write("\n".join(out))
        for ln, line in enumerate(out, 1):
            for name in IDENT.findall(strip_comments(line)):
                if name in env:
                    print(f"{f}:{ln}: remaining use of {name}: {line.strip()}")


if __name__ == "__main__":
    main(sys.argv[1:])
