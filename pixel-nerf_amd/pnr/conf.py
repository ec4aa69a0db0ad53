"""Config access for the hot-path constructors.

The reference reads pyhocon ``ConfigTree`` objects through ``get_int / get_float /
get_bool / get_string / get_list`` and ``conf["subtree"]`` (args.py:99,
models.py:21-74, nerf.py:340-352).  ``make_model`` / ``NeRFRenderer.from_conf``
here accept a real pyhocon tree unchanged, a plain dict, or a :class:`Conf`.

pyhocon is not installed in this image, so :func:`parse_file` implements the
HOCON subset the shipped ``conf/*.conf`` files use (objects, ``=``/``:``,
lists, ``include required("...")``, ``#``/``//`` comments, object merging).
"""
import os
import re

__all__ = ["Conf", "as_conf", "parse_file", "parse_string"]

_MISSING = object()


class Conf(dict):
    """dict with pyhocon-style typed getters; nested dicts come back as Conf."""

    def __getitem__(self, k):
        if not dict.__contains__(self, k) and isinstance(k, str) and "." in k:
            return self._get(k)   # conf["loss.rgb"] reaches into subtrees, as pyhocon does (train.py:111)
        v = dict.__getitem__(self, k)
        return Conf(v) if isinstance(v, dict) and not isinstance(v, Conf) else v

    def _get(self, k, default=_MISSING):
        cur = self
        for part in str(k).split("."):
            if not isinstance(cur, dict) or part not in cur:
                if default is _MISSING:
                    raise KeyError(k)
                return default
            cur = dict.__getitem__(cur, part)
        return Conf(cur) if isinstance(cur, dict) and not isinstance(cur, Conf) else cur

    def get(self, k, default=None):
        return self._get(k, default)

    def get_int(self, k, default=_MISSING):
        v = self._get(k, default)
        return None if v is None else int(v)

    def get_float(self, k, default=_MISSING):
        v = self._get(k, default)
        return None if v is None else float(v)

    def get_bool(self, k, default=_MISSING):
        v = self._get(k, default)
        if isinstance(v, str):
            return v.strip().lower() in ("true", "yes", "on", "1")
        return None if v is None else bool(v)

    def get_string(self, k, default=_MISSING):
        v = self._get(k, default)
        return None if v is None else str(v)

    def get_list(self, k, default=_MISSING):
        v = self._get(k, default)
        return None if v is None else list(v)

    def get_config(self, k, default=_MISSING):
        return self._get(k, default)


def as_conf(c):
    """Accept pyhocon ConfigTree, Conf or dict."""
    if hasattr(c, "get_int") and hasattr(c, "get_bool"):
        return c
    return Conf(c or {})


# --------------------------------------------------------------- parser ----
_TOKEN = re.compile(r'''\s*(?:
    (?P<comment>(?:\#|//)[^\n]*) |
    (?P<include>include\s+(?:required\()?\s*"(?P<inc>[^"]+)"\s*\)?) |
    (?P<str>"(?:[^"\\]|\\.)*") |
    (?P<punct>[{}\[\],=:]) |
    (?P<nl>\n) |
    (?P<word>[^\s{}\[\],=:\#"]+(?:[ \t]+[^\s{}\[\],=:\#"]+)*)
)''', re.X)


def _tokens(text):
    pos = 0
    out = []
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            if text[pos:].strip() == "":
                break
            raise ValueError("HOCON parse error near: %r" % text[pos:pos + 40])
        pos = m.end()
        if m.group("comment"):
            continue
        if m.group("include"):
            out.append(("include", m.group("inc")))
        elif m.group("str"):
            out.append(("val", bytes(m.group("str")[1:-1], "utf-8").decode("unicode_escape")))
        elif m.group("punct"):
            out.append(("p", m.group("punct")))
        elif m.group("nl"):
            out.append(("nl", None))
        elif m.group("word"):
            out.append(("val", m.group("word").strip()))
    return out


def _scalar(s):
    if not isinstance(s, str):
        return s
    low = s.lower()
    if low in ("true", "yes", "on"):
        return True
    if low in ("false", "no", "off"):
        return False
    if low == "null":
        return None
    try:
        return int(s)
    except ValueError:
        pass
    try:
        return float(s)
    except ValueError:
        return s


def _merge(dst, src):
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = v
    return dst


class _Parser:
    def __init__(self, toks, base_dir):
        self.t = toks
        self.i = 0
        self.base = base_dir

    def peek(self):
        while self.i < len(self.t) and self.t[self.i][0] == "nl":
            self.i += 1
        return self.t[self.i] if self.i < len(self.t) else (None, None)

    def take(self):
        tok = self.peek()
        self.i += 1
        return tok

    def obj(self, closing):
        d = {}
        while True:
            kind, val = self.peek()
            if kind is None:
                if closing:
                    raise ValueError("unterminated object")
                return d
            if kind == "p" and val == "}" and closing:
                self.take()
                return d
            if kind == "p" and val == ",":
                self.take()
                continue
            if kind == "include":
                self.take()
                _merge(d, parse_file(os.path.join(self.base, val)))
                continue
            key = self.take()[1]
            kind, val = self.peek()
            if kind == "p" and val in ("=", ":"):
                self.take()
            value = self.value()
            cur = d
            parts = str(key).split(".")
            for p in parts[:-1]:
                cur = cur.setdefault(p, {})
            if isinstance(value, dict) and isinstance(cur.get(parts[-1]), dict):
                _merge(cur[parts[-1]], value)
            else:
                cur[parts[-1]] = value

    def value(self):
        kind, val = self.take()
        if kind == "p" and val == "{":
            return self.obj(True)
        if kind == "p" and val == "[":
            items = []
            while True:
                k2, v2 = self.peek()
                if k2 == "p" and v2 == "]":
                    self.take()
                    return items
                if k2 == "p" and v2 == ",":
                    self.take()
                    continue
                items.append(self.value())
        return _scalar(val)


def parse_string(text, base_dir="."):
    return Conf(_Parser(_tokens(text), base_dir).obj(False))


def parse_file(path):
    with open(path) as f:
        return parse_string(f.read(), os.path.dirname(os.path.abspath(path)))
