"""Fortran namelist reader (the subset offline drivers use).

The reference reads run/case.nml with f90nml (offline/noahmp_config.py:69-70),
which is not available here; this is our own reader for the same files:

    &GROUP  key = value, key2 = 'text', arr = 1, 2, 3*0.5, flag = .true. /

* group names and keys are case-insensitive (returned lower-case);
* values: integers, reals (``1.5``, ``1e3``, ``1.0d-3``), quoted strings
  (``'..'`` or ``".."``, doubled quote escapes), logicals (``.true.``/``T``),
  ``r*value`` repeat counts; several values make a list;
* ``!`` starts a comment outside strings; ``/`` (or ``&end``) ends a group.
"""
from __future__ import annotations

import re

__all__ = ["read", "reads", "NamelistError"]


class NamelistError(ValueError):
    pass


_TOKEN = re.compile(r"""
    (?P<str>'(?:[^']|'')*'|"(?:[^"]|"")*")
  | (?P<group>&[A-Za-z_][A-Za-z0-9_]*)
  | (?P<end>/)
  | (?P<eq>=)
  | (?P<comma>,)
  | (?P<word>[^\s,=/'"!]+)
""", re.VERBOSE)


def _strip_comments(text: str) -> str:
    out, q = [], None
    for line in text.splitlines():
        buf = []
        for ch in line:
            if q:
                buf.append(ch)
                if ch == q:
                    q = None
            elif ch in "'\"":
                q = ch
                buf.append(ch)
            elif ch == "!":
                break
            else:
                buf.append(ch)
        out.append("".join(buf))
    return "\n".join(out)


def _scalar(word: str):
    w = word.strip()
    lw = w.lower()
    if lw in (".true.", ".t.", "t", "true"):
        return True
    if lw in (".false.", ".f.", "f", "false"):
        return False
    try:
        return int(w)
    except ValueError:
        pass
    try:
        return float(lw.replace("d", "e"))
    except ValueError as exc:
        raise NamelistError(f"cannot parse value {word!r}") from exc


def _value(tok):
    kind, text = tok
    if kind == "str":
        q = text[0]
        return text[1:-1].replace(q + q, q)
    m = re.fullmatch(r"(\d+)\*(.*)", text)
    if m:
        return ("repeat", int(m.group(1)), _scalar(m.group(2)) if m.group(2) else None)
    return _scalar(text)


def reads(text: str) -> dict:
    """Parse namelist text -> {group: {key: value}} (lower-case names)."""
    toks = [(m.lastgroup, m.group(m.lastgroup)) for m in _TOKEN.finditer(_strip_comments(text))]
    groups: dict = {}
    i, n = 0, len(toks)
    while i < n:
        kind, text = toks[i]
        if kind != "group":
            i += 1  # text outside groups is ignored, as Fortran readers do
            continue
        name = text[1:].lower()
        if name == "end":
            i += 1
            continue
        grp = groups.setdefault(name, {})
        i += 1
        key, vals = None, []

        def flush():
            if key is None:
                return
            flat = []
            for v in vals:
                if isinstance(v, tuple) and v and v[0] == "repeat":
                    flat.extend([v[2]] * v[1])
                else:
                    flat.append(v)
            grp[key] = flat[0] if len(flat) == 1 else flat

        while i < n:
            kind, text = toks[i]
            if kind == "end" or (kind == "group" and text.lower() == "&end"):
                i += 1
                break
            if kind == "group":
                raise NamelistError(f"group &{name} not terminated before {text}")
            if kind == "word" and i + 1 < n and toks[i + 1][0] == "eq":
                flush()
                key, vals = text.lower(), []
                i += 2
                continue
            if kind == "comma":
                i += 1
                continue
            if key is None:
                raise NamelistError(f"value {text!r} before any key in &{name}")
            vals.append(_value((kind, text)))
            i += 1
        else:
            flush()
            raise NamelistError(f"group &{name} has no terminating '/'")
        flush()
    return groups


def read(path: str) -> dict:
    with open(path) as f:
        return reads(f.read())
