"""Independent restatement of nrgrep's k = 0 "simple" engine.  TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module.  It works on the nrgrep pattern STRING
(what ``patmatch_to_nrgrep.pl`` prints) with its own parser -- it shares no
code with ``patmatchdocker_amd.regex`` -- so a compiler bug cannot hide behind
an oracle that consumes the same compiled program.  Every rule below is read
from the disassembly of the reference's ``www/bin/nrgrep_coords`` (nrgrep 1.1;
``objdump -d``, never executed; addresses in DESIGN.md §1):

* main(): a leading ``^`` / trailing ``$`` are stripped and become the
  OptStartLine / OptEndLine anchors (0x4012a1, 0x4012bd);
* getAchar (0x419510): ``\\n`` ``\\t`` ``\\xHH`` and ``\\c`` = literal c;
  getAclass (0x419640): ``.`` = all 256 bytes, ``#`` = every non-isalnum byte,
  ``[...]`` with ranges (a reversed range adds nothing), ``[^...]`` = all 256
  minus the listed bytes; ``-i`` adds the other case of every letter a class
  holds, or -- for a negated class -- removes the other case of every letter
  it lacks (0x4196b8, 0x4197fb);
* simpleScan + checkMatch (0x416600, 0x416790): a window is checked against
  the region [R, end of text), never against its record, so a match may span
  a line break; the first window found (leftmost start) is reported;
* recSearchFile (0x402250): after a report the next scan starts at its end.

Grouping parentheses are accepted only when they hold a plain sequence (what
the converter wraps every pattern in); anything with ``? * + |`` is not a
simple pattern and raises :class:`NotSimple`.
"""

from __future__ import annotations

from typing import List, Tuple


class NotSimple(ValueError):
    """The pattern is not a plain class sequence (nrgrep would not use the simple engine)."""


def _isalnum(b: int) -> bool:
    return 48 <= b <= 57 or 65 <= b <= 90 or 97 <= b <= 122


def _get_char(p: bytes, i: int) -> Tuple[int, int]:
    """getAchar: (byte, next index)."""
    c = p[i]
    if c != 0x5C:   # '\\'
        return c, i + 1
    if i + 1 >= len(p):
        raise NotSimple("dangling escape")
    e = p[i + 1]
    if e == ord("n"):
        return 10, i + 2
    if e == ord("t"):
        return 9, i + 2
    if e in (ord("x"), ord("X")):
        h = p[i + 2:i + 4]
        if len(h) != 2:
            raise NotSimple("bad \\x escape")
        try:
            return int(h.decode("ascii"), 16), i + 4
        except ValueError:
            raise NotSimple("bad \\x escape") from None
    return e, i + 2


def _case(members: set, negated: bool) -> set:
    out = set(members)
    for up in range(65, 91):
        lo = up + 32
        if not negated:
            if up in members:
                out.add(lo)
            if lo in members:
                out.add(up)
        else:
            if up not in members:
                out.discard(lo)
            if lo not in members:
                out.discard(up)
    return out


def parse(pattern: str, icase: bool = True):
    """(classes, anchor_start, anchor_end): classes = list of 256-byte sets."""
    p = pattern.encode("latin-1")
    a_start = p[:1] == b"^"
    if a_start:
        p = p[1:]
    a_end = p[-1:] == b"$"
    if a_end:
        p = p[:-1]
    classes: List[set] = []
    i = 0
    depth = 0
    while i < len(p):
        c = p[i]
        if c == ord("("):
            depth += 1
            i += 1
            continue
        if c == ord(")"):
            depth -= 1
            if depth < 0:
                raise NotSimple("unbalanced ')'")
            i += 1
            continue
        if c in (ord("?"), ord("*"), ord("+"), ord("|")):
            raise NotSimple("operator %r" % chr(c))
        if c == ord("."):
            members, neg = set(range(256)), False
            i += 1
        elif c == ord("#"):
            members, neg = {b for b in range(256) if not _isalnum(b)}, False
            i += 1
        elif c == ord("["):
            i += 1
            neg = i < len(p) and p[i] == ord("^")
            if neg:
                i += 1
            listed = set()
            while i < len(p) and p[i] != ord("]"):
                lo, i = _get_char(p, i)
                if i + 1 < len(p) and p[i] == ord("-") and p[i + 1] != ord("]"):
                    hi, i = _get_char(p, i + 1)
                    listed.update(range(lo, hi + 1))   # reversed: empty
                else:
                    listed.add(lo)
            if i >= len(p):
                raise NotSimple("unterminated class")
            i += 1
            members = (set(range(256)) - listed) if neg else listed
        else:
            b, i = _get_char(p, i)
            members, neg = {b}, False
        classes.append(_case(members, neg) if icase else members)
    if depth != 0:
        raise NotSimple("unbalanced '('")
    if not classes:
        raise NotSimple("empty pattern")
    return classes, a_start, a_end


def scan(text: bytes, pattern: str, icase: bool = True):
    """[(beg, end)] that nrgrep_coords prints for a k = 0 simple pattern."""
    classes, a_start, a_end = parse(pattern, icase)
    m, n = len(classes), len(text)
    out, R, s = [], 0, 0
    while s + m <= n:
        if all(text[s + j] in classes[j] for j in range(m)):
            e = s + m
            ok = not a_end or e == n or text[e] == 10
            ok = ok and (not a_start or s == R or s == 0 or text[s - 1] == 10)
            if ok:
                out.append((s, e))
                R = e
                s = e
                continue
        s += 1
    return out
