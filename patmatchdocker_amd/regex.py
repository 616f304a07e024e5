"""nrgrep pattern syntax -> position automaton (Glushkov NFA) with bitmasks.

This is the "pattern compiler" half of the scan path.  The reference hands
the converted pattern to the prebuilt ``nrgrep_coords`` binary
(``www/FlaskApp/FlaskApp/patmatch.py:733-742``), whose syntax is documented by
its own ``-H`` help text (nrgrep 1.1, G. Navarro, GPL): ``.`` any character,
``#`` any separator, ``[..]`` classes with ``^`` complement and ``a-z`` ranges,
postfix ``?`` ``*`` ``+``, union ``|``, grouping ``( )`` and the escapes
``\\t`` ``\\n`` ``\\xdd`` ``\\c``.  Details read from the binary's code
(``www/bin/nrgrep_coords``, disassembled, never run):

* ``.`` sets all 256 bytes, the delimiter ``'\\n'`` included (getAclass
  0x4198c0); ``[^..]`` starts from all 256 and clears the listed bytes
  (0x419988); ``#`` is every non-``isalnum`` byte (0x419780); with ``-i`` a
  class gains the other case of each letter it holds (0x4196b8), a negated
  class loses the other case of each letter it lacks (0x4197fb) -- i.e.
  membership of the case-folded byte;
* a reversed range ``[z-a]`` adds nothing (0x419aac), it is no error;
* a ``^`` as the FIRST character of the pattern and a ``$`` as its LAST are
  anchors, stripped before parsing (main 0x4012a1 / 0x4012bd, OptStartLine /
  OptEndLine); anywhere else they are ordinary characters, as are
  ``{`` ``}`` ``<`` ``>``.

The compiled :class:`Program` is what the HIP library consumes: every
position of the regular expression gets a 256-bit membership set over the
(case-folded) byte alphabet, and the automaton's ``first``/``last``/``follow``
sets are 64-bit masks (bit *i* = position *i*), i.e. the per-character
bitmask tables of bit-parallel Shift-And/Glushkov simulation.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

__all__ = ["RegexSyntaxError", "Program", "compile_pattern", "fold_byte",
           "MAX_POSITIONS"]

MAX_POSITIONS = 4096        # parser bound; the GPU kernels take up to 256 (engine.route)
DELIMITER = 0x0A            # record delimiter (nrgrep default '\n')
ALL_BYTES = frozenset(range(256))   # '.' (the delimiter included)


class RegexSyntaxError(ValueError):
    """nrgrep would print "Syntax error in pattern" and report nothing."""


def fold_byte(b: int) -> int:
    """Case folding used for ``-i``: ASCII lower case -> upper case."""
    return b - 32 if 97 <= b <= 122 else b


def _fold_set(s) -> frozenset:
    return frozenset(fold_byte(b) for b in s)


def _isalnum(b: int) -> bool:
    return 48 <= b <= 57 or 65 <= b <= 90 or 97 <= b <= 122


SEPARATORS = frozenset(b for b in range(256) if not _isalnum(b))


# --------------------------------------------------------------------------
# parser: recursive descent over the byte string -> small AST
#   ('sym', frozenset) | ('cat', [..]) | ('alt', [..]) | ('opt'|'star'|'plus', node)
# --------------------------------------------------------------------------

class _Parser:
    def __init__(self, text: bytes, ignore_case: bool):
        self.s = text
        self.i = 0
        self.icase = ignore_case

    def peek(self):
        return self.s[self.i] if self.i < len(self.s) else None

    def take(self):
        b = self.peek()
        if b is None:
            raise RegexSyntaxError("unexpected end of pattern")
        self.i += 1
        return b

    def escape(self) -> int:
        b = self.take()
        if b == ord("t"):
            return 9
        if b == ord("n"):
            return 10
        if b == ord("x"):
            digits = self.s[self.i:self.i + 2]
            try:
                value = int(digits.decode("ascii"), 16)
            except (UnicodeDecodeError, ValueError):
                raise RegexSyntaxError("bad \\x escape") from None
            if len(digits) != 2:
                raise RegexSyntaxError("bad \\x escape")
            self.i += 2
            return value
        return b

    def sym(self, members) -> tuple:
        members = frozenset(members)
        if self.icase:
            members = _fold_set(members)
        return ("sym", members)

    def klass(self) -> tuple:
        negate = self.peek() == ord("^")
        if negate:
            self.i += 1
        members = set()
        while True:
            b = self.take()
            if b == ord("]"):
                break
            lo = self.escape() if b == ord("\\") else b
            if self.peek() == ord("-") and self.i + 1 < len(self.s) and self.s[self.i + 1] != ord("]"):
                self.i += 1
                hb = self.take()
                hi = self.escape() if hb == ord("\\") else hb
                members.update(range(lo, hi + 1))   # reversed: empty (0x419aac)
            else:
                members.add(lo)
        if self.icase:
            members = set(_fold_set(members)) | {b + 32 for b in _fold_set(members) if 65 <= b <= 90}
        if negate:
            members = set(ALL_BYTES) - members
        return self.sym(members)

    def atom(self) -> tuple:
        b = self.take()
        if b == ord("("):
            node = self.alternation()
            if self.take() != ord(")"):
                raise RegexSyntaxError("missing ')'")
            return node
        if b == ord("["):
            return self.klass()
        if b == ord("."):
            return self.sym(ALL_BYTES)
        if b == ord("#"):
            return self.sym(SEPARATORS)
        if b == ord("\\"):
            return self.sym({self.escape()})
        if b in (ord("?"), ord("*"), ord("+"), ord(")"), ord("|")):
            raise RegexSyntaxError("operator %r without operand" % chr(b))
        return self.sym({b})

    def factor(self) -> tuple:
        node = self.atom()
        while self.peek() in (ord("?"), ord("*"), ord("+")):
            op = {ord("?"): "opt", ord("*"): "star", ord("+"): "plus"}[self.take()]
            node = (op, node)
        return node

    def concatenation(self) -> tuple:
        items = []
        while self.peek() is not None and self.peek() not in (ord("|"), ord(")")):
            items.append(self.factor())
        if not items:
            raise RegexSyntaxError("empty expression")
        return items[0] if len(items) == 1 else ("cat", items)

    def alternation(self) -> tuple:
        branches = [self.concatenation()]
        while self.peek() == ord("|"):
            self.i += 1
            branches.append(self.concatenation())
        return branches[0] if len(branches) == 1 else ("alt", branches)


# --------------------------------------------------------------------------
# Glushkov construction
# --------------------------------------------------------------------------

@dataclass
class Program:
    """A compiled pattern: position automaton + bitmask tables.

    ``classes[i]``   set of (folded) bytes position *i* accepts
    ``first``        positions a match can begin with (64-bit mask)
    ``last``         positions a match can end with
    ``follow[i]``    positions that may come right after position *i*
    ``nullable``     the empty string matches (never reported)
    ``min_len``/``max_len``   match length bounds (``max_len`` None = unbounded)
    ``linear``       True when the pattern is a plain sequence of classes
                     (fixed length, no ``? * + |``) -- the bit-sliced fast path;
                     nrgrep's "simple" engine at k = 0 (detClass() == 1)
    ``anchor_start``/``anchor_end``  the stripped leading ``^`` / trailing ``$``
    """

    source: str
    classes: List[frozenset]
    first: int
    last: int
    follow: List[int]
    nullable: bool
    min_len: int
    max_len: Optional[int]
    linear: bool
    ignore_case: bool = True
    precede: List[int] = field(default_factory=list)
    anchor_start: bool = False   # leading '^' (OptStartLine)
    anchor_end: bool = False     # trailing '$' (OptEndLine)
    kind: str = "simple"         # nrgrep engine class: simple / extended / regular

    @property
    def m(self) -> int:
        return len(self.classes)

    def byte_masks(self) -> List[int]:
        """B[c]: 64-bit mask of positions accepting byte ``c`` (Shift-And table)."""
        table = [0] * 256
        for i, cls in enumerate(self.classes):
            for b in cls:
                table[b] |= 1 << i
        return table


def _glushkov(node, classes: list):
    """Returns (first, last, nullable, follow-pairs) for ``node``."""
    kind = node[0]
    if kind == "sym":
        i = len(classes)
        if i >= MAX_POSITIONS:
            raise RegexSyntaxError("pattern longer than %d positions" % MAX_POSITIONS)
        classes.append(node[1])
        return 1 << i, 1 << i, False, []
    if kind == "cat":
        first, last, nullable, pairs = _glushkov(node[1][0], classes)
        for child in node[1][1:]:
            f2, l2, n2, p2 = _glushkov(child, classes)
            pairs = pairs + p2 + [(last, f2)]
            first = first | f2 if nullable else first
            last = last | l2 if n2 else l2
            nullable = nullable and n2
        return first, last, nullable, pairs
    if kind == "alt":
        first = last = 0
        nullable, pairs = False, []
        for child in node[1]:
            f2, l2, n2, p2 = _glushkov(child, classes)
            first, last, nullable, pairs = first | f2, last | l2, nullable or n2, pairs + p2
        return first, last, nullable, pairs
    f, l, n, pairs = _glushkov(node[1], classes)
    if kind == "opt":
        return f, l, True, pairs
    loop = pairs + [(l, f)]
    return f, l, (True if kind == "star" else n), loop


def _length_bounds(node) -> Tuple[int, Optional[int]]:
    kind = node[0]
    if kind == "sym":
        return 1, 1
    if kind == "cat":
        lo, hi = 0, 0
        for child in node[1]:
            a, b = _length_bounds(child)
            lo += a
            hi = None if hi is None or b is None else hi + b
        return lo, hi
    if kind == "alt":
        bounds = [_length_bounds(c) for c in node[1]]
        his = [b for _, b in bounds]
        return min(a for a, _ in bounds), (None if None in his else max(his))
    a, b = _length_bounds(node[1])
    if kind == "opt":
        return 0, b
    if kind == "star":
        return 0, (0 if b == 0 else None)
    return a, (0 if b == 0 else None)


def _kind(node) -> str:
    """nrgrep's engine class (detClass, called by searchPreproc 0x4025b5):
    "simple" = a sequence of classes, "extended" = a sequence of classes
    each optionally followed by ``? * +``, "regular" = anything else."""
    items = node[1] if node[0] == "cat" else [node]
    if all(c[0] == "sym" for c in items):
        return "simple"
    if all(c[0] == "sym" or (c[0] in ("opt", "star", "plus") and c[1][0] == "sym") for c in items):
        return "extended"
    return "regular"


# the line searchPreproc puts() before scanning (0x402654 .. 0x40275d):
# "SIMPLE search" .. "EREGULAR search"; 'E' = with errors (-k > 0)
def engine_banner(prog: "Program", k: int) -> str:
    return ("E" if k else "") + prog.kind.upper() + " search"


def _is_linear(node) -> bool:
    if node[0] == "sym":
        return True
    if node[0] == "cat":
        return all(_is_linear(c) for c in node[1])
    return False


def split_anchors(text: bytes):
    """nrgrep main(): a leading ``^`` sets OptStartLine and is skipped
    (0x4012a1 / 0x40164d), then a trailing ``$`` sets OptEndLine and is cut
    (0x4012bd / 0x40162a).  Returns (core, anchor_start, anchor_end)."""
    start = text[:1] == b"^"
    if start:
        text = text[1:]
    end = text[-1:] == b"$"
    if end:
        text = text[:-1]
    return text, start, end


def compile_pattern(pattern, ignore_case: bool = True) -> Program:
    """Compile an nrgrep-syntax pattern (e.g. ``(GAA[CT]TC)``)."""
    source = pattern.encode("latin-1") if isinstance(pattern, str) else bytes(pattern)
    text, a_start, a_end = split_anchors(source)
    parser = _Parser(text, ignore_case)
    if not text:
        raise RegexSyntaxError("empty pattern")
    ast = parser.alternation()
    if parser.i != len(text):
        raise RegexSyntaxError("unbalanced ')' in pattern")
    classes: list = []
    first, last, nullable, pairs = _glushkov(ast, classes)
    follow = [0] * len(classes)
    for src, dst in pairs:
        for i in range(len(classes)):
            if src >> i & 1:
                follow[i] |= dst
    precede = [0] * len(classes)
    for i, f in enumerate(follow):
        for j in range(len(classes)):
            if f >> j & 1:
                precede[j] |= 1 << i
    lo, hi = _length_bounds(ast)
    return Program(source=source.decode("latin-1"), classes=classes, first=first,
                   last=last, follow=follow, nullable=nullable, min_len=lo,
                   max_len=hi, linear=_is_linear(ast), ignore_case=ignore_case,
                   precede=precede, anchor_start=a_start, anchor_end=a_end, kind=_kind(ast))
