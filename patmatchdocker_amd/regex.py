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
# parser: nrgrep's own tree (parse 0x41ae90 / parseOr 0x41a530 / parseConc
# 0x41a760), then its simplify pass (0x41a170), then a small AST
#   ('sym', frozenset) | ('eps',) | ('cat', [..]) | ('alt', [..])
#   | ('opt'|'star'|'plus', node)
# --------------------------------------------------------------------------

# node types of nrgrep's tree (the jump tables at 0x41d4c0 / 0x41d4f0)
_LEAF, _STAR, _OR, _CAT, _OPT, _PLUS = 0, 1, 2, 3, 4, 5


class _Node:
    """A node of nrgrep's parse tree: ``type`` (above), ``nullable`` (the
    parse-time flag at +0x8: an empty leaf, '?', '*', a nullable '+' / '|' /
    concatenation), ``cls`` (a leaf's byte set; None = an empty leaf) and the
    children ``a`` / ``b`` (+0x10 / +0x18)."""

    __slots__ = ("type", "nullable", "cls", "a", "b")

    def __init__(self, type_, nullable, cls=None, a=None, b=None):
        self.type, self.nullable, self.cls, self.a, self.b = type_, nullable, cls, a, b


_EMPTY_AT = (None, ord(")"), ord("*"), ord("+"), ord("?"), ord("|"))


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

    def sym(self, members) -> frozenset:
        members = frozenset(members)
        return _fold_set(members) if self.icase else members

    def klass(self) -> frozenset:
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

    def leaf(self) -> frozenset:
        b = self.take()
        if b == ord("["):
            return self.klass()
        if b == ord("."):
            return self.sym(ALL_BYTES)
        if b == ord("#"):
            return self.sym(SEPARATORS)
        if b == ord("\\"):
            return self.sym({self.escape()})
        if b == ord("("):   # (parseConc handles a group before the leaf)
            raise RegexSyntaxError("unexpected '('")
        return self.sym({b})

    def alternatives(self) -> _Node:
        """parse / parseOr: c1 | c2 | ... as right-deep '|' nodes, each
        nullable when either side is."""
        items = [self.conc()]
        while self.peek() == ord("|"):
            self.i += 1
            items.append(self.conc())
        node = items[-1]
        for it in reversed(items[:-1]):
            node = _Node(_OR, it.nullable or node.nullable, a=it, b=node)
        return node

    def conc(self) -> _Node:
        """parseConc: one atom -- a group, an empty leaf (at end, ')', '|'
        or a postfix operator, nothing consumed: 0x41a830) or a class --, its
        postfix operators, then the rest of the concatenation (right-deep;
        built here from a list, the binary recurses)."""
        items = []
        while True:
            c = self.peek()
            if c == ord("("):
                self.i += 1
                node = self.alternatives()
                if self.peek() != ord(")"):
                    raise RegexSyntaxError("missing ')'")
                self.i += 1
            elif c in _EMPTY_AT:
                node = _Node(_LEAF, True)
            else:
                node = _Node(_LEAF, False, cls=self.leaf())
            while self.peek() in (ord("+"), ord("?"), ord("*")):
                op = self.take()
                if op == ord("+"):
                    node = _Node(_PLUS, node.nullable, a=node)
                else:
                    node = _Node(_OPT if op == ord("?") else _STAR, True, a=node)
            items.append(node)
            if self.peek() in (None, ord(")"), ord("|")):
                break
            if len(items) > MAX_POSITIONS:
                raise RegexSyntaxError("pattern longer than %d positions" % MAX_POSITIONS)
        node = items[-1]
        for it in reversed(items[:-1]):
            node = _Node(_CAT, it.nullable and node.nullable, a=it, b=node)
        return node


def _empty_leaf() -> _Node:
    return _Node(_LEAF, True)


def _simplify(n: _Node, left: bool, right: bool) -> _Node:
    """nrgrep's simplify (0x41a170), applied by parse() with both edge flags
    set (no -w / -x, 0x41aec3): a nullable subexpression at the left or
    right edge of the pattern becomes an empty leaf and drops out, a '+' at
    an edge loses its repetition, nested postfix operators merge, and a '|'
    of two single classes becomes one class.  Only the first element of a
    concatenation sees the left edge, the last the right edge (0x41a1c8,
    0x41a2f8); a '|' passes (left, 0) / (0, right) to its two sides."""
    if n.nullable and (left or right):                 # 0x41a190 -> 0x41a260
        return _empty_leaf()
    t = n.type
    if t == _LEAF:
        return n
    if t == _STAR:                                     # 0x41a378
        c = _simplify(n.a, left, right)
        if c.type in (_STAR, _OPT, _PLUS):
            return _Node(_STAR, True, a=c.a)           # 0x41a480: the child becomes '*'
        if c.type == _LEAF and c.nullable:
            return c
        n.a = c
        return n
    if t == _OPT:                                      # 0x41a2a0
        c = _simplify(n.a, left, right)
        if c.type in (_STAR, _PLUS):
            return _Node(_STAR, True, a=c.a)           # 0x41a458
        if c.type == _OPT or (c.type == _LEAF and c.nullable):
            return c
        n.a = c
        return n
    if t == _PLUS:                                     # 0x41a3d8 / 0x41a410
        if n.nullable:
            c = _simplify(n.a, False, False)
        else:
            c = _simplify(n.a, left, right)
            if left or right:
                return c                               # a '+' at an edge: its operand once
        if c.type in (_STAR, _OPT):
            return _Node(_STAR, True, a=c.a)
        if c.type == _PLUS or (c.type == _LEAF and c.nullable):
            return c
        n.a = c
        return n
    if t == _CAT:
        return _simplify_chain(n, left, right)
    a = _simplify(n.a, left, False)
    b = _simplify(n.b, False, right)
    if t == _OR:                                       # 0x41a1c8
        n.a, n.b = a, b
        if a.type != _LEAF or b.type != _LEAF:
            return n
        if a.nullable == b.nullable:                   # 0x41a498: one class
            cls = None if a.nullable else frozenset(a.cls | b.cls)
            return _Node(_LEAF, a.nullable, cls=cls)
        return _Node(_OPT, True, a=b if a.nullable else a)   # 0x41a501 / 0x41a51f
    raise AssertionError("node type %d" % t)


def _simplify_chain(n: _Node, left: bool, right: bool) -> _Node:
    """simplify of a right-deep concatenation a1 (a2 (.. an)) (0x41a2f8),
    without recursing along it: a1 gets (left, 0), each suffix node
    (a_i .. a_n) gets (0, right) -- the first nullable one touching the right
    edge becomes an empty leaf --, the elements before it (0, 0) and a_n
    (0, right); an empty leaf on either side of a node drops out."""
    items, suffix = [], []
    x = n
    while x.type == _CAT:
        items.append(x.a)
        suffix.append(x)
        x = x.b
    items.append(x)
    suffix.append(x)
    out = [_simplify(items[0], left, False)]
    for i in range(1, len(items)):
        s_node = suffix[i]
        if right and s_node.nullable:                   # the suffix node's own check
            break
        last = i == len(items) - 1
        out.append(_simplify(items[i], False, right if last else False))
    # rebuild right-deep, dropping empty leaves (0x41a32d / 0x41a342)
    node = None
    for it in reversed(out):
        if it.type == _LEAF and it.nullable:
            if node is None:
                node = it
            continue
        if node is None or (node.type == _LEAF and node.nullable):
            node = it
        else:
            node = _Node(_CAT, it.nullable and node.nullable, a=it, b=node)
    return node


def _det_class(n: _Node) -> int:
    """detClass (0x41ac90): 1 a class sequence, 2 classes each with an
    optional '? * +', 3 anything else."""
    best = 1
    stack = [n]
    while stack:
        x = stack.pop()
        if x.type == _LEAF:
            continue
        if x.type == _OR:
            return 3
        if x.type == _CAT:
            stack += [x.a, x.b]
        elif x.a.type == _LEAF:                        # 0x41acf8
            best = max(best, 2)
        else:
            return 3
    return best


def _serialize(n: _Node):
    """Preorder node list of a simplified tree (``Program.tree``): leaves are
    numbered in the order _glushkov numbers ``classes`` (left to right,
    regularLength 0x40b2a0 numbers nrgrep's states the same way, from 1)."""
    nodes, nulls = [], []
    pos = [0]

    def walk(x) -> int:
        i = len(nodes)
        nodes.append(None)
        nulls.append(1 if x.nullable else 0)
        if x.type == _LEAF:
            p = -1
            if x.cls is not None:
                p = pos[0]
                pos[0] += 1
            nodes[i] = (x.type, -1, -1, p)
            return i
        a = walk(x.a)
        b = walk(x.b) if x.type in (_OR, _CAT) else -1
        nodes[i] = (x.type, a, b, -1)
        return i

    walk(n)
    return tuple(nodes), tuple(nulls)


def _to_ast(n: _Node):
    if n.type == _LEAF:
        return ("eps",) if n.cls is None else ("sym", n.cls)
    if n.type in (_OR, _CAT):
        kind = "alt" if n.type == _OR else "cat"
        items = []
        x = n
        while x.type == n.type:      # a right-deep chain, flattened
            sub = _to_ast(x.a)
            items.extend(sub[1] if sub[0] == kind else [sub])
            x = x.b
        sub = _to_ast(x)
        items.extend(sub[1] if sub[0] == kind else [sub])
        return (kind, items)
    return ({_STAR: "star", _OPT: "opt", _PLUS: "plus"}[n.type], _to_ast(n.a))


def _extended_flags(n: _Node):
    """(opt, rep) position masks of a class-2 tree (extendedTreeLoad
    0x411970): '?' optional, '+' repeatable, '*' both."""
    opt = rep = 0
    pos = 0
    stack = [n]
    order = []
    while stack:
        x = stack.pop()
        if x.type == _CAT:
            stack.append(x.b)
            stack.append(x.a)
        else:
            order.append(x)
    for x in order:
        leaf = x if x.type == _LEAF else x.a
        if leaf.cls is None:
            continue
        if x.type in (_OPT, _STAR):
            opt |= 1 << pos
        if x.type in (_PLUS, _STAR):
            rep |= 1 << pos
        pos += 1
    return opt, rep


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
    opt_mask: int = 0            # extended: optional positions ('?', '*')
    rep_mask: int = 0            # extended: repeatable positions ('+', '*')
    # nrgrep's simplified tree (regular patterns' minCost / detClass run over
    # it): node i = (type, left, right, position) in preorder, node 0 the
    # root, position = the leaf's index into ``classes`` (-1: an empty
    # leaf, -1 children); ``tree_nullable[i]`` = the parse-time flag
    tree: Tuple[Tuple[int, int, int, int], ...] = ()
    tree_nullable: Tuple[int, ...] = ()

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
    if kind == "eps":
        return 0, 0, True, []
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
    if kind == "eps":
        return 0, 0
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


_KINDS = {1: "simple", 2: "extended", 3: "regular"}


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
    """Compile an nrgrep-syntax pattern (e.g. ``(GAA[CT]TC)``) as nrgrep_coords
    does: anchors stripped (main), parsed into nrgrep's tree and simplified
    (parse 0x41ae90, simplify 0x41a170: e.g. ``(GAATTC.?.?)`` becomes the class
    sequence ``GAATTC``), its engine class from detClass (0x41ac90), then the
    position automaton of what is left."""
    source = pattern.encode("latin-1") if isinstance(pattern, str) else bytes(pattern)
    text, a_start, a_end = split_anchors(source)
    parser = _Parser(text, ignore_case)
    if not text:
        raise RegexSyntaxError("empty pattern")
    tree = parser.alternatives()
    if parser.i != len(text):
        # parse() stops at a top-level ')' (0x41af3a) -- the converter never
        # emits one; a user pattern that nrgrep would cut there is refused
        raise RegexSyntaxError("unbalanced ')' in pattern")
    tree = _simplify(tree, True, True)
    ast = _to_ast(tree)
    if ast[0] == "eps":
        raise RegexSyntaxError("the pattern matches only the empty string")
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
    kind = _KINDS[_det_class(tree)]
    opt, rep = _extended_flags(tree) if kind == "extended" else (0, 0)
    tnodes, tnull = _serialize(tree)
    return Program(source=source.decode("latin-1"), classes=classes, first=first,
                   last=last, follow=follow, nullable=nullable, min_len=lo,
                   max_len=hi, linear=_is_linear(ast), ignore_case=ignore_case,
                   precede=precede, anchor_start=a_start, anchor_end=a_end, kind=kind,
                   opt_mask=opt, rep_mask=rep, tree=tnodes, tree_nullable=tnull)
