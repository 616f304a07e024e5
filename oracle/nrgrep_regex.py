"""Independent restatement of the scan candidates for ANY nrgrep pattern.  TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module.  It covers what ``nrgrep_simple``
refuses -- ``? * + |`` and groups, i.e. nrgrep's extended and regular
engines -- and k > 0 with any of the i / d / s error types.  It works on the
pattern STRING with its own parser and a different algorithm from the
product's and from ``pm_oracle.c``: no position automaton at all, but a
recursive relation over the parse tree, for every start s of a record,

    reach(node, {(i, u): e}) = {(j, u'): the fewest edits e' with which node
                                turns text[i:j] into a word of its language}

(u: a pattern position was used on the way -- matched, substituted or
deleted: the empty word of a nullable pattern is never a match, as in the
position automata, where only a last position reports)

composed node by node (concatenation = relation product, ``|`` = union,
``?`` / ``*`` / ``+`` = union with the empty relation / fixpoint).  A class
consumes one byte of its set (0 edits) or any other byte (1, substitution),
or none (1, deletion); insertions (1 per extra byte) go before every class
and after the last one.  The candidate of s is the shortest non-empty
text[s, e) inside the record with at most k edits -- the rule
``pm_oracle.c``'s header states (pmo_scan: records between '\\n', every
start, its shortest end).  Anchors (``^`` / ``$``) are stripped here as
nrgrep's main() does (0x4012a1, 0x4012bd) and returned to the caller.

Syntax (getAchar 0x419510 / getAclass 0x419640, shared with
``nrgrep_simple``): ``\\n \\t \\xHH \\c``, ``.``, ``#``, ``[...]`` with ranges and
``[^...]``; ``-i`` extends every class with the other case of its letters.
"""

from __future__ import annotations

from typing import Dict, List, Tuple

from oracle.nrgrep_simple import _case, _get_char, _isalnum


class PatternError(ValueError):
    """Not a pattern this restatement parses."""


def _class_at(p: bytes, i: int, icase: bool):
    c = p[i]
    if c == ord("."):
        members, neg, i = set(range(256)), False, i + 1
    elif c == ord("#"):
        members, neg, i = {b for b in range(256) if not _isalnum(b)}, False, i + 1
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
                listed.update(range(lo, hi + 1))
            else:
                listed.add(lo)
        if i >= len(p):
            raise PatternError("unterminated class")
        i += 1
        members = (set(range(256)) - listed) if neg else listed
    else:
        b, i = _get_char(p, i)
        members, neg = {b}, False
    return frozenset(_case(members, neg) if icase else members), i


def parse(pattern: str, icase: bool = True):
    """(tree, anchor_start, anchor_end).  tree: ('sym', set) | ('cat', [..])
    | ('alt', [..]) | ('opt' | 'star' | 'plus', node) | ('eps',)."""
    p = pattern.encode("latin-1")
    a_start = p[:1] == b"^"
    if a_start:
        p = p[1:]
    a_end = p[-1:] == b"$" and p[-2:-1] != b"\\"
    if a_end:
        p = p[:-1]
    pos = [0]

    def peek():
        return p[pos[0]] if pos[0] < len(p) else None

    def alt():
        items = [cat()]
        while peek() == ord("|"):
            pos[0] += 1
            items.append(cat())
        return items[0] if len(items) == 1 else ("alt", items)

    def cat():
        items = []
        while peek() is not None and peek() not in (ord("|"), ord(")")):
            items.append(post())
        if not items:
            return ("eps",)
        return items[0] if len(items) == 1 else ("cat", items)

    def post():
        node = atom()
        while peek() in (ord("?"), ord("*"), ord("+")):
            op = {ord("?"): "opt", ord("*"): "star", ord("+"): "plus"}[p[pos[0]]]
            pos[0] += 1
            node = (op, node)
        return node

    def atom():
        c = peek()
        if c == ord("("):
            pos[0] += 1
            node = alt()
            if peek() != ord(")"):
                raise PatternError("unbalanced '('")
            pos[0] += 1
            return node
        if c in (ord("?"), ord("*"), ord("+")):
            raise PatternError("operator without operand")
        members, pos[0] = _class_at(p, pos[0], icase)
        return ("sym", members)

    tree = alt()
    if pos[0] != len(p):
        raise PatternError("unbalanced ')'")
    return simplify(tree), a_start, a_end


def _nullable(node) -> bool:
    k = node[0]
    if k in ("eps", "opt", "star"):
        return True
    if k == "sym":
        return False
    if k == "plus":
        return _nullable(node[1])
    if k == "cat":
        return all(_nullable(c) for c in node[1])
    return any(_nullable(c) for c in node[1])


def simplify(tree):
    """nrgrep's simplify pass (the binary's 0x41a170, called by parse with
    both edges set), restated on this module's n-ary tree: a nullable
    subexpression touching an edge of the pattern is dropped -- at the left
    edge only the first element of a concatenation sees it, at the right
    edge the whole nullable tail goes; a '+' touching an edge keeps one
    copy of its operand; a postfix operator over '*', '+' or '?' merges
    into '*' or '?'; a '|' of two single classes is one class, a '|' with an
    empty side is '?' of the other.  Nested concatenations and alternations
    are right-deep binary nodes in the binary, which fixes who sees an edge."""

    def simp(node, left, right):
        k = node[0]
        if _nullable(node) and (left or right):
            return ("eps",)
        if k in ("sym", "eps"):
            return node
        if k in ("cat", "alt") and len(node[1]) > 2:
            node = (k, [node[1][0], (k, node[1][1:])])
        if k in ("cat", "alt") and len(node[1]) == 1:
            return simp(node[1][0], left, right)
        if k == "cat":
            a, b = simp(node[1][0], left, False), simp(node[1][1], False, right)
            if a[0] == "eps":
                return b
            if b[0] == "eps":
                return a
            return ("cat", [a, b])
        if k == "alt":
            a, b = simp(node[1][0], left, False), simp(node[1][1], False, right)
            leafy = lambda x: x[0] in ("sym", "eps")
            if leafy(a) and leafy(b):
                if a[0] == b[0] == "sym":
                    return ("sym", frozenset(a[1] | b[1]))
                if a[0] == b[0] == "eps":
                    return a
                return ("opt", b if a[0] == "eps" else a)
            return ("alt", [a, b])
        if k == "plus" and not _nullable(node):
            c = simp(node[1], left, right)
            if left or right:
                return c
        else:
            c = simp(node[1], False, False) if k == "plus" else simp(node[1], left, right)
        if c[0] == "eps":
            return c
        if k == "star":
            return ("star", c[1]) if c[0] in ("star", "opt", "plus") else ("star", c)
        if k == "opt":
            if c[0] in ("star", "plus"):
                return ("star", c[1])
            return c if c[0] == "opt" else ("opt", c)
        # plus
        if c[0] in ("star", "opt"):
            return ("star", c[1])
        return c if c[0] == "plus" else ("plus", c)

    return simp(tree, True, True)


Rel = Dict[Tuple[int, bool], int]


def _merge(a: Rel, b: Rel) -> Rel:
    out = dict(a)
    for j, e in b.items():
        if e < out.get(j, 1 << 30):
            out[j] = e
    return out


class _Matcher:
    def __init__(self, text: bytes, end: int, k: int, ins: bool, dele: bool, sub: bool):
        self.t, self.end, self.k = text, end, k
        self.ins, self.dele, self.sub = ins, dele, sub

    def insert(self, I: Rel) -> Rel:
        if not self.ins:
            return I
        out = dict(I)
        for (i, u), e in I.items():
            for t in range(1, self.k - e + 1):
                if i + t > self.end:
                    break
                if e + t < out.get((i + t, u), 1 << 30):
                    out[(i + t, u)] = e + t
        return out

    def reach(self, node, I: Rel) -> Rel:
        kind = node[0]
        if not I:
            return {}
        if kind == "eps":
            return dict(I)
        if kind == "sym":
            S = node[1]
            out: Rel = {}
            for (i, _), e in self.insert(I).items():
                cands = []
                if i < self.end:
                    if self.t[i] in S:
                        cands.append((i + 1, e))
                    elif self.sub and e < self.k:
                        cands.append((i + 1, e + 1))
                if self.dele and e < self.k:
                    cands.append((i, e + 1))
                for j, ee in cands:
                    if ee < out.get((j, True), 1 << 30):
                        out[(j, True)] = ee
            return out
        if kind == "cat":
            for child in node[1]:
                I = self.reach(child, I)
            return I
        if kind == "alt":
            out = {}
            for child in node[1]:
                out = _merge(out, self.reach(child, I))
            return out
        if kind == "opt":
            return _merge(I, self.reach(node[1], I))
        if kind in ("star", "plus"):
            acc = {} if kind == "plus" else dict(I)
            frontier = I
            while frontier:
                nxt = self.reach(node[1], frontier)
                new = {j: e for j, e in nxt.items() if e < acc.get(j, 1 << 30)}
                acc = _merge(acc, new)
                frontier = new
            return acc
        raise PatternError("node %r" % (kind,))


def candidates(text: bytes, pattern: str, k: int = 0, types: str = "ids", icase: bool = True) -> List[Tuple[int, int]]:
    """pmo_scan's candidate list, restated: every start s of every record
    (lines between '\\n') with its shortest non-empty end."""
    tree, _, _ = parse(pattern, icase)
    ins, dele, sub = ("i" in types, "d" in types, "s" in types) if k else (False, False, False)
    out = []
    n = len(text)
    rec = 0
    while rec <= n:
        nl = text.find(b"\n", rec)
        end = nl if nl >= 0 else n
        m = _Matcher(text, end, k, ins, dele, sub)
        for s in range(rec, end):
            ends = m.insert(m.reach(tree, {(s, False): 0}))
            best = [j for (j, u), e in ends.items() if u and j > s and e <= k]
            if best:
                out.append((s, min(best)))
        rec = end + 1
    return out


def reported(text: bytes, pattern: str, k: int = 0, types: str = "ids", icase: bool = True) -> List[Tuple[int, int]]:
    """The report rule over the candidates (pm_oracle.c header;
    recSearchFile 0x402250): regions [R, n) from R = 0, the first candidate
    with s >= R is printed and R becomes its end; '^' wants s == R, s == 0 or
    a '\\n' before s (recCheckLeftContext 0x402170), '$' an end at the line
    end -- the forward verification extends to it (extended checkMatch
    0x411eb0), so the candidate of s is then the line end itself when it is
    reachable.  Line-bounded candidates only (not the k = 0 simple engine's
    whole-text windows, ``nrgrep_simple``)."""
    tree, a_start, a_end = parse(pattern, icase)
    ins, dele, sub = ("i" in types, "d" in types, "s" in types) if k else (False, False, False)
    out = []
    n = len(text)
    R = 0
    rec = 0
    while rec <= n:
        nl = text.find(b"\n", rec)
        end = nl if nl >= 0 else n
        m = _Matcher(text, end, k, ins, dele, sub)
        for s in range(rec, end):
            if s < R:
                continue
            if a_start and not (s == R or s == 0 or text[s - 1] == 10):
                continue
            ends = m.insert(m.reach(tree, {(s, False): 0}))
            ok = [j for (j, u), e in ends.items() if u and j > s and e <= k]
            if a_end:
                ok = [j for j in ok if j == end]
            if not ok:
                continue
            e = min(ok)
            out.append((s, e))
            R = e
        rec = end + 1
    return out
