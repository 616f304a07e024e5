"""A second statement of nrgrep's extended engine at k = 0 (test helper).

``oracle/pm_nrgrep_ext.c`` replays the binary's bit-parallel loops word for
word.  This model states the same rule with explicit position SETS and no
bit tricks, so a slip in the replay's shifts, masks or borrows shows up as a
disagreement (tests/test_nrgrep_extended.py):

* the plan (window / prefix, L) is taken from the oracle (its cost model is
  checked separately against the library's C++ restatement);
* type 2: every window start s in [R, n - fwd] whose ``fwd`` characters,
  read right to left, lead from some window position back to the window's
  first position is a candidate -- the replay's backward scan skips windows
  (BDM shifts), the model tries them all, which is the same set if the
  shifts never skip a candidate;
* type 3: every end p + 1 of a prefix occurrence inside a line (a fresh
  state at R and after each '\\n');
* verify: the left part read back from the candidate, the right part read
  forward, each stopping at the nearest accepting boundary, from the state
  {first position} when it is optional and without the optional-block
  closure before the first character.

Patterns whose scanned part starts with an optional position (the binary
marks the "position before" at bit 63 there) are outside the model.
"""

from __future__ import annotations

from typing import List, Tuple


def _fold(c: int) -> int:
    return c - 32 if 97 <= c <= 122 else c


class ExtendedModel:
    def __init__(self, prog, plan: dict):
        self.m = prog.m
        self.cls = [set(c) for c in prog.classes]
        self.icase = prog.ignore_case
        self.opt = [bool(prog.opt_mask >> i & 1) for i in range(self.m)]
        self.rep = [bool(prog.rep_mask >> i & 1) for i in range(self.m)]
        self.start_anchor, self.end_anchor = prog.anchor_start, prog.anchor_end
        self.type, self.fwd = plan["type"], plan["fwd"]
        self.beg, self.end = plan["window"]
        self.L = plan["L"]
        self.simple = plan["simple"]

    def accepts(self, c: int, p: int) -> bool:
        return (_fold(c) if self.icase else c) in self.cls[p]

    # -- verification ------------------------------------------------------
    def _part(self, left: bool):
        """(positions, optional block members, X) of the left (reversed) or
        right part, r -> pattern position: an optional first position is X
        (matched by nothing: the part may start after it), every other
        optional position belongs to the block of optional positions it is
        in (extendedLoadVerif 0x412c60)."""
        pos = list(range(self.L - 1, -1, -1)) if left else list(range(self.L, self.m))
        block = {r for r, p in enumerate(pos) if r > 0 and self.opt[p]}
        x = {0} if pos and self.opt[pos[0]] else set()
        return pos, block, x

    def _phase(self, text: bytes, pos: int, bound: int, left: bool, recbeg: int, recend: int):
        parts, block, x = self._part(left)
        n = len(parts)
        if n == 0:
            ok = self._left_ok(text, pos, recbeg) if left else self._right_ok(text, pos, recend)
            return pos if ok else None
        D = set(x)
        first = True
        p = pos
        while True:
            ok = self._left_ok(text, p, recbeg) if left else self._right_ok(text, p, recend)
            if n - 1 in D and ok:
                return p
            if p == bound:
                return None
            c = text[p - 1] if left else text[p]
            p = p - 1 if left else p + 1
            nxt = set()
            srcs = set(D) | ({-1} if first else set())
            for r in srcs:
                q = r + 1
                if q < n and self.accepts(c, parts[q]):
                    nxt.add(q)
            for r in D:
                if self.rep[parts[r]] and self.accepts(c, parts[r]):
                    nxt.add(r)
            if not nxt:
                return None
            D = set(nxt)
            for r in sorted(nxt):       # an active position opens the rest of its block
                q = r + 1
                while q < n and q in block:
                    D.add(q)
                    q += 1
            first = False

    def _left_ok(self, text, p, recbeg):
        return not (self.start_anchor and p > recbeg and text[p - 1] != 10)

    def _right_ok(self, text, q, recend):
        return not (self.end_anchor and q < recend and text[q] != 10)

    def verify(self, text: bytes, c: int, R: int):
        rp = c - 1 if self.type == 3 else c
        if rp < R:
            return None
        nl = text.rfind(b"\n", R, rp)
        recbeg = nl + 1 if nl >= 0 else R
        e = text.find(b"\n", rp)
        recend = e if e >= 0 else len(text)
        if rp >= recend:
            return None
        s = self._phase(text, c, recbeg, True, recbeg, recend)
        if s is None:
            return None
        e = self._phase(text, c, recend, False, recbeg, recend)
        if e is None:
            return None
        return s, e

    # -- candidates --------------------------------------------------------
    def _window_cond(self, text: bytes, s: int) -> bool:
        win = list(range(self.beg, self.end))
        block = set()
        for p in win:
            if self.opt[p]:
                block.add(p)
        last = text[s + self.fwd - 1]
        D = {p for p in win if self.accepts(last, p)}
        for i in range(self.fwd - 2, -1, -1):
            # closure: an active position may skip the optional ones before it
            cl = set(D)
            for p in D:
                q = p - 1
                while q >= self.beg and q in block:
                    cl.add(q)
                    q -= 1
            c = text[s + i]
            D = {p - 1 for p in cl if p - 1 >= self.beg and self.accepts(c, p - 1)}
            D |= {p for p in cl if self.rep[p] and self.accepts(c, p)}
            if not D:
                return False
        return self.beg in D

    def candidates(self, text: bytes, R: int):
        n = len(text)
        if self.type == 2:
            for s in range(R, n - self.fwd + 1):
                if self._window_cond(text, s):
                    yield s
            return
        # type 3, extended prefix: fresh at R and after every '\n'
        pre = list(range(0, self.end))
        D = set()
        for p in range(R, n):
            c = text[p]
            if c == 10:
                D = set()
                continue
            nxt = {0} if self.accepts(c, 0) else set()
            nxt |= {q + 1 for q in D if q + 1 < len(pre) and self.accepts(c, q + 1)}
            nxt |= {q for q in D if self.rep[q] and self.accepts(c, q)}
            D = set(nxt)
            for q in sorted(nxt):
                r = q + 1
                while r < len(pre) and self.opt[r]:
                    D.add(r)
                    r += 1
            if len(pre) - 1 in D:
                yield p + 1

    def report(self, text: bytes) -> List[Tuple[int, int]]:
        out, R, n = [], 0, len(text)
        while R < n:
            hit = None
            for c in self.candidates(text, R):
                hit = self.verify(text, c, R)
                if hit:
                    break
            if not hit:
                break
            out.append(hit)
            if hit[1] == n:
                break
            R = hit[1]
        return out

    @staticmethod
    def covers(prog, plan) -> bool:
        """The model leaves out a scanned part that starts optional, type 3
        with a simple prefix (a pattern over 64 positions), and a window
        scanned by simpleScan is modelled by the general window rule."""
        scanned0 = plan["window"][0] if plan["type"] == 2 else 0
        if prog.opt_mask >> scanned0 & 1:
            return False
        if plan["type"] == 3 and plan["simple"]:
            return False
        return True
