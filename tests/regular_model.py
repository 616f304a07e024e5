"""A second statement of nrgrep's regular engine at k = 0 (what
oracle/pm_nrgrep_reg.c replays literally): the report written over state
SETS instead of the binary's loops, so the backward scanner's window shifts,
the forward scanner's restarts and the checkMatch order are checked against
their meaning.  TEST INFRASTRUCTURE ONLY.

* backward plan (type 2): from R, the first window start ws (ws + ell <= n)
  whose window set D -- the window states q reading t[ws] with a path of ell
  characters inside the window -- meets the window's initial states and
  whose checkMatch succeeds (every window start that can pass is examined in
  increasing order whatever the shifts were: pm_regular.hip relies on it);
* forward plan (type 3): the first end pointer p (R < p < n; a '\\n' restarts
  the automaton) where the states reached from some start in [R, p) of the
  line meet the window's final states, checkMatch over those;
* checkMatch: inside the line around the candidate (never before R), for
  each state in state order, the shortest end forward and the nearest start
  backward around it; the first state with both wins.

The plan (window, initial / final states, ell) comes from the library
(engine.regular_plan), checked against the oracle's separately."""

from typing import List, Tuple


def _fold(c: int) -> int:
    return c - 32 if 97 <= c <= 122 else c


class Model:
    def __init__(self, prog, plan):
        self.m = prog.m + 1
        self.arrows = [prog.first << 1] + [f << 1 for f in prog.follow]
        self.final = prog.last << 1
        bm = prog.byte_masks()
        self.B = [bm[_fold(c)] << 1 for c in range(256)]
        self.rev = [0] * self.m
        for s in range(self.m):
            for q in range(self.m):
                if self.arrows[s] >> q & 1:
                    self.rev[q] |= 1 << s
        self.plan = plan
        self.win = plan["window"]
        self.start = prog.anchor_start
        self.end = prog.anchor_end

    def _step(self, D: int, tab) -> int:
        out = 0
        s = 0
        while D:
            if D & 1:
                out |= tab[s]
            D >>= 1
            s += 1
        return out

    def _record(self, t: bytes, rp: int, R: int) -> Tuple[int, int]:
        nl = t.rfind(b"\n", 0, rp)
        rb = nl + 1 if nl >= R else R
        re_ = t.find(b"\n", rp)
        return rb, (len(t) if re_ < 0 else re_)

    def _fwd(self, t, p, lim, s):
        D = 1 << s
        while True:
            if D & self.final and not (self.end and p + 1 < lim + 1 and t[p + 1] != 10):
                return p
            if p == lim:
                return None
            p += 1
            D = self._step(D, self.arrows) & self.B[t[p]]
            if not D:
                return None

    def _bwd(self, t, p, lim, s):
        D = 1 << s
        while True:
            if D & 1 and not (self.start and p > lim and t[p - 1] != 10):
                return p
            if p == lim:
                return None
            p -= 1
            D = self._step(D & self.B[t[p]], self.rev)
            if not D:
                return None

    def _check(self, t, pos, R, states: List[int]):
        fwd_type = self.plan["type"] == 3
        rp = pos - 1 if fwd_type else pos
        rb, re_ = self._record(t, rp, R)
        if rp < rb or rp >= re_:
            return None
        for s in states:
            if fwd_type:
                st = self._bwd(t, pos, rb, s)
                en = None if st is None else self._fwd(t, pos - 1, re_ - 1, s)
            else:
                en = self._fwd(t, pos, re_ - 1, s)
                st = None if en is None else self._bwd(t, pos + 1, rb, s)
            if st is not None and en is not None:
                return st, en + 1
        return None

    def _window_set(self, t, ws):
        ell = self.plan["ell"]
        alive = self.win & self.B[t[ws + ell - 1]]          # any window state may end the window
        for j in range(ell - 2, -1, -1):
            alive = self.win & self.B[t[ws + j]] & self._step(alive, self.rev)
        return alive

    def _scan(self, t: bytes, R: int):
        n = len(t)
        if self.plan["type"] == 2:
            ell = self.plan["ell"]
            init = self.plan["init"]
            for ws in range(R, n - ell + 1):
                D = self._window_set(t, ws)
                if D & init:
                    hit = self._check(t, ws, R, [s for s in range(self.m) if D >> s & 1])
                    if hit:
                        return hit
            return None
        final = self.plan["final"]
        D = 0
        for p in range(R, n):
            c = t[p]
            if c == 10:
                D = 0
                continue
            D = (self._step(D, self.arrows) | self.arrows[0]) & self.win & self.B[c]
            if p + 1 < n and D & final:
                hit = self._check(t, p + 1, R, [s for s in range(self.m) if (D & final) >> s & 1])
                if hit:
                    return hit
        return None

    def report(self, text: bytes):
        """One region [0, n): the printed matches."""
        if self.plan["cls"] != 3:
            return []
        out, R = [], 0
        while R < len(text):
            hit = self._scan(text, R)
            if hit is None:
                break
            out.append(hit)
            if hit[1] == len(text):
                break
            R = hit[1]
        return out
