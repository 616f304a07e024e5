"""A second, independent statement of nrgrep's esimple report (test helper).

``oracle/pm_nrgrep.c`` replays the binary's own loops (its BNDM / ABNDM /
shift-or scanners and the bit-parallel rows of checkMatch1 0x414190).  This
module states the same behaviour the way the GPU walk (pm_esimple.hip) uses
it, and computes every phase with a plain edit-distance table instead of
bit-parallel rows:

* candidates, in scan order from the region start R:
    type 1  positions pos (then piece i = 0..k) where the pieces that match
            exactly at pos, as BNDM's surviving bits, intersect piece i's
            test mask (esimpleScan 0x41384b: a 32-bit ``1 << bit``);
    type 2  every pos below n - (window length - k - 1), L = window start;
    type 3  every end position e > R, L = the window end, the record taken
            from e - 1;
* verify: the record is the line around the candidate, never starting
  before R (recGetRecord 0x402030).  Left of pos the pattern part
  [0, L) is aligned backward, right of pos the part [L, m) forward; the
  text character next to pos on either side is never an insertion (the
  phases inject their start state only on their first step).  The left
  phase takes the start p nearest to pos among those with the fewest
  errors (<= k); the right phase the nearest end among those with the
  fewest errors (<= k - left errors); '^' / '$' restrict p / the end to
  the record bounds (recCheckLeft/RightContext 0x402170 / 0x4021e0);
* report: the first verified candidate; R = its end; restart at R; stop
  when a match ends at the end of the text (recSearchFile 0x402250).
"""

from __future__ import annotations

INF = 1 << 30


def _fold(c: int) -> int:
    return c - 32 if 97 <= c <= 122 else c


def _phase(prog, text: bytes, pos: int, lo: int, hi: int, L: int, left: bool, kmax: int, types: str,
           anchor: bool):
    """Nearest boundary with the fewest errors, or None.  Left: the pattern
    part [0, L) reversed against text[p, pos) for p in [lo, pos]; right: the
    part [L, m) against text[pos, q) for q in [pos, hi]."""
    part = list(range(L - 1, -1, -1)) if left else list(range(L, prog.m))
    span = (pos - lo) if left else (hi - pos)
    chars = [_fold(text[pos - 1 - j]) if left else _fold(text[pos + j]) for j in range(span)]
    n_a = len(part)
    ins, dele, sub = "i" in types, "d" in types, "s" in types
    # D[i][j]: part[:i] against chars[:j]; no insertion before part[0]
    prev = [INF] * (span + 1)
    prev[0] = 0
    for j in range(1, span + 1):
        # an empty part may still take insertions up to a context boundary
        # (the len == 0 loops of checkMatch1, 0x4141ef / 0x414eae)
        prev[j] = j if (n_a == 0 and ins) else INF
    best = None
    cols = [prev[:]]
    for i in range(1, n_a + 1):
        cur = [INF] * (span + 1)
        cur[0] = prev[0] + 1 if dele else INF
        cls = prog.classes[part[i - 1]]
        for j in range(1, span + 1):
            v = prev[j - 1] + (0 if chars[j - 1] in cls else (1 if sub else INF))
            if ins:
                v = min(v, cur[j - 1] + 1)
            if dele:
                v = min(v, prev[j] + 1)
            cur[j] = min(v, INF)
        prev = cur
        cols.append(cur)
    final = prev
    bound_ok = (lambda j: pos - j == lo) if left else (lambda j: pos + j == hi)
    dmin = INF
    for j in range(span + 1):
        if anchor and not bound_ok(j):
            continue
        if final[j] < dmin:
            dmin = final[j]
            best = j
    if dmin > kmax:
        return None
    return (pos - best if left else pos + best), dmin


def _record(text: bytes, rp: int, R: int):
    nl = text.rfind(b"\n", R, rp)
    lo = nl + 1 if nl >= 0 else R
    e = text.find(b"\n", rp)
    hi = e if e >= 0 else len(text)
    return lo, hi


def _verify(prog, text, plan, k, types, typ, L, pos, R):
    rp = pos - 1 if typ == 3 else pos
    if rp < 0 or rp >= len(text):
        return None
    lo, hi = _record(text, rp, R)
    if not (lo <= rp < hi):
        return None
    left = _phase(prog, text, pos, lo, hi, L, True, k, types, prog.anchor_start)
    if left is None:
        return None
    right = _phase(prog, text, pos, lo, hi, L, False, k - left[1], types, prog.anchor_end)
    if right is None:
        return None
    return left[0], right[0]


def _piece_bits(prog, text, plan, pos):
    mpc = plan["piece_len"]
    D = 0
    for r, L in enumerate(plan["L"]):
        if pos + mpc > len(text):
            return 0
        if all(_fold(text[pos + j]) in prog.classes[L + j] for j in range(mpc)):
            D |= 1 << (r * mpc + mpc - 1)
    return D


def _test_mask(bit: int) -> int:
    v = (1 << (bit & 31)) & 0xFFFFFFFF
    if v & 0x80000000:
        v |= 0xFFFFFFFF00000000
    return v


def report(text: bytes, prog, k: int, types: str, plan: dict):
    """nrgrep_coords' matches for a class sequence at k > 0."""
    n = len(text)
    typ = plan["type"]
    out, R = [], 0
    while R < n:
        found = None
        if typ == 1:
            mpc = plan["piece_len"]
            for pos in range(R, n - mpc + 1):
                D = _piece_bits(prog, text, plan, pos)
                if not D:
                    continue
                for i, L in enumerate(plan["L"]):
                    if D & _test_mask(i * mpc + mpc - 1):
                        found = _verify(prog, text, plan, k, types, 1, L, pos, R)
                        if found:
                            break
                if found:
                    break
        elif typ == 2:
            wb, we = plan["window"]
            for pos in range(R, n - (we - wb - k - 1)):
                found = _verify(prog, text, plan, k, types, 2, plan["L"][0], pos, R)
                if found:
                    break
        else:
            for pos in range(R + 1, n + 1):
                found = _verify(prog, text, plan, k, types, 3, plan["L"][0], pos, R)
                if found:
                    break
        if not found:
            break
        out.append(found)
        if found[1] == n:
            break
        R = found[1]
    return out
