// pm_extended.hip -- what nrgrep_coords reports for an extended pattern at
// k = 0 (nrgrep's "extended" engine), on the GPU.
//
// The reference runs `nrgrep_coords -i -b 1600000 -k 0 '<pattern>'`
// (www/FlaskApp/FlaskApp/patmatch.py:733-743); every PatMatch range X{m,n}
// becomes X..?.? (patmatch_to_nrgrep.pl:476-486), so a pattern with a range
// is a sequence of classes with '?', '*' or '+' (detClass() == 2) and
// searchPreproc (0x4026b7) picks extendedPreproc.  The binary's code
// (disassembled, never run; DESIGN.md §1, oracle/pm_nrgrep_ext.c):
//
//  * plan (extendedPreproc 0x413260): extendedFindBest (0x411fe0) prices
//    every window [beg, end) of <= 64 positions with letterProb (.data
//    0x621120); the cheapest under 0.7 is scanned backward (type 2, the
//    candidate is a window start, L = beg), else the prefix [0, end) is
//    scanned forward (type 3, the candidate is a prefix end, L = end).  A
//    window with no '?*+' uses simpleScan (0x416600), else extendedScan
//    (0x4116f0), whose backward window reads `fwd` characters (the window's
//    non-optional positions) with the optional-block closure
//    D |= S & ((D | F) ^ ~((D | F) - I)) before each step;
//  * verify (checkMatch 0x411aa0): inside the line around the candidate
//    (never before R), the L positions left of it are matched backward from
//    it and the other m - L forward, each phase stopping at the NEAREST
//    accepting boundary; each phase starts from the part's first position
//    when optional (X) without the closure;
//  * report (recSearchFile 0x402250): the first verified candidate in scan
//    order is printed, R = its end, the scan restarts at R.
//
// GPU form.  The automaton kernels (pm_nfa.hip) produce every start of a
// match.  A printed match [s, e) is a match, so s is one of them, and its
// candidate c lies in [s, e] (the left phase reads back from c to s, the
// right phase forward from c to e).  Starts more than 2 max_len + 2 apart
// (bounded patterns) or on different lines (unbounded: '*', '+') therefore
// fall into independent clusters: the candidates that can print a cluster's
// starts lie in [first, last + max_len] and no earlier print reaches back to
// them.  One thread per cluster replays the scanner and checkMatch over the
// cluster's text from R = first - max_len - 1 (or its line start); the
// matches it prints are written in place and compacted by the report pass's
// scatter (k_rep_scatter), as the esimple walk does.
#include "pm_internal.h"

#include <algorithm>

namespace pm {

namespace {

#pragma clang fp contract(off)

inline bool has_bit(const uint64_t* w, int i) { return (w[i >> 6] >> (i & 63)) & 1; }
inline void set_bit(uint64_t* w, int i) { w[i >> 6] |= 1ull << (i & 63); }

}  // namespace

// extendedFindBest 0x411fe0 (K = 0 from extendedPreproc, K = k from
// eextendedPreproc 0x40ff33): prob / aprob per position, P1 / P2 over
// [m + 1][m][m + 1]; returns the window's cost (1.0 for the prefix)
double find_best_ext(const std::vector<double>& prob, const std::vector<double>& aprob, const uint64_t* opt, int m,
                     int K, int* fwd, int* beg, int* end) {
    // the binary's third index runs to m; t never exceeds a window's 64
    // non-optional positions, so 65 slots hold the same values
    const size_t T1 = (size_t)std::min(m, 64) + 1, MM = (size_t)m * T1;
    std::vector<double> P1(((size_t)m + 1) * MM, 0.0), P2(((size_t)m + 1) * MM, 0.0);
    std::vector<int> pos(m, 0);
    auto idx = [&](int a, int b, int c) { return (size_t)a * MM + (size_t)b * T1 + (size_t)c; };
    for (int i = 0; i < m; ++i) {                        // 0x412168
        for (int t = 0; t <= i; ++t) P1[idx(t, i, 0)] = P2[idx(t, i, 0)] = 1.0;
        P1[idx(i + 1, i, 0)] = P2[idx(i + 1, i, 0)] = 0.0;
    }
    double best = 0.7;                                   // 0x41d410
    *fwd = *beg = *end = 0;
    for (int i = 0; i < m; ++i) {
        int len = 0;
        for (int j = i; j < m; ++j) {                    // 0x412345
            if ((unsigned)(j - i + 1) > 64u) continue;
            if (!has_bit(opt, j)) {
                ++len;
                if (len <= 2 * K) continue;
            } else if (2 * K >= len) {
                continue;
            }
            double sum = (double)K + 1.0;
            const int lk = len - K;
            const double lim = (double)(lk + 1);
            if (!(sum >= lim)) {
                const double dlk = (double)lk;
                double q = sum / ((dlk - sum) + 1.0);
                if (!(q >= best)) {
                    for (int t = 1;;) {                  // 0x4124a8
                        if (pos[j] < t) {
                            P2[idx(j + 1, j, t)] = 0.0;
                            P1[idx(j + 1, j, t)] = 0.0;
                            for (int l = j; l >= 0; --l) {
                                double v = prob[l] * P1[idx(l + 1, j, t - 1)] + aprob[l] * P1[idx(l, j, t - 1)];
                                v = has_bit(opt, l) ? P1[idx(l + 1, j, t)] + v : 0.0 + v;
                                double r;
                                if (v > 1.0) {
                                    P1[idx(l, j, t)] = 1.0;
                                    r = 0.0;
                                } else {
                                    P1[idx(l, j, t)] = v;
                                    r = 1.0 - v;
                                }
                                P2[idx(l, j, t)] = 1.0 - (1.0 - P2[idx(l + 1, j, t)]) * r;
                            }
                            pos[j] = t;
                        }
                        sum = sum + P2[idx(i, j, t)];
                        ++t;
                        if (t > len || sum >= lim) break;
                        q = sum / ((dlk - sum) + 1.0);
                        if (!(q < best)) break;
                    }
                }
            }
            if (lim > sum) {                             // 0x41268d
                const double q = sum / (1.0 + ((double)lk - sum));
                if (best > q) {
                    best = q;
                    *beg = i;
                    *end = j + 1;
                    *fwd = len;
                }
            }
        }
    }
    if (*fwd > 0) {                                      // 0x4127f9: optional ends trimmed
        while (*beg < *end && has_bit(opt, *beg)) ++*beg;
        while (*beg < *end && has_bit(opt, *end - 1)) --*end;
        if (*beg == *end) *fwd = 0;
        else return best;
    }
    *end = m <= 64 ? m : 64;                             // 0x4128d4: the prefix
    while (*end > 0 && has_bit(opt, *end - 1)) --*end;
    return 1.0;
}

#pragma clang fp contract(on)

XtPlan xt_plan(const uint64_t* B, int W, int m, const uint64_t* opt, const uint64_t* rep) {
    require(W >= 1 && W <= 4 && m >= 1 && m <= 64 * W, "extended plan: m / words out of range");
    double lp[256];
    letter_probs(lp);
    // bytes in increasing order (0x412058); B holds the folded byte's set
    // and -i gives a class both cases (getAclass)
    std::vector<double> prob(m, 0.0), aprob(m, 0.0);
    for (int i = 0; i < m; ++i)
        for (int c = 0; c < 256; ++c)
            if ((B[(size_t)fold((uint8_t)c) * W + (i >> 6)] >> (i & 63)) & 1) {
                prob[i] += lp[c];
                if (has_bit(rep, i)) aprob[i] += lp[c];
            }
    XtPlan P{};
    find_best_ext(prob, aprob, opt, m, 0, &P.fwd, &P.beg, &P.end);
    P.type = P.fwd ? 2 : 3;                              // 0x41336b
    P.L = P.fwd ? P.beg : P.end;
    P.simple = 1;                                        // 0x413485: detClass over the window
    for (int p = P.beg; p < P.end; ++p)
        if (has_bit(opt, p) || has_bit(rep, p)) P.simple = 0;
    return P;
}

void xt_build(const uint64_t* B, int W, int m, const uint64_t* opt, const uint64_t* rep, int64_t max_len,
              uint32_t flags, int32_t pid, Upload& up, size_t& o_slot, size_t& o_tab) {
    const XtPlan P = xt_plan(B, W, m, opt, rep);
    const int len = P.end - P.beg;
    require(len >= 1 && len <= 64, "extended plan: empty window");
    auto cls = [&](int c, int p) { return ((B[(size_t)fold((uint8_t)c) * W + (p >> 6)] >> (p & 63)) & 1) != 0; };
    auto rp = [&](int c, int p) { return has_bit(rep, p) && cls(c, p); };
    XtSlot S{};
    S.m = m;
    S.type = P.type;
    S.fwd = P.fwd;
    S.len = len;
    S.simple = P.simple;
    S.L = P.L;
    S.anchors = (int32_t)(flags & (PM_ANCHOR_START | PM_ANCHOR_END));
    S.pid = pid;
    S.max_len = max_len;
    std::vector<uint64_t> tab;
    // scanner tables (extendedLoadFast 0x413060 / simpleLoadFast 0x417520)
    S.o_T = tab.size();
    tab.resize(tab.size() + 256, 0);
    S.o_TA = tab.size();
    tab.resize(tab.size() + 256, 0);
    uint64_t* T = tab.data() + S.o_T;
    uint64_t* TA = tab.data() + S.o_TA;
    if (P.simple && P.fwd) {
        for (int r = 0; r < len; ++r)
            for (int c = 0; c < 256; ++c)
                if (cls(c, P.end - 1 - r)) T[c] |= 1ull << (64 - len + r);
    } else if (P.simple) {
        const uint64_t full = len == 64 ? ~0ull : (1ull << len) - 1;
        for (int c = 0; c < 256; ++c) T[c] = full;
        for (int r = 0; r < len; ++r)
            for (int c = 0; c < 256; ++c)
                if (cls(c, P.beg + r)) T[c] &= ~(1ull << r);
    } else {
        int b = P.fwd ? 64 - len : 0, p = P.fwd ? P.end - 1 : P.beg;
        for (int r = 0; r < len; ++r, ++b, p += P.fwd ? -1 : 1) {
            const uint64_t bit = 1ull << b;
            for (int c = 0; c < 256; ++c) {
                if (cls(c, p)) T[c] |= bit;
                if (rp(c, p)) TA[c] |= bit;
            }
            if (has_bit(opt, p)) {                       // 0x4131ba
                const uint64_t pbit = 1ull << ((b - 1) & 63);
                S.fS |= bit;
                if (S.fF & pbit) {
                    S.fF = (S.fF & ~pbit) | bit;
                } else {
                    S.fI |= pbit;
                    S.fF |= bit;
                }
            }
        }
    }
    // verify parts (extendedLoadVerif 0x412c60): left = [0, L) from L - 1
    // down, right = [L, m) up
    for (int side = 0; side < 2; ++side) {
        const int plen = side == 0 ? P.L : m - P.L, p0 = side == 0 ? P.L - 1 : P.L, dir = side == 0 ? -1 : 1;
        const int pw = std::max(1, (plen + 63) >> 6);
        S.plen[side] = plen;
        S.pw[side] = pw;
        S.o_vB[side] = tab.size();
        tab.resize(tab.size() + (size_t)256 * pw, 0);
        S.o_vA[side] = tab.size();
        tab.resize(tab.size() + (size_t)256 * pw, 0);
        uint64_t* vB = tab.data() + S.o_vB[side];
        uint64_t* vA = tab.data() + S.o_vA[side];
        bool opened = false;
        for (int r = 0; r < plen; ++r) {
            const int p = p0 + r * dir;
            for (int c = 0; c < 256; ++c) {
                if (cls(c, p)) set_bit(vB + (size_t)c * pw, r);
                if (rp(c, p)) set_bit(vA + (size_t)c * pw, r);
            }
            if (!has_bit(opt, p)) continue;
            if (r > 0) {
                if (has_bit(S.vF[side], r - 1)) {        // 0x412ff1: the block goes on
                    S.vF[side][(r - 1) >> 6] &= ~(1ull << ((r - 1) & 63));
                    set_bit(S.vF[side], r);
                } else {
                    set_bit(S.vI[side], r - 1);
                    set_bit(S.vF[side], r);
                    set_bit(S.vS[side], r);
                    opened = true;
                    continue;
                }
            }
            if (opened) set_bit(S.vS[side], r);          // 0x413015
            else set_bit(S.vX[side], r);
        }
    }
    o_slot = up.add(&S, sizeof(S));
    o_tab = up.add(tab.data(), tab.size() * 8);
}

// ---------------------------------------------------------------------------
// device: the per-cluster replay
// ---------------------------------------------------------------------------
namespace {

constexpr uint64_t XT_POS_MASK = (1ull << 48) - 1;
constexpr uint64_t XT_SCAN = 1ull << 16;   // unbounded patterns: how far a head looks back for a line break
constexpr uint32_t XT_T = 256;

__global__ __launch_bounds__(XT_T) void k_xt_heads(XtPrep X, const uint64_t* __restrict__ keys, const uint64_t* total_d,
                                                   uint64_t total_h, uint8_t* __restrict__ acc, TextView tv) {
    const uint64_t total = total_d ? *total_d : total_h;
    const XtSlot& S = *X.slot;
    for (uint64_t i = blockIdx.x * (uint64_t)XT_T + threadIdx.x; i < total; i += (uint64_t)gridDim.x * XT_T) {
        bool head = i == 0 || (keys[i] >> 48) != (keys[i - 1] >> 48);
        if (!head) {
            const uint64_t a = keys[i - 1] & XT_POS_MASK, b = keys[i] & XT_POS_MASK;
            if (xt_region(tv, a) != xt_region(tv, b)) head = true;
            else if (S.max_len >= 0) head = b - a > 2 * (uint64_t)S.max_len + 2;
            else head = xt_brk_between(tv, a, b, XT_SCAN);
        }
        acc[i] = head ? 2 : 0;
    }
}

// one walk: nrgrep's scanner and checkMatch over [R, n), candidates up to
// `stop`
// WB: the verify parts' words; SC: the scanner (xt_scanner: one scanner and
// one inlined checkMatch per kernel)
template <int WB, int SC>
struct XtWalk {
    const XtSlot* S;
    const uint64_t* tab;
    TextView tv;
    uint64_t n;        // the region end
    uint64_t R;
    uint64_t nl_lo;    // the last '\n' seen below the record cursor (~0: none since the walk began)
    uint64_t nl_hi;    // the first '\n' at or after it (n: none)
    mutable TxtCache tc;   // the thread's text window (LDS)

    __device__ uint8_t at(uint64_t p) const { return tc.get(tv, p); }
    __device__ bool is_nl(uint64_t p) const { return xt_brk(tv, p) && at(p) == (uint8_t)'\n'; }
    __device__ uint64_t next_nl(uint64_t p) const { return xt_next_nl(tv, p, n); }
    // recGetRecord 0x402030 for rp (non-decreasing over a walk): the last
    // '\n' before rp searched back to R only, the first at or after it
    __device__ void record(uint64_t rp, uint64_t& recbeg, uint64_t& recend) {
        while (nl_hi < rp) {
            nl_lo = nl_hi;
            nl_hi = next_nl(nl_hi + 1);
        }
        recbeg = (nl_lo != ~0ull && nl_lo >= R) ? nl_lo + 1 : R;
        recend = nl_hi;
    }
    __device__ bool left_ok(uint64_t p, uint64_t recbeg) const {
        return !((S->anchors & PM_ANCHOR_START) && p > recbeg && at(p - 1) != (uint8_t)'\n');
    }
    __device__ bool right_ok(uint64_t q, uint64_t recend) const {
        return !((S->anchors & PM_ANCHOR_END) && q < recend && at(q) != (uint8_t)'\n');
    }

    // one phase of checkMatch: D from X, then (D << 1 | carry) & B | D & A
    // and the closure per character (0x411c98 / 0x411eb0); the next step's
    // character and table words are read before the step's arithmetic
    __device__ __forceinline__ bool phase(int side, uint64_t pos, uint64_t bound, bool left, uint64_t& out) const {
        const int W = S->pw[side], len = S->plen[side];
        const uint64_t fin = 1ull << ((len - 1) & 63);
        const uint64_t* vB = tab + S->o_vB[side];
        const uint64_t* vA = tab + S->o_vA[side];
        uint64_t D[WB];
#pragma unroll
        for (int w = 0; w < WB; ++w) D[w] = w < W ? S->vX[side][w] : 0ull;
        uint64_t carry = 1;
        uint64_t p = pos;   // left: the boundary is p; right: p is the last character read + 1
        uint64_t Bc[WB], Ac[WB];
        {
            const uint8_t c0 = p != bound ? (left ? at(p - 1) : at(p)) : (uint8_t)0;
#pragma unroll
            for (int w = 0; w < WB; ++w) {
                Bc[w] = w < W ? vB[(size_t)c0 * W + w] : 0ull;
                Ac[w] = w < W ? vA[(size_t)c0 * W + w] : 0ull;
            }
        }
        for (;;) {
            const bool ok = left ? left_ok(p, bound) : right_ok(p, bound);
            uint64_t dl = 0;   // D[W - 1] without a run-time index (no scratch)
#pragma unroll
            for (int w = 0; w < WB; ++w)
                if (w == W - 1) dl = D[w];
            if ((dl & fin) && ok) {
                out = p;
                return true;
            }
            if (p == bound) return false;
            p = left ? p - 1 : p + 1;
            uint64_t Bn[WB], An[WB];
            {
                const uint8_t cn = p != bound ? (left ? at(p - 1) : at(p)) : (uint8_t)0;
#pragma unroll
                for (int w = 0; w < WB; ++w) {
                    Bn[w] = w < W ? vB[(size_t)cn * W + w] : 0ull;
                    An[w] = w < W ? vA[(size_t)cn * W + w] : 0ull;
                }
            }
            bool any = false;
#pragma unroll
            for (int w = 0; w < WB; ++w) {
                if (w >= W) break;
                const uint64_t old = D[w];
                D[w] = (((old << 1) | carry) & Bc[w]) | (old & Ac[w]);
                any |= D[w] != 0;
                carry = old >> 63;
            }
            if (!any) return false;
            uint64_t borrow = 0;
#pragma unroll
            for (int w = 0; w < WB; ++w) {
                if (w >= W) break;
                const uint64_t d = D[w], xx = d | S->vF[side][w];
                const uint64_t sub = xx - borrow - S->vI[side][w];
                D[w] = ((~sub ^ xx) & S->vS[side][w]) | d;
                const uint64_t bi = borrow + S->vI[side][w];
                borrow = (bi < borrow) | (xx < bi);
            }
            carry = 0;
#pragma unroll
            for (int w = 0; w < WB; ++w) {
                Bc[w] = Bn[w];
                Ac[w] = An[w];
            }
        }
    }

    __device__ __forceinline__ bool check(uint64_t pos, uint64_t& mb, uint64_t& me) {
        const uint64_t rp = S->type == 3 ? pos - 1 : pos;   // 0x411b90
        if (pos == 0 && S->type == 3) return false;
        uint64_t recbeg, recend;
        record(rp, recbeg, recend);
        if (rp < recbeg || rp >= recend) return false;
        uint64_t start = pos;
        if (S->plen[0] == 0) {
            if (!left_ok(pos, recbeg)) return false;
        } else if (!phase(0, pos, recbeg, true, start)) {
            return false;
        }
        uint64_t end = pos;
        if (S->plen[1] == 0) {
            if (!right_ok(pos, recend)) return false;
        } else if (!phase(1, pos, recend, false, end)) {
            return false;
        }
        mb = start;
        me = end;
        return true;
    }

    // the scanners (pm_nrgrep_ext.c); false when no candidate <= stop verifies
    __device__ bool scan(uint64_t stop, uint64_t& mb, uint64_t& me) {
        const uint64_t* T = tab + S->o_T;
        const uint64_t* TA = tab + S->o_TA;
        if constexpr (SC == 0) {                         // extendedScan 0x4116f0, window
            const uint64_t len = (uint64_t)S->fwd;
            if (n < len) return false;
            const uint64_t limit = n - len;
            uint64_t r11 = R;   // the window start (r11 + 1 in the binary)
            while (r11 <= limit) {
                if (r11 > stop) return false;
                uint64_t D = T[at(r11 + len - 1)];
                if (!D) {
                    r11 += len;
                    continue;
                }
                uint64_t c = r11 + len - 1;
                bool dead = false;
                for (uint64_t e = len - 1; e > 0; --e) {
                    --c;
                    const uint64_t xx = D | S->fF;
                    const uint64_t Dc = ((~(xx - S->fI) ^ xx) & S->fS) | D;
                    const uint8_t ch = at(c);
                    D = ((Dc << 1) & T[ch]) | (Dc & TA[ch]);
                    if (!D) {
                        r11 = c + 1;
                        dead = true;
                        break;
                    }
                }
                if (dead) continue;
                if ((D >> 63) && check(r11, mb, me)) return true;
                ++r11;
            }
            return false;
        }
        if constexpr (SC == 1) {                         // simpleScan 0x4166d2, window
            const uint64_t len = (uint64_t)S->len;
            if (n < len) return false;
            const uint64_t r8 = n - len;
            uint64_t s0 = R;    // the window start (rsi + 1 in the binary)
            while (s0 <= r8) {
                if (s0 > stop) return false;
                uint64_t D = T[at(s0 + len - 1)];
                if (!D) {
                    s0 += len;
                    continue;
                }
                uint64_t c = s0 + len - 1;
                uint64_t e = len;
                // the table word of the next character read, a step ahead
                uint64_t Tn = c > s0 ? T[at(c - 1)] : 0ull;
                for (;;) {
                    const uint64_t sh = D << 1;
                    --e;
                    --c;
                    const uint64_t Tc = Tn;
                    Tn = c > s0 ? T[at(c - 1)] : 0ull;
                    // reading s0 - 1 only meets a shifted-out state
                    D = sh ? sh & Tc : 0ull;
                    if (!D) break;
                }
                if (e == 0) {
                    if (check(s0, mb, me)) return true;
                    ++s0;
                } else {
                    s0 = c + 1;
                }
            }
            return false;
        }
        const uint64_t fin = 1ull << (S->len - 1);
        if constexpr (SC == 2) {                         // simpleScan 0x41663d, prefix: the START goes on
            const uint64_t len = (uint64_t)S->len;
            uint64_t D = ~0ull;
            for (uint64_t q = R; q < n; ++q) {
                D = (D << 1) | T[at(q)];
                if (!(D & fin)) {
                    const uint64_t c = q + 1 - len;
                    if (c > stop) return false;
                    if (check(c, mb, me)) return true;
                }
            }
            return false;
        }
        uint64_t D = 0;                                  // extendedScan 0x41184f, prefix
        bool fresh = true;
        // the next character and its table words are read a step ahead
        uint8_t cn = R < n ? at(R) : (uint8_t)0;
        uint64_t Tn = T[cn], TAn = TA[cn];
        for (uint64_t p = R; p < n; ++p) {
            if (p >= stop) return false;   // the candidate p + 1 is past it
            const uint8_t c = cn;
            const uint64_t Tc = Tn, TAc = TAn;
            cn = p + 1 < n ? at(p + 1) : (uint8_t)0;
            Tn = T[cn];
            TAn = TA[cn];
            if (c == (uint8_t)'\n') {
                fresh = true;
                continue;
            }
            if (fresh) {
                D = 0;
                fresh = false;
            }
            D = (D & TAc) | (((D << 1) | 1ull) & Tc);
            const uint64_t xx = D | S->fF;
            D |= (~(xx - S->fI) ^ xx) & S->fS;
            if ((D & fin) && check(p + 1, mb, me)) return true;
        }
        return false;
    }
};

// One thread per cluster head: the printed matches are written in place
// from the head on (acc bit 0), every other entry of the cluster is cleared.
template <int WB, int SC>
__global__ __launch_bounds__(WALK_T) void k_xt_walk(XtPrep X, uint64_t* __restrict__ keys, uint32_t* __restrict__ lens,
                                                    const uint64_t* total_d, uint64_t total_h,
                                                    uint8_t* __restrict__ acc, TextView tv) {
    extern __shared__ __attribute__((aligned(16))) uint8_t walk_lds[];
    const uint64_t total = total_d ? *total_d : total_h;
    const XtSlot* S = X.slot;
    // the tables in LDS when they fit, then the thread's text window
    const size_t tb = walk_tab_bytes(X.tab_words);
    const uint64_t* tab = X.tab;
    if (tb) {
        uint64_t* lt = reinterpret_cast<uint64_t*>(walk_lds);
        for (uint32_t q = threadIdx.x; q < X.tab_words; q += blockDim.x) lt[q] = X.tab[q];
        tab = lt;
    }
    __syncthreads();
    uint8_t* const tcbuf = walk_lds + tb + threadIdx.x * TC_WIN;
    for (uint64_t i = blockIdx.x * (uint64_t)WALK_T + threadIdx.x; i < total; i += (uint64_t)gridDim.x * WALK_T) {
        if (!(acc[i] & 2)) continue;
        uint64_t j = i + 1;   // the next cluster's head keeps bit 1 whatever its owner writes
        while (j < total && !(acc[j] & 2)) ++j;
        const uint64_t pid = keys[i] >> 48;
        const uint64_t first = keys[i] & XT_POS_MASK, last = keys[j - 1] & XT_POS_MASK;
        uint64_t nout = 0;
        const uint64_t nmax = j - i;
        if ((int64_t)pid == X.pid) {
            uint64_t R0 = 0, n = tv.n;
            if (tv.reg.n > 1) {
                const uint32_t r = region_of(tv.reg, first);
                R0 = tv.reg.t[r];
                n = tv.reg.e[r];
            }
            XtWalk<WB, SC> w{S, tab, tv, n, R0, ~0ull, n, TxtCache{tcbuf, 0, 0}};
            uint64_t stop;
            if (S->max_len >= 0) {
                // candidates in [first, last + max_len] can print the
                // cluster's starts; no earlier print reaches first - max_len
                const uint64_t back = (uint64_t)S->max_len + 1;
                if (first > R0 + back) w.R = first - back;
                stop = last + (uint64_t)S->max_len;
            } else {
                // unbounded: the cluster's lines, from the first one's start
                uint64_t p = first;
                while (p > R0 && !w.is_nl(p - 1)) --p;
                w.R = p;
                stop = w.next_nl(last);
            }
            w.nl_hi = w.next_nl(w.R);
            for (;;) {
                uint64_t mb = 0, me = 0;
                if (!w.scan(stop, mb, me)) break;
                if (!xt_header(tv, mb) && nout < nmax) {   // a printed start is one of the cluster's
                    keys[i + nout] = (pid << 48) | mb;
                    lens[i + nout] = (uint32_t)(me - mb);
                    acc[i + nout] = (nout == 0 ? 2 : 0) | 1;
                    ++nout;
                }
                if (me >= n) break;                      // 0x4022eb
                w.R = me;
            }
        }
        for (uint64_t q = i + nout; q < j; ++q) acc[q] = q == i ? 2 : 0;
    }
}

// kept entries (acc bit 0) per chunk of C = ceil(total / G) entries, for
// k_rep_scatter
__global__ __launch_bounds__(256) void k_xt_count(const uint64_t* total_d, uint64_t total_h,
                                                  const uint8_t* __restrict__ acc, uint32_t* __restrict__ bcnt) {
    __shared__ uint32_t red[4];
    const uint64_t total = total_d ? *total_d : total_h;
    const uint64_t C = (total + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = blockIdx.x * C, b1 = umin64(total, b0 + C);
    uint32_t c = 0;
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += blockDim.x) c += acc[i] & 1;
    for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) bcnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

}  // namespace

int xt_scanner(const Upload& up, size_t o_slot) {
    XtSlot S;
    memcpy(&S, up.blob.data() + o_slot, sizeof(S));
    if (S.type == 2) return S.simple ? 1 : 0;
    return S.simple ? 2 : 3;
}

void xt_launch(const XtPrep& X, uint64_t* keys, uint32_t* lens, const uint64_t* total_d, uint64_t total_h,
               uint8_t* acc, uint32_t* bcnt, uint32_t G, const TextView& tv, hipStream_t s) {
    const uint32_t blocks = 1024;
    if (X.rg) {
        rg_launch(X, keys, lens, total_d, total_h, acc, tv, s);
    } else if (X.ee) {
        ee_launch(X, keys, lens, total_d, total_h, acc, tv, X.words, s);
    } else {
        hipLaunchKernelGGL(k_xt_heads, dim3(blocks), dim3(XT_T), 0, s, X, keys, total_d, total_h, acc, tv);
        // the verify parts' words and the scanner are template arguments
        const size_t lds = walk_tab_bytes(X.tab_words) + WALK_T * TC_WIN;
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(WALK_T), lds, s, X, keys, lens, total_d, total_h, acc, tv);
        };
        auto by_sc = [&](auto wb) {
            constexpr int WB = decltype(wb)::value;
            switch (X.scanner) {
                case 0: go(k_xt_walk<WB, 0>); break;
                case 1: go(k_xt_walk<WB, 1>); break;
                case 2: go(k_xt_walk<WB, 2>); break;
                default: go(k_xt_walk<WB, 3>); break;
            }
        };
        if (X.words <= 1) by_sc(std::integral_constant<int, 1>{});
        else by_sc(std::integral_constant<int, 4>{});
    }
    hipLaunchKernelGGL(k_xt_count, dim3(G), dim3(256), 0, s, total_d, total_h, acc, bcnt);
    HIPCHK(hipGetLastError());
}

}  // namespace pm

using namespace pm;

extern "C" int pm_extended_plan(int m, int words, const uint64_t* byte_mask, const uint64_t* opt_mask,
                                const uint64_t* rep_mask, int32_t* out) {
    return guarded([&] {
        require(byte_mask != nullptr && opt_mask != nullptr && rep_mask != nullptr && out != nullptr, "null argument");
        require(words >= 1 && words <= 4 && m >= 1 && m <= 64 * words, "m / words out of range");
        const XtPlan P = xt_plan(byte_mask, words, m, opt_mask, rep_mask);
        out[0] = P.type;
        out[1] = P.fwd;
        out[2] = P.beg;
        out[3] = P.end;
        out[4] = P.L;
        out[5] = P.simple;
    });
}
