// pm_regular.hip -- what nrgrep_coords reports for a regular pattern at k = 0
// (nrgrep's "regular" engine), on the GPU.
//
// The reference runs `nrgrep_coords -i -b 1600000 -k 0 '<pattern>'`
// (www/FlaskApp/FlaskApp/patmatch.py:733-743); a PatMatch pattern that
// repeats a parenthesised group -- GA(TC){1,2}A becomes (GA(TC)(TC)?A)
// (patmatch_to_nrgrep.pl:307-348, :462-495) -- or a user pattern with '|' is
// a general regular expression (detClass() == 3) and searchPreproc picks
// regularPreproc (0x40c880).  The binary's code (disassembled, never run;
// DESIGN.md §1, oracle/pm_nrgrep_reg.c):
//
//  * plan (regularFindBest 0x40a500, minCost 0x409940): every state's
//    distance to a final state; per state and length, the chance a random
//    text (letterProb, .data 0x621120) runs along the automaton; minCost
//    over nrgrep's tree: a leaf opens a window of l levels (the states
//    reachable within l - 1 arrows), '|' joins both sides' windows, a
//    concatenation takes its cheaper side, '*' / '?' cannot hold one; the
//    best cost / (l - cost + 1) under 0.65 is scanned backward (type 2),
//    else the whole automaton forward (type 3);
//  * detClass (0x41ac90) of the window: a class sequence (1) or an extended
//    sequence (2) runs simpleScan / extendedScan, which never set the state
//    word checkMatch reads (P->match, +0x28, zeroed at 0x40cb91): nothing is
//    ever printed.  A regular window (3) runs regularScan (0x4091d0);
//  * scan: backward, windows of l characters read right to left over the
//    window's reversed automaton with every state initial (a factor test:
//    a dead character moves the window past it); a whole window whose last
//    set leads back to the window's initial states goes to checkMatch with
//    that set.  Forward: the window automaton with state 0 looping, fresh
//    after each '\n', never tested after the region's last byte;
//  * verify (checkMatch 0x408ec0): for each state of the set in state order,
//    inside the line (never before R): the shortest end forward (fwdCheck
//    0x408bc0) and the nearest start backward (bwdCheck 0x408d50) around it
//    on the whole automaton (transition tables in slices of W states of one
//    word: SLICE 0x41b8e0 loses the states of a slice that straddles a word);
//  * report (recSearchFile 0x402250): the first verified candidate is
//    printed, R = its end.
//
// GPU form.  The automaton kernels (pm_nfa.hip) give every start of a match;
// a printed match is a match, so its start is one of them and the window
// that printed it starts inside it.  Every window start that can pass the
// factor test is examined in increasing order whatever the shifts were, so
// the result from R depends on R only: starts more than 2 max_len + 2 apart
// form independent clusters, one thread replays the scanner and checkMatch
// over a cluster from R = first - max_len - 1 (forward: the automaton's
// final states are the window's, so an earlier start only matters through
// a match that ends before it).  Unbounded patterns ('*', '+') and forward
// plans over more than 64 states walk whole lines.  The printed matches are
// written in place and compacted by the report pass's scatter.
#include "pm_internal.h"

#include <algorithm>
#include <array>

namespace pm {

namespace {

#pragma clang fp contract(off)

enum { T_LEAF = 0, T_STAR = 1, T_OR = 2, T_CAT = 3, T_OPT = 4, T_PLUS = 5 };

using Set = std::array<uint64_t, RG_NW>;

inline bool has(const Set& s, int i) { return (s[i >> 6] >> (i & 63)) & 1; }
inline void put(Set& s, int i) { s[i >> 6] |= 1ull << (i & 63); }
inline void join(Set& d, const Set& s) {
    for (int q = 0; q < RG_NW; ++q) d[q] |= s[q];
}
inline bool meets(const Set& a, const Set& b) {
    uint64_t x = 0;
    for (int q = 0; q < RG_NW; ++q) x |= a[q] & b[q];
    return x != 0;
}
inline int bits(const Set& s) {
    int n = 0;
    for (int q = 0; q < RG_NW; ++q) n += __builtin_popcountll(s[q]);
    return n;
}

struct Node {
    int type, a, b, state;
    bool nullable;
    Set pm{}, first{}, last{};
};

// the automaton over nrgrep's states (regularLength 0x40b2a0: state 0 is
// the initial one, leaves are numbered 1.. left to right)
struct Automaton {
    int ms = 0;
    std::vector<Node> nd;
    std::vector<Set> arrows, rev;
    Set final_{}, vis{};
    std::vector<Set> B;   // [256] by folded byte

    void masks(int i) {   // firstLast 0x4086b0 / setMaskPos 0x41ad90
        Node& e = nd[i];
        if (e.type == T_LEAF) {
            put(e.pm, e.state);
            put(e.first, e.state);
            put(e.last, e.state);
            return;
        }
        masks(e.a);
        const Node& a = nd[e.a];
        e.pm = a.pm;
        if (e.type == T_OR || e.type == T_CAT) {
            masks(e.b);
            const Node& b = nd[e.b];
            join(e.pm, b.pm);
            if (e.type == T_OR) {
                e.first = a.first;
                join(e.first, b.first);
                e.last = a.last;
                join(e.last, b.last);
            } else {
                e.first = a.first;
                if (a.nullable) join(e.first, b.first);
                e.last = b.last;
                if (b.nullable) join(e.last, a.last);
            }
        } else {
            e.first = a.first;
            e.last = a.last;
        }
    }
    void follow(int i, int s, Set& out) const {   // follow 0x4089b0
        const Node& e = nd[i];
        if (e.type == T_LEAF) return;
        if (e.type == T_OPT) return follow(e.a, s, out);
        if (e.type == T_STAR || e.type == T_PLUS) {
            follow(e.a, s, out);
            if (has(nd[e.a].last, s)) join(out, nd[e.a].first);
            return;
        }
        if (e.type == T_CAT && has(nd[e.a].last, s)) join(out, nd[e.b].first);
        if (has(nd[e.a].pm, s)) follow(e.a, s, out);
        if (has(nd[e.b].pm, s)) follow(e.b, s, out);
    }
};

Automaton make_automaton(const RgTree& t, const uint64_t* B, int W, int npos) {
    Automaton A;
    require(t.nodes >= 1 && t.tree && t.nullable, "regular: no tree");
    require(npos >= 1 && npos + 1 <= 64 * RG_NW, "regular: positions out of range");
    A.ms = npos + 1;
    A.nd.resize(t.nodes);
    int leaves = 0;
    for (int i = 0; i < t.nodes; ++i) {
        Node& e = A.nd[i];
        e.type = t.tree[4 * i];
        e.a = t.tree[4 * i + 1];
        e.b = t.tree[4 * i + 2];
        e.nullable = t.nullable[i] != 0;
        require(e.type >= 0 && e.type <= 5, "regular: bad node type");
        if (e.type == T_LEAF) {
            // an empty leaf inside the tree has no state (its minCost would
            // read an unset field): refused
            require(t.tree[4 * i + 3] == leaves, "regular: leaves must be numbered left to right", PM_E_UNSUPPORTED);
            e.state = ++leaves;
        } else {
            require(e.a > i && e.a < t.nodes, "regular: bad child");
            require(!(e.type == T_OR || e.type == T_CAT) || (e.b > i && e.b < t.nodes), "regular: bad child");
        }
    }
    require(leaves == npos, "regular: the tree's leaves are not the automaton's positions");
    A.masks(0);
    A.arrows.assign(A.ms, Set{});
    A.rev.assign(A.ms, Set{});
    A.arrows[0] = A.nd[0].first;
    for (int s = 1; s < A.ms; ++s) A.follow(0, s, A.arrows[s]);
    A.final_ = A.nd[0].last;
    for (int s = 0; s < A.ms; ++s)
        for (int q = 0; q < A.ms; ++q)
            if (has(A.arrows[s], q)) put(A.rev[q], s);
    A.B.assign(256, Set{});
    for (int c = 0; c < 256; ++c) {
        const uint64_t* bp = B + (size_t)fold((uint8_t)c) * W;
        for (int p = 0; p < npos; ++p)
            if ((bp[p >> 6] >> (p & 63)) & 1) put(A.B[c], p + 1);
    }
    const int ntab = (A.ms + 15) / 16, Wd = (A.ms - 1 + ntab) / ntab;   // regularPreproc 0x40cb26
    for (int tb = 0; tb < ntab; ++tb)
        for (int b = tb * Wd; b < tb * Wd + Wd && b < A.ms; ++b)
            if ((b >> 6) == ((tb * Wd) >> 6)) put(A.vis, b);
    return A;
}

struct Costs {
    int L = 0;
    std::vector<int> dist;
    std::vector<double> C;       // [ms][L]
    std::vector<Set> M50, M70;   // [ms][L]
};

double min_cost(const Automaton& A, const Costs& c, int i, int ell, Set& win, Set& ini, Set& fin) {
    const Node& e = A.nd[i];
    switch (e.type) {
    case T_LEAF: {
        if (c.dist[e.state] < ell) return ell + 1.0;
        win = c.M70[(size_t)e.state * c.L + ell];
        ini = Set{};
        put(ini, e.state);
        fin = c.M50[(size_t)e.state * c.L + ell];
        return c.C[(size_t)e.state * c.L + ell];
    }
    case T_STAR:
    case T_OPT:
        return ell + 1.0;
    case T_PLUS:
        return min_cost(A, c, e.a, ell, win, ini, fin);
    case T_OR: {
        Set w2{}, i2{}, f2{};
        const double c1 = min_cost(A, c, e.a, ell, win, ini, fin);
        const double c2 = min_cost(A, c, e.b, ell, w2, i2, f2);
        join(win, w2);
        join(ini, i2);
        fin = f2;
        if (bits(win) > 64) {
            win = ini = fin = Set{};
            return ell + 1.0;
        }
        return std::max(c1, c2);
    }
    default: {
        Set w2{}, i2{}, f2{};
        const double c1 = min_cost(A, c, e.a, ell, win, ini, fin);
        const double c2 = min_cost(A, c, e.b, ell, w2, i2, f2);
        if (c2 >= c1) return c1;
        win = w2;
        ini = i2;
        fin = f2;
        return c2;
    }
    }
}

int det_class(const Automaton& A, int i, const Set& pos) {   // detClass 0x41ac90 / detClass1 0x418420
    const Node& e = A.nd[i];
    if (!meets(e.pm, pos)) return 1;
    if (e.type == T_LEAF) return 1;
    if (e.type == T_OR) return 3;
    if (e.type == T_CAT) return std::max(det_class(A, e.a, pos), det_class(A, e.b, pos));
    int r = det_class(A, e.a, pos);
    if (r == 1) r = 2;
    return A.nd[e.a].type == T_LEAF ? r : 3;
}

struct Plan {
    int type = 3, ell = 0, cls = 3;
    double best = 0.65;   // regularFindBest's return value (xmm0)
    Set win{}, winit{}, wfinal{};
};

Plan plan_of(const Automaton& A, int K = 0) {   // regularFindBest 0x40a500 (its cost C carries + K)
    const int ms = A.ms;
    Costs c;
    c.dist.assign(ms, 1);
    for (int i = 0; i < ms; ++i) {
        Set S{};
        put(S, i);
        while (!meets(S, A.final_) && c.dist[i] <= ms + 1) {
            ++c.dist[i];
            Set T{};
            for (int j = 0; j < ms; ++j)
                if (has(S, j)) join(T, A.arrows[j]);
            join(S, T);
        }
    }
    const int L = std::min(c.dist[0], 64);
    c.L = L;
    double lp[256];
    letter_probs(lp);
    std::vector<double> prob(ms, 0.0);
    for (int i = 0; i < ms; ++i)
        for (int ch = 0; ch < 256; ++ch)
            if (has(A.B[ch], i)) prob[i] += lp[ch];
    const size_t ML = (size_t)ms * L;
    std::vector<double> cost(ML, 0.0);
    c.M50.assign(ML, Set{});
    c.M70.assign(ML, Set{});
    for (int i = 0; i < ms; ++i) {
        cost[(size_t)i * L] = 1.0;
        if (L > 1) {
            cost[(size_t)i * L + 1] = prob[i];
            put(c.M50[(size_t)i * L + 1], i);
            put(c.M70[(size_t)i * L + 1], i);
        }
    }
    for (int l = 1; l + 1 < L; ++l)
        for (int i = 0; i < ms; ++i) {
            double s = 0.0;
            Set M{};
            for (int j = 0; j < ms; ++j)
                if (has(A.arrows[i], j)) {
                    s += cost[(size_t)j * L + l];
                    join(M, c.M50[(size_t)j * L + l]);
                }
            s *= prob[i];
            cost[(size_t)i * L + l + 1] = 1.0 < s ? 1.0 : s;
            c.M50[(size_t)i * L + l + 1] = M;
            c.M70[(size_t)i * L + l + 1] = c.M70[(size_t)i * L + l];
            join(c.M70[(size_t)i * L + l + 1], M);
        }
    std::vector<double> P((size_t)ms * L * L, 0.0);
    auto pi = [&](int i, int l, int a) -> double& { return P[((size_t)i * L + l) * L + a]; };
    for (int i = 0; i < ms; ++i)
        for (int l = 0; l < L; ++l) pi(i, l, 0) = 1.0;
    for (int l = 1; l < L; ++l)
        for (int a = 1; a <= l; ++a)
            for (int i = 0; i < ms; ++i) {
                double v = cost[(size_t)i * L + a];
                if (a < l)
                    for (int j = 0; j < ms; ++j)
                        if (has(A.arrows[i], j)) v = 1.0 - (1.0 - v) * (1.0 - pi(j, l - 1, a));
                pi(i, l, a) = v;
            }
    c.C.assign(ML, 0.0);
    for (int i = 0; i < ms; ++i)
        for (int l = 0; l < L; ++l) {
            double s = (double)K;
            for (int a = 0; a <= l; ++a) s += pi(i, l, a);
            c.C[(size_t)i * L + l] = s;
        }
    Plan p;
    double best = 0.65;
    int ell = L - 1;
    if (ell > 0 && !(1.0 >= 0.65 * ell)) {
        for (;;) {
            Set w{}, in{}, fi{};
            const double cc = min_cost(A, c, 0, ell, w, in, fi);
            if (ell + 1.0 > cc) {
                const double r = cc / ((double)ell - cc + 1.0);
                if (best > r) {
                    best = r;
                    p.win = w;
                    p.winit = in;
                    p.wfinal = fi;
                    p.ell = ell;
                }
            }
            if (--ell == 0 || 1.0 >= best * ell) break;
        }
    }
    p.best = best;
    if (0.65 > best) {
        p.type = 2;
    } else {
        p.type = 3;
        p.ell = 0;
        p.win = p.winit = Set{};
        put(p.winit, 0);
        if (ms <= 64) {
            for (int s = 0; s < ms; ++s) put(p.win, s);
            p.wfinal = A.final_;
        } else {   // 0x40b175: breadth-first layers while at most 64 states are reached
            Set reach = p.winit, layer{};
            while (bits(reach) <= 64) {
                for (int q = 0; q < RG_NW; ++q) layer[q] = reach[q] & ~p.win[q];
                join(p.win, reach);
                reach = Set{};
                for (int s = 0; s < ms; ++s)
                    if (has(p.win, s)) join(reach, A.arrows[s]);
            }
            p.wfinal = layer;
            join(p.wfinal, A.final_);
            for (int q = 0; q < RG_NW; ++q) p.wfinal[q] &= p.win[q];
        }
    }
    p.cls = det_class(A, 0, p.win);
    return p;
}

int window_states(const Plan& p, int ms) {
    int mp = 1;
    for (int s = 1; s < ms; ++s) mp += has(p.win, s);
    return mp;
}

// ---------------------------------------------------------------------------
// eregular (k > 0): eregularPreproc 0x406a20
// ---------------------------------------------------------------------------

// eregularPreproc's successor sets (over the arrows, exact)
inline Set reach_of(const Automaton& A, const Set& d) {
    Set r{};
    for (int s = 0; s < A.ms; ++s)
        if (has(d, s)) join(r, A.arrows[s]);
    return r;
}

struct EPlan {
    int etype = 3, ell = 0, cls = 3, npieces = 1;
    bool pieces_computed = false, defined = true;
    Set pwin[PM_MAX_K + 1] = {}, pini[PM_MAX_K + 1] = {}, pfin[PM_MAX_K + 1] = {};
    int first[PM_MAX_K + 1] = {};
    uint64_t match0 = 0;   // class 1: P->0x28
};

// fwdCheck / bwdCheck's transition tables (regularMakeDet 0x40bfc0 in slices
// of W = ceil(m / ceil(m / 16)) states, OptDetWidth .data 0x621920): table t
// holds the states t W + b, but the checks index it by SLICE(D, off, W)
// (0x41b8e0, one word) with off moving on by W or, when the next slice would
// cross a word, to the next word (0x403530).  src[q] = the state whose
// transitions state q takes, -1 when no slice reads q (identity for m <=
// 64).  False when a slice would read past the set's words.
bool slice_map(int m, std::vector<int>& src) {
    const int nt0 = (m + 16 - 1) / 16, W = (m + nt0 - 1) / nt0, ntab = (m + W - 1) / W;
    src.assign(64 * RG_NW, -1);
    int off = 0;
    for (int t = 0; t < ntab; ++t) {
        if ((off >> 6) >= (m + 63) / 64 || (off >> 6) >= RG_NW) return false;
        for (int b = 0; b < W; ++b) {
            const int q = off + b, from = t * W + b;
            if ((q >> 6) == (off >> 6) && from < m && q < 64 * RG_NW) src[q] = from;
        }
        off += W;
        if (((off + W - 1) >> 6) != (off >> 6)) off = (off & ~63) + 64;
    }
    return true;
}

// regularFindBest with K, the breadth-first levels, the piece DP against
// 0.78 and (K + 1) 1.3 fb, detClass of windows[0] (oracle/pm_nrgrep_reg.c
// eplan; transpositions off, PatMatch's letters are i/d/s)
EPlan eplan_of(const Automaton& A, int K) {
    require(K >= 1 && K <= PM_MAX_K, "eregular: k out of range");
    {
        std::vector<int> src;
        require(slice_map(A.ms, src), "eregular: a transition table slice past the state set", PM_E_UNSUPPORTED);
    }
    const Plan fb = plan_of(A, K);
    const int m = A.ms, transp = 0;
    Set seen{};
    seen[0] = 1;
    int nlev = 1;
    while (!meets(seen, A.final_)) {   // 0x406db8
        ++nlev;
        join(seen, reach_of(A, seen));
        require(nlev <= m + 2, "eregular: no final state reachable");
    }
    const int minlen = nlev - 1;
    std::vector<Set> lev(nlev + 1, Set{});
    lev[0][0] = 1;
    seen = Set{};
    seen[0] = 1;
    for (int i = 1; i <= minlen; ++i) {   // 0x406f69
        const Set succ = reach_of(A, seen);
        for (int q = 0; q < RG_NW; ++q) lev[i][q] = succ[q] & ~seen[q];
        join(seen, succ);
    }
    int pl0 = minlen - K * transp;   // 0x406e54
    if ((unsigned)pl0 > 64u) pl0 = 64;
    pl0 = pl0 / (K + 1);
    const int PL1 = pl0 + 1;
    double best = 0.78;
    int chosen = 0;
    Set pieces[PM_MAX_K + 1] = {};
    if (PL1 > 1 && pl0 != 1 && !(1.0 / (double)pl0 > 0.78)) {
        double lp[256];
        letter_probs(lp);
        std::vector<double> prob(m, 0.0);
        for (int i = 0; i < m; ++i)
            for (int c = 0; c < 256; ++c)
                if (has(A.B[c], i)) prob[i] += lp[c];
        std::vector<double> Av((size_t)m * PL1, 0.0);
        for (int i = 0; i < m; ++i) {
            Av[(size_t)i * PL1] = 1.0;
            Av[(size_t)i * PL1 + 1] = prob[i];
        }
        for (int l = 2; l < PL1; ++l)   // 0x407118
            for (int i = 0; i < m; ++i) {
                double sum = 0.0;
                for (int j = 0; j < m; ++j)
                    if (has(A.arrows[i], j)) sum += Av[(size_t)j * PL1 + l - 1];
                sum *= prob[i];
                Av[(size_t)i * PL1 + l] = 1.0 < sum ? 1.0 : sum;
            }
        std::vector<double> Bt((size_t)m * PL1 * PL1, 0.0);
        auto bt = [&](int i, int l, int a) -> double& { return Bt[((size_t)i * PL1 + l) * PL1 + a]; };
        for (int i = 0; i < m; ++i)
            for (int l = 0; l < PL1; ++l) bt(i, l, 0) = 1.0;
        for (int l = 1; l < PL1; ++l)   // 0x4072a0
            for (int a = 1; a <= l; ++a)
                for (int i = 0; i < m; ++i) {
                    double v = Av[(size_t)i * PL1 + a];
                    if (a < l)
                        for (int j = 0; j < m; ++j)
                            if (has(A.arrows[i], j)) v = 1.0 - (1.0 - v) * (1.0 - bt(j, l - 1, a));
                    bt(i, l, a) = v;
                }
        std::vector<double> C((size_t)nlev * PL1, 0.0);
        for (int lv = 0; lv < nlev; ++lv)   // 0x40742d
            for (int l = 0; l < PL1; ++l) {
                double sum = 1.0;
                for (int i = 0; i < m; ++i)
                    if (has(lev[lv], i) && l != 0)
                        for (int a = 1; a <= l; ++a) sum += bt(i, l, a);
                C[(size_t)lv * PL1 + l] = sum;
            }
        const int W2 = K + 2;
        std::vector<double> D((size_t)(nlev + 1) * W2, 0.0);
        std::vector<int> E((size_t)(nlev + 1) * W2, 0);
        for (int pl = pl0;;) {   // 0x40772e
            for (int r = 1; r <= nlev; ++r) D[(size_t)r * W2] = 0.0;
            for (int c = 1, esi = nlev - pl; c <= K + 1; ++c, esi -= pl + transp)
                for (int r = (esi < 0 ? 0 : esi) + 1; r <= nlev; ++r) D[(size_t)r * W2 + c] = 1.0;
            for (int c = 1; c <= K + 1; ++c) {   // 0x407850
                const int r11 = nlev - pl - (c - 1) * (pl + transp);
                for (int r = r11; r >= 1; --r) {
                    double v = C[(size_t)r * PL1 + pl];
                    if ((double)(pl + 1) > v) {
                        v = v / ((double)pl - v + 1.0);
                        v = 1.0 < v ? 1.0 : v;
                    } else {
                        v = 1.0;
                    }
                    if (c > 1) v = 1.0 - (1.0 - v) * (1.0 - D[(size_t)(r + pl + transp) * W2 + c - 1]);
                    E[(size_t)r * W2 + c] = r;
                    const double y = D[(size_t)(r + 1) * W2 + c];
                    if (v > y) {
                        v = y;
                        E[(size_t)r * W2 + c] = E[(size_t)(r + 1) * W2 + c];
                    }
                    D[(size_t)r * W2 + c] = v;
                }
            }
            if (best > D[W2 + K + 1]) {   // 0x407a0b
                int r = 1;
                for (int i = 0, c = K + 1; c >= 1; ++i, --c) {
                    const int st = E[(size_t)r * W2 + c];
                    pieces[i] = lev[st];
                    r = st + pl + transp;
                }
                best = D[W2 + K + 1];
                chosen = pl;
            }
            if (--pl == 1) break;
            if (!(1.0 / (double)pl <= best)) break;
        }
    }
    EPlan e;
    bool use_pieces = false;
    if (best < 0.78) {   // 0x4082c9
        e.pieces_computed = true;
        for (int i = 0; i <= K; ++i) {
            Set w = pieces[i], last{};
            for (int st = 0; st < chosen; ++st) {
                last = reach_of(A, w);
                join(w, last);
            }
            e.pwin[i] = w;
            e.pini[i] = pieces[i];
            e.pfin[i] = last;
        }
        use_pieces = !(best >= (double)(K + 1) * 1.3 * fb.best) && chosen != 0;   // 0x40842a
    }
    if (use_pieces) {
        e.etype = 1;
        e.ell = chosen;
        e.npieces = K + 1;
    } else {   // 0x407bb9
        e.etype = fb.ell == 0 ? 3 : 2;
        e.ell = fb.ell;
        e.npieces = 1;
        e.pwin[0] = fb.win;
        e.pini[0] = fb.winit;
        e.pfin[0] = fb.wfinal;
    }
    e.cls = det_class(A, 0, e.pwin[0]);
    if (e.cls == 1) {   // 0x407e4b: the first state of each window (windows[1 .. K] unset for a window plan)
        const int nw = (e.etype == 1 || e.pieces_computed) ? K + 1 : 1;
        e.defined = nw == K + 1;
        for (int i = 0; i < nw; ++i) {
            int f = 0;
            while (f < m && !has(e.pwin[i], f)) ++f;
            e.first[i] = f;
            if (e.ell != 0) {   // shl %cl: the count mod 64 (0x407ef0)
                e.match0 |= 1ull << (f & 63);
            } else {
                int r = f + 1;
                while (r < m && has(e.pwin[i], r)) ++r;
                e.match0 |= 1ull << (r & 63);
            }
        }
    }
    return e;
}

// The window automaton's tables (regularRemapStates 0x40bab0 +
// regularLoadFast 0x40c4f0): window states 1.. in state order, 0 the virtual
// initial one; backward (ell > 0): reversed, every state initial; forward:
// state 0 loops on every byte.
void window_tables(const Automaton& A, const Set& win, const Set& winit, const Set& wfinal, int ell, RgSlot& S,
                   std::vector<uint64_t>& tab, bool eregular) {
    const int ms = A.ms;
    int mp = 1;
    for (int q = 1; q < ms; ++q) mp += has(win, q);
    require(mp <= 64, "regular: a window of more than 64 states", PM_E_UNSUPPORTED);
    S.mp = mp;
    std::vector<int> map(ms, 0);
    int k = 0;
    for (int q = 1; q < ms; ++q)
        if (has(win, q)) map[q] = ++k;
    for (int i = 0; i < 64; ++i) S.unmap[i] = eregular ? -1 : 0;
    for (int q = 0; q < ms; ++q)
        if (has(win, q)) S.unmap[map[q]] = q;
    uint64_t* fw = tab.data() + S.o_fw;
    for (int q = 0; q < ms; ++q)
        if (has(winit, q)) fw[0] |= 1ull << map[q];
    for (int q = 0; q < ms; ++q)
        if (has(win, q))
            for (int t = 0; t < ms; ++t)
                if (has(win, t) && has(A.arrows[q], t)) fw[map[q]] |= 1ull << map[t];
    uint64_t fin = 0;
    for (int q = 0; q < ms; ++q)
        if (has(wfinal, q)) fin |= 1ull << map[q];
    uint64_t* Bw = tab.data() + S.o_Bw;
    for (int c = 0; c < 256; ++c)
        for (int q = 0; q < ms; ++q)
            if (has(win, q) && has(A.B[c], q)) Bw[c] |= 1ull << map[q];
    const uint64_t all = mp >= 64 ? ~0ull : (1ull << mp) - 1;
    if (ell > 0) {   // regularLoadFast 0x40c5dd: reversed, every state initial
        uint64_t* rw = tab.data() + S.o_rw;
        for (int a = 0; a < mp; ++a)
            for (int b = 0; b < mp; ++b)
                if ((fw[a] >> b) & 1) rw[b] |= 1ull << a;
        S.finit = all;
        S.ffinal = 1;
        uint64_t* Av = tab.data() + S.o_A;
        for (int c = 0; c < 256; ++c) {
            const uint64_t d = all & Bw[c];
            for (int q = 0; q < mp; ++q)
                if ((d >> q) & 1) Av[c] |= rw[q];
        }
    } else {         // 0x40c771: state 0 loops on every byte
        fw[0] |= 1;
        for (int c = 0; c < 256; ++c) Bw[c] |= 1;
        S.finit = 1;
        S.ffinal = fin;
    }
}

}  // namespace

bool rg_build(const RgTree& t, const uint64_t* B, int W, int npos, int64_t max_len, int k, int errs, uint32_t flags,
              int32_t pid, Upload& up, size_t& o_slot, size_t& o_tab) {
    const Automaton A = make_automaton(t, B, W, npos);
    const int ms = A.ms;
    RgSlot S{};
    S.ms = ms;
    S.anchors = (int32_t)(flags & (PM_ANCHOR_START | PM_ANCHOR_END));
    S.pid = pid;
    S.k = k;
    S.errs = errs;
    std::vector<uint64_t> tab;
    auto take = [&](size_t words) {
        const uint64_t o = tab.size();
        tab.resize(tab.size() + words, 0);
        return o;
    };
    if (k > 0) {
        const EPlan E = eplan_of(A, k);
        // class 2: eregularPreproc stores through a null pointer (0x4081ed),
        // nrgrep_coords dies before the scan: nothing prints
        if (E.cls == 2) return false;
        const int nw = ms <= 64 ? 1 : RG_NW;
        S.nw = nw;
        S.type = E.etype;
        S.ell = E.ell;
        S.cls = E.cls;
        S.match0 = E.match0;
        for (int i = 0; i <= PM_MAX_K; ++i) S.first[i] = E.first[i];
        // a match covers at most max_len + k characters (insertions); the
        // walk replays from span + 4 before a cluster, clusters break at
        // 2 span + 4 or at a line break
        S.max_len = max_len < 0 ? -1 : max_len + k;
        S.gap = max_len < 0 ? -1 : 2 * S.max_len + 4;
        S.lines = 1;
        for (int q = 0; q < RG_NW; ++q) S.final_[q] = A.final_[q];
        S.o_arr = take((size_t)ms * nw);
        S.o_rev = take((size_t)ms * nw);
        S.o_B = take((size_t)256 * nw);
        S.o_Bw = take(256);
        S.o_A = take(256);
        S.o_fw = take(64);
        S.o_rw = take(64);
        S.o_T0 = take(256);
        S.o_T2 = take(256);
        // fwdCheck / bwdCheck's transitions with the slice layout baked in:
        // row q = the arrows of the state whose table slot q's bit indexes
        // (slice_map; the identity up to 64 states)
        std::vector<int> src;
        require(slice_map(ms, src), "eregular: a transition table slice past the state set", PM_E_UNSUPPORTED);
        for (int q = 0; q < ms; ++q)
            if (src[q] >= 0)
                for (int w = 0; w < nw; ++w) {
                    tab[S.o_arr + (size_t)q * nw + w] = A.arrows[src[q]][w];
                    tab[S.o_rev + (size_t)q * nw + w] = A.rev[src[q]][w];
                }
        for (int c = 0; c < 256; ++c)
            for (int w = 0; w < nw; ++w) tab[S.o_B + (size_t)c * nw + w] = A.B[c][w];
        if (E.cls == 3) {   // eregularLoadFast 0x406860: the union of the windows
            Set uw{}, ui{}, uf{};
            for (int i = 0; i < E.npieces; ++i) {
                join(uw, E.pwin[i]);
                join(ui, E.pini[i]);
                join(uf, E.pfin[i]);
            }
            window_tables(A, uw, ui, uf, E.ell, S, tab, true);
            S.nstates = S.mp;
        } else {            // esimpleLoadFast 0x415370 over the states first[r] ..
            // P->0x858 is the identity over every state (0x407f67): the
            // walk takes state i for slot i (no unmap beyond 64 states)
            S.nstates = ms;
            S.mp = ms;
            for (int i = 0; i < 64; ++i) S.unmap[i] = i < ms ? i : -1;
            uint64_t* T0 = tab.data() + S.o_T0;
            uint64_t* T2 = tab.data() + S.o_T2;
            for (int c = 0; c < 256; ++c) {
                if (E.etype == 1) {   // 0x4153fa: the pieces, bit r * pl + pp (ISSET: every state)
                    for (int r = 0; r <= k; ++r)
                        for (int pp = 0; pp < E.ell; ++pp) {
                            const int st = E.first[r] + E.ell - 1 - pp;
                            if (st < ms && has(A.B[c], st)) {
                                const uint64_t bit = 1ull << (r * E.ell + pp);
                                T0[c] |= bit;
                                if (pp > 0) T2[c] |= bit;
                            }
                        }
                } else {              // simpleLoadFast 0x417561: the window backward
                    for (int r = 0; r < E.ell; ++r) {
                        const int st = E.first[0] + E.ell - 1 - r;
                        if (st < ms && has(A.B[c], st)) T0[c] |= 1ull << (64 - E.ell + r);
                    }
                }
            }
        }
        o_slot = up.add(&S, sizeof(S));
        o_tab = up.add(tab.data(), tab.size() * 8);
        return true;
    }
    const Plan P = plan_of(A);
    if (P.cls != 3) return false;   // simpleScan / extendedScan never leave P->match set: nothing prints
    S.nw = ms <= 64 ? 1 : RG_NW;
    S.type = P.type;
    S.ell = P.ell;
    S.cls = 3;
    // bounded clusters unless the pattern is unbounded or the forward
    // window's final states are not the automaton's (more than 64 states)
    S.max_len = (max_len < 0 || (P.type == 3 && ms > 64)) ? -1 : max_len;
    S.gap = S.max_len < 0 ? -1 : 2 * S.max_len + 2;
    for (int q = 0; q < RG_NW; ++q) {
        S.final_[q] = A.final_[q];
        S.vis[q] = A.vis[q];
    }
    const int nw = S.nw;
    S.o_arr = take((size_t)ms * nw);
    S.o_rev = take((size_t)ms * nw);
    S.o_B = take((size_t)256 * nw);
    S.o_Bw = take(256);
    S.o_A = take(256);
    S.o_fw = take(64);
    S.o_rw = take(64);
    for (int s = 0; s < ms; ++s)
        for (int q = 0; q < nw; ++q) {
            tab[S.o_arr + (size_t)s * nw + q] = A.arrows[s][q];
            tab[S.o_rev + (size_t)s * nw + q] = A.rev[s][q];
        }
    for (int c = 0; c < 256; ++c)
        for (int q = 0; q < nw; ++q) tab[S.o_B + (size_t)c * nw + q] = A.B[c][q];
    window_tables(A, P.win, P.winit, P.wfinal, P.type == 2 ? P.ell : 0, S, tab, false);
    o_slot = up.add(&S, sizeof(S));
    o_tab = up.add(tab.data(), tab.size() * 8);
    return true;
}

// ---------------------------------------------------------------------------
// device: the per-cluster replay
// ---------------------------------------------------------------------------
namespace {

constexpr uint64_t RG_POS_MASK = (1ull << 48) - 1;
constexpr uint64_t RG_SCAN = 1ull << 16;   // lines mode: how far a head looks back for a line break
constexpr uint32_t RG_T = 256;
constexpr uint64_t RG_NONE = ~0ull;

__global__ __launch_bounds__(RG_T) void k_rg_heads(XtPrep X, const uint64_t* __restrict__ keys, const uint64_t* total_d,
                                                   uint64_t total_h, uint8_t* __restrict__ acc, TextView tv) {
    const uint64_t total = total_d ? *total_d : total_h;
    const RgSlot& S = *X.rg;
    for (uint64_t i = blockIdx.x * (uint64_t)RG_T + threadIdx.x; i < total; i += (uint64_t)gridDim.x * RG_T) {
        bool head = i == 0 || (keys[i] >> 48) != (keys[i - 1] >> 48);
        if (!head) {
            const uint64_t a = keys[i - 1] & RG_POS_MASK, b = keys[i] & RG_POS_MASK;
            if (xt_region(tv, a) != xt_region(tv, b)) head = true;
            else if (S.gap >= 0 && b - a > (uint64_t)S.gap) head = true;
            // (a break at a itself: every position is a key when deletions
            // can empty the pattern)
            else if (S.gap < 0 || S.lines) head = xt_brk(tv, a) || xt_brk_between(tv, a, b, RG_SCAN);
        }
        acc[i] = head ? 2 : 0;
    }
}

template <int NW>
struct RgWalk {
    const RgSlot* S;
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
    // recGetRecord 0x402030 (rp non-decreasing over a walk)
    __device__ void record(uint64_t rp, uint64_t& rb, uint64_t& re) {
        while (nl_hi < rp) {
            nl_lo = nl_hi;
            nl_hi = next_nl(nl_hi + 1);
        }
        rb = (nl_lo != ~0ull && nl_lo >= R) ? nl_lo + 1 : R;
        re = nl_hi;
    }
    __device__ bool left_ok(uint64_t p, uint64_t lim) const {
        return !((S->anchors & PM_ANCHOR_START) && p > lim && at(p - 1) != (uint8_t)'\n');
    }
    __device__ bool right_ok(uint64_t q, uint64_t lim) const {
        return !((S->anchors & PM_ANCHOR_END) && q < lim && at(q) != (uint8_t)'\n');
    }
    // one step of the whole automaton over the states SLICE sees
    __device__ void step(const uint64_t (&D)[NW], const uint64_t* tr, uint64_t (&T)[NW]) const {
#pragma unroll
        for (int q = 0; q < NW; ++q) T[q] = 0;
#pragma unroll
        for (int q = 0; q < NW; ++q) {
            uint64_t b = D[q] & S->vis[q];
            while (b) {
                const int s = 64 * q + __builtin_ctzll(b);
                b &= b - 1;
                const uint64_t* row = tr + (size_t)s * NW;
#pragma unroll
                for (int w = 0; w < NW; ++w) T[w] |= row[w];
            }
        }
    }
    // fwdCheck 0x408bc0: the shortest end from state s reading t[p]
    __device__ uint64_t fwd(uint64_t p, uint64_t lim, int s) const {
        uint64_t D[NW], T[NW];
#pragma unroll
        for (int q = 0; q < NW; ++q) D[q] = q == (s >> 6) ? 1ull << (s & 63) : 0ull;
        const uint64_t* B = tab + S->o_B;
        for (;;) {
            uint64_t hit = 0;
#pragma unroll
            for (int q = 0; q < NW; ++q) hit |= D[q] & S->final_[q];
            if (hit && right_ok(p + 1, lim + 1)) return p;
            if (p == lim) return RG_NONE;
            step(D, tab + S->o_arr, T);
            ++p;
            const uint64_t* b = B + (size_t)at(p) * NW;
            uint64_t any = 0;
#pragma unroll
            for (int q = 0; q < NW; ++q) {
                D[q] = T[q] & b[q];
                any |= D[q];
            }
            if (!any) return RG_NONE;
        }
    }
    // bwdCheck 0x408d50: the nearest start, state s reading t[p - 1]
    __device__ uint64_t bwd(uint64_t p, uint64_t lim, int s) const {
        uint64_t D[NW], T[NW];
#pragma unroll
        for (int q = 0; q < NW; ++q) D[q] = q == (s >> 6) ? 1ull << (s & 63) : 0ull;
        const uint64_t* B = tab + S->o_B;
        for (;;) {
            if ((D[0] & 1) && left_ok(p, lim)) return p;
            if (p == lim) return RG_NONE;
            --p;
            const uint64_t* b = B + (size_t)at(p) * NW;
#pragma unroll
            for (int q = 0; q < NW; ++q) D[q] &= b[q];
            step(D, tab + S->o_rev, T);
            uint64_t any = 0;
#pragma unroll
            for (int q = 0; q < NW; ++q) {
                D[q] = T[q];
                any |= T[q];
            }
            if (!any) return RG_NONE;
        }
    }
    // checkMatch 0x408ec0: the states of `match` in state order
    __device__ bool check(uint64_t pos, uint64_t match, uint64_t& mb, uint64_t& me) {
        if (S->type == 3 && pos == 0) return false;
        const uint64_t rp = S->type == 3 ? pos - 1 : pos;
        uint64_t rb, re;
        record(rp, rb, re);
        if (rp < rb || rp >= re) return false;
        const uint64_t lim = S->mp >= 64 ? ~0ull : (1ull << S->mp) - 1;
        match &= lim;
        while (match) {
            const int i = __builtin_ctzll(match);
            match &= match - 1;
            const int s = S->unmap[i];
            uint64_t st, en;
            if (S->type == 3) {
                st = bwd(pos, rb, s);
                if (st == RG_NONE) continue;
                en = fwd(pos - 1, re - 1, s);
                if (en == RG_NONE) continue;
            } else {
                en = fwd(pos, re - 1, s);
                if (en == RG_NONE) continue;
                st = bwd(pos + 1, rb, s);
                if (st == RG_NONE) continue;
            }
            mb = st;
            me = en + 1;
            return true;
        }
        return false;
    }
    __device__ static uint64_t wtrans(const uint64_t* tb, uint64_t d) {
        uint64_t r = 0;
        while (d) {
            r |= tb[__builtin_ctzll(d)];
            d &= d - 1;
        }
        return r;
    }
    // regularScan 0x4091d0 from R; false when no candidate <= stop verifies
    __device__ bool scan(uint64_t stop, uint64_t& mb, uint64_t& me) {
        const uint64_t* Bw = tab + S->o_Bw;
        if (S->type == 2) {   // backward windows (0x40921c)
            const uint64_t ell = (uint64_t)S->ell;
            const uint64_t* A = tab + S->o_A;
            const uint64_t* rw = tab + S->o_rw;
            uint64_t ws = R;
            while (ws + ell <= n) {
                if (ws > stop) return false;
                uint64_t rsi = A[at(ws + ell - 1)];
                if (!rsi) {
                    ws += ell;
                    continue;
                }
                uint64_t D = 0;
                bool dead = false;
                for (uint64_t e = ell - 1; e > 0; --e) {   // positions ws + ell - 2 .. ws
                    const uint64_t c = ws + e - 1;
                    D = rsi & Bw[at(c)];
                    rsi = wtrans(rw, D);
                    if (!rsi) {
                        ws = c + 1;
                        dead = true;
                        break;
                    }
                }
                if (dead) continue;
                if ((rsi & S->ffinal) && check(ws, D, mb, me)) return true;
                ++ws;
            }
            return false;
        }
        const uint64_t* fw = tab + S->o_fw;   // forward (0x409500)
        uint64_t p = R, D = S->finit;
        if (p < n && (D & S->ffinal) && check(p, D & S->ffinal, mb, me)) return true;
        while (p < n) {
            if (p >= stop) return false;   // the next candidate p + 1 is past it
            const uint8_t c = at(p++);
            if (c == (uint8_t)'\n') {
                if (p >= n) return false;
                D = S->finit;
            } else {
                D = wtrans(fw, D) & Bw[c];
                if (p == n) return false;
            }
            const uint64_t f = D & S->ffinal;
            if (f && check(p, f, mb, me)) return true;
        }
        return false;
    }
};

// A state set of the eregular verify: NW words (1 up to 64 states, RG_NW
// beyond)
template <int NW>
struct WS {
    uint64_t w[NW];
};
template <int NW>
__device__ __forceinline__ WS<NW> ws_zero() {
    WS<NW> r;
#pragma unroll
    for (int q = 0; q < NW; ++q) r.w[q] = 0;
    return r;
}
template <int NW>
__device__ __forceinline__ WS<NW> ws_bit(int s) {
    WS<NW> r;
#pragma unroll
    for (int q = 0; q < NW; ++q) r.w[q] = q == (s >> 6) ? 1ull << (s & 63) : 0ull;
    return r;
}
template <int NW>
__device__ __forceinline__ WS<NW> ws_or(const WS<NW>& a, const WS<NW>& b) {
    WS<NW> r;
#pragma unroll
    for (int q = 0; q < NW; ++q) r.w[q] = a.w[q] | b.w[q];
    return r;
}
template <int NW>
__device__ __forceinline__ WS<NW> ws_and(const WS<NW>& a, const WS<NW>& b) {
    WS<NW> r;
#pragma unroll
    for (int q = 0; q < NW; ++q) r.w[q] = a.w[q] & b.w[q];
    return r;
}
template <int NW>
__device__ __forceinline__ bool ws_meets(const WS<NW>& a, const WS<NW>& b) {
    uint64_t x = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) x |= a.w[q] & b.w[q];
    return x != 0;
}
template <int NW>
__device__ __forceinline__ bool ws_any(const WS<NW>& a) {
    uint64_t x = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) x |= a.w[q];
    return x != 0;
}
template <int NW>
__device__ __forceinline__ WS<NW> ws_load(const uint64_t* p) {
    WS<NW> r;
#pragma unroll
    for (int q = 0; q < NW; ++q) r.w[q] = p[q];
    return r;
}

// eregular (k > 0): the scanners and checkMatch of oracle/pm_nrgrep_reg.c
// over the cluster's text.  The scanners run over one word (the window
// remapped, or esimple's piece bits); checkMatch's rows hold NW words, their
// transitions through the tables rg_build baked the slice layout into
// (slice_map: fwdCheck / bwdCheck's regularMakeDet tables indexed by SLICE)
template <int KR, int SC, int NW>
struct ErgWalk {
    const RgSlot* S;
    const uint64_t* tab;
    TextView tv;
    uint64_t n;        // the region end
    uint64_t R;
    uint64_t nl_lo, nl_hi;

    mutable TxtCache tc;   // the thread's text window (LDS)

    // SC is the scanner (erg_scanner: a kernel holds one scanner and one
    // inlined checkMatch); KR the row count the kernel was built for: k
    // itself for k <= 3 (row loops unroll, the rows stay in registers),
    // PM_MAX_K otherwise (loops bounded by the run-time k)
    __device__ __forceinline__ int kk() const { return KR < PM_MAX_K ? KR : S->k; }
    template <int N>
    __device__ __forceinline__ static uint64_t pick(const uint64_t (&a)[N], int i) {
        uint64_t v = 0;
#pragma unroll
        for (int j = 0; j < N; ++j)
            if (j == i) v = a[j];
        return v;
    }

    __device__ uint8_t at(uint64_t p) const { return tc.get(tv, p); }
    __device__ uint64_t next_nl(uint64_t p) const { return xt_next_nl(tv, p, n); }
    __device__ void record(uint64_t rp, uint64_t& rb, uint64_t& re) {   // recGetRecord 0x402030
        while (nl_hi < rp) {
            nl_lo = nl_hi;
            nl_hi = next_nl(nl_hi + 1);
        }
        rb = (nl_lo != ~0ull && nl_lo >= R) ? nl_lo + 1 : R;
        re = nl_hi;
    }
    __device__ bool left_ok(uint64_t p, uint64_t lim) const {
        return !((S->anchors & PM_ANCHOR_START) && p > lim && at(p - 1) != (uint8_t)'\n');
    }
    __device__ bool right_ok(uint64_t q, uint64_t lim) const {
        return !((S->anchors & PM_ANCHOR_END) && q < lim && at(q) != (uint8_t)'\n');
    }
    // the window scanners' one-word transitions
    __device__ static uint64_t tr(const uint64_t* tb, uint64_t d) {
        uint64_t r = 0;
        while (d) {
            r |= tb[__builtin_ctzll(d)];
            d &= d - 1;
        }
        return r;
    }
    // checkMatch's transitions: row q of tb (NW words) for every state q of d
    __device__ static WS<NW> trn(const uint64_t* tb, const WS<NW>& d) {
        WS<NW> r = ws_zero<NW>();
#pragma unroll
        for (int q = 0; q < NW; ++q) {
            uint64_t x = d.w[q];
            while (x) {
                const uint64_t* row = tb + (size_t)(q * 64 + __builtin_ctzll(x)) * NW;
                x &= x - 1;
#pragma unroll
                for (int w = 0; w < NW; ++w) r.w[w] |= row[w];
            }
        }
        return r;
    }
    __device__ WS<NW> bmask(uint64_t p) const { return ws_load<NW>(tab + S->o_B + (size_t)at(p) * NW); }
    // fwdCheck 0x403310: from state s (it read t[p]) forward; kio: budget in,
    // errors used out
    __device__ uint64_t efwd(uint64_t p, uint64_t lim, int s, int& kio) const {
        const int K = kio, ins = S->errs & PM_ERR_INS, del = S->errs & PM_ERR_DEL, sub = S->errs & PM_ERR_SUB;
        const uint64_t* arr = tab + S->o_arr;
        WS<NW> F;
#pragma unroll
        for (int q = 0; q < NW; ++q) F.w[q] = S->final_[q];
        WS<NW> rows[KR + 1];
        rows[0] = ws_bit<NW>(s);
        if (ws_meets(rows[0], F)) {   // 0x40339d: insertions up to the right context
            kio = 0;
            for (uint64_t q = p + 1;; ++q) {
                if (right_ok(q, lim + 1)) return q - 1;
                if (q == lim + 1 || !ins) return RG_NONE;
                if (++kio > K) return RG_NONE;
            }
        }
        int kmax = K;
        uint64_t best = RG_NONE;
#pragma unroll
        for (int j = 1; j <= KR; ++j) {   // 0x4034c0 (rows left unset without OptDel: row 0)
            if (j > kmax) break;
            rows[j] = del ? ws_or(rows[j - 1], trn(arr, rows[j - 1])) : rows[j - 1];
            if (del && ws_meets(rows[j], F) && right_ok(p + 1, lim + 1)) {
                kio = j;
                kmax = j - 1;
                best = p;
            }
        }
        if (p == lim) return best;
        for (uint64_t cur = p;;) {
            ++cur;
            const WS<NW> bc = bmask(cur);
            const WS<NW> n0 = ws_and(trn(arr, rows[0]), bc);
            if (ws_meets(n0, F) && right_ok(cur + 1, lim + 1)) {
                kio = 0;
                return cur;
            }
            WS<NW> oldp = rows[0], last = n0;
            rows[0] = n0;
#pragma unroll
            for (int j = 1; j <= KR; ++j) {   // 0x4037a0
                if (j > kmax) break;
                WS<NW> v = del ? trn(arr, last) : ws_zero<NW>();
                if (ins) v = ws_or(v, oldp);
                if (sub) v = ws_or(v, trn(arr, oldp));
                v = ws_or(v, ws_and(trn(arr, rows[j]), bc));
                const WS<NW> oj = rows[j];
                rows[j] = v;
                last = v;
                if (ws_meets(v, F) && right_ok(cur + 1, lim + 1)) {   // 0x403a01: the fewest errors
                    int c = j;
#pragma unroll
                    for (int d = KR - 1; d >= 0; --d)   // while rows[c - 1] is final: --c
                        if (d == c - 1 && ws_meets(rows[d], F)) c = d;
                    if (c == 0) {
                        kio = 0;
                        return cur;
                    }
                    kio = c;
                    kmax = c - 1;
                    best = cur;
                    break;
                }
                oldp = oj;
            }
            if (!ws_any(last) || cur == lim) return best;
        }
    }
    // bwdCheck 0x403df0: from state s (it reads t[p - 1]) backward
    __device__ uint64_t ebwd(uint64_t p, uint64_t lim, int s, int& kio) const {
        const int K = kio, ins = S->errs & PM_ERR_INS, del = S->errs & PM_ERR_DEL, sub = S->errs & PM_ERR_SUB;
        const uint64_t* rev = tab + S->o_rev;
        WS<NW> rows[KR + 1];
        rows[0] = ws_bit<NW>(s);
        if (rows[0].w[0] & 1) {   // 0x403e71: insertions down to the left context
            kio = 0;
            for (uint64_t q = p;;) {
                if (left_ok(q, lim)) return q;
                if (q == lim) return RG_NONE;
                --q;
                if (!ins) return RG_NONE;
                if (++kio > K) return RG_NONE;
            }
        }
        int kmax = K;
        uint64_t best = RG_NONE;
#pragma unroll
        for (int j = 1; j <= KR; ++j) {   // 0x403f80
            if (j > kmax) break;
            rows[j] = del ? ws_or(rows[j - 1], trn(rev, rows[j - 1])) : rows[j - 1];
            if (del && (rows[j].w[0] & 1) && left_ok(p, lim)) {
                kio = j;
                kmax = j - 1;
                best = p;
            }
        }
        if (p == lim) return best;
        for (uint64_t cur = p;;) {
            --cur;
            const WS<NW> bc = bmask(cur);
            const WS<NW> n0 = trn(rev, ws_and(rows[0], bc));
            if ((n0.w[0] & 1) && left_ok(cur, lim)) {
                kio = 0;
                return cur;
            }
            WS<NW> oldp = rows[0], last = n0;
            rows[0] = n0;
#pragma unroll
            for (int j = 1; j <= KR; ++j) {   // 0x404230
                if (j > kmax) break;
                WS<NW> v = del ? trn(rev, last) : ws_zero<NW>();
                if (ins) v = ws_or(v, oldp);
                if (sub) v = ws_or(v, trn(rev, oldp));
                v = ws_or(v, trn(rev, ws_and(rows[j], bc)));
                const WS<NW> oj = rows[j];
                rows[j] = v;
                last = v;
                if ((v.w[0] & 1) && left_ok(cur, lim)) {
                    int c = j;
#pragma unroll
                    for (int d = KR - 1; d >= 0; --d)   // while rows[c - 1] is final: --c
                        if (d == c - 1 && (rows[d].w[0] & 1)) c = d;
                    if (c == 0) {
                        kio = 0;
                        return cur;
                    }
                    kio = c;
                    kmax = c - 1;
                    best = cur;
                    break;
                }
                oldp = oj;
            }
            if (!ws_any(last) || cur == lim) return best;
        }
    }
    // one state of checkMatch's loop: 1 printed (mb, me), 0 the candidate
    // fails (a failed second phase), -1 the next state
    __device__ int attempt(int s, uint64_t pos, uint64_t rb, uint64_t re, uint64_t& mb, uint64_t& me) {
        int k1 = S->k, k2;
        uint64_t st, en;
        if (S->type != 3) {
            en = efwd(pos, re - 1, s, k1);
            if (en == RG_NONE) return -1;
            k2 = S->k - k1;
            st = ebwd(pos + 1, rb, s, k2);
        } else {
            st = ebwd(pos, rb, s, k1);
            if (st == RG_NONE) return -1;
            k2 = S->k - k1;
            en = efwd(pos - 1, re - 1, s, k2);
        }
        if (st == RG_NONE || en == RG_NONE) return 0;   // 0x406248: the second phase fails the candidate
        mb = st;
        me = en + 1;
        return 1;
    }
    // checkMatch 0x406010: the slots i < P->0x24 whose bit of `match` is set
    // (`bt`: the bit number mod 64), in order; the first whose first phase
    // succeeds decides
    __device__ bool check(uint64_t pos, uint64_t match, uint64_t& mb, uint64_t& me) {
        if (S->type == 3 && pos == 0) return false;
        const uint64_t rp = S->type == 3 ? pos - 1 : pos;
        uint64_t rb, re;
        record(rp, rb, re);
        if (rp < rb || rp >= re) return false;
        if (S->nstates <= 64) {
            if (S->nstates < 64) match &= (1ull << S->nstates) - 1;
            while (match) {
                const int i = __builtin_ctzll(match);
                match &= match - 1;
                const int s = S->unmap[i];
                if (s < 0) continue;
                const int r = attempt(s, pos, rb, re, mb, me);
                if (r >= 0) return r == 1;
            }
            return false;
        }
        // class 1 over more than 64 states: slot i = state i (P->0x858 the
        // identity), tested by bit i mod 64 -- states i, i + 64, ... per bit
        for (int base = 0; base < S->nstates; base += 64) {
            uint64_t mm = match;
            while (mm) {
                const int s = base + __builtin_ctzll(mm);
                mm &= mm - 1;
                if (s >= S->nstates) break;
                const int r = attempt(s, pos, rb, re, mb, me);
                if (r >= 0) return r == 1;
            }
        }
        return false;
    }
    // eregularScan / esimpleScan from R; false when no candidate at or
    // before stop verifies
    __device__ bool scan(uint64_t stop, uint64_t& mb, uint64_t& me) {
        const int K = kk(), ell = S->ell;
        if constexpr (SC == 0) {             // esimpleScan's pieces (0x413780)
            const uint64_t* T0 = tab + S->o_T0;
            const uint64_t* T2 = tab + S->o_T2;
            const int np = K + 1;
            if (n < (uint64_t)ell) return false;
            int64_t r9 = (int64_t)R - 1;
            const int64_t limit = (int64_t)n - ell;
            while (r9 < limit) {
                if ((uint64_t)(r9 + 1) > stop) return false;
                uint64_t D = T0[at((uint64_t)(r9 + ell))];
                if (!D) {
                    r9 += ell;
                    continue;
                }
                int64_t a = r9 + ell - 1;
                int kk = ell - 1;
                do {
                    D = (D << 1) & T2[at((uint64_t)a)];
                    --kk;
                    --a;
                } while (D && kk);
                if (D) {
                    bool any = false;
                    for (int i = 0; i < np; ++i) {   // 0x41384b: a 32-bit shift
                        const int bit = i * ell + ell - 1;
                        any |= (D & (uint64_t)(int64_t)(int32_t)(1u << (bit & 31))) != 0;
                    }
                    if (any && check((uint64_t)(r9 + 1), S->match0, mb, me)) return true;
                }
                r9 += kk + 1;
            }
            return false;
        }
        if constexpr (SC == 1) {             // esimpleScan's ABNDM window (0x413b6f)
            const uint64_t* T = tab + S->o_T0;
            const uint64_t top = ~0ull << (64 - ell);
            const int W = ell - K;
            if (n < (uint64_t)(ell - K - 1)) return false;
            const uint64_t limit = n - (uint64_t)(ell - K - 1);
            uint64_t Rr[KR + 1], Tr[KR + 1];
            for (uint64_t s = R; s < limit;) {
                if (s > stop) return false;
                const uint64_t b0 = T[at(s + W - 1)];
                Rr[0] = b0;
#pragma unroll
                for (int j = 1; j <= KR; ++j) {
                    if (j > K) break;
                    Rr[j] = top;
                    Tr[j] = b0;
                }
                int64_t rb = W - 2;
                for (;;) {
                    const uint64_t bc = T[at(s + (uint64_t)rb)];
                    uint64_t oldp = Rr[0], newp = (oldp << 1) & bc;
                    Rr[0] = newp;
#pragma unroll
                    for (int j = 1; j <= KR; ++j) {
                        if (j > K) break;
                        const uint64_t trans = (bc << 1) & Tr[j];
                        uint64_t v = ((newp | oldp) << 1) | oldp;
                        Tr[j] = (oldp << 2) & bc;
                        v |= trans;
                        const uint64_t oldj = Rr[j];
                        v |= (oldj << 1) & bc;
                        Rr[j] = v;
                        oldp = oldj;
                        newp = v;
                    }
                    if (rb == 0) {
                        if ((pick(Rr, K) >> 63) && check(s, S->match0, mb, me)) return true;
                        break;
                    }
                    if (!pick(Rr, K) && !pick(Tr, K)) break;
                    --rb;
                }
                s += (uint64_t)(rb + 1);
            }
            return false;
        }
        const uint64_t* Bw = tab + S->o_Bw;
        const uint64_t* Av = tab + S->o_A;
        const uint64_t* rw = tab + S->o_rw;
        const uint64_t* fw = tab + S->o_fw;
        if constexpr (SC == 2) {             // the pieces exactly (0x4052b9)
            if (n < (uint64_t)ell) return false;
            int64_t pos = (int64_t)R - 1;
            const int64_t lim = (int64_t)n - ell;
            while (pos < lim) {
                if ((uint64_t)(pos + 1) > stop) return false;
                uint64_t rcx = Av[at((uint64_t)(pos + ell))];
                if (!rcx) {
                    pos += ell;
                    continue;
                }
                uint64_t D = 0;
                int64_t c = pos + ell - 1;
                bool dead = false;
                for (;;) {
                    D = rcx & Bw[at((uint64_t)c)];
                    rcx = tr(rw, D);
                    if (!rcx) {
                        dead = true;
                        break;
                    }
                    if (--c == pos) break;
                }
                if (dead) {
                    pos = c;
                    continue;
                }
                if ((rcx & S->ffinal) && check((uint64_t)(pos + 1), D, mb, me)) return true;
                ++pos;
            }
            return false;
        }
        uint64_t rows[KR + 1], old[KR + 1];
        if constexpr (SC == 3) {             // bwdScanrk 0x402d50
            const int W = ell - K;
            if (n < (uint64_t)W) return false;
            int64_t pos = (int64_t)R - 1;
            const int64_t lim = (int64_t)n - W;
            while (pos < lim) {
                if ((uint64_t)(pos + 1) > stop) return false;
                const uint8_t c0 = at((uint64_t)(pos + W));
                uint64_t bprev = Bw[c0];
                rows[0] = Av[c0];
#pragma unroll
                for (int j = 1; j <= KR; ++j)
                    if (j <= K) rows[j] = S->finit;
#pragma unroll
                for (int j = 0; j <= KR; ++j)
                    if (j <= K) old[j] = S->finit;
                int64_t cur = pos + W - 1;
                for (;;) {
                    const uint64_t bc = Bw[at((uint64_t)cur)];
                    uint64_t po = rows[0], pn = tr(rw, bc & po);
                    rows[0] = pn;
#pragma unroll
                    for (int j = 1; j <= KR; ++j) {   // 0x4030d0
                        if (j > K) break;
                        const uint64_t oj = rows[j];
                        uint64_t v = po | tr(rw, pn | po) | tr(rw, bc & oj);
                        v |= tr(rw, tr(rw, bc & old[j - 1]) & bprev);
                        old[j - 1] = po;
                        rows[j] = v;
                        po = oj;
                        pn = v;
                    }
                    if (!pn) {               // 0x403230
                        pos = cur;
                        break;
                    }
                    if (--cur == pos) {      // 0x4031ed
                        if ((pn & S->ffinal) && check((uint64_t)(pos + 1), po, mb, me)) return true;
                        ++pos;
                        break;
                    }
                    bprev = bc;
                }
            }
            return false;
        }
        uint64_t cur = R;                    // fwdScanrk 0x402830
        for (;;) {
            if (cur >= n || cur + 1 > stop) return false;
            uint8_t c = at(cur++);
            while (c == (uint8_t)'\n') {
                if (cur == n) return false;
                c = at(cur++);
            }
            uint64_t st = S->finit;
            rows[0] = old[0] = st;
#pragma unroll
            for (int j = 1; j <= KR; ++j) {
                if (j > K) break;
                st |= tr(fw, st);
                rows[j] = old[j] = st;
            }
            uint64_t bc = Bw[c];
            uint64_t po = rows[0], pn = tr(fw, po) & bc;
            rows[0] = pn;
#pragma unroll
            for (int j = 1; j <= KR; ++j) {   // 0x402a31
                if (j > K) break;
                const uint64_t r = pn | po, oj = rows[j];
                const uint64_t v = r | (tr(fw, oj) & bc) | tr(fw, r);
                rows[j] = v;
                po = oj;
                pn = v;
            }
            if (cur >= n) return false;
            uint64_t bprev = bc;
            if ((pn & S->ffinal) && check(cur, pn & S->ffinal, mb, me)) return true;
            for (;;) {                       // 0x402ac0
                if (cur + 1 > stop) return false;
                c = at(cur++);
                if (c == (uint8_t)'\n') break;
                bc = Bw[c];
                po = rows[0];
                pn = tr(fw, po) & bc;
                rows[0] = pn;
#pragma unroll
                for (int j = 1; j <= KR; ++j) {   // 0x402b68
                    if (j > K) break;
                    const uint64_t oj = rows[j];
                    uint64_t v = po | (tr(fw, oj) & bc) | tr(fw, pn | po);
                    v |= tr(fw, tr(fw, old[j - 1]) & bc) & bprev;
                    old[j - 1] = po;
                    rows[j] = v;
                    po = oj;
                    pn = v;
                }
                if (cur == n) return false;
                if ((pn & S->ffinal) && check(cur, pn & S->ffinal, mb, me)) return true;
                bprev = bc;
            }
        }
    }
};

template <int KR, int SC, int NW>
__global__ __launch_bounds__(WALK_T) void k_erg_walk(XtPrep X, uint64_t* __restrict__ keys, uint32_t* __restrict__ lens,
                                                     const uint64_t* total_d, uint64_t total_h,
                                                     uint8_t* __restrict__ acc, TextView tv) {
    extern __shared__ __attribute__((aligned(16))) uint8_t walk_lds[];
    const size_t tb = walk_tab_bytes(X.tab_words);
    const uint64_t* tab = X.tab;
    if (tb) {
        uint64_t* lt = reinterpret_cast<uint64_t*>(walk_lds);
        for (uint32_t q = threadIdx.x; q < X.tab_words; q += blockDim.x) lt[q] = X.tab[q];
        tab = lt;
    }
    __syncthreads();
    uint8_t* const tcbuf = walk_lds + tb + threadIdx.x * TC_WIN;
    const uint64_t total = total_d ? *total_d : total_h;
    const RgSlot* S = X.rg;
    for (uint64_t i = blockIdx.x * (uint64_t)WALK_T + threadIdx.x; i < total; i += (uint64_t)gridDim.x * WALK_T) {
        if (!(acc[i] & 2)) continue;
        uint64_t j = i + 1;
        while (j < total && !(acc[j] & 2)) ++j;
        const uint64_t pid = keys[i] >> 48;
        const uint64_t first = keys[i] & RG_POS_MASK, last = keys[j - 1] & RG_POS_MASK;
        uint64_t nout = 0;
        const uint64_t nmax = j - i;
        if ((int64_t)pid == X.pid) {
            uint64_t R0 = 0, n = tv.n;
            if (tv.reg.n > 1) {
                const uint32_t r = region_of(tv.reg, first);
                R0 = tv.reg.t[r];
                n = tv.reg.e[r];
            }
            ErgWalk<KR, SC, NW> w{S, tab, tv, n, R0, ~0ull, n, TxtCache{tcbuf, 0, 0}};
            // from the start of first's line, at most span + 4 before it
            // (the scanners' rows then agree with the whole scan's, and no
            // match found before first can start at another cluster's key)
            uint64_t lo = R0;
            if (S->max_len >= 0 && first > R0 + (uint64_t)S->max_len + 4) lo = first - (uint64_t)S->max_len - 4;
            uint64_t p = first;
            while (p > lo && !(xt_brk(tv, p - 1) && w.at(p - 1) == (uint8_t)'\n')) --p;
            w.R = p;
            // up to last's line end, at most span + 2 after it
            uint64_t stop = w.next_nl(last);
            if (S->max_len >= 0) stop = umin64(stop, last + (uint64_t)S->max_len + 2);
            w.nl_hi = w.next_nl(w.R);
            for (;;) {
                uint64_t mb = 0, me = 0;
                if (!w.scan(stop, mb, me)) break;
                // process_output drops a start on a header line, its '\n'
                // included (an empty or erroneous first character can start
                // there at k > 0)
                const bool hdr = xt_header(tv, mb) || (mb > 0 && w.at(mb) == (uint8_t)'\n' && xt_header(tv, mb - 1));
                if (!hdr && nout < nmax) {
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

// One thread per cluster head: the printed matches are written in place
// from the head on (acc bit 0), every other entry of the cluster is cleared.
template <int NW>
__global__ __launch_bounds__(WALK_T) void k_rg_walk(XtPrep X, uint64_t* __restrict__ keys, uint32_t* __restrict__ lens,
                                                    const uint64_t* total_d, uint64_t total_h,
                                                    uint8_t* __restrict__ acc, TextView tv) {
    extern __shared__ __attribute__((aligned(16))) uint8_t walk_lds[];
    const size_t tb = walk_tab_bytes(X.tab_words);
    const uint64_t* tab = X.tab;
    if (tb) {
        uint64_t* lt = reinterpret_cast<uint64_t*>(walk_lds);
        for (uint32_t q = threadIdx.x; q < X.tab_words; q += blockDim.x) lt[q] = X.tab[q];
        tab = lt;
    }
    __syncthreads();
    uint8_t* const tcbuf = walk_lds + tb + threadIdx.x * TC_WIN;
    const uint64_t total = total_d ? *total_d : total_h;
    const RgSlot* S = X.rg;
    for (uint64_t i = blockIdx.x * (uint64_t)WALK_T + threadIdx.x; i < total; i += (uint64_t)gridDim.x * WALK_T) {
        if (!(acc[i] & 2)) continue;
        uint64_t j = i + 1;
        while (j < total && !(acc[j] & 2)) ++j;
        const uint64_t pid = keys[i] >> 48;
        const uint64_t first = keys[i] & RG_POS_MASK, last = keys[j - 1] & RG_POS_MASK;
        uint64_t nout = 0;
        const uint64_t nmax = j - i;
        if ((int64_t)pid == X.pid) {
            uint64_t R0 = 0, n = tv.n;
            if (tv.reg.n > 1) {
                const uint32_t r = region_of(tv.reg, first);
                R0 = tv.reg.t[r];
                n = tv.reg.e[r];
            }
            RgWalk<NW> w{S, tab, tv, n, R0, ~0ull, n, TxtCache{tcbuf, 0, 0}};
            uint64_t stop;
            if (S->max_len >= 0) {
                const uint64_t back = (uint64_t)S->max_len + 1;
                if (first > R0 + back) w.R = first - back;
                stop = last + (uint64_t)S->max_len;
            } else {
                uint64_t p = first;
                while (p > R0 && !w.is_nl(p - 1)) --p;
                w.R = p;
                stop = w.next_nl(last);
            }
            w.nl_hi = w.next_nl(w.R);
            for (;;) {
                uint64_t mb = 0, me = 0;
                if (!w.scan(stop, mb, me)) break;
                if (!xt_header(tv, mb) && nout < nmax) {
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

}  // namespace

int erg_scanner(const Upload& up, size_t o_slot) {
    RgSlot S;
    memcpy(&S, up.blob.data() + o_slot, sizeof(S));
    if (S.cls == 1) return S.type == 1 ? 0 : 1;
    return S.type == 1 ? 2 : S.type == 2 ? 3 : 4;
}

void rg_launch(const XtPrep& X, uint64_t* keys, uint32_t* lens, const uint64_t* total_d, uint64_t total_h,
               uint8_t* acc, const TextView& tv, hipStream_t s) {
    const uint32_t blocks = 1024;
    hipLaunchKernelGGL(k_rg_heads, dim3(blocks), dim3(RG_T), 0, s, X, keys, total_d, total_h, acc, tv);
    const size_t lds = walk_tab_bytes(X.tab_words) + WALK_T * TC_WIN;
    if (X.eregular) {
        // the scanner and the row count (below 4 errors: rows in registers)
        // are template arguments
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(WALK_T), lds, s, X, keys, lens, total_d, total_h, acc, tv);
        };
        // (and the verify's words: one up to 64 states)
        auto by_k = [&](auto sc) {
            constexpr int SC = decltype(sc)::value;
            if (X.words == 1) {
                X.k == 1   ? go(k_erg_walk<1, SC, 1>)
                : X.k == 2 ? go(k_erg_walk<2, SC, 1>)
                : X.k == 3 ? go(k_erg_walk<3, SC, 1>)
                           : go(k_erg_walk<PM_MAX_K, SC, 1>);
            } else {
                X.k == 1   ? go(k_erg_walk<1, SC, RG_NW>)
                : X.k == 2 ? go(k_erg_walk<2, SC, RG_NW>)
                : X.k == 3 ? go(k_erg_walk<3, SC, RG_NW>)
                           : go(k_erg_walk<PM_MAX_K, SC, RG_NW>);
            }
        };
        switch (X.scanner) {
            case 0: by_k(std::integral_constant<int, 0>{}); break;
            case 1: by_k(std::integral_constant<int, 1>{}); break;
            case 2: by_k(std::integral_constant<int, 2>{}); break;
            case 3: by_k(std::integral_constant<int, 3>{}); break;
            default: by_k(std::integral_constant<int, 4>{}); break;
        }
    } else if (X.words == 1)
        hipLaunchKernelGGL(k_rg_walk<1>, dim3(blocks), dim3(WALK_T), lds, s, X, keys, lens, total_d, total_h, acc, tv);
    else
        hipLaunchKernelGGL(k_rg_walk<RG_NW>, dim3(blocks), dim3(WALK_T), lds, s, X, keys, lens, total_d, total_h, acc,
                           tv);
    HIPCHK(hipGetLastError());
}

}  // namespace pm

using namespace pm;

extern "C" int pm_regular_plan(int m, int words, const uint64_t* byte_mask, int nodes, const int32_t* tree,
                               const int32_t* tree_nullable, int32_t* out, uint64_t* masks) {
    return guarded([&] {
        require(byte_mask != nullptr && tree != nullptr && tree_nullable != nullptr && out != nullptr &&
                    masks != nullptr,
                "null argument");
        require(words >= 1 && words <= 4 && m >= 1 && m <= 64 * words, "m / words out of range");
        const Automaton A = make_automaton(RgTree{nodes, tree, tree_nullable}, byte_mask, words, m);
        const Plan P = plan_of(A);
        out[0] = P.type;
        out[1] = P.ell;
        out[2] = P.cls;
        out[3] = P.cls == 3 ? window_states(P, A.ms) : 0;
        for (int q = 0; q < RG_NW; ++q) {
            masks[q] = P.win[q];
            masks[RG_NW + q] = P.winit[q];
            masks[2 * RG_NW + q] = P.wfinal[q];
        }
    });
}

extern "C" int pm_eregular_plan(int m, int words, const uint64_t* byte_mask, int nodes, const int32_t* tree,
                                const int32_t* tree_nullable, int k, int32_t* out, uint64_t* masks) {
    return guarded([&] {
        require(byte_mask != nullptr && tree != nullptr && tree_nullable != nullptr && out != nullptr &&
                    masks != nullptr,
                "null argument");
        require(words >= 1 && words <= 4 && m >= 1 && m <= 64 * words, "m / words out of range");
        const Automaton A = make_automaton(RgTree{nodes, tree, tree_nullable}, byte_mask, words, m);
        const EPlan E = eplan_of(A, k);
        out[0] = E.etype;
        out[1] = E.ell;
        out[2] = E.cls;
        out[3] = E.defined ? 1 : 0;
        out[4] = E.npieces;
        for (int i = 0; i < E.npieces; ++i)
            for (int q = 0; q < RG_NW; ++q) {
                masks[(3 * i) * RG_NW + q] = E.pwin[i][q];
                masks[(3 * i + 1) * RG_NW + q] = E.pini[i][q];
                masks[(3 * i + 2) * RG_NW + q] = E.pfin[i][q];
            }
        masks[3 * (PM_MAX_K + 1) * RG_NW] = E.match0;
    });
}
