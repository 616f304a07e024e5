/*
 * pm_nrgrep_reg.c -- nrgrep's regular engine at k = 0 (detClass 3: a pattern
 * with '|' or a repeated group), the engine nrgrep_coords runs for every
 * PatMatch pattern that repeats a parenthesised group: GA(TC){1,2}A becomes
 * (GA(TC)(TC)?A) (patmatch_to_nrgrep.pl:307-348 pops the group, :462-495
 * repeats it), searched per strand by patmatch.py:733-743.
 *
 * TEST INFRASTRUCTURE ONLY (like pm_oracle.c / pm_nrgrep.c / pm_nrgrep_ext.c):
 * only tests/, smoke() and bench.py's cpu_baseline leg may load it, and only
 * as the checker.
 *
 * Round 5: restated from the binary's disassembly (www/bin/nrgrep_coords,
 * `objdump -d`, never executed).  This file simulates the binary's loops
 * literally; the GPU engine (pm_regular.hip) replays the same rule per
 * cluster of candidate starts, and tests compare the two.
 *
 *   searchPreproc: detClass == 3, OptErrors == 0 -> regularPreproc 0x40c880
 *   regularPreproc:
 *     regularLength 0x40b2a0: states 1.. in leaf order (state 0 = initial)
 *     regularLoadMasks 0x40b730: B[c] by getAclass (-i: both cases),
 *       firstLast 0x4086b0, follow 0x4089b0: arrows[0] = first,
 *       arrows[s] = follow(s), final = last; reverse arrows (0x40ca65)
 *     regularFindBest 0x40a500: dist to a final state, per-state costs over
 *       letterProb (.data 0x621120), minCost 0x409940 over the tree (a leaf
 *       starts a window of l levels, '|' joins its sides, a concatenation
 *       takes its cheaper side, '*' / '?' cannot hold one), the best
 *       cost / (l - cost + 1) under 0.65 -> a window scanned backward
 *       (type 2), else the automaton scanned forward (type 3)
 *     regularMakeDet 0x40bfc0: the forward / backward transition tables of
 *       the whole automaton in slices of W = ceil(m / ceil(m / 16)) states
 *     detClass 0x41ac90 over the window's states: 1 -> simpleLoadFast +
 *       simpleScan, 2 -> extendedLoadFast + extendedScan, 3 ->
 *       regularLoadFast 0x40c4f0 (regularRemapStates 0x40bab0) + regularScan
 *       0x4091d0
 *   regularSearch 0x40ce90: P->scan(beg, end, checkMatch 0x408ec0, P, fast)
 *
 * Quirks restated as they are:
 *   - checkMatch 0x408ec0 verifies only the window states the scanner left
 *     in P->match (+0x28, a 64-bit word): regularScan stores its last state
 *     set there (0x4093aa, 0x4095f8, 0x40976e, 0x409870, 0x409924) but
 *     simpleScan and extendedScan never do, and regularPreproc zeroes it
 *     (0x40cb91).  A regular pattern whose best window is a class sequence
 *     or an extended sequence is therefore never printed: nrgrep_coords
 *     prints its banner and no match.
 *   - the backward scanner hands checkMatch every window state of its last
 *     set (not only the window's initial ones); checkMatch tries them in
 *     state order: the shortest end forward (fwdCheck 0x408bc0) and the
 *     nearest start backward (bwdCheck 0x408d50) around the state.
 *   - the forward scanner never tests a state set after the last character
 *     of the search region (0x4095c4), and restarts after every '\n'.
 *   - SLICE 0x41b8e0 takes W bits of ONE 64-bit word: for m > 64 states a
 *     table slice that straddles a word boundary loses the states past it,
 *     so their transitions are never taken in fwdCheck / bwdCheck.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PMR_NW 5                    /* 64-bit words per state set: 257 states */
#define PMR_MAXS (64 * PMR_NW)
#define PMR_START 2                 /* '^' (OptStartLine) */
#define PMR_END 4                   /* '$' (OptEndLine) */

/* nrgrep's tree node types (regex.py _LEAF.. : the jump tables 0x41d4f0) */
enum { T_LEAF = 0, T_STAR = 1, T_OR = 2, T_CAT = 3, T_OPT = 4, T_PLUS = 5 };

extern const double pmn_letter_prob[256];   /* pm_nrgrep.c: letterProb, .data 0x621120 */

typedef struct { uint64_t w[PMR_NW]; } rset;

static inline int rs_has(const rset* s, int i) { return (int)((s->w[i >> 6] >> (i & 63)) & 1); }
static inline void rs_set(rset* s, int i) { s->w[i >> 6] |= 1ull << (i & 63); }
static inline void rs_or(rset* d, const rset* s) { for (int q = 0; q < PMR_NW; ++q) d->w[q] |= s->w[q]; }
static inline int rs_any(const rset* s) {
    uint64_t a = 0;
    for (int q = 0; q < PMR_NW; ++q) a |= s->w[q];
    return a != 0;
}
static inline int rs_inter(const rset* a, const rset* b) {
    uint64_t x = 0;
    for (int q = 0; q < PMR_NW; ++q) x |= a->w[q] & b->w[q];
    return x != 0;
}
static inline int rs_count(const rset* s) {
    int n = 0;
    for (int q = 0; q < PMR_NW; ++q) n += __builtin_popcountll(s->w[q]);
    return n;
}

typedef struct {
    int type, a, b, state, nullable;
    rset pm, first, last;
} rnode;

typedef struct {
    int m;                          /* states (positions + 1) */
    int nn;
    rnode* nd;
    rset arrows[PMR_MAXS], rev[PMR_MAXS], final, B[256];
    rset vis;                       /* states SLICE can see (all for m <= 64) */
    /* plan */
    int type, ell, cls;
    rset win, winit, wfinal;
    double best;
    /* window tables (regularRemapStates: one word) */
    int mp;
    int map[PMR_MAXS], unmap[64];
    uint64_t Bw[256], A[256], fw[64], rw[64], ffinal, finit;
    /* text */
    const uint8_t* t;
    int64_t n;
    const int64_t* nl;
    int64_t nnl;
    int mode;
} rctx_t;

/* ------------------------------------------------------------------------
 * the automaton (regularLength, firstLast, follow, regularLoadMasks)
 * ---------------------------------------------------------------------- */

static void first_last(rctx_t* x, int i) {                 /* firstLast 0x4086b0 + setMaskPos 0x41ad90 */
    rnode* e = &x->nd[i];
    memset(&e->pm, 0, sizeof(rset));
    memset(&e->first, 0, sizeof(rset));
    memset(&e->last, 0, sizeof(rset));
    if (e->type == T_LEAF) {
        if (e->state > 0) {
            rs_set(&e->pm, e->state);
            rs_set(&e->first, e->state);
            rs_set(&e->last, e->state);
        }
        return;
    }
    first_last(x, e->a);
    const rnode* a = &x->nd[e->a];
    if (e->type == T_OR || e->type == T_CAT) {
        first_last(x, e->b);
        const rnode* b = &x->nd[e->b];
        e->pm = a->pm;
        rs_or(&e->pm, &b->pm);
        if (e->type == T_OR) {
            e->first = a->first;
            rs_or(&e->first, &b->first);
            e->last = a->last;
            rs_or(&e->last, &b->last);
        } else {                                           /* 0x4087f0 */
            e->first = a->first;
            if (a->nullable) rs_or(&e->first, &b->first);
            e->last = b->last;
            if (b->nullable) rs_or(&e->last, &a->last);
        }
        return;
    }
    e->pm = a->pm;                                         /* '*', '?', '+' (0x408768) */
    e->first = a->first;
    e->last = a->last;
}

static void follow_of(const rctx_t* x, int i, int s, rset* out) {   /* follow 0x4089b0 */
    const rnode* e = &x->nd[i];
    switch (e->type) {
    case T_LEAF:
        return;
    case T_OPT:
        follow_of(x, e->a, s, out);
        return;
    case T_STAR:
    case T_PLUS:                                           /* 0x408af0 */
        follow_of(x, e->a, s, out);
        if (rs_has(&x->nd[e->a].last, s)) rs_or(out, &x->nd[e->a].first);
        return;
    case T_OR:
        if (rs_has(&x->nd[e->a].pm, s)) follow_of(x, e->a, s, out);
        if (rs_has(&x->nd[e->b].pm, s)) follow_of(x, e->b, s, out);
        return;
    default:                                               /* T_CAT 0x408a38 */
        if (rs_has(&x->nd[e->a].last, s)) rs_or(out, &x->nd[e->b].first);
        if (rs_has(&x->nd[e->a].pm, s)) follow_of(x, e->a, s, out);
        if (rs_has(&x->nd[e->b].pm, s)) follow_of(x, e->b, s, out);
        return;
    }
}

static inline uint8_t fold(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }

/* tree: nodes * 4 int32 (type, a, b, pos), node 0 the root; pos = the
 * regex.py position of a leaf (state pos + 1), -1 for an empty leaf.
 * Bpos: [256][4] regex.py position sets by folded byte. */
static int build(rctx_t* x, const int32_t* tree, int nodes, const int32_t* nullable, const uint64_t* Bpos,
                 int npos, int icase) {
    if (nodes < 1 || npos < 1 || npos + 1 > PMR_MAXS) return -1;
    x->m = npos + 1;
    x->nn = nodes;
    x->nd = calloc((size_t)nodes, sizeof(rnode));
    if (!x->nd) return -1;
    int next = 1;
    for (int i = 0; i < nodes; ++i) {
        rnode* e = &x->nd[i];
        e->type = tree[4 * i];
        e->a = tree[4 * i + 1];
        e->b = tree[4 * i + 2];
        e->nullable = nullable[i];
        e->state = tree[4 * i + 3] >= 0 ? tree[4 * i + 3] + 1 : 0;
        if (e->type < 0 || e->type > 5) return -1;
        if (e->type == T_LEAF && e->state == 0) return -1;   /* an empty leaf inside: no position (refused) */
        if (e->type != T_LEAF && (e->a <= i || e->a >= nodes)) return -1;
        if ((e->type == T_OR || e->type == T_CAT) && (e->b <= i || e->b >= nodes)) return -1;
        (void)next;
    }
    first_last(x, 0);
    x->arrows[0] = x->nd[0].first;                        /* regularLoadMasks 0x40b8b8 */
    for (int s = 1; s < x->m; ++s) follow_of(x, 0, s, &x->arrows[s]);
    x->final = x->nd[0].last;
    for (int s = 0; s < x->m; ++s)
        for (int t = 0; t < x->m; ++t)
            if (rs_has(&x->arrows[s], t)) rs_set(&x->rev[t], s);
    for (int c = 0; c < 256; ++c) {                        /* getAclass: -i gives both cases */
        const uint64_t* bp = Bpos + (size_t)(icase ? fold((uint8_t)c) : c) * 4;
        for (int p = 0; p < npos; ++p)
            if ((bp[p >> 6] >> (p & 63)) & 1) rs_set(&x->B[c], p + 1);
    }
    /* SLICE 0x41b8e0: slices of W bits of one word */
    const int ntab = (x->m + 16 - 1) / 16, W = (x->m - 1 + ntab) / ntab;
    for (int t = 0; t < ntab; ++t)
        for (int b = t * W; b < t * W + W && b < x->m; ++b)
            if ((b >> 6) == ((t * W) >> 6)) rs_set(&x->vis, b);
    return 0;
}

/* ------------------------------------------------------------------------
 * regularFindBest 0x40a500 + minCost 0x409940
 * ---------------------------------------------------------------------- */

typedef struct {
    int L, m;
    const int* dist;
    double* C;                  /* [m][L] */
    rset *M50, *M70;            /* [m][L]: states exactly / within l - 1 arrows away */
} mc_t;

static double min_cost(const rctx_t* x, const mc_t* c, int i, int ell, rset* win, rset* ini, rset* fin) {
    const rnode* e = &x->nd[i];
    switch (e->type) {
    case T_LEAF: {                                         /* 0x409b10 */
        const int p = e->state;
        if (c->dist[p] < ell) return (double)(ell + 1);
        *win = c->M70[(size_t)p * c->L + ell];
        memset(ini, 0, sizeof(rset));
        rs_set(ini, p);
        *fin = c->M50[(size_t)p * c->L + ell];
        return c->C[(size_t)p * c->L + ell];
    }
    case T_STAR:
    case T_OPT:                                            /* 0x409aef */
        return (double)(ell + 1);
    case T_PLUS:                                           /* 0x409bb0 */
        return min_cost(x, c, e->a, ell, win, ini, fin);
    case T_OR: {                                           /* 0x409978 */
        rset w2, i2, f2;
        memset(&w2, 0, sizeof w2);
        memset(&i2, 0, sizeof i2);
        memset(&f2, 0, sizeof f2);
        const double c1 = min_cost(x, c, e->a, ell, win, ini, fin);
        const double c2 = min_cost(x, c, e->b, ell, &w2, &i2, &f2);
        rs_or(win, &w2);
        rs_or(ini, &i2);
        *fin = f2;
        if (rs_count(win) > 64) {                          /* 0x409ac8 */
            memset(win, 0, sizeof(rset));
            memset(ini, 0, sizeof(rset));
            memset(fin, 0, sizeof(rset));
            return (double)(ell + 1);
        }
        return c1 > c2 ? c1 : c2;                          /* maxsd */
    }
    default: {                                             /* T_CAT 0x409bc0 */
        rset w2, i2, f2;
        memset(&w2, 0, sizeof w2);
        memset(&i2, 0, sizeof i2);
        memset(&f2, 0, sizeof f2);
        const double c1 = min_cost(x, c, e->a, ell, win, ini, fin);
        const double c2 = min_cost(x, c, e->b, ell, &w2, &i2, &f2);
        if (c2 >= c1) return c1;
        *win = w2;
        *ini = i2;
        *fin = f2;
        return c2;
    }
    }
}

static int find_best(rctx_t* x, int K) {
    const int m = x->m;
    int* dist = calloc((size_t)m, sizeof(int));
    for (int i = 0; i < m; ++i) {                          /* 0x40a57e */
        rset S, T;
        memset(&S, 0, sizeof S);
        rs_set(&S, i);
        dist[i] = 1;
        while (!rs_inter(&S, &x->final)) {
            ++dist[i];
            memset(&T, 0, sizeof T);
            for (int j = 0; j < m; ++j)
                if (rs_has(&S, j)) rs_or(&T, &x->arrows[j]);
            rs_or(&S, &T);
            if (dist[i] > m + 1) break;                     /* (no final state reachable) */
        }
    }
    int L = dist[0] > 64 ? 64 : dist[0];
    double* prob = calloc((size_t)m, sizeof(double));
    for (int i = 0; i < m; ++i)                            /* 0x40a6b0 */
        for (int ch = 0; ch < 256; ++ch)
            if (rs_has(&x->B[ch], i)) prob[i] += pmn_letter_prob[ch];
    const size_t ML = (size_t)m * L;
    double* cost = calloc(ML, sizeof(double));
    rset* M50 = calloc(ML, sizeof(rset));
    rset* M70 = calloc(ML, sizeof(rset));
    for (int i = 0; i < m; ++i) {                          /* 0x40a79b */
        cost[(size_t)i * L] = 1.0;
        if (L > 1) {
            cost[(size_t)i * L + 1] = prob[i];
            rs_set(&M70[(size_t)i * L + 1], i);
            rs_set(&M50[(size_t)i * L + 1], i);
        }
    }
    for (int l = 1; l + 1 < L; ++l)                        /* 0x40a8af */
        for (int i = 0; i < m; ++i) {
            double s = 0.0;
            rset M;
            memset(&M, 0, sizeof M);
            for (int j = 0; j < m; ++j)
                if (rs_has(&x->arrows[i], j)) {
                    s += cost[(size_t)j * L + l];
                    rs_or(&M, &M50[(size_t)j * L + l]);
                }
            s *= prob[i];
            cost[(size_t)i * L + l + 1] = 1.0 < s ? 1.0 : s;
            M50[(size_t)i * L + l + 1] = M;
            M70[(size_t)i * L + l + 1] = M70[(size_t)i * L + l];
            rs_or(&M70[(size_t)i * L + l + 1], &M);
        }
    /* P[i][l][a], l, a < L: idx (i L + l) L + a (0x40aa30) */
    double* P = calloc((size_t)m * L * L, sizeof(double));
#define PI(i, l, a) P[((size_t)(i) * L + (l)) * L + (a)]
    for (int i = 0; i < m; ++i)
        for (int l = 0; l < L; ++l) PI(i, l, 0) = 1.0;
    for (int l = 1; l < L; ++l)                            /* 0x40aad1 */
        for (int a = 1; a <= l; ++a)
            for (int i = 0; i < m; ++i) {
                double v = cost[(size_t)i * L + a];
                if (a < l)
                    for (int j = 0; j < m; ++j)
                        if (rs_has(&x->arrows[i], j)) v = 1.0 - (1.0 - v) * (1.0 - PI(j, l - 1, a));
                PI(i, l, a) = v;
            }
    double* C = calloc(ML, sizeof(double));
    for (int i = 0; i < m; ++i)                            /* 0x40ac2f */
        for (int l = 0; l < L; ++l) {
            double s = (double)K;
            for (int a = 0; a <= l; ++a) s += PI(i, l, a);
            C[(size_t)i * L + l] = s;
        }
#undef PI
    mc_t mc = {L, m, dist, C, M50, M70};
    double best = 0.65;                                    /* .rodata 0x41d288 */
    int bell = 0;
    rset bw, bi, bf;
    memset(&bw, 0, sizeof bw);
    memset(&bi, 0, sizeof bi);
    memset(&bf, 0, sizeof bf);
    int ell = L - 1;
    if (ell > 0 && !(1.0 >= 0.65 * (double)ell)) {         /* 0x40ad20 */
        for (;;) {
            rset w, in, fi;
            memset(&w, 0, sizeof w);
            memset(&in, 0, sizeof in);
            memset(&fi, 0, sizeof fi);
            const double c = min_cost(x, &mc, 0, ell, &w, &in, &fi);
            if ((double)(ell + 1) > c) {
                const double r = c / ((double)ell - c + 1.0);
                if (best > r) {
                    best = r;
                    bw = w;
                    bi = in;
                    bf = fi;
                    bell = ell;
                }
            }
            if (--ell == 0) break;
            if (1.0 >= best * (double)ell) break;
        }
    }
    x->best = best;
    if (0.65 > best) {                                     /* 0x40aec3 */
        x->type = 2;
        x->ell = bell;
        x->win = bw;
        x->winit = bi;
        x->wfinal = bf;
    } else {                                               /* 0x40b0a7: the automaton forward */
        x->type = 3;
        x->ell = 0;
        memset(&x->win, 0, sizeof(rset));
        memset(&x->winit, 0, sizeof(rset));
        rs_set(&x->winit, 0);
        if (m <= 64) {
            for (int s = 0; s < m; ++s) rs_set(&x->win, s);
            x->wfinal = x->final;
        } else {                                           /* 0x40b175: BFS layers while <= 64 states */
            rset reach = x->winit, layer;
            memset(&layer, 0, sizeof layer);
            while (rs_count(&reach) <= 64) {
                for (int q = 0; q < PMR_NW; ++q) layer.w[q] = reach.w[q] & ~x->win.w[q];
                rs_or(&x->win, &reach);
                memset(&reach, 0, sizeof reach);
                for (int s = 0; s < m; ++s)
                    if (rs_has(&x->win, s)) rs_or(&reach, &x->arrows[s]);
            }
            x->wfinal = layer;
            rs_or(&x->wfinal, &x->final);
            for (int q = 0; q < PMR_NW; ++q) x->wfinal.w[q] &= x->win.w[q];
        }
    }
    free(dist);
    free(prob);
    free(cost);
    free(M50);
    free(M70);
    free(P);
    free(C);
    return 0;
}

/* detClass 0x41ac90 / detClass1 0x418420 over the states of `pos` */
static int det_class1(const rctx_t* x, int i, const rset* pos) {
    const rnode* e = &x->nd[i];
    if (!rs_inter(&e->pm, pos)) return 1;
    switch (e->type) {
    case T_LEAF:
        return 1;
    case T_OR:
        return 3;
    case T_CAT: {
        const int a = det_class1(x, e->a, pos), b = det_class1(x, e->b, pos);
        return a > b ? a : b;
    }
    default: {
        int r = det_class1(x, e->a, pos);
        if (r == 1) r = 2;
        return x->nd[e->a].type == T_LEAF ? r : 3;
    }
    }
}

/* regularRemapStates 0x40bab0 + regularLoadFast 0x40c4f0 */
static int load_fast(rctx_t* x) {
    x->mp = 1;
    for (int s = 1; s < x->m; ++s) x->mp += rs_has(&x->win, s);
    if (x->mp > 64) return -1;                             /* the tables keep one word (0x40c5b4) */
    x->map[0] = 0;
    int k = 0;
    for (int s = 1; s < x->m; ++s)
        if (rs_has(&x->win, s)) x->map[s] = ++k;
    memset(x->unmap, 0, sizeof x->unmap);
    for (int s = 0; s < x->m; ++s)
        if (rs_has(&x->win, s)) x->unmap[x->map[s]] = s;   /* regularPreproc 0x40cd00: P->0x860 */
    memset(x->fw, 0, sizeof x->fw);
    for (int s = 0; s < x->m; ++s)
        if (rs_has(&x->winit, s)) x->fw[0] |= 1ull << x->map[s];
    for (int s = 0; s < x->m; ++s)
        if (rs_has(&x->win, s))
            for (int t = 0; t < x->m; ++t)
                if (rs_has(&x->win, t) && rs_has(&x->arrows[s], t)) x->fw[x->map[s]] |= 1ull << x->map[t];
    uint64_t fin = 0;
    for (int s = 0; s < x->m; ++s)
        if (rs_has(&x->wfinal, s)) fin |= 1ull << x->map[s];
    for (int ch = 0; ch < 256; ++ch) {
        uint64_t b = 0;
        for (int s = 0; s < x->m; ++s)
            if (rs_has(&x->win, s) && rs_has(&x->B[ch], s)) b |= 1ull << x->map[s];
        x->Bw[ch] = b;
    }
    if (x->ell > 0) {                                      /* backward: reverse arrows, every state initial */
        memset(x->rw, 0, sizeof x->rw);
        for (int a = 0; a < x->mp; ++a)
            for (int b = 0; b < x->mp; ++b)
                if ((x->fw[a] >> b) & 1) x->rw[b] |= 1ull << a;
        const uint64_t all = x->mp >= 64 ? ~0ull : (1ull << x->mp) - 1;
        x->finit = all;
        x->ffinal = 1;                                     /* init' = {0} */
        for (int ch = 0; ch < 256; ++ch) {                 /* 0x40c700 */
            uint64_t d = all & x->Bw[ch], r = 0;
            for (int q = 0; q < x->mp; ++q)
                if ((d >> q) & 1) r |= x->rw[q];
            x->A[ch] = r;
        }
    } else {                                               /* forward: state 0 loops on every byte */
        x->fw[0] |= 1;
        for (int ch = 0; ch < 256; ++ch) x->Bw[ch] |= 1;
        x->finit = 1;
        x->ffinal = fin;
    }
    return 0;
}

static inline uint64_t wtrans(const uint64_t* tab, int mp, uint64_t d) {
    uint64_t r = 0;
    for (int q = 0; q < mp; ++q)
        if ((d >> q) & 1) r |= tab[q];
    return r;
}

/* ------------------------------------------------------------------------
 * checkMatch 0x408ec0, fwdCheck 0x408bc0, bwdCheck 0x408d50
 * ---------------------------------------------------------------------- */

static void full_trans(const rctx_t* x, const rset* D, const rset* tab, rset* out) {
    memset(out, 0, sizeof(rset));
    for (int s = 0; s < x->m; ++s)
        if (rs_has(D, s) && rs_has(&x->vis, s)) rs_or(out, &tab[s]);
}

static int left_ok(const rctx_t* x, int64_t p, int64_t lim) {      /* recCheckLeftContext 0x402170 */
    return !((x->mode & PMR_START) && p > lim && x->t[p - 1] != '\n');
}
static int right_ok(const rctx_t* x, int64_t q, int64_t lim) {     /* recCheckRightContext 0x4021e0 */
    return !((x->mode & PMR_END) && q < lim && x->t[q] != '\n');
}

/* the nearest p >= ... forward from state set {s} read at p: a final state
 * with the right context; -1 if none before lim */
static int64_t fwd_check(const rctx_t* x, int64_t p, int64_t lim, int s) {
    rset D, T;
    memset(&D, 0, sizeof D);
    rs_set(&D, s);
    for (;;) {
        if (rs_inter(&D, &x->final) && right_ok(x, p + 1, lim + 1)) return p;
        if (p == lim) return -1;
        full_trans(x, &D, x->arrows, &T);
        ++p;
        const rset* b = &x->B[x->t[p]];
        int any = 0;
        for (int q = 0; q < PMR_NW; ++q) {
            T.w[q] &= b->w[q];
            any |= T.w[q] != 0;
        }
        if (!any) return -1;
        D = T;
    }
}

/* the nearest start: from {s} (state s reads t[p - 1]) backward */
static int64_t bwd_check(const rctx_t* x, int64_t p, int64_t lim, int s) {
    rset D, T, init;
    memset(&D, 0, sizeof D);
    memset(&init, 0, sizeof init);
    rs_set(&init, 0);
    rs_set(&D, s);
    for (;;) {
        if (rs_inter(&D, &init) && left_ok(x, p, lim)) return p;
        if (p == lim) return -1;
        --p;
        const rset* b = &x->B[x->t[p]];
        for (int q = 0; q < PMR_NW; ++q) D.w[q] &= b->w[q];
        full_trans(x, &D, x->rev, &T);
        if (!rs_any(&T)) return -1;
        D = T;
    }
}

static int check_match(const rctx_t* x, int64_t pos, int64_t R, uint64_t match, int64_t* mb, int64_t* me) {
    const int64_t rp = x->type == 3 ? pos - 1 : pos;
    /* recGetRecord 0x402030: the last '\n' before rp (back to R only), the
     * first at or after it */
    int64_t lo = 0, hi = x->nnl;
    while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if (x->nl[mid] < rp) lo = mid + 1; else hi = mid;
    }
    int64_t rb = R;
    if (lo > 0 && x->nl[lo - 1] >= R) rb = x->nl[lo - 1] + 1;
    const int64_t re = lo < x->nnl ? x->nl[lo] : x->n;
    if (rp < rb || rp >= re) return 0;
    for (int i = 0; i < x->mp; ++i) {                      /* 0x408f6a */
        if (!((match >> i) & 1)) continue;
        const int s = x->unmap[i];
        int64_t st, en;
        if (x->type == 3) {                                /* 0x4090f0 */
            st = bwd_check(x, pos, rb, s);
            if (st < 0) continue;
            en = fwd_check(x, pos - 1, re - 1, s);
            if (en < 0) continue;
        } else {                                           /* 0x408f89 */
            en = fwd_check(x, pos, re - 1, s);
            if (en < 0) continue;
            st = bwd_check(x, pos + 1, rb, s);
            if (st < 0) continue;
        }
        *mb = st;
        *me = en + 1;
        return 1;
    }
    return 0;
}

/* ------------------------------------------------------------------------
 * regularScan 0x4091d0 over the region [R, n)
 * ---------------------------------------------------------------------- */

/* backward (0x40921c): windows of ell characters read right to left over
 * the window's reversed automaton with every state initial (a factor test);
 * a dead character moves the window past it, a whole window whose last set
 * leads to the window's initial states goes to checkMatch */
static int scan_backward(const rctx_t* x, int64_t R, int64_t* mb, int64_t* me) {
    const int ell = x->ell;
    const uint8_t* t = x->t;
    int64_t r8 = R - 1;
    const int64_t r13 = x->n - ell;
    while (r13 > r8) {
        uint64_t D0 = x->A[t[r8 + ell]];
        if (!D0) {
            r8 += ell;
            continue;
        }
        uint64_t rsi = D0, D = 0;
        int64_t c = r8 + ell - 1;
        int dead = 0;
        for (; c > r8; --c) {                              /* 0x409319 */
            D = rsi & x->Bw[t[c]];
            rsi = wtrans(x->rw, x->mp, D);
            if (!rsi) {
                dead = 1;
                break;
            }
        }
        if (dead) {
            r8 = c;
            continue;
        }
        if (ell == 1) D = 0;                               /* (never chosen: cost >= 1) */
        if (rsi & x->ffinal) {
            if (check_match(x, r8 + 1, R, D, mb, me)) return 1;
        }
        r8 = r8 + 1;
    }
    return 0;
}

/* forward (0x409500): the automaton with state 0 looping, a fresh state
 * after every '\n' (OptRecChar), no test after the region's last byte */
static int scan_forward(const rctx_t* x, int64_t R, int64_t* mb, int64_t* me) {
    const uint8_t* t = x->t;
    int64_t p = R;
    uint64_t D = x->finit;
    if ((D & x->ffinal) && p < x->n && check_match(x, p, R, D & x->ffinal, mb, me)) return 1;
    while (p < x->n) {
        const uint8_t c = t[p++];
        if (c == '\n') {
            if (p >= x->n) return 0;
            D = x->finit;
        } else {
            D = wtrans(x->fw, x->mp, D) & x->Bw[c];
            if (p == x->n) return 0;
        }
        const uint64_t f = D & x->ffinal;
        if (f && check_match(x, p, R, f, mb, me)) return 1;
    }
    return 0;
}

static void ctx_free(rctx_t* x) {
    free(x->nd);
    free(x);
}

static rctx_t* ctx_new(const int32_t* tree, const int32_t* nullable, int nodes, const uint64_t* Bpos, int npos,
                       int icase, int mode) {
    rctx_t* x = calloc(1, sizeof(rctx_t));
    if (!x) return NULL;
    x->mode = mode;
    if (build(x, tree, nodes, nullable, Bpos, npos, icase) < 0 || find_best(x, 0) < 0) {
        ctx_free(x);
        return NULL;
    }
    x->cls = det_class1(x, 0, &x->win);
    if (x->cls == 3 && load_fast(x) < 0) {
        ctx_free(x);
        return NULL;
    }
    return x;
}

/* out[0] = type (2 backward window, 3 forward), out[1] = ell, out[2] =
 * detClass of the window (1 / 2: nothing is ever printed), out[3] = window
 * states m'; masks[0..4] window, [5..9] its initial, [10..14] its final
 * states (nrgrep state numbering: regex position + 1) */
int pmr_plan(const int32_t* tree, const int32_t* nullable, int nodes, const uint64_t* Bpos, int npos, int icase,
             int* out, uint64_t* masks) {
    rctx_t* x = ctx_new(tree, nullable, nodes, Bpos, npos, icase, 0);
    if (!x) return -1;
    out[0] = x->type;
    out[1] = x->ell;
    out[2] = x->cls;
    out[3] = x->cls == 3 ? x->mp : 0;
    for (int q = 0; q < PMR_NW; ++q) {
        masks[q] = x->win.w[q];
        masks[PMR_NW + q] = x->winit.w[q];
        masks[2 * PMR_NW + q] = x->wfinal.w[q];
    }
    ctx_free(x);
    return 0;
}

/* What nrgrep_coords prints for a class-3 pattern at k = 0 over one region
 * (recSearchFile 0x402250: print, R = match end, stop when it ends at n).
 * Returns the number of matches (may exceed cap), -1 if refused. */
int64_t pmr_regular(const uint8_t* text, int64_t n, const int32_t* tree, const int32_t* nullable, int nodes,
                    const uint64_t* Bpos, int npos, int icase, int mode, int64_t* out_beg, int64_t* out_end,
                    int64_t cap) {
    rctx_t* x = ctx_new(tree, nullable, nodes, Bpos, npos, icase, mode);
    if (!x) return -1;
    if (x->cls != 3) {                                     /* P->match stays 0: checkMatch never succeeds */
        ctx_free(x);
        return 0;
    }
    x->t = text;
    x->n = n;
    int64_t nnl = 0;
    for (int64_t p = 0; p < n; ++p) nnl += text[p] == '\n';
    int64_t* nl = malloc(sizeof(int64_t) * (size_t)(nnl + 1));
    nnl = 0;
    for (int64_t p = 0; p < n; ++p)
        if (text[p] == '\n') nl[nnl++] = p;
    x->nl = nl;
    x->nnl = nnl;
    int64_t count = 0, R = 0;
    while (R < n) {
        int64_t mb = 0, me = 0;
        const int ok = x->type == 2 ? scan_backward(x, R, &mb, &me) : scan_forward(x, R, &mb, &me);
        if (!ok) break;
        if (count < cap) {
            out_beg[count] = mb;
            out_end[count] = me;
        }
        ++count;
        if (me == n) break;                                /* 0x4022eb */
        R = me;
    }
    free(nl);
    ctx_free(x);
    return count;
}

/* ========================================================================
 * eregular: the same patterns at k > 0 (searchPreproc: OptErrors != 0 and
 * detClass == 3 -> eregularPreproc 0x406a20).  Restated for automata of up
 * to 319 positions (round 6: more than one word of states, the sliced
 * transition tables of fwdCheck / bwdCheck included -- etab below).
 *
 *   eregularPreproc 0x406a20:
 *     regularFindBest 0x40a500 with K (its cost C carries + K) -> a window
 *       plan and its ratio fb;
 *     the breadth-first levels of the automaton from state 0 to the first
 *       level holding a final state (0x406db8 / 0x406f69), the piece length
 *       pl = min(minlen - K * OptTransp, 64) / (K + 1) (0x406e54);
 *     per state and length the chance a random text runs along it (A,
 *       0x40707a), its factor chance per window position (Bt, 0x4072a0) and
 *       per level the cost C = 1 + sum over the level's states (0x40742d);
 *     a DP over K + 1 pieces of pl characters starting on levels >= 1, each
 *       piece (pl + OptTransp) levels after the previous (0x4076a0 ..
 *       0x407b5e): cost x = C / (pl - C + 1) (1 when C >= pl + 1), pieces
 *       combined as 1 - (1 - x)(1 - rest), best under 0.78, pl shrinking
 *       while 1 / pl <= best;
 *     pieces win (type 1) when their cost < 0.78 and < (K + 1) 1.3 fb
 *       (0x40842a); piece i's window = the states within pl arrows of its
 *       level, its final states those 1 .. pl arrows away (0x408337);
 *       otherwise regularFindBest's window (type 2 backward when ell > 0,
 *       3 forward);
 *     detClass of windows[0]: 1 -> esimpleLoadFast 0x415370 + esimpleScan
 *       0x4136d0 with checkMatch's state word P->0x28 = the first state of
 *       each piece window (0x407e4b); 2 -> a store through a null pointer
 *       (0x4081ed: the process dies, nothing is printed); 3 ->
 *       eregularLoadFast 0x406860 (regularLoadFast over the union of the
 *       windows) + eregularScan 0x4048b0.
 *   eregularScan: type 1 the pieces exactly, backward windows of pl
 *     characters (0x4052b9, like regularScan); type 2 bwdScanrk 0x402d50:
 *     windows of ell - K characters, K + 1 rows of at most j errors with
 *     every edit and transpositions (a filter), P->0x28 = row K before the
 *     window's first character; type 3 fwdScanrk 0x402830: the same rows
 *     forward, fresh after every run of '\n', the final states of row K
 *     after each character except the region's last.
 *   checkMatch 0x406010: for each state s of P->0x28 in order (at most
 *     P->0x24, mapped back by P->0x858): type 1/2 fwdCheck 0x403310 from s
 *     reading t[pos + 1] on (budget K), then bwdCheck 0x403df0 from s reading
 *     t[pos] back (the rest of the budget); type 3 the other way round from
 *     pos - 1.  The first state whose first phase succeeds decides: a failed
 *     second phase fails the candidate.  fwdCheck / bwdCheck keep K + 1 rows
 *     (OptIns, OptDel, OptSubs as given): the nearest boundary with the
 *     fewest errors, row 0 ends the phase at once, a find at j errors caps
 *     the rows at j - 1 (0x403a01).
 *
 * Two places where the binary reads memory it never wrote (parity unpinned,
 * restated as noted):
 *   - without OptDel, fwdCheck / bwdCheck never initialise rows 1 .. K
 *     (0x4034d3 / 0x403f93): they hold whatever the previous check left (the
 *     first time: fresh heap).  Restated as rows 1 .. K = row 0 (the state
 *     the phase starts from, reached with at most j errors).
 *   - class 1 reads windows[1 .. K] (0x407e95) even for a window plan, where
 *     only windows[0] was set unless the piece DP filled them.  Restated as
 *     windows[0] alone.
 * ====================================================================== */

#define PME_MAXK 16
#define PME_INS 1
#define PME_DEL 2
#define PME_SUB 4

typedef struct {
    rctx_t* x;
    int K, errs;
    int etype, ell, cls, npieces, pieces_computed, defined;
    double pbest, fbest;
    rset pwin[PME_MAXK + 1], pini[PME_MAXK + 1], pfin[PME_MAXK + 1];
    int first[PME_MAXK + 1];
    int m;
    /* fwdCheck / bwdCheck's transition tables (regularMakeDet 0x40bfc0,
     * called at 0x407c4c / 0x407c63): ntab tables, table t = the states
     * t W .. t W + W - 1, W = ceil(m / ceil(m / OptDetWidth)) (0x407c1d;
     * OptDetWidth .data 0x621920 = 16) */
    int W, ntab;
    /* checkMatch */
    uint64_t match0;            /* class 1: P->0x28 */
    int nstates;                /* P->0x24 */
    int unmap[PMR_MAXS];        /* P->0x858 */
} ectx_t;

/* eregularPreproc's successor sets (ISSET / OR over the arrows: exact) */
static void ereach(const rctx_t* x, const rset* D, rset* out) {
    memset(out, 0, sizeof(rset));
    for (int s = 0; s < x->m; ++s)
        if (rs_has(D, s)) rs_or(out, &x->arrows[s]);
}

/* fwdCheck / bwdCheck's transition (the seven slice loops of each, e.g.
 * 0x403508 .. 0x40354f and 0x403fc8 .. 0x40400f): table t is indexed by
 * SLICE(D, off, W) (0x41b8e0: W bits of ONE 64-bit word from bit off), off
 * starting at 0 and moving on by W -- or, when the next slice would cross a
 * word (0x403530: (off + W - 1) / 64 != off / 64), to the next word's first
 * bit.  The tables are built for the states t W + b (no such jump), so after
 * a jump the states off + b take the transitions of the states t W + b, and
 * the states a jump skips take none (m <= 64: no slice crosses a word, the
 * identity).  k = 0's fwdCheck (0x408c90) has no jump: rctx_t's vis. */
static void etab(const ectx_t* e, const rset* tab, const rset* D, rset* out) {
    memset(out, 0, sizeof(rset));
    const uint64_t msk = e->W >= 64 ? ~0ull : (1ull << e->W) - 1;
    int off = 0;
    for (int t = 0; t < e->ntab; ++t) {
        uint64_t sl = (D->w[off >> 6] >> (off & 63)) & msk;
        while (sl) {
            const int src = t * e->W + __builtin_ctzll(sl);
            sl &= sl - 1;
            if (src < e->m) rs_or(out, &tab[src]);
        }
        off += e->W;
        if (((off + e->W - 1) >> 6) != (off >> 6)) off = (off & ~63) + 64;
    }
}

/* the table layout fwdCheck / bwdCheck read: -1 if a slice would read past
 * the state set's words (SLICE on memory the binary never allocated) */
static int etab_layout(ectx_t* e) {
    const int m = e->m;
    const int nt0 = (m + 16 - 1) / 16;
    e->W = (m + nt0 - 1) / nt0;
    e->ntab = (m + e->W - 1) / e->W;
    const int words = (m + 63) / 64;
    int off = 0;
    for (int t = 0; t < e->ntab; ++t) {
        if ((off >> 6) >= words || (off >> 6) >= PMR_NW) return -1;
        off += e->W;
        if (((off + e->W - 1) >> 6) != (off >> 6)) off = (off & ~63) + 64;
    }
    return 0;
}

/* eregularPreproc's plan (transpositions off: PatMatch's -k letters are
 * i/d/s only, patmatch.py:299-314) */
static int eplan(ectx_t* e, int K) {
    rctx_t* x = e->x;
    const int m = x->m;
    if (K < 1 || K > PME_MAXK) return -1;
    e->m = m;
    e->K = K;
    if (etab_layout(e) < 0) return -1;
    if (find_best(x, K) < 0) return -1;                     /* 0x406d39 */
    e->fbest = x->best;
    const int transp = 0;
    /* levels (0x406db8) */
    rset seen, succ;
    memset(&seen, 0, sizeof seen);
    rs_set(&seen, 0);
    int nlev = 1;
    while (!rs_inter(&seen, &x->final)) {
        ++nlev;
        ereach(x, &seen, &succ);
        rs_or(&seen, &succ);
        if (nlev > m + 2) return -1;
    }
    const int minlen = nlev - 1;
    rset* lev = calloc((size_t)nlev + 1, sizeof(rset));
    rs_set(&lev[0], 0);
    memset(&seen, 0, sizeof seen);
    rs_set(&seen, 0);
    for (int i = 1; i <= minlen; ++i) {                    /* 0x406f69 */
        ereach(x, &seen, &succ);
        for (int q = 0; q < PMR_NW; ++q) lev[i].w[q] = succ.w[q] & ~seen.w[q];
        rs_or(&seen, &succ);
    }
    int pl0 = minlen - K * transp;                         /* 0x406e54 */
    if ((unsigned)pl0 > 64u) pl0 = 64;
    pl0 = pl0 / (K + 1);
    const int PL1 = pl0 + 1;
    double best = 0.78;                                    /* .rodata 0x41d1e8 */
    int chosen = 0;
    rset pieces[PME_MAXK + 1];
    memset(pieces, 0, sizeof pieces);
    if (PL1 > 1 && pl0 != 1 && !(1.0 / (double)pl0 > 0.78)) {
        double* prob = calloc((size_t)m, sizeof(double));
        for (int i = 0; i < m; ++i) {                      /* 0x407031 */
            for (int c = 0; c < 256; ++c)
                if (rs_has(&x->B[c], i)) prob[i] += pmn_letter_prob[c];
        }
        double* A = calloc((size_t)m * PL1, sizeof(double));
        for (int i = 0; i < m; ++i) {
            A[(size_t)i * PL1] = 1.0;
            A[(size_t)i * PL1 + 1] = prob[i];
        }
        for (int l = 2; l < PL1; ++l)                      /* 0x407118 */
            for (int i = 0; i < m; ++i) {
                double s = 0.0;
                for (int j = 0; j < m; ++j)
                    if (rs_has(&x->arrows[i], j)) s += A[(size_t)j * PL1 + l - 1];
                s *= prob[i];
                A[(size_t)i * PL1 + l] = 1.0 < s ? 1.0 : s;
            }
        double* Bt = calloc((size_t)m * PL1 * PL1, sizeof(double));
#define BT(i, l, a) Bt[((size_t)(i) * PL1 + (l)) * PL1 + (a)]
        for (int i = 0; i < m; ++i)
            for (int l = 0; l < PL1; ++l) BT(i, l, 0) = 1.0;
        for (int l = 1; l < PL1; ++l)                      /* 0x4072a0 */
            for (int a = 1; a <= l; ++a)
                for (int i = 0; i < m; ++i) {
                    double v = A[(size_t)i * PL1 + a];
                    if (a < l)
                        for (int j = 0; j < m; ++j)
                            if (rs_has(&x->arrows[i], j)) v = 1.0 - (1.0 - v) * (1.0 - BT(j, l - 1, a));
                    BT(i, l, a) = v;
                }
        double* C = calloc((size_t)nlev * PL1, sizeof(double));
        for (int lv = 0; lv < nlev; ++lv)                  /* 0x40742d */
            for (int l = 0; l < PL1; ++l) {
                double s = 1.0;
                for (int i = 0; i < m; ++i)
                    if (rs_has(&lev[lv], i) && l != 0)
                        for (int a = 1; a <= l; ++a) s += BT(i, l, a);
                C[(size_t)lv * PL1 + l] = s;
            }
#undef BT
        const int W2 = K + 2;
        double* D = calloc((size_t)(nlev + 1) * W2, sizeof(double));
        int* E = calloc((size_t)(nlev + 1) * W2, sizeof(int));
        for (int pl = pl0;;) {                             /* 0x40772e */
            for (int r = 1; r <= nlev; ++r) D[(size_t)r * W2] = 0.0;
            for (int c = 1, esi = nlev - pl; c <= K + 1; ++c, esi -= pl + transp)
                for (int r = (esi < 0 ? 0 : esi) + 1; r <= nlev; ++r) D[(size_t)r * W2 + c] = 1.0;
            for (int c = 1; c <= K + 1; ++c) {             /* 0x407850 */
                const int r11 = nlev - pl - (c - 1) * (pl + transp);
                for (int r = r11; r >= 1; --r) {
                    double v = C[(size_t)r * PL1 + pl];
                    if ((double)(pl + 1) > v) {
                        v = v / ((double)pl - v + 1.0);
                        v = 1.0 < v ? 1.0 : v;             /* minsd */
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
            if (best > D[W2 + K + 1]) {                    /* 0x407a0b */
                int r = 1;
                for (int i = 0, c = K + 1; c >= 1; ++i, --c) {
                    const int s = E[(size_t)r * W2 + c];
                    pieces[i] = lev[s];
                    r = s + pl + transp;
                }
                best = D[W2 + K + 1];
                chosen = pl;
            }
            if (--pl == 1) break;                          /* 0x407ae0 */
            if (!(1.0 / (double)pl <= best)) break;
        }
        free(prob);
        free(A);
        free(Bt);
        free(C);
        free(D);
        free(E);
    }
    free(lev);
    e->pbest = best;
    int use_pieces = 0;
    if (best < 0.78) {                                     /* 0x4082c9 */
        e->pieces_computed = 1;
        for (int i = 0; i <= K; ++i) {
            rset w = pieces[i], last;
            memset(&last, 0, sizeof last);
            for (int st = 0; st < chosen; ++st) {
                ereach(x, &w, &last);
                rs_or(&w, &last);
            }
            e->pwin[i] = w;
            e->pini[i] = pieces[i];
            e->pfin[i] = last;
        }
        if (!(best >= (double)(K + 1) * 1.3 * e->fbest) && chosen != 0) use_pieces = 1;   /* 0x40842a */
    }
    if (use_pieces) {
        e->etype = 1;
        e->ell = chosen;
        e->npieces = K + 1;
    } else {                                               /* 0x407bb9 */
        e->etype = x->ell == 0 ? 3 : 2;
        e->ell = x->ell;
        e->npieces = 1;
        e->pwin[0] = x->win;
        e->pini[0] = x->winit;
        e->pfin[0] = x->wfinal;
    }
    e->cls = det_class1(x, 0, &e->pwin[0]);                /* 0x407c97 */
    e->defined = 1;
    for (int i = 0; i < PMR_MAXS; ++i) e->unmap[i] = -1;
    if (e->cls == 1) {                                     /* 0x407e4b */
        const int nw = (e->etype == 1 || e->pieces_computed) ? K + 1 : 1;
        if (nw < K + 1) e->defined = 0;
        e->match0 = 0;
        for (int i = 0; i < nw; ++i) {
            int f = 0;
            while (f < m && !rs_has(&e->pwin[i], f)) ++f;
            e->first[i] = f;
            /* 0x407ef0 / 0x407f39: shl %cl (the count taken mod 64) */
            if (e->ell != 0) e->match0 |= 1ull << (f & 63);
            else {
                int r = f + 1;
                while (r < m && rs_has(&e->pwin[i], r)) ++r;
                e->match0 |= 1ull << (r & 63);
            }
        }
        e->nstates = m;                                    /* P->0x858[i] = i, i < P->0x20 (0x407f67) */
        for (int i = 0; i < m; ++i) e->unmap[i] = i;
    } else if (e->cls == 3) {                              /* 0x407fe9 */
        rset uw, ui, uf;
        memset(&uw, 0, sizeof uw);
        memset(&ui, 0, sizeof ui);
        memset(&uf, 0, sizeof uf);
        for (int i = 0; i < e->npieces; ++i) {
            rs_or(&uw, &e->pwin[i]);
            rs_or(&ui, &e->pini[i]);
            rs_or(&uf, &e->pfin[i]);
        }
        x->win = uw;
        x->winit = ui;
        x->wfinal = uf;
        x->ell = e->ell;
        if (load_fast(x) < 0) return -1;
        e->nstates = x->mp;
        for (int s = 0; s < m; ++s)
            if (rs_has(&uw, s)) e->unmap[x->map[s]] = s;   /* 0x40807f */
    }
    return 0;
}

/* ------------------------------------------------------------------------
 * fwdCheck 0x403310 / bwdCheck 0x403df0 with K + 1 rows of state sets (the
 * transitions through the sliced tables: etab); *kio: the budget in, the
 * errors used out.  -1: none.
 * ---------------------------------------------------------------------- */

static inline void rs_and(rset* d, const rset* s) { for (int q = 0; q < PMR_NW; ++q) d->w[q] &= s->w[q]; }

static int64_t efwd(const ectx_t* e, int64_t p, int64_t lim, int s, int* kio) {
    const rctx_t* x = e->x;
    const int K = *kio, ins = e->errs & PME_INS, del = e->errs & PME_DEL, sub = e->errs & PME_SUB;
    rset rows[PME_MAXK + 1], T;
    memset(&rows[0], 0, sizeof(rset));
    rs_set(&rows[0], s);
    if (rs_inter(&rows[0], &x->final)) {                   /* 0x40339d: insertions to the right context */
        *kio = 0;
        for (int64_t q = p + 1;; ++q) {
            if (right_ok(x, q, lim + 1)) return q - 1;
            if (q == lim + 1 || !ins) return -1;
            if (++*kio > K) return -1;
        }
    }
    int kmax = K;
    int64_t best = -1;
    for (int j = 1; j <= kmax; ++j) {                      /* 0x4034c0 */
        rows[j] = rows[j - 1];                             /* (unset in the binary without OptDel: see the header) */
        if (!del) continue;
        etab(e, x->arrows, &rows[j - 1], &T);
        rs_or(&rows[j], &T);
        if (rs_inter(&rows[j], &x->final) && right_ok(x, p + 1, lim + 1)) {   /* 0x403d82 */
            *kio = j;
            kmax = j - 1;
            best = p;
        }
    }
    if (p == lim) return best;
    for (int64_t cur = p;;) {
        ++cur;
        const rset* bc = &x->B[x->t[cur]];
        rset n0;
        etab(e, x->arrows, &rows[0], &n0);
        rs_and(&n0, bc);
        if (rs_inter(&n0, &x->final) && right_ok(x, cur + 1, lim + 1)) {
            *kio = 0;
            return cur;
        }
        rset oldp = rows[0], last = n0;
        rows[0] = n0;
        for (int j = 1; j <= kmax; ++j) {                  /* 0x4037a0 */
            rset v;
            memset(&v, 0, sizeof v);
            if (del) etab(e, x->arrows, &last, &v);
            if (ins) rs_or(&v, &oldp);
            if (sub) {
                etab(e, x->arrows, &oldp, &T);
                rs_or(&v, &T);
            }
            etab(e, x->arrows, &rows[j], &T);
            rs_and(&T, bc);
            rs_or(&v, &T);
            const rset oj = rows[j];
            rows[j] = v;
            last = v;
            if (rs_inter(&v, &x->final) && right_ok(x, cur + 1, lim + 1)) {   /* 0x403a01: the fewest errors */
                int c = j;
                while (c - 1 >= 0 && rs_inter(&rows[c - 1], &x->final)) --c;
                if (c == 0) {
                    *kio = 0;
                    return cur;
                }
                *kio = c;
                kmax = c - 1;
                best = cur;
                break;
            }
            oldp = oj;
        }
        if (!rs_any(&last)) return best;                   /* 0x403afc */
        if (cur == lim) return best;
    }
}

static int64_t ebwd(const ectx_t* e, int64_t p, int64_t lim, int s, int* kio) {
    const rctx_t* x = e->x;
    const int K = *kio, ins = e->errs & PME_INS, del = e->errs & PME_DEL, sub = e->errs & PME_SUB;
    rset rows[PME_MAXK + 1], T;
    memset(&rows[0], 0, sizeof(rset));
    rs_set(&rows[0], s);
    if (rs_has(&rows[0], 0)) {                             /* 0x403e71: insertions to the left context */
        *kio = 0;
        for (int64_t q = p;;) {
            if (left_ok(x, q, lim)) return q;
            if (q == lim) return -1;
            --q;
            if (!ins) return -1;
            if (++*kio > K) return -1;
        }
    }
    int kmax = K;
    int64_t best = -1;
    for (int j = 1; j <= kmax; ++j) {                      /* 0x403f80 */
        rows[j] = rows[j - 1];
        if (!del) continue;
        etab(e, x->rev, &rows[j - 1], &T);
        rs_or(&rows[j], &T);
        if (rs_has(&rows[j], 0) && left_ok(x, p, lim)) {   /* 0x40484e */
            *kio = j;
            kmax = j - 1;
            best = p;
        }
    }
    if (p == lim) return best;
    for (int64_t cur = p;;) {
        --cur;
        const rset* bc = &x->B[x->t[cur]];
        rset n0, a = rows[0];
        rs_and(&a, bc);
        etab(e, x->rev, &a, &n0);
        if (rs_has(&n0, 0) && left_ok(x, cur, lim)) {
            *kio = 0;
            return cur;
        }
        rset oldp = rows[0], last = n0;
        rows[0] = n0;
        for (int j = 1; j <= kmax; ++j) {                  /* 0x404230 */
            rset v;
            memset(&v, 0, sizeof v);
            if (del) etab(e, x->rev, &last, &v);
            if (ins) rs_or(&v, &oldp);
            if (sub) {
                etab(e, x->rev, &oldp, &T);
                rs_or(&v, &T);
            }
            a = rows[j];
            rs_and(&a, bc);
            etab(e, x->rev, &a, &T);
            rs_or(&v, &T);
            const rset oj = rows[j];
            rows[j] = v;
            last = v;
            if (rs_has(&v, 0) && left_ok(x, cur, lim)) {   /* 0x404479 */
                int c = j;
                while (c - 1 >= 0 && rs_has(&rows[c - 1], 0)) --c;
                if (c == 0) {
                    *kio = 0;
                    return cur;
                }
                *kio = c;
                kmax = c - 1;
                best = cur;
                break;
            }
            oldp = oj;
        }
        if (!rs_any(&last)) return best;                   /* 0x404579 */
        if (cur == lim) return best;
    }
}

/* checkMatch 0x406010 */
static int echeck(const ectx_t* e, int64_t pos, int64_t R, uint64_t match, int64_t* mb, int64_t* me) {
    const rctx_t* x = e->x;
    const int64_t rp = e->etype == 3 ? pos - 1 : pos;
    int64_t lo = 0, hi = x->nnl;
    while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if (x->nl[mid] < rp) lo = mid + 1; else hi = mid;
    }
    int64_t rb = R;
    if (lo > 0 && x->nl[lo - 1] >= R) rb = x->nl[lo - 1] + 1;
    const int64_t re = lo < x->nnl ? x->nl[lo] : x->n;
    if (rp < rb || rp >= re) return 0;
    /* 0x4060b9: every i < P->0x24, its bit tested by `bt %rbx` (the bit
     * number taken mod 64: class 1 over more than 64 states tries the states
     * i, i + 64, ... of each set bit) */
    for (int i = 0; i < e->nstates; ++i) {
        if (!((match >> (i & 63)) & 1) || e->unmap[i] < 0) continue;
        const int s = e->unmap[i];
        int k1 = e->K, k2;
        int64_t st, en;
        if (e->etype != 3) {
            en = efwd(e, pos, re - 1, s, &k1);
            if (en < 0) continue;
            k2 = e->K - k1;
            st = ebwd(e, pos + 1, rb, s, &k2);
            if (st < 0) return 0;                          /* 0x406248 */
        } else {                                           /* 0x406320 */
            st = ebwd(e, pos, rb, s, &k1);
            if (st < 0) continue;
            k2 = e->K - k1;
            en = efwd(e, pos - 1, re - 1, s, &k2);
            if (en < 0) return 0;
        }
        *mb = st;
        *me = en + 1;
        return 1;
    }
    return 0;
}

/* ------------------------------------------------------------------------
 * eregularScan 0x4048b0 (class 3) and esimpleScan 0x4136d0 (class 1) over
 * the region [R, n)
 * ---------------------------------------------------------------------- */

/* type 1: the pieces exactly (0x4052b9) */
static int escan_pieces3(const ectx_t* e, int64_t R, int64_t* mb, int64_t* me) {
    const rctx_t* x = e->x;
    const int ell = e->ell;
    const uint8_t* t = x->t;
    int64_t pos = R - 1;
    const int64_t lim = x->n - ell;
    while (pos < lim) {
        uint64_t rcx = x->A[t[pos + ell]];
        if (!rcx) {
            pos += ell;
            continue;
        }
        uint64_t D = 0;
        int64_t c = pos + ell - 1;
        int dead = 0;
        for (;;) {
            D = rcx & x->Bw[t[c]];
            rcx = wtrans(x->rw, x->mp, D);
            if (!rcx) {
                dead = 1;
                break;
            }
            if (--c == pos) break;
        }
        if (dead) {
            pos = c;
            continue;
        }
        if ((rcx & x->ffinal) && echeck(e, pos + 1, R, D, mb, me)) return 1;
        ++pos;
    }
    return 0;
}

/* type 2: bwdScanrk 0x402d50 */
static int escan_backward(const ectx_t* e, int64_t R, int64_t* mb, int64_t* me) {
    const rctx_t* x = e->x;
    const int K = e->K, W = e->ell - K;
    const uint8_t* t = x->t;
    uint64_t rows[PME_MAXK + 1], old[PME_MAXK + 1];
    int64_t pos = R - 1;
    const int64_t lim = x->n - W;
    while (pos < lim) {                                    /* 0x402f21 */
        const uint8_t c0 = t[pos + W];
        uint64_t bprev = x->Bw[c0];
        rows[0] = x->A[c0];
        for (int j = 1; j <= K; ++j) rows[j] = x->finit;
        for (int j = 0; j <= K; ++j) old[j] = x->finit;
        int64_t cur = pos + W - 1;
        for (;;) {                                         /* 0x403044 */
            const uint64_t bc = x->Bw[t[cur]];
            uint64_t po = rows[0];
            uint64_t pn = wtrans(x->rw, x->mp, bc & po);
            rows[0] = pn;
            for (int j = 1; j <= K; ++j) {                 /* 0x4030d0 */
                const uint64_t r10 = pn | po;
                const uint64_t oj = rows[j];
                uint64_t v = po | wtrans(x->rw, x->mp, r10) | wtrans(x->rw, x->mp, bc & oj);
                const uint64_t tr = wtrans(x->rw, x->mp, bc & old[j - 1]) & bprev;
                v |= wtrans(x->rw, x->mp, tr);
                old[j - 1] = po;
                rows[j] = v;
                po = oj;
                pn = v;
            }
            if (!pn) {                                     /* 0x403230: dead */
                pos = cur;
                break;
            }
            if (--cur == pos) {                            /* 0x4031ed */
                if ((pn & x->ffinal) && echeck(e, pos + 1, R, po, mb, me)) return 1;
                ++pos;
                break;
            }
            bprev = bc;
        }
    }
    return 0;
}

/* type 3: fwdScanrk 0x402830 */
static int escan_forward(const ectx_t* e, int64_t R, int64_t* mb, int64_t* me) {
    const rctx_t* x = e->x;
    const int K = e->K;
    const uint8_t* t = x->t;
    const int64_t n = x->n;
    uint64_t rows[PME_MAXK + 1], old[PME_MAXK + 1];
    int64_t cur = R;
    for (;;) {
        /* a record start (0x4028db): the next character that is not '\n' */
        if (cur >= n) return 0;
        uint8_t c = t[cur++];
        while (c == '\n') {
            if (cur == n) return 0;
            c = t[cur++];
        }
        uint64_t s = x->finit;                             /* 0x402911 */
        rows[0] = old[0] = s;
        for (int j = 1; j <= K; ++j) {
            s |= wtrans(x->fw, x->mp, s);
            rows[j] = old[j] = s;
        }
        uint64_t bc = x->Bw[c];
        uint64_t po = rows[0], pn = wtrans(x->fw, x->mp, po) & bc;
        rows[0] = pn;
        for (int j = 1; j <= K; ++j) {                     /* 0x402a31 */
            const uint64_t r = pn | po;
            const uint64_t oj = rows[j];
            const uint64_t v = r | (wtrans(x->fw, x->mp, oj) & bc) | wtrans(x->fw, x->mp, r);
            rows[j] = v;
            po = oj;
            pn = v;
        }
        if (cur >= n) return 0;
        uint64_t bprev = bc;
        if ((pn & x->ffinal) && echeck(e, cur, R, pn & x->ffinal, mb, me)) return 1;
        for (;;) {                                         /* 0x402ac0 */
            c = t[cur++];
            if (c == '\n') break;
            bc = x->Bw[c];
            po = rows[0];
            pn = wtrans(x->fw, x->mp, po) & bc;
            rows[0] = pn;
            for (int j = 1; j <= K; ++j) {                 /* 0x402b68 */
                const uint64_t r10 = pn | po;
                const uint64_t oj = rows[j];
                uint64_t v = po | (wtrans(x->fw, x->mp, oj) & bc) | wtrans(x->fw, x->mp, r10);
                const uint64_t tr = wtrans(x->fw, x->mp, old[j - 1]) & bc;
                v |= wtrans(x->fw, x->mp, tr) & bprev;
                old[j - 1] = po;
                rows[j] = v;
                po = oj;
                pn = v;
            }
            if (cur == n) return 0;                        /* 0x402c3c */
            if ((pn & x->ffinal) && echeck(e, cur, R, pn & x->ffinal, mb, me)) return 1;
            bprev = bc;
        }
    }
}

/* class 1, type 1: esimpleScan's multi-piece BNDM (0x413780) over the
 * pieces' states first[r] .. first[r] + pl - 1 (esimpleLoadFast 0x4153fa) */
static int escan_pieces1(const ectx_t* e, int64_t R, int64_t* mb, int64_t* me) {
    const rctx_t* x = e->x;
    const int mpc = e->ell, np = e->K + 1;
    uint64_t T0[256], T2[256];
    for (int c = 0; c < 256; ++c) {
        T0[c] = T2[c] = 0;
        for (int r = 0; r < np; ++r)
            for (int pp = 0; pp < mpc; ++pp) {
                const int st = e->first[r] + mpc - 1 - pp;
                if (st < e->m && rs_has(&x->B[c], st)) {
                    const uint64_t bit = 1ull << (r * mpc + pp);
                    T0[c] |= bit;
                    if (pp > 0) T2[c] |= bit;
                }
            }
    }
    const uint8_t* t = x->t;
    int64_t r9 = R - 1;
    const int64_t limit = x->n - mpc;
    while (r9 < limit) {
        uint64_t D = T0[t[r9 + mpc]];
        if (!D) {
            r9 += mpc;
            continue;
        }
        int64_t a = r9 + mpc - 1;
        int k = mpc - 1;
        do {
            D = (D << 1) & T2[t[a]];
            --k;
            --a;
        } while (D && k);
        if (D) {
            for (int i = 0; i < np; ++i) {                 /* 0x41384b: 32-bit shift */
                const int bit = i * mpc + mpc - 1;
                const uint64_t msk = (uint64_t)(int64_t)(int32_t)(1u << (bit & 31));
                if ((D & msk) && echeck(e, r9 + 1, R, e->match0, mb, me)) return 1;
            }
        }
        r9 += k + 1;
    }
    return 0;
}

/* class 1, type 2: esimpleScan's ABNDM (0x413b6f) over the window's states
 * first .. first + ell - 1 (simpleLoadFast 0x417561) */
static int escan_window1(const ectx_t* e, int64_t R, int64_t* mb, int64_t* me) {
    const rctx_t* x = e->x;
    const int beg = e->first[0], Lw = e->ell, k = e->K;
    uint64_t T[256];
    for (int c = 0; c < 256; ++c) {
        T[c] = 0;
        for (int r = 0; r < Lw; ++r) {
            const int st = beg + Lw - 1 - r;
            if (st < e->m && rs_has(&x->B[c], st)) T[c] |= 1ull << (64 - Lw + r);
        }
    }
    const uint64_t top = ~0ull << (64 - Lw);
    const int W = Lw - k;
    const int64_t limit = x->n - (Lw - k - 1);
    uint64_t Rr[PME_MAXK + 1], Tr[PME_MAXK + 1];
    const uint8_t* t = x->t;
    for (int64_t s = R; s < limit;) {
        const uint64_t b0 = T[t[s + W - 1]];
        Rr[0] = b0;
        for (int j = 1; j <= k; ++j) {
            Rr[j] = top;
            Tr[j] = b0;
        }
        int64_t rb = W - 2;
        for (;;) {
            const uint64_t bc = T[t[s + rb]];
            uint64_t oldp = Rr[0];
            uint64_t newp = (oldp << 1) & bc;
            Rr[0] = newp;
            for (int j = 1; j <= k; ++j) {
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
                if ((Rr[k] >> 63) && echeck(e, s, R, e->match0, mb, me)) return 1;
                break;
            }
            if (!Rr[k] && !Tr[k]) break;
            --rb;
        }
        s += rb + 1;
    }
    return 0;
}

static ectx_t* ectx_new(const int32_t* tree, const int32_t* nullable, int nodes, const uint64_t* Bpos, int npos,
                        int icase, int mode, int K, int errs) {
    ectx_t* e = calloc(1, sizeof(ectx_t));
    if (!e) return NULL;
    e->x = calloc(1, sizeof(rctx_t));
    if (!e->x) {
        free(e);
        return NULL;
    }
    e->x->mode = mode;
    e->errs = errs;
    if (build(e->x, tree, nodes, nullable, Bpos, npos, icase) < 0 || eplan(e, K) < 0) {
        ctx_free(e->x);
        free(e);
        return NULL;
    }
    return e;
}

static void ectx_free(ectx_t* e) {
    ctx_free(e->x);
    free(e);
}

/* out[0] = type (1 pieces, 2 backward window, 3 forward), out[1] = the
 * pieces' length or the window's ell, out[2] = detClass of windows[0],
 * out[3] = P->0x24, out[4] = 1 unless nrgrep reads memory it never wrote,
 * out[5] = the number of windows; masks[(3 i + j) PMR_NW ..] (PMR_NW words
 * each) = window i, its initial and its final states (j = 0, 1, 2);
 * masks[51 PMR_NW] = P->0x28 (class 1) */
int pmr_eplan(const int32_t* tree, const int32_t* nullable, int nodes, const uint64_t* Bpos, int npos, int icase,
              int K, int errs, int* out, uint64_t* masks) {
    ectx_t* e = ectx_new(tree, nullable, nodes, Bpos, npos, icase, 0, K, errs);
    if (!e) return -1;
    out[0] = e->etype;
    out[1] = e->ell;
    out[2] = e->cls;
    out[3] = e->nstates;
    out[4] = e->defined;
    out[5] = e->npieces;
    for (int i = 0; i < e->npieces; ++i)
        for (int q = 0; q < PMR_NW; ++q) {
            masks[(3 * i) * PMR_NW + q] = e->pwin[i].w[q];
            masks[(3 * i + 1) * PMR_NW + q] = e->pini[i].w[q];
            masks[(3 * i + 2) * PMR_NW + q] = e->pfin[i].w[q];
        }
    masks[3 * (PME_MAXK + 1) * PMR_NW] = e->match0;
    ectx_free(e);
    return 0;
}

/* What nrgrep_coords prints for a class-3 pattern at k = K > 0 over one
 * region (recSearchFile 0x402250).  errs: 1 insertions, 2 deletions, 4
 * substitutions.  Returns the number of matches (may exceed cap), -1 if
 * refused (a window union of more than 64 states, or a table slice past the
 * state set's words). */
int64_t pmr_eregular(const uint8_t* text, int64_t n, const int32_t* tree, const int32_t* nullable, int nodes,
                     const uint64_t* Bpos, int npos, int icase, int mode, int K, int errs, int64_t* out_beg,
                     int64_t* out_end, int64_t cap) {
    ectx_t* e = ectx_new(tree, nullable, nodes, Bpos, npos, icase, mode, K, errs);
    if (!e) return -1;
    if (e->cls == 2) {                                     /* 0x4081ed: the process dies before the scan */
        ectx_free(e);
        return 0;
    }
    rctx_t* x = e->x;
    x->t = text;
    x->n = n;
    int64_t nnl = 0;
    for (int64_t p = 0; p < n; ++p) nnl += text[p] == '\n';
    int64_t* nl = malloc(sizeof(int64_t) * (size_t)(nnl + 1));
    nnl = 0;
    for (int64_t p = 0; p < n; ++p)
        if (text[p] == '\n') nl[nnl++] = p;
    x->nl = nl;
    x->nnl = nnl;
    int64_t count = 0, R = 0;
    while (R < n) {
        int64_t mb = 0, me = 0;
        int ok;
        if (e->cls == 1) ok = e->etype == 1 ? escan_pieces1(e, R, &mb, &me) : escan_window1(e, R, &mb, &me);
        else if (e->etype == 1) ok = escan_pieces3(e, R, &mb, &me);
        else if (e->etype == 2) ok = escan_backward(e, R, &mb, &me);
        else ok = escan_forward(e, R, &mb, &me);
        if (!ok) break;
        if (count < cap) {
            out_beg[count] = mb;
            out_end[count] = me;
        }
        ++count;
        if (me == n) break;
        R = me;
    }
    free(nl);
    ectx_free(e);
    return count;
}
