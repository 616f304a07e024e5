/*
 * pm_nrgrep_ext.c -- nrgrep's extended engine at k = 0 (class 2: a sequence
 * of classes each with an optional '?', '*' or '+'), the engine nrgrep_coords
 * runs for every PatMatch pattern with a range X{m,n} (patmatch_to_nrgrep.pl
 * :476-486 unrolls it into X..?.?) -- e.g. configs[3]'s PROSITE
 * C-x(2,4)-C-x(3)-[LIVMFYWC].
 *
 * TEST INFRASTRUCTURE ONLY (like pm_oracle.c / pm_nrgrep.c): only tests/,
 * smoke() and bench.py's cpu_baseline leg may load it, and only as the
 * checker.
 *
 * Round 4: restated from the binary's disassembly (www/bin/nrgrep_coords,
 * `objdump -d`, never executed).  This file simulates the binary's loops
 * literally; the GPU engine (pm_extended.hip) replays the same loops per
 * cluster of candidate starts, and tests compare the two.
 *
 *   searchPreproc 0x4026b7: detClass == 2, OptErrors == 0 -> extendedPreproc
 *   extendedPreproc 0x413260:
 *     extendedLoadMasks 0x412af0 / extendedTreeLoad 0x411970: B[c] (classes),
 *       A[c] (repeatable positions: '+', '*'), S (optional: '?', '*')
 *     extendedFindBest 0x411fe0: a window [beg, end) of the pattern priced by
 *       letterProb (.data 0x621120), best < 0.7; none -> the prefix [0, end)
 *     window found: type 2, L = beg; else type 3, L = end        (0x41337a)
 *     extendedLoadVerif 0x412c60: the left part [0, L) reversed and the
 *       right part [L, m) as bit-parallel tables with the optional-block
 *       masks I, F, S and the initial state X
 *     detClass over the window's positions (0x413485): with no '?*+' in it
 *       simpleLoadFast 0x417520 + simpleScan 0x416600, else
 *       extendedLoadFast 0x413060 + extendedScan 0x4116f0
 *   extendedSearch 0x4136b0: P->scan(beg, end, checkMatch 0x411aa0, P, fast)
 *
 * Quirks restated as they are:
 *   - checkMatch starts each phase from the state X (the part's first
 *     position when it is optional) without the optional-block closure, so
 *     two or more optional positions right next to the candidate cannot all
 *     be skipped before the first character is read: C..?.?C read back from
 *     the second C never takes the two '.?' as empty (0x411bfa, 0x411e1f).
 *   - the prefix scanner of a prefix with no '?*+' (simpleScan, forward)
 *     hands checkMatch the START of the prefix occurrence (r15 at 0x4166a2),
 *     which checkMatch takes as the prefix END (type 3: the record of
 *     pos - 1, the left part read back from pos).
 *   - extendedLoadFast / extendedLoadVerif mark the position before an
 *     optional block at bit b - 1; for b = 0 that is bit 63 (a 64-bit shift
 *     by -1 & 63).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PMX_NW 4            /* 64-bit words per position set: 256 positions */
#define PMX_START 2         /* '^' (OptStartLine) */
#define PMX_END 4           /* '$' (OptEndLine) */

extern const double pmn_letter_prob[256];   /* pm_nrgrep.c: letterProb, .data 0x621120 */

static inline uint8_t fold(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }
static inline int isset(const uint64_t* w, int i) { return (int)((w[i >> 6] >> (i & 63)) & 1); }
static inline void setb(uint64_t* w, int i) { w[i >> 6] |= 1ull << (i & 63); }

typedef struct {
    int len;                         /* positions of the part */
    uint64_t B[256][PMX_NW], A[256][PMX_NW];
    uint64_t I[PMX_NW], F[PMX_NW], S[PMX_NW], X[PMX_NW];
} xpart_t;

typedef struct {
    const uint8_t* t;
    int64_t n;
    int m, icase, mode;
    const uint64_t* Bp;              /* [256][PMX_NW] class of each folded byte */
    uint64_t opt[PMX_NW], rep[PMX_NW];
    /* plan */
    int win, beg, end, type, L, simple;
    /* scanner tables (one word) */
    int len;
    uint64_t T[256], TA[256], fI, fF, fS;
    /* verification: [0] left (reversed), [1] right */
    xpart_t v[2];
    const int64_t* nl;
    int64_t nnl;
} xctx_t;

/* B[c] / A[c] as extendedLoadMasks builds them: -i gives a class both cases,
 * i.e. the text byte's folded value indexes the table */
static inline int cls_has(const xctx_t* x, int c, int p) {
    return isset(x->Bp + (size_t)(x->icase ? fold((uint8_t)c) : c) * PMX_NW, p);
}
static inline int rep_has(const xctx_t* x, int c, int p) { return isset(x->rep, p) && cls_has(x, c, p); }

/* ------------------------------------------------------------------------
 * extendedFindBest 0x411fe0 (K = 0 here: extendedPreproc passes r8d = 0)
 * ---------------------------------------------------------------------- */
static double find_best(const xctx_t* x, int K, int* fwd, int* beg, int* end) {
    const int m = x->m;
    double* prob = calloc((size_t)m, sizeof(double));
    double* aprob = calloc((size_t)m, sizeof(double));
    for (int i = 0; i < m; ++i)                          /* 0x412058 */
        for (int c = 0; c < 256; ++c) {
            if (cls_has(x, c, i)) prob[i] += pmn_letter_prob[c];
            if (rep_has(x, c, i)) aprob[i] += pmn_letter_prob[c];
        }
    /* P1 / P2: the binary's [m + 1][m][m + 1], idx(a, b, c) = a m (m + 1) +
     * b (m + 1) + c; c (t) never exceeds 64, so the last index holds
     * min(m, 64) + 1 slots here (same values, less memory at m = 256) */
    const size_t M1 = (size_t)(m < 64 ? m : 64) + 1, MM = (size_t)m * M1;
    double* P1 = malloc(sizeof(double) * MM * ((size_t)m + 1));
    double* P2 = malloc(sizeof(double) * MM * ((size_t)m + 1));
    int* pos = calloc((size_t)m, sizeof(int));
#define IDX(a, b, c) ((size_t)(a) * MM + (size_t)(b) * M1 + (size_t)(c))
    for (int i = 0; i < m; ++i) {                        /* 0x412168 */
        for (int t = 0; t <= i; ++t) P1[IDX(t, i, 0)] = P2[IDX(t, i, 0)] = 1.0;
        P1[IDX(i + 1, i, 0)] = P2[IDX(i + 1, i, 0)] = 0.0;
    }
    double best = 0.7;                                   /* 0x41d410 */
    *fwd = 0;
    *beg = 0;
    *end = 0;
    for (int i = 0; i < m; ++i) {                        /* 0x412260 */
        int len = 0;
        for (int j = i; j < m; ++j) {                    /* 0x412345 */
            if ((unsigned)(j - i + 1) > 64u) continue;
            if (!isset(x->opt, j)) {
                ++len;
                if (len <= 2 * K) continue;
            } else if (2 * K >= len) {
                continue;
            }
            double sum = (double)K + 1.0;                /* 0x412389 / 0x412729 */
            const int lk = len - K;
            const double lim = (double)(lk + 1);
            if (!(sum >= lim)) {
                const double dlk = (double)lk;
                double q = sum / ((dlk - sum) + 1.0);
                if (!(q >= best)) {
                    for (int t = 1;;) {                  /* 0x4124a8 */
                        if (pos[j] < t) {
                            P2[IDX(j + 1, j, t)] = 0.0;
                            P1[IDX(j + 1, j, t)] = 0.0;
                            for (int l = j; l >= 0; --l) {   /* 0x412595 */
                                double v = prob[l] * P1[IDX(l + 1, j, t - 1)] + aprob[l] * P1[IDX(l, j, t - 1)];
                                v = isset(x->opt, l) ? P1[IDX(l + 1, j, t)] + v : 0.0 + v;
                                double r;
                                if (v > 1.0) {
                                    P1[IDX(l, j, t)] = 1.0;
                                    r = 0.0;
                                } else {
                                    P1[IDX(l, j, t)] = v;
                                    r = 1.0 - v;
                                }
                                P2[IDX(l, j, t)] = 1.0 - (1.0 - P2[IDX(l + 1, j, t)]) * r;
                            }
                            pos[j] = t;
                        }
                        sum = sum + P2[IDX(i, j, t)];    /* 0x41261b */
                        ++t;
                        if (t > len) break;
                        if (sum >= lim) break;
                        q = sum / ((dlk - sum) + 1.0);
                        if (!(q < best)) break;
                    }
                }
            }
            if (lim > sum) {                             /* 0x41268d */
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
#undef IDX
    free(prob);
    free(aprob);
    free(P1);
    free(P2);
    free(pos);
    if (*fwd > 0) {                                      /* 0x4127f9: trim optional ends */
        while (*beg < *end && isset(x->opt, *beg)) ++*beg;
        while (*beg < *end && isset(x->opt, *end - 1)) --*end;
        if (*beg == *end) *fwd = 0;
        else return best;
    }
    if (*fwd == 0) {                                     /* 0x4128d4: the prefix */
        *end = m <= 64 ? m : 64;
        while (*end > 0 && isset(x->opt, *end - 1)) --*end;
        return 1.0;
    }
    return best;
}

/* extendedLoadVerif 0x412c60: `len` positions from pattern position p0
 * stepping dir; an optional position after a non-optional one opens a
 * block (I = the bit before it, F = its last bit, S its bits), the part's
 * first position goes to X when optional (0x41301d) */
static void load_verif(const xctx_t* x, xpart_t* v, int len, int p0, int dir) {
    memset(v, 0, sizeof(*v));
    v->len = len;
    int opened = 0;
    for (int r = 0; r < len; ++r) {
        const int p = p0 + r * dir;
        for (int c = 0; c < 256; ++c) {
            if (cls_has(x, c, p)) setb(v->B[c], r);
            if (rep_has(x, c, p)) setb(v->A[c], r);
        }
        if (!isset(x->opt, p)) continue;
        if (r > 0) {
            if (isset(v->F, r - 1)) {                    /* 0x412ff1: the block goes on */
                v->F[(r - 1) >> 6] &= ~(1ull << ((r - 1) & 63));
                setb(v->F, r);
            } else {
                setb(v->I, r - 1);
                setb(v->F, r);
                opened = 1;
                setb(v->S, r);
                continue;
            }
        }
        if (opened) setb(v->S, r);                       /* 0x413015 */
        else setb(v->X, r);
    }
}

/* extendedLoadFast 0x413060 (window: win != 0, bits top-aligned and
 * reversed) or simpleLoadFast 0x417520 */
static void load_fast(xctx_t* x) {
    const int len = x->len;
    memset(x->T, 0, sizeof(x->T));
    memset(x->TA, 0, sizeof(x->TA));
    x->fI = x->fF = x->fS = 0;
    if (x->simple) {
        if (x->win) {                                    /* 0x417561 */
            for (int r = 0; r < len; ++r)
                for (int c = 0; c < 256; ++c)
                    if (cls_has(x, c, x->end - 1 - r)) x->T[c] |= 1ull << (64 - len + r);
        } else {                                         /* 0x417615: shift-or */
            const uint64_t full = len == 64 ? ~0ull : (1ull << len) - 1;
            for (int c = 0; c < 256; ++c) x->T[c] = full;
            for (int r = 0; r < len; ++r)
                for (int c = 0; c < 256; ++c)
                    if (cls_has(x, c, x->beg + r)) x->T[c] &= ~(1ull << r);
        }
        return;
    }
    const int step = x->win ? -1 : 1;
    int b = x->win ? 64 - len : 0;
    int p = x->win ? x->end - 1 : x->beg;
    for (int r = 0; r < len; ++r, ++b, p += step) {      /* 0x413168 */
        const uint64_t bit = 1ull << b;
        for (int c = 0; c < 256; ++c) {
            if (cls_has(x, c, p)) x->T[c] |= bit;
            if (rep_has(x, c, p)) x->TA[c] |= bit;
        }
        if (isset(x->opt, p)) {
            const int pb = (b - 1) & 63;
            const uint64_t pbit = 1ull << pb;
            x->fS |= bit;
            if ((x->fF >> pb) & 1) {
                x->fF = (x->fF & ~pbit) | bit;
            } else {
                x->fI |= pbit;
                x->fF |= bit;
            }
        }
    }
}

/* the window (or prefix) holds a '?', '*' or '+' (detClass over its
 * positions, 0x413485) */
static int window_extended(const xctx_t* x) {
    for (int p = x->beg; p < x->end; ++p)
        if (isset(x->opt, p) || isset(x->rep, p)) return 1;
    return 0;
}

/* ------------------------------------------------------------------------
 * checkMatch 0x411aa0
 * ---------------------------------------------------------------------- */
static int left_ok(const xctx_t* x, int64_t p, int64_t recbeg) {
    return !((x->mode & PMX_START) && p > recbeg && x->t[p - 1] != '\n');
}
static int right_ok(const xctx_t* x, int64_t q, int64_t recend) {
    return !((x->mode & PMX_END) && q < recend && x->t[q] != '\n');
}

/* one step of a phase: D = ((D << 1 | carry) & B[c]) | (D & A[c]); returns
 * whether D is not empty */
static int step(uint64_t* D, int W, const xpart_t* v, uint8_t c, uint64_t carry) {
    int any = 0;
    for (int w = 0; w < W; ++w) {
        const uint64_t old = D[w];
        D[w] = (((old << 1) | carry) & v->B[c][w]) | (old & v->A[c][w]);
        any |= D[w] != 0;
        carry = old >> 63;
    }
    return any;
}

/* D |= S & ((D | F) ^ ~((D | F) - I)), multiword with a borrow (0x411d58) */
static void closure(uint64_t* D, int W, const xpart_t* v) {
    uint64_t borrow = 0;
    for (int w = 0; w < W; ++w) {
        const uint64_t d = D[w], xx = d | v->F[w];
        const uint64_t sub = xx - borrow - v->I[w];
        D[w] = ((~sub ^ xx) & v->S[w]) | d;
        const uint64_t bi = borrow + v->I[w];
        borrow = (bi < borrow) | (xx < bi);
    }
}

static int check_match(const xctx_t* x, int64_t pos, int64_t R, int64_t* mb, int64_t* me) {
    const int64_t rp = x->type == 3 ? pos - 1 : pos;
    /* recGetRecord 0x402030: the last '\n' before rp (back to R only), the
     * first at or after it */
    int64_t lo = 0, hi = x->nnl;
    while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if (x->nl[mid] < rp) lo = mid + 1; else hi = mid;
    }
    int64_t recbeg = R;
    if (lo > 0 && x->nl[lo - 1] >= R) recbeg = x->nl[lo - 1] + 1;
    const int64_t recend = lo < x->nnl ? x->nl[lo] : x->n;
    if (rp < recbeg || rp >= recend) return 0;
    int64_t start;
    const xpart_t* lv = &x->v[0];
    if (lv->len == 0) {                                  /* 0x411b48 */
        if (!left_ok(x, pos, recbeg)) return 0;
        start = pos;
    } else {
        const int W = (lv->len + 63) >> 6;
        const uint64_t fin = 1ull << ((lv->len - 1) & 63);
        uint64_t D[PMX_NW];
        memcpy(D, lv->X, sizeof(D));
        uint64_t carry = 1;
        int64_t p = pos;
        for (;;) {                                       /* 0x411c98 */
            if ((D[W - 1] & fin) && left_ok(x, p, recbeg)) break;
            if (p == recbeg) return 0;
            --p;
            const uint8_t c = x->t[p];
            if (!step(D, W, lv, c, carry)) return 0;
            closure(D, W, lv);
            carry = 0;
        }
        start = p;
    }
    const xpart_t* rv = &x->v[1];
    if (rv->len == 0) {                                  /* 0x411dd4 */
        if (!right_ok(x, pos, recend)) return 0;
        *mb = start;
        *me = pos;
        return 1;
    }
    const int W = (rv->len + 63) >> 6;
    const uint64_t fin = 1ull << ((rv->len - 1) & 63);
    uint64_t D[PMX_NW];
    memcpy(D, rv->X, sizeof(D));
    uint64_t carry = 1;
    int64_t q = pos - 1;
    for (;;) {                                           /* 0x411eb0 */
        if ((D[W - 1] & fin) && right_ok(x, q + 1, recend)) break;
        if (q == recend - 1) return 0;
        ++q;
        const uint8_t c = x->t[q];
        if (!step(D, W, rv, c, carry)) return 0;
        closure(D, W, rv);
        carry = 0;
    }
    *mb = start;
    *me = q + 1;
    return 1;
}

/* ------------------------------------------------------------------------
 * scanners over the region [R, n)
 * ---------------------------------------------------------------------- */

/* extendedScan 0x4116f0, window: backward over `fwd` characters -- the
 * window's non-optional positions, its shortest match (extendedLoadFast
 * keeps extendedFindBest's count at +0x1018, 0x41312c; the bits are laid
 * out over all end - beg positions) -- the optional-block closure before
 * each step but the first */
static int scan_ext_window(const xctx_t* x, int64_t R, int64_t* mb, int64_t* me) {
    const int len = x->win;
    const uint8_t* t = x->t;
    int64_t r11 = R - 1;
    const int64_t limit = x->n - len;
    while (r11 < limit) {                                /* 0x411760 */
        uint64_t D = x->T[t[r11 + len]];
        if (!D) {
            r11 += len;
            continue;
        }
        int64_t c = r11 + len - 1;
        int dead = 0;
        for (int e = len - 1; e > 0; --e) {              /* 0x4117a0 */
            const uint64_t xx = D | x->fF;
            const uint64_t Dc = ((((xx - x->fI) ^ ~0ull) ^ xx) & x->fS) | D;
            const uint8_t ch = t[c];
            D = ((Dc << 1) & x->T[ch]) | (Dc & x->TA[ch]);
            if (!D) {
                r11 = c;
                dead = 1;
                break;
            }
            --c;
        }
        if (dead) continue;
        ++r11;
        if ((D >> 63) && check_match(x, r11, R, mb, me)) return 1;
    }
    return 0;
}

/* extendedScan 0x41184f, prefix: forward, a fresh state after every '\n'
 * (OptRecChar) and at R, the closure after each step */
static int scan_ext_prefix(const xctx_t* x, int64_t R, int64_t* mb, int64_t* me) {
    const uint64_t fin = 1ull << (x->len - 1);
    const uint8_t* t = x->t;
    uint64_t D = 0;
    int fresh = 1;
    for (int64_t p = R; p < x->n; ++p) {
        const uint8_t c = t[p];
        if (c == '\n') {
            fresh = 1;
            continue;
        }
        if (fresh) {
            D = 0;
            fresh = 0;
        }
        D = (D & x->TA[c]) | (((D << 1) | 1) & x->T[c]);
        const uint64_t xx = D | x->fF;
        D |= (((xx - x->fI) ^ ~0ull) ^ xx) & x->fS;
        if ((D & fin) && check_match(x, p + 1, R, mb, me)) return 1;
    }
    return 0;
}

/* simpleScan 0x4166d2, window: backward, exact; a candidate once the whole
 * window matched */
static int scan_simple_window(const xctx_t* x, int64_t R, int64_t* mb, int64_t* me) {
    const int len = x->len;
    const uint8_t* t = x->t;
    int64_t rsi = R - 1;
    const int64_t r8 = x->n - len;
    while (rsi < r8) {                                   /* 0x4166e0 */
        uint64_t D = x->T[t[rsi + len]];
        if (!D) {
            rsi += len;
            continue;
        }
        int64_t c = rsi + len - 1, r11 = c;
        int e = len;
        for (;;) {                                       /* 0x416720 */
            const uint64_t sh = D << 1;
            --e;
            r11 = c;
            /* the read past the window (rsi, possibly R - 1) only meets a
             * shifted-out state */
            D = sh ? sh & x->T[t[c]] : 0;
            --c;
            if (!D) break;
        }
        if (e == 0) {
            if (check_match(x, rsi + 1, R, mb, me)) return 1;
            rsi = rsi + 1;
        } else {
            rsi = r11;
        }
    }
    return 0;
}

/* simpleScan 0x41663d, prefix: forward shift-or; the candidate handed on
 * is the occurrence's START (r15) */
static int scan_simple_prefix(const xctx_t* x, int64_t R, int64_t* mb, int64_t* me) {
    const int len = x->len;
    const uint64_t fin = 1ull << (len - 1);
    uint64_t D = ~0ull;
    for (int64_t q = R; q < x->n; ++q) {
        D = (D << 1) | x->T[x->t[q]];
        if (!(D & fin) && check_match(x, q - len + 1, R, mb, me)) return 1;
    }
    return 0;
}

static int plan_ctx(xctx_t* x) {
    find_best(x, 0, &x->win, &x->beg, &x->end);
    x->type = x->win ? 2 : 3;                            /* 0x41336b */
    x->L = x->win ? x->beg : x->end;
    x->len = x->end - x->beg;
    if (x->len < 1 || x->len > 64) return -1;
    x->simple = !window_extended(x);
    load_verif(x, &x->v[0], x->L, x->L - 1, -1);
    load_verif(x, &x->v[1], x->m - x->L, x->L, 1);
    load_fast(x);
    return 0;
}

static int ctx_init(xctx_t* x, const uint64_t* B, int m, const uint64_t* opt, const uint64_t* rep, int icase,
                    int mode) {
    if (m < 1 || m > 64 * PMX_NW) return -1;
    memset(x, 0, sizeof(*x));
    x->Bp = B;
    x->m = m;
    x->icase = icase;
    x->mode = mode;
    memcpy(x->opt, opt, sizeof(x->opt));
    memcpy(x->rep, rep, sizeof(x->rep));
    return plan_ctx(x);
}

/* out[0] = type (2 window, 3 prefix), out[1] = window length fwd (0: none),
 * out[2] = beg, out[3] = end, out[4] = L, out[5] = simple scanner */
int pmx_plan(const uint64_t* B, int m, const uint64_t* opt, const uint64_t* rep, int icase, int* out) {
    xctx_t* x = malloc(sizeof(xctx_t));
    if (!x) return -1;
    const int rc = ctx_init(x, B, m, opt, rep, icase, 0);
    if (rc == 0) {
        out[0] = x->type;
        out[1] = x->win;
        out[2] = x->beg;
        out[3] = x->end;
        out[4] = x->L;
        out[5] = x->simple;
    }
    free(x);
    return rc;
}

/* What nrgrep_coords prints for a class-2 pattern at k = 0 over one region
 * (recSearchFile 0x402250: print, R = match end, stop when it ends at n).
 * B: [256][4] position sets of the folded bytes; opt / rep: [4] masks.
 * Returns the number of matches (may exceed cap), -1 if out of range. */
int64_t pmx_extended(const uint8_t* text, int64_t n, const uint64_t* B, int m, const uint64_t* opt,
                     const uint64_t* rep, int icase, int mode, int64_t* out_beg, int64_t* out_end, int64_t cap) {
    xctx_t* x = malloc(sizeof(xctx_t));
    if (!x) return -1;
    if (ctx_init(x, B, m, opt, rep, icase, mode) < 0) {
        free(x);
        return -1;
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
        int64_t mb = 0, me = 0, ok;
        if (x->simple) ok = x->win ? scan_simple_window(x, R, &mb, &me) : scan_simple_prefix(x, R, &mb, &me);
        else ok = x->win ? scan_ext_window(x, R, &mb, &me) : scan_ext_prefix(x, R, &mb, &me);
        if (!ok) break;
        if (count < cap) {
            out_beg[count] = mb;
            out_end[count] = me;
        }
        ++count;
        if (me == n) break;                              /* 0x4022eb */
        R = me;
    }
    free(nl);
    free(x);
    return count;
}
