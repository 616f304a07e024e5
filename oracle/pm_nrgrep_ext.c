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

/* ========================================================================
 * k > 0: the eextended engine (searchPreproc 0x402710: OptErrors != 0 and
 * detClass == 2 -> eextendedPreproc 0x40fe30; eextendedSearch 0x4116d0:
 * P->scan(beg, end, checkMatch 0x40f910, P, P->fast)).
 *
 *   eextendedPreproc 0x40fe30:
 *     extendedFindBest (K = k) -> a window [beg, end) and its cost `prob`
 *     a piece DP like esimple's: tab[t][i] = the pattern end after t
 *       "units" (optional* mandatory) from i (0x4100fb), cost[i][e] from
 *       extendedFindBest's P1/P2 recurrence (0x4102cd), the DP over k + 1
 *       pieces of L units (0x410929), threshold 0.95 (.rodata 0x41d2a0)
 *     pieces trimmed of optional ends (0x410cc7); split when best < 0.95,
 *       no piece empties and best < (k + 1) prob (0x410d7d)
 *     scanned positions without '?*+' (detClass != 2 over them, 0x4110d9 /
 *       0x4112e5): esimpleLoadFast + esimpleScan 0x4136d0 (the esimple
 *       scanners of pm_nrgrep.c); else eextendedLoadFast 0x40fac0 +
 *       eextendedScan 0x40ceb0
 *   verify: checkMatch 0x40f910 -> recGetRecord -> checkMatch1 0x40e340
 *
 * Quirks restated as they are:
 *   - checkMatch1 reads text[pos - 1] leftward and text[pos] rightward, but
 *     a boundary found after reading at least one character is recorded one
 *     position further out: the left phase records the look-ahead pointer
 *     (0x40e877, [rsp+0xf8] = the position left of the character just read;
 *     recCheckLeftContext is asked about it too, 0x40e98b), the right phase
 *     `p + 1` past the position after the character just read (0x40f3da,
 *     0x40ed59).  A match both of whose phases read characters is printed as
 *     [s - 1, e + 1) around its alignment [s, e); a phase that reads nothing
 *     (an empty part, or a boundary found before the first character)
 *     records the natural position.
 *   - the window scanner (type 2) reads fwd - k characters from p and hands
 *     checkMatch p + 1 (0x40d80d).
 *   - the prefix scanner (type 3) feeds each character with the next one as
 *     a look-ahead; a character followed by '\n' is never fed (0x40d25d,
 *     0x40d9ab, 0x40df51: the scan restarts after the '\n').
 *   - the general prefix scanner (k >= 3) has no repeat term in row 0
 *     (0x40d275); its k = 1 and k = 2 specializations do.
 *   - checkMatch1's substitution term carries 1 into every word after the
 *     first (0x40eb7d / 0x40f5ed `mov esi, 1`): parts over 64 positions.
 * Transpositions (OptTransp) are never requested by PatMatch; the scanners'
 * own transposition banks are restated since they run unconditionally.
 * ====================================================================== */

#define PMX_MAXK 16
#define PMX_INS 1
#define PMX_DEL 2
#define PMX_SUB 4

typedef struct {
    xctx_t x;                        /* m, tables, opt / rep, icase, mode, text, records */
    int k, errs;
    int type, simple, np, plen;      /* 1 pieces, 2 window, 3 prefix; esimple scanners; pieces; piece length */
    int fwd, wbeg, wend;             /* extendedFindBest's window */
    int off[PMX_MAXK + 1], pend[PMX_MAXK + 1];
    xpart_t* lv;                     /* [np] left parts (reversed) */
    xpart_t* rv;                     /* [np] right parts */
    /* eextendedLoadFast: X->T / X->TA / I F S (one word), F+8 (type 1), tops */
    int flen, fspan;
    uint64_t T[256], TA[256], T2[256], fI, fF, fS, top[PMX_MAXK + 1];
} ectx_t;

/* ------------------------------------------------------------------------
 * the plan (eextendedPreproc 0x40fe30)
 * ---------------------------------------------------------------------- */
static int eplan(ectx_t* e) {
    xctx_t* x = &e->x;
    const int m = x->m, k = e->k;
    int fwd, beg, end;
    const double prob = find_best(x, k, &fwd, &beg, &end);      /* 0x40ff33 */
    e->fwd = fwd;
    e->wbeg = beg;
    e->wend = end;
    const int ml = m > 64 ? 64 : m;
    const int mp = ml / (k + 1);                                /* 0x40ffda (no transpositions) */
    double best = 0.95;                                         /* .rodata 0x41d2a0 */
    int bestL = 0, offs[PMX_MAXK + 1], ends[PMX_MAXK + 1];
    if (mp > 1 && !(1.0 / (double)mp > 0.95)) {                 /* 0x410798 */
        double* pr = calloc((size_t)m, sizeof(double));
        double* apr = calloc((size_t)m, sizeof(double));
        for (int i = 0; i < m; ++i)                             /* 0x41000f */
            for (int c = 0; c < 256; ++c) {
                if (cls_has(x, c, i)) pr[i] += pmn_letter_prob[c];
                if (rep_has(x, c, i)) apr[i] += pmn_letter_prob[c];
            }
        /* tab[t][i], t = 0 .. mp: the end after t units from i (0x4100fb) */
        int* tab = malloc(sizeof(int) * (size_t)(mp + 1) * (size_t)m);
        for (int i = 0; i < m; ++i) {
            int r = i;
            for (int t = 0;; ++t) {
                if (r > m) {
                    r = m;
                } else if (r > 0 && r < m) {
                    while (isset(x->opt, r - 1)) {
                        ++r;
                        if (r == m) break;
                    }
                }
                tab[(size_t)t * m + i] = r;
                if (t + 1 > mp) break;
                ++r;
            }
        }
        /* cost[i * mp + e] (rows overlap as in the binary: stride mp, column
         * e up to m - 1; a span over 64 / (k + 1) writes 1.0 at i m + 1 + e),
         * from extendedFindBest's recurrence (0x4102cd .. 0x410715) */
        const int cap = 64 / (k + 1);
        const int tc = cap < m ? cap : m;
        const size_t T1 = (size_t)tc + 1, EM = (size_t)m * T1;
#define PIDX(l, ee, t) ((size_t)(l) * EM + (size_t)(ee) * T1 + (size_t)(t))
        double* P1 = malloc(sizeof(double) * EM * ((size_t)m + 1));
        double* P2 = malloc(sizeof(double) * EM * ((size_t)m + 1));
        int* pos = calloc((size_t)m, sizeof(int));
        for (int i = 0; i < m; ++i)                             /* 0x4101de */
            for (int t = 0; t <= i + 1; ++t) P1[PIDX(t, i, 0)] = P2[PIDX(t, i, 0)] = 1.0;
        /* heap read before write is taken as 0.0 (see header of pm_nrgrep.c) */
        double* C = calloc((size_t)m * (size_t)m + 2, sizeof(double));
        for (int i = 0; i < m; ++i)
            for (int ee = i; ee < m; ++ee) {
                const int j = ee - i + 1;
                if (j > cap) {                                  /* 0x4106a0 */
                    C[(size_t)i * m + 1 + ee] = 1.0;
                    continue;
                }
                double sum = 1.0;
                for (int t = 1; t <= j; ++t) {
                    if (pos[ee] < t) {                          /* 0x410470 */
                        P2[PIDX(ee + 1, ee, t)] = 0.0;
                        P1[PIDX(ee + 1, ee, t)] = 0.0;
                        for (int l = ee; l >= 0; --l) {
                            double v = pr[l] * P1[PIDX(l + 1, ee, t - 1)] + apr[l] * P1[PIDX(l, ee, t - 1)];
                            v = isset(x->opt, l) ? P1[PIDX(l + 1, ee, t)] + v : 0.0 + v;
                            double r;
                            if (v > 1.0) {
                                P1[PIDX(l, ee, t)] = 1.0;
                                r = 0.0;
                            } else {
                                P1[PIDX(l, ee, t)] = v;
                                r = 1.0 - v;
                            }
                            P2[PIDX(l, ee, t)] = 1.0 - (1.0 - P2[PIDX(l + 1, ee, t)]) * r;
                        }
                        pos[ee] = t;
                    }
                    sum = sum + P2[PIDX(i, ee, t)];
                }
                C[(size_t)i * mp + ee] = sum;
            }
#undef PIDX
        free(P1);
        free(P2);
        free(pos);
        free(pr);
        free(apr);
        /* the piece DP (0x410929): D[p][c] = the cost of c pieces from p */
        const int K2 = k + 2;
        double* D = malloc(sizeof(double) * (size_t)(m + 1) * K2);
        int* Wc = calloc((size_t)(m + 1) * K2, sizeof(int));
        for (int L = mp;;) {
            for (int q = 0; q <= m; ++q) D[(size_t)q * K2] = 0.0;
            for (int c = 1; c <= k + 1; ++c) D[(size_t)m * K2 + c] = 1.0;
            for (int c = 1; c <= k + 1; ++c)                    /* 0x410ac0 */
                for (int p = m - 1; p >= 0; --p) {
                    const int en = tab[(size_t)L * m + p];
                    const int len = en - p;
                    const double x1 = C[(size_t)p * mp + en - 1];
                    double q = 0.0;
                    if ((double)(len + 1) > x1) {
                        const double xx = x1 / (((double)len - x1) + 1.0);
                        q = xx <= 1.0 ? 1.0 - xx : 0.0;
                    }
                    double val = 1.0 - q * (1.0 - D[(size_t)en * K2 + c - 1]);
                    Wc[(size_t)p * K2 + c] = p;
                    if (val > D[(size_t)(p + 1) * K2 + c]) {
                        val = D[(size_t)(p + 1) * K2 + c];
                        Wc[(size_t)p * K2 + c] = Wc[(size_t)(p + 1) * K2 + c];
                    }
                    D[(size_t)p * K2 + c] = val;
                }
            const double v = D[k + 1];                          /* 0x410bbe */
            if (best > v) {
                int p = 0;
                for (int c = k + 1, idx = 0; c >= 1; --c, ++idx) {
                    const int o = Wc[(size_t)p * K2 + c];
                    offs[idx] = o;
                    ends[idx] = tab[(size_t)L * m + o];
                    p = tab[(size_t)L * m + o];
                }
                best = v;
                bestL = L;
            }
            --L;                                                /* 0x410c44 */
            if (L == 1) break;
            if (1.0 / (double)L > best) break;
        }
        free(D);
        free(Wc);
        free(C);
        free(tab);
    }
    int split = 0;
    if (!(best >= 0.95) && bestL != 0) {                        /* 0x410cbd */
        split = 1;
        for (int i = 0; i <= k && split; ++i) {                 /* 0x410cc7: trim optional ends */
            while (offs[i] < ends[i] && isset(x->opt, offs[i])) ++offs[i];
            while (ends[i] > offs[i] && isset(x->opt, ends[i] - 1)) --ends[i];
            if (offs[i] == ends[i]) split = 0;
        }
        if (split && best >= (double)(k + 1) * prob) split = 0;   /* 0x410d95 */
    }
    int Ls[PMX_MAXK + 1];
    uint64_t scanned[PMX_NW] = {0};
    if (split) {
        e->type = 1;
        e->np = k + 1;
        e->plen = bestL;
        for (int i = 0; i <= k; ++i) {
            e->off[i] = offs[i];
            e->pend[i] = ends[i];
            Ls[i] = offs[i];
            for (int p = offs[i]; p < ends[i]; ++p) setb(scanned, p);
        }
    } else {
        e->type = fwd >= 1 ? 2 : 3;                             /* 0x411087 */
        e->np = 1;
        e->plen = 0;
        e->off[0] = beg;
        e->pend[0] = end;
        Ls[0] = fwd ? beg : end;                                /* 0x41120f / 0x411379 */
        if (end - beg < 1 || end - beg > 64) return -1;
        for (int p = beg; p < end; ++p) setb(scanned, p);
    }
    e->simple = 1;                                              /* detClass over them */
    for (int p = 0; p < m; ++p)
        if (isset(scanned, p) && (isset(x->opt, p) || isset(x->rep, p))) e->simple = 0;
    e->lv = malloc(sizeof(xpart_t) * (size_t)e->np);
    e->rv = malloc(sizeof(xpart_t) * (size_t)e->np);
    for (int i = 0; i < e->np; ++i) {                           /* 0x410e8c: extendedLoadVerif x 2 */
        load_verif(x, &e->lv[i], Ls[i], Ls[i] - 1, -1);
        load_verif(x, &e->rv[i], m - Ls[i], Ls[i], 1);
    }
    /* the scanner's tables */
    memset(e->T, 0, sizeof(e->T));
    memset(e->TA, 0, sizeof(e->TA));
    memset(e->T2, 0, sizeof(e->T2));
    e->fI = e->fF = e->fS = 0;
    if (e->simple) {                                            /* esimpleLoadFast 0x415370 */
        if (e->type == 1) {
            for (int r = 0; r < e->np; ++r)
                for (int pp = 0; pp < e->plen; ++pp)
                    for (int c = 0; c < 256; ++c)
                        if (e->off[r] + e->plen - 1 - pp < m && cls_has(x, c, e->off[r] + e->plen - 1 - pp)) {
                            const uint64_t bit = 1ull << (r * e->plen + pp);
                            e->T[c] |= bit;
                            if (pp > 0) e->T2[c] |= bit;
                        }
        } else {
            x->win = e->type == 2;                              /* simpleLoadFast(win, B, beg, end) */
            x->beg = beg;
            x->end = end;
            x->len = end - beg;
            x->simple = 1;
            load_fast(x);
            memcpy(e->T, x->T, sizeof(e->T));
        }
        return 0;
    }
    if (e->type == 1) {                                         /* eextendedLoadFast 0x40fb79 */
        e->flen = e->plen;
        int b = 0;
        for (int q = 0; q <= k; ++q) {
            const int plen = e->pend[q] - e->off[q];
            for (int r = 0; r < plen; ++r, ++b) {
                const int p = e->pend[q] - 1 - r;
                const uint64_t bit = 1ull << (b & 63);
                for (int c = 0; c < 256; ++c) {
                    if (cls_has(x, c, p)) {
                        e->T[c] |= bit;
                        if (r > 0) e->T2[c] |= bit;
                    }
                    if (rep_has(x, c, p)) e->TA[c] |= bit;
                }
                if (isset(x->opt, p)) {                         /* 0x40fd0e */
                    const uint64_t pbit = 1ull << ((b - 1) & 63);
                    e->fS |= bit;
                    if (e->fF & pbit) {
                        e->fF = (e->fF & ~pbit) | bit;
                    } else {
                        e->fI |= pbit;
                        e->fF |= bit;
                    }
                }
            }
            e->top[q] = 1ull << ((b - 1) & 63);                 /* 0x40fd7c */
        }
        return 0;
    }
    x->win = fwd;                                               /* extendedLoadFast(fwd, B, A, S, beg, end) */
    x->beg = beg;
    x->end = end;
    x->len = end - beg;
    x->simple = 0;
    load_fast(x);
    memcpy(e->T, x->T, sizeof(e->T));
    memcpy(e->TA, x->TA, sizeof(e->TA));
    e->fI = x->fI;
    e->fF = x->fF;
    e->fS = x->fS;
    e->flen = fwd;                                              /* X->len (+0x1018) */
    e->fspan = end - beg;                                       /* F->len (+0x80c) */
    return 0;
}

/* ------------------------------------------------------------------------
 * checkMatch1 0x40e340 (and checkMatch 0x40f910)
 * ---------------------------------------------------------------------- */

/* D |= S & ((D | F) ^ ~((D | F) - I)) over W words, as a row update */
static void eclosure(uint64_t* D, int W, const xpart_t* v) { closure(D, W, v); }

/* one row-set update of a phase: row 0 then rows 1 .. maxk (0x40e8ad,
 * 0x40e9b0; 0x40f2fd, 0x40f418); R[j] updated in place, returns the lowest
 * row whose new value holds `fin` in the last word (-1: none), rows above
 * are still updated up to the first hit, as the binary breaks there */
typedef struct {
    int W;
    uint64_t fin, alive;
    uint64_t R[PMX_MAXK + 1][PMX_NW];
} erows_t;

static void erows_init(erows_t* s, const xpart_t* v, int errs, int kmax) {
    s->W = (v->len + 63) >> 6;
    s->fin = 1ull << ((v->len - 1) & 63);
    s->alive = s->fin * 2 - 1;
    memcpy(s->R[0], v->X, sizeof(s->R[0]));
    for (int j = 1; j <= kmax; ++j) {                           /* 0x40e658 */
        if (errs & PMX_DEL) {
            uint64_t carry = 1;
            for (int w = 0; w < s->W; ++w) {
                const uint64_t old = s->R[j - 1][w];
                s->R[j][w] = (old << 1) | carry;
                carry = old >> 63;
            }
            eclosure(s->R[j], s->W, v);
        } else {
            memcpy(s->R[j], s->R[j - 1], sizeof(s->R[j]));       /* 0x40ee3f */
        }
    }
}

/* row 0 with character c (inj: the first character) */
static void erow0(erows_t* s, const xpart_t* v, uint8_t c, uint64_t inj, uint64_t* tmp1, uint64_t* tmp2) {
    uint64_t carry = inj;
    for (int w = 0; w < s->W; ++w) {
        const uint64_t old = s->R[0][w];
        tmp1[w] = old;
        tmp2[w] = (((old << 1) | carry) & v->B[c][w]) | (old & v->A[c][w]);
        carry = old >> 63;
    }
    eclosure(tmp2, s->W, v);
    memcpy(s->R[0], tmp2, sizeof(uint64_t) * (size_t)s->W);
}

/* row j >= 1: tmp2 holds the new row j - 1, tmp1 the old one */
static void erowj(erows_t* s, const xpart_t* v, int j, uint8_t c, uint64_t inj, int errs, uint64_t* tmp1,
                  uint64_t* tmp2) {
    uint64_t dc = 0, sc = inj, mc = inj;
    uint64_t nw[PMX_NW];
    for (int w = 0; w < s->W; ++w) {
        uint64_t r = 0;
        if (errs & PMX_DEL) {
            r = (tmp2[w] << 1) | dc;
            dc = tmp2[w] >> 63;
        }
        if (errs & PMX_INS) r |= tmp1[w];
        if (errs & PMX_SUB) {
            r |= sc | (tmp1[w] << 1);
            sc = 1;                                             /* 0x40eb7d: mov esi, 1 */
        }
        const uint64_t old = s->R[j][w];
        r |= (((old << 1) | mc) & v->B[c][w]) | (old & v->A[c][w]);
        mc = old >> 63;
        nw[w] = r;
        tmp1[w] = old;
    }
    eclosure(nw, s->W, v);
    memcpy(tmp2, nw, sizeof(uint64_t) * (size_t)s->W);
    memcpy(s->R[j], nw, sizeof(uint64_t) * (size_t)s->W);
}

static int erows_alive(const erows_t* s, int maxk) {            /* 0x40edb9 / 0x40f6eb */
    for (int w = 0; w < s->W - 1; ++w)
        if (s->R[maxk][w]) return 1;
    return (s->R[maxk][s->W - 1] & s->alive) != 0;
}

/* the left phase: `len` = L positions read backward from pos; *start and
 * the errors spent, or 0 */
static int eleft(const ectx_t* e, const xpart_t* v, int64_t pos, int64_t recbeg, int* nerr, int64_t* start) {
    const xctx_t* x = &e->x;
    const int k = e->k;
    if (v->len == 0) {                                          /* 0x40e3a0 */
        for (int q = 0; q <= k; ++q) {
            if (left_ok(x, pos - q, recbeg)) {
                *start = pos - q;
                *nerr = q;
                return 1;
            }
            if (pos - q == recbeg || !(e->errs & PMX_INS)) return 0;
        }
        return 0;
    }
    erows_t s;
    erows_init(&s, v, e->errs, k);
    int maxk = k, best = k, found = 0;
    int64_t fpos = 0;
    for (int j = 1; j <= maxk; ++j)                             /* 0x40e6f3 */
        if ((s.R[j][s.W - 1] & s.fin) && left_ok(x, pos, recbeg)) {
            found = 1;
            fpos = pos;
            best = j;
            maxk = j - 1;
        }
    if (pos != recbeg) {
        uint64_t tmp1[PMX_NW], tmp2[PMX_NW];
        uint64_t inj = 1;
        uint8_t c = x->t[pos - 1];
        for (int64_t X = pos - 2; X != recbeg - 2; --X) {       /* 0x40e849 */
            const uint8_t look = X + 1 != recbeg ? x->t[X] : 0;
            erow0(&s, v, c, inj, tmp1, tmp2);
            if ((tmp2[s.W - 1] & s.fin) && left_ok(x, X, recbeg)) {   /* 0x40e964 */
                *start = X;
                *nerr = 0;
                return 1;
            }
            for (int j = 1; j <= maxk; ++j) {                   /* 0x40e9b0 */
                erowj(&s, v, j, c, inj, e->errs, tmp1, tmp2);
                if ((tmp2[s.W - 1] & s.fin) && left_ok(x, X, recbeg)) {
                    int cc = j;                                 /* 0x40ec54: walk down */
                    while (cc - 1 >= 0 && (s.R[cc - 1][s.W - 1] & s.fin)) --cc;
                    if (cc == 0) {
                        *start = X;
                        *nerr = 0;
                        return 1;
                    }
                    found = 1;
                    fpos = X;
                    best = cc;
                    maxk = cc - 1;
                    break;
                }
            }
            if (!erows_alive(&s, maxk)) break;
            inj = 0;
            c = look;
        }
    }
    if (!found) return 0;                                       /* 0x40ee6e */
    *start = fpos;
    *nerr = best;
    return 1;
}

/* the right phase: m - L positions read forward from pos with kmax errors */
static int eright(const ectx_t* e, const xpart_t* v, int64_t pos, int64_t recend, int kmax, int64_t* end) {
    const xctx_t* x = &e->x;
    if (v->len == 0) {                                          /* 0x40ecd5 */
        for (int q = 0; q <= kmax; ++q) {
            if (right_ok(x, pos + q, recend)) {
                *end = pos + q;
                return 1;
            }
            if (q == recend - pos || !(e->errs & PMX_INS)) return 0;
        }
        return 0;
    }
    if (kmax < 0) return 0;
    erows_t s;
    erows_init(&s, v, e->errs, kmax);
    int maxk = kmax, found = 0;
    int64_t fend = 0;
    for (int j = 1; j <= maxk; ++j)                             /* 0x40f176 */
        if ((s.R[j][s.W - 1] & s.fin) && right_ok(x, pos, recend)) {
            found = 1;
            fend = pos;
            maxk = j - 1;
        }
    if (pos != recend) {
        uint64_t tmp1[PMX_NW], tmp2[PMX_NW];
        uint64_t inj = 1;
        uint8_t c = x->t[pos];
        for (int64_t Y = pos + 1;; ++Y) {                       /* 0x40f2a3: Y - 1 = the character read */
            const int64_t q = Y - 1;
            const uint8_t look = q != recend - 1 ? x->t[Y] : 0;
            erow0(&s, v, c, inj, tmp1, tmp2);
            if ((tmp2[s.W - 1] & s.fin) && right_ok(x, Y + 1, recend)) {   /* 0x40f3ca */
                *end = Y + 1;
                return 1;
            }
            for (int j = 1; j <= maxk; ++j) {                   /* 0x40f418 */
                erowj(&s, v, j, c, inj, e->errs, tmp1, tmp2);
                if ((tmp2[s.W - 1] & s.fin) && right_ok(x, Y + 1, recend)) {
                    int cc = j;                                 /* 0x40f6ae */
                    while (cc - 1 >= 0 && (s.R[cc - 1][s.W - 1] & s.fin)) --cc;
                    if (cc == 0) {
                        *end = Y + 1;
                        return 1;
                    }
                    found = 1;
                    fend = Y + 1;
                    maxk = cc - 1;
                    break;
                }
            }
            if (!erows_alive(&s, maxk)) break;
            if (q == recend - 1) break;                         /* 0x40f76d */
            inj = 0;
            c = look;
        }
    }
    if (!found) return 0;                                       /* 0x40f7be */
    *end = fend;
    return 1;
}

/* checkMatch 0x40f910: the record (from pos - 1 for the prefix scanner),
 * then checkMatch1's two phases for piece q */
static int echeck(const ectx_t* e, int q, int64_t pos, int64_t R, int64_t* mb, int64_t* me) {
    const xctx_t* x = &e->x;
    const int64_t rp = e->type == 3 ? pos - 1 : pos;
    int64_t lo = 0, hi = x->nnl;
    while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if (x->nl[mid] < rp) lo = mid + 1; else hi = mid;
    }
    int64_t recbeg = R;
    if (lo > 0 && x->nl[lo - 1] >= R) recbeg = x->nl[lo - 1] + 1;
    const int64_t recend = lo < x->nnl ? x->nl[lo] : x->n;
    if (rp < recbeg || rp >= recend) return 0;
    int64_t start, end;
    int eL;
    if (!eleft(e, &e->lv[q], pos, recbeg, &eL, &start)) return 0;
    if (!eright(e, &e->rv[q], pos, recend, e->k - eL, &end)) return 0;
    *mb = start;
    *me = end;
    return 1;
}

/* ------------------------------------------------------------------------
 * scanners over the region [R, n)
 * ---------------------------------------------------------------------- */

static inline uint64_t fclose1(const ectx_t* e, uint64_t D) {
    const uint64_t xx = D | e->fF;
    return D | ((xx ^ ~(xx - e->fI)) & e->fS);
}

/* eextendedScan type 1 (0x40cf05): k + 1 pieces with '?*+' searched
 * exactly, backward over plen characters, the closure before each step */
static int escan_xpieces(const ectx_t* e, int64_t R, int64_t* mb, int64_t* me) {
    const uint8_t* t = e->x.t;
    const int len = e->flen;
    int64_t pos = R - 1;
    const int64_t lim = e->x.n - len;
    while (pos < lim) {                                         /* 0x40cf82 */
        uint64_t D = e->T[t[pos + len]];
        while (!D) {
            pos += len;
            if (!(pos < lim)) return 0;
            D = e->T[t[pos + len]];
        }
        int ebp = len - 1;
        int64_t c = pos + len - 1;
        do {                                                    /* 0x40cff4 */
            --ebp;
            const uint8_t ch = t[c];
            --c;
            const uint64_t Dc = fclose1(e, D);
            D = (Dc & e->TA[ch]) | ((Dc << 1) & e->T2[ch]);
        } while (D && ebp != 0);
        if (D)
            for (int q = 0; q < e->np; ++q)                     /* 0x40d081 */
                if ((e->top[q] & D) && echeck(e, q, pos + 1, R, mb, me)) return 1;
        pos = pos + ebp + 1;
    }
    return 0;
}

/* eextendedScan type 2 (0x40d3c6; k = 1 0x40e0b2, k = 2 0x40db73, the same
 * rule): a window of fwd - k characters from p read backward with k errors,
 * checkMatch at p + 1 */
static int escan_xwindow(const ectx_t* e, int64_t R, int64_t* mb, int64_t* me) {
    const uint8_t* t = e->x.t;
    const int k = e->k;
    const int W = e->flen - k - 1;
    const uint64_t top = e->fspan >= 64 ? ~0ull : ~0ull << (64 - e->fspan);
    uint64_t Rr[PMX_MAXK + 1], Tr[PMX_MAXK + 1];
    if (W < 1) return 0;
    for (int64_t pos = R; pos < e->x.n - W;) {                  /* 0x40d5a1 */
        const uint8_t c1 = t[pos + W], c2 = t[pos + W - 1];
        Rr[0] = fclose1(e, e->T[c1]);
        const uint64_t tr0 = (fclose1(e, e->T[c2]) << 1) & e->T[c1];
        for (int j = 1; j <= k; ++j) {
            Rr[j] = top;
            Tr[j] = tr0;
        }
        int64_t ptr = pos + W - 1;
        int cnt = W - 1;
        uint8_t c = c2, look = 0;
        for (;;) {                                              /* 0x40d6d0 */
            --cnt;
            if (cnt + 1 > 0) look = t[ptr - 1];
            uint64_t pold = Rr[0];
            uint64_t pnew = fclose1(e, (Rr[0] & e->TA[c]) | ((Rr[0] << 1) & e->T[c]));
            Rr[0] = pnew;
            for (int j = 1; j <= k; ++j) {                      /* 0x40d740 */
                const uint64_t old = Rr[j];
                const uint64_t v = ((old << 1) & e->T[c]) | (old & e->TA[c]) | pold | ((pnew | pold) << 1) | Tr[j];
                Tr[j] = (fclose1(e, (pold & e->TA[look]) | ((pold << 1) & e->T[look])) << 1) & e->T[c];
                Rr[j] = fclose1(e, v);
                pold = old;
                pnew = Rr[j];
            }
            if (cnt < 0) {                                      /* 0x40d7ea */
                if ((Rr[k] >> 63) && echeck(e, 0, pos + 1, R, mb, me)) return 1;
                break;
            }
            if (!Rr[k] && !Tr[k]) break;                        /* 0x40d7c2 */
            --ptr;
            c = look;
        }
        pos = pos + cnt + 2;                                    /* 0x40d833 */
    }
    return 0;
}

/* eextendedScan type 3 (0x40d0f4; k = 1 0x40de5e, k = 2 0x40d888): the
 * prefix forward with k errors, every character fed with the next one as a
 * look-ahead, fresh rows at R and after '\n'; checkMatch at the position
 * after the character */
static int escan_xprefix(const ectx_t* e, int64_t R, int64_t* mb, int64_t* me) {
    const uint8_t* t = e->x.t;
    const int64_t n = e->x.n;
    const int k = e->k;
    const int ta0 = k <= 2;                                     /* row 0's repeat term: 0x40da6f / 0x40df9d only */
    const uint64_t fin = 1ull << ((e->fspan - 1) & 63);
    uint64_t Rr[PMX_MAXK + 1], Tr[PMX_MAXK + 1];
    if (R == n) return 0;                                       /* 0x40d17b */
    int64_t p = R;
    for (;;) {                                                  /* 0x40d1ae */
        if (p > n) return 0;
        if (p == n) return 0;                                   /* t[n] is read and dropped: 0x40d1c0 .. 0x40e2fa */
        uint8_t c = t[p];
        ++p;
        while (c == '\n') {                                     /* 0x40d37e */
            if (p == n) return 0;                               /* t[n] read, '\n' or not the scan ends */
            ++p;
            c = t[p - 1];
        }
        for (int j = 0; j <= k; ++j) {                          /* 0x40d1f8 */
            Rr[j] = j ? ~(~0ull << j) : 0;
            Tr[j] = 0;
        }
        int64_t nxt = p;
        int restart = 0;
        for (;;) {                                              /* 0x40d240 */
            uint8_t look = c;
            if (nxt < n) {
                look = t[nxt];
                if (look == '\n') {                             /* the character before '\n' is dropped */
                    p = nxt + 1;
                    restart = 1;
                    break;
                }
            }
            uint64_t pold = Rr[0];
            uint64_t raw0 = ((Rr[0] << 1) | 1) & e->T[c];
            if (ta0) raw0 |= Rr[0] & e->TA[c];
            uint64_t pnew = fclose1(e, raw0);
            Rr[0] = pnew;
            for (int j = 1; j <= k; ++j) {                      /* 0x40d2c8 */
                const uint64_t old = Rr[j];
                const uint64_t v = (((old << 1) | 1) & e->T[c]) | (old & e->TA[c]) | ((pnew | pold) << 1) | pold |
                                   1 | Tr[j];
                const uint64_t u = fclose1(e, (pold & e->TA[look]) | (((pold << 1) | 1) & e->T[look]));
                Tr[j] = (u & e->TA[c]) | ((u << 1) & e->T[c]);
                Rr[j] = fclose1(e, v);
                pold = old;
                pnew = Rr[j];
            }
            if ((Rr[k] & fin) && echeck(e, 0, nxt, R, mb, me)) return 1;   /* 0x40d35d */
            if (n < nxt + 1) return 0;                          /* 0x40d364 */
            c = look;
            ++nxt;
        }
        if (restart) continue;
    }
}

/* esimpleScan 0x4136d0 over an extended pattern's simple pieces / window /
 * prefix (the loops of pm_nrgrep.c: scan_pieces, scan_backward,
 * scan_forward), verified by the eextended checkMatch */
static int escan_spieces(const ectx_t* e, int64_t R, int64_t* mb, int64_t* me) {
    const int mpc = e->plen, np = e->np;
    const uint8_t* t = e->x.t;
    int64_t r9 = R - 1;
    const int64_t limit = e->x.n - mpc;
    while (r9 < limit) {                                        /* 0x413780 */
        uint64_t D = e->T[t[r9 + mpc]];
        if (!D) {
            r9 += mpc;
            continue;
        }
        int64_t a = r9 + mpc - 1;
        int q = mpc - 1;
        do {
            D = (D << 1) & e->T2[t[a]];
            --q;
            --a;
        } while (D && q);
        if (D)
            for (int i = 0; i < np; ++i) {                      /* 0x41384b: 32-bit shift */
                const int bit = i * mpc + mpc - 1;
                const uint64_t msk = (uint64_t)(int64_t)(int32_t)(1u << (bit & 31));
                if ((D & msk) && echeck(e, i, r9 + 1, R, mb, me)) return 1;
            }
        r9 += q + 1;
    }
    return 0;
}

static int escan_swindow(const ectx_t* e, int64_t R, int64_t* mb, int64_t* me) {
    const int Lw = e->wend - e->wbeg, k = e->k;
    const uint64_t top = ~0ull << (64 - Lw);
    const int W = Lw - k;
    const int64_t limit = e->x.n - (Lw - k - 1);
    uint64_t Rr[PMX_MAXK + 1], Tr[PMX_MAXK + 1];
    const uint8_t* t = e->x.t;
    if (W < 2) return 0;
    for (int64_t s = R; s < limit;) {                           /* 0x413b6f */
        const uint64_t b0 = e->T[t[s + W - 1]];
        Rr[0] = b0;
        for (int j = 1; j <= k; ++j) {
            Rr[j] = top;
            Tr[j] = b0;
        }
        int64_t rb = W - 2;
        for (;;) {
            const uint64_t bc = e->T[t[s + rb]];
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
            if (rb == 0) {                                      /* 0x413ca1 */
                if ((Rr[k] >> 63) && echeck(e, 0, s, R, mb, me)) return 1;
                break;
            }
            if (!Rr[k] && !Tr[k]) break;
            --rb;
        }
        s += rb + 1;                                            /* 0x413cfa */
    }
    return 0;
}

static int escan_sprefix(const ectx_t* e, int64_t R, int64_t* mb, int64_t* me) {
    const int Lw = e->wend - e->wbeg, k = e->k;
    const uint64_t fin = 1ull << (Lw - 1);
    uint64_t Rr[PMX_MAXK + 1], Tr[PMX_MAXK + 1];
    for (int j = 0; j <= k; ++j) {                              /* 0x413905 */
        Rr[j] = ~0ull << j;
        Tr[j] = ~0ull;
    }
    const uint8_t* t = e->x.t;
    for (int64_t p = R; p < e->x.n;) {                          /* 0x413932 */
        const uint64_t bc = e->T[t[p]];
        ++p;
        uint64_t oldp = Rr[0];
        uint64_t newp = (oldp << 1) | bc;
        Rr[0] = newp;
        const uint64_t r9 = (bc << 1) | 1;
        for (int j = 1; j <= k; ++j) {
            const uint64_t tr = r9 | Tr[j];
            uint64_t v = ((newp & oldp) << 1) & oldp;
            Tr[j] = (oldp << 2) | bc;
            v &= tr;
            const uint64_t oldj = Rr[j];
            v &= (oldj << 1) | bc;
            Rr[j] = v;
            oldp = oldj;
            newp = v;
        }
        if (!(Rr[k] & fin) && echeck(e, 0, p, R, mb, me)) return 1;
    }
    return 0;
}

static int ectx_init(ectx_t* e, const uint64_t* B, int m, int k, int errs, const uint64_t* opt, const uint64_t* rep,
                     int icase, int mode) {
    if (m < 1 || m > 64 * PMX_NW || k < 1 || k > PMX_MAXK) return -1;
    memset(e, 0, sizeof(*e));
    e->x.Bp = B;
    e->x.m = m;
    e->x.icase = icase;
    e->x.mode = mode;
    memcpy(e->x.opt, opt, sizeof(e->x.opt));
    memcpy(e->x.rep, rep, sizeof(e->x.rep));
    e->k = k;
    e->errs = errs;
    return eplan(e);
}

static void ectx_free(ectx_t* e) {
    free(e->lv);
    free(e->rv);
}

/* out[0] = type (1 pieces, 2 window, 3 prefix), out[1] = simple scanner,
 * out[2] = pieces, out[3] = piece length (type 1) / window fwd, out[4] = beg,
 * out[5] = end (extendedFindBest's window), out[6 ..] = {off, end} of every
 * piece (or of the window) */
int pmx_eplan(const uint64_t* B, int m, int k, const uint64_t* opt, const uint64_t* rep, int icase, int* out) {
    ectx_t* e = malloc(sizeof(ectx_t));
    if (!e) return -1;
    const int rc = ectx_init(e, B, m, k, PMX_INS | PMX_DEL | PMX_SUB, opt, rep, icase, 0);
    if (rc == 0) {
        out[0] = e->type;
        out[1] = e->simple;
        out[2] = e->np;
        out[3] = e->type == 1 ? e->plen : e->fwd;
        out[4] = e->wbeg;
        out[5] = e->wend;
        for (int i = 0; i < e->np; ++i) {
            out[6 + 2 * i] = e->off[i];
            out[7 + 2 * i] = e->pend[i];
        }
    }
    ectx_free(e);
    free(e);
    return rc;
}

/* What nrgrep_coords prints for a class-2 pattern at k > 0 over one region
 * (recSearchFile 0x402250).  Returns the number of matches (may exceed cap),
 * -1 if out of range. */
int64_t pmx_eextended(const uint8_t* text, int64_t n, const uint64_t* B, int m, int k, int errs, const uint64_t* opt,
                      const uint64_t* rep, int icase, int mode, int64_t* out_beg, int64_t* out_end, int64_t cap) {
    ectx_t* e = malloc(sizeof(ectx_t));
    if (!e) return -1;
    if (ectx_init(e, B, m, k, errs, opt, rep, icase, mode) < 0) {
        free(e);
        return -1;
    }
    e->x.t = text;
    e->x.n = n;
    int64_t nnl = 0;
    for (int64_t p = 0; p < n; ++p) nnl += text[p] == '\n';
    int64_t* nl = malloc(sizeof(int64_t) * (size_t)(nnl + 1));
    nnl = 0;
    for (int64_t p = 0; p < n; ++p)
        if (text[p] == '\n') nl[nnl++] = p;
    e->x.nl = nl;
    e->x.nnl = nnl;
    int64_t count = 0, R = 0;
    while (R < n) {
        int64_t mb = 0, me = 0;
        int ok;
        if (e->simple)
            ok = e->type == 1 ? escan_spieces(e, R, &mb, &me)
                              : e->type == 2 ? escan_swindow(e, R, &mb, &me) : escan_sprefix(e, R, &mb, &me);
        else
            ok = e->type == 1 ? escan_xpieces(e, R, &mb, &me)
                              : e->type == 2 ? escan_xwindow(e, R, &mb, &me) : escan_xprefix(e, R, &mb, &me);
        if (!ok) break;
        if (count < cap) {
            out_beg[count] = mb;
            out_end[count] = me;
        }
        ++count;
        if (me >= n) break;                                     /* 0x4022eb */
        R = me;
    }
    free(nl);
    ectx_free(e);
    free(e);
    return count;
}
