/*
 * pm_nrgrep.c -- nrgrep's approximate class-sequence engine ("esimple"), the
 * engine nrgrep_coords runs for `-k <k><ids>` on a plain class sequence.
 *
 * TEST INFRASTRUCTURE ONLY (like pm_oracle.c): only tests/, smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker.
 *
 * Round 3: restated from the binary's disassembly (www/bin/nrgrep_coords,
 * `objdump -d`, never executed).  Every step cites the address it follows.
 * This file deliberately simulates the binary's own loops literally (its
 * BNDM / ABNDM / shift-or scanners, record lookup and two-phase verify);
 * the GPU engine reaches the same report through a different route (event
 * keys + a per-cluster walk), and tests compare the two.
 *
 *   searchPreproc 0x402710: OptErrors != 0 and detClass == 1 -> esimplePreproc
 *   esimpleSearch 0x4165e0: P->scan(beg, end, checkMatch 0x4151d0, P->fast, P)
 *   P->scan is always esimpleScan 0x4136d0 (esimplePreproc 0x4162df); it
 *   switches on P->fast->type (0x80c):
 *     1: k+1 pieces of one length, searched exactly by one multi-piece BNDM
 *     2: one pattern window [beg, end), backward (ABNDM) with k errors
 *     3: the pattern prefix [0, min(m,64)), forward shift-or with k errors
 *   The choice is nrgrep's cost model over letterProb (.data 0x621120):
 *   simpleFindBest 0x416a10 and the piece DP in esimplePreproc 0x415540.
 *
 *   A candidate (pos, piece i) is verified by checkMatch 0x4151d0 ->
 *   recGetRecord 0x402030 (the line around pos; its start is never before
 *   the search region start R) -> checkMatch1 0x414190: the part of the
 *   pattern left of the piece (L = off[i] positions) is matched BACKWARD
 *   from pos, the rest (m - L positions, the piece included) FORWARD from
 *   pos; each phase takes the nearest boundary with the fewest errors
 *   (row 0 ends the phase at once), the right phase gets what the left
 *   phase left of k.  recSearchFile 0x402250 prints the first verified
 *   match and resumes at its end.
 *
 * Two places where the binary's own code is not well defined, restated as
 * noted:
 *   - esimplePreproc 0x415a74 reads pprob[(l-1)*(mp+1)] before anything
 *     writes it (fresh heap); restated as 0.0 (the intended "no factor").
 *   - esimpleScan 0x41384b tests piece i with a 32-bit `1 << bit` (shll +
 *     cltq); restated exactly, i.e. for bit >= 32 the test mask is
 *     sign_extend_32(1 << (bit & 31)).
 * Transpositions (OptTransp) are never requested by PatMatch
 * (patmatch.py:299-314 builds only i/d/s), so their banks are left out.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PMN_NW 4            /* 64-bit words per position set: 256 positions */
#define PMN_MAXK 16
#define PMN_INS 1
#define PMN_DEL 2
#define PMN_SUB 4
#define PMN_START 2         /* '^' (OptStartLine) */
#define PMN_END 4           /* '$' (OptEndLine) */

/* letterProb, .data 0x621120 (256 doubles); pm_nrgrep_ext.c shares it */
const double pmn_letter_prob[256] = {
    0, 0, 0, 0, 0, 0, 0, 0,
    0, 0.000344, 0.020793, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0,
    0.146588, 4.3e-05, 0.00046, 0.000398, 0.01143, 0.003034, 0.001013, 0.001707,
    0.004156, 0.004162, 0.000506, 0.000998, 0.008441, 0.003342, 0.009616, 0.000903,
    0.002255, 0.004002, 0.002441, 0.001222, 0.000937, 0.001102, 0.000874, 0.000828,
    0.00097, 0.00181, 0.000679, 0.000168, 0.00019, 0.001562, 0.000143, 3.5e-05,
    8.6e-05, 0.002093, 0.001334, 0.00153, 0.000818, 0.000981, 0.001181, 0.000571,
    0.000754, 0.001534, 0.000156, 0.000228, 0.000656, 0.001308, 0.000922, 0.001299,
    0.001202, 0.000261, 0.000689, 0.001809, 0.003403, 0.000669, 0.00034, 0.000961,
    0.000158, 0.00039, 0.000234, 0.000847, 0.01584, 0.000846, 0.001258, 0.001695,
    0.000715, 0.053857, 0.011376, 0.0279, 0.021596, 0.094887, 0.015707, 0.013246,
    0.030408, 0.054368, 0.000933, 0.003729, 0.028211, 0.020693, 0.048064, 0.047054,
    0.018812, 0.002436, 0.044806, 0.048118, 0.065831, 0.016154, 0.006572, 0.008692,
    0.005656, 0.007099, 0.001124, 0.008146, 0.000445, 0.008146, 0.001852, 0,
    0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0,
    1e-06, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0,
    0, 0, 0, 0, 0, 0, 0, 0,
    0, 3.5e-05, 0, 0, 0, 0, 0, 0,
    0, 1.9e-05, 0, 0, 0, 3.2e-05, 0, 0,
    0, 9e-06, 0, 4e-05, 0, 0, 0, 0,
    0, 0, 2.7e-05, 0, 0, 0, 0, 0,
};

#define letterProb pmn_letter_prob

static inline uint8_t fold(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }

/* the class table nrgrep builds for byte c (simpleLoadMasks 0x4172b0 via
 * getAclass): with -i a class holds both cases, i.e. the folded byte's set.
 * B is [256][PMN_NW], bit i = pattern position i. */
static inline const uint64_t* cls(const uint64_t* B, int icase, uint8_t c) {
    return B + (size_t)(icase ? fold(c) : c) * PMN_NW;
}
static inline int isset(const uint64_t* w, int i) { return (int)((w[i >> 6] >> (i & 63)) & 1); }

/* ------------------------------------------------------------------------
 * cost model
 * ---------------------------------------------------------------------- */

/* pr[i]: sum of letterProb over the bytes position i accepts, bytes in
 * increasing order (simpleFindBest 0x416a70, esimplePreproc 0x4156b8) */
static void class_probs(const uint64_t* B, int m, int icase, double* pr) {
    for (int i = 0; i < m; ++i) {
        double s = 0.0;
        for (int c = 0; c < 256; ++c)
            if (isset(cls(B, icase, (uint8_t)c), i)) s += letterProb[c];
        pr[i] = s;
    }
}

/* simpleFindBest 0x416a10 (K = the error count): best pattern window for a
 * backward scan; returns the window's cost (1.0 if none beats 0.8). */
static double find_best(const double* pr, int m, int K, int* fwd, int* beg, int* end) {
    static double mprob[(256 + 1) * (256 + 1)];
    double pprob[256];
    int pos[256];
    const int M1 = m + 1;
    /* mprob[i][j] = pr[i] * .. * pr[i+j-1], 0 past m (0x416ad0 .. 0x416cb4) */
    mprob[m * M1] = 1.0;
    for (int s = 1; s <= m; ++s) mprob[m * M1 + s] = 0.0;
    for (int i = m - 1; i >= 0; --i) {
        mprob[i * M1] = 1.0;
        for (int s = 0; s < m; ++s) mprob[i * M1 + 1 + s] = pr[i] * mprob[(i + 1) * M1 + s];
    }
    *end = 0;
    *beg = 0;
    double best = 0.8;                                   /* 0x41d420 */
    for (int i = 0; i < m; ++i) {
        for (int d = 0; d < m; ++d) { pprob[d] = 0.0; pos[d] = i - 1 + d; }   /* 0x417135 */
        int j = K + 1 + i;                               /* r10 */
        if (m < j || j - i > 64) continue;
        int len = j - i;                                 /* r11 */
        for (;;) {
            const double k1 = (double)(K + 1);           /* xmm6 */
            const int lk = len - K;                      /* r14 */
            const double lim = (double)(lk + 1);         /* xmm4 */
            double sum = k1;                             /* xmm3 */
            if (len > 0 && !(k1 >= lim)) {
                const double x13 = (double)lk;
                const double x = k1 / ((x13 - k1) + 1.0);
                if (!(x >= best)) {
                    for (int t = 1;; ) {                 /* 0x416f70 */
                        int e = pos[t - 1] + 1;
                        double v = pprob[t - 1];
                        for (; e <= j; ++e) {
                            const double a = 1.0 - mprob[(e - t + 1) * M1 + t];
                            const double b = 1.0 - v;
                            v = 1.0 - b * a;
                            pprob[t - 1] = v;
                        }
                        pos[t - 1] = j;
                        sum = sum + v;
                        ++t;
                        if (t > len) break;
                        if (sum >= lim) break;
                        const double x1 = sum / ((x13 - sum) + 1.0);
                        if (!(x1 < best)) break;
                    }
                }
            }
            if (lim > sum) {                             /* 0x417012 */
                const double x = sum / (((double)lk - sum) + 1.0);
                if (best > x) { best = x; *beg = i; *end = j; }
            }
            if (m < j + 1) break;                        /* 0x417047 */
            ++j;
            len = j - i;
            if (len > 64) break;
        }
    }
    if (*end - *beg <= K + 1) { *end = 0; *beg = 0; }    /* 0x4170ba */
    *fwd = *end != 0;
    if (*end == 0) *end = m >= 65 ? 64 : m;
    return best < 0.8 ? best : 1.0;
}

/* out[0] = type, out[1] = piece length (type 1), out[2] = window beg,
 * out[3] = window end, out[4 ..] = L (left length) of each piece; returns
 * the number of pieces.  esimplePreproc 0x415540 (transpositions off). */
int pmn_plan(const uint64_t* B, int m, int k, int icase, int* out) {
    if (m < 1 || m > 256 || k < 1 || k > PMN_MAXK) return -1;
    double pr[256];
    class_probs(B, m, icase, pr);
    int fwd, wbeg, wend;
    const double prob = find_best(pr, m, k, &fwd, &wbeg, &wend);   /* 0x415601 */
    int ml = m;                                          /* m - k * OptTransp */
    if ((unsigned)ml > 64u) ml = 64;
    const int mp = ml / (k + 1);                         /* 0x41567a */
    const int P1 = mp + 1;
    static double mprob[257 * 257];
    static double cost[256 * 256];
    mprob[m * P1] = 1.0;
    for (int j = 1; j <= mp; ++j) mprob[m * P1 + j] = 0.0;
    for (int i = m - 1; i >= 0; --i) {                   /* 0x415761 */
        mprob[i * P1] = 1.0;
        for (int j = 1; j <= mp; ++j) mprob[i * P1 + j] = pr[i] * mprob[(i + 1) * P1 + j - 1];
    }
    /* cost[i][l]: 1 + sum_t P(a (t+1)-gram is a factor of pattern[i, i+l)) (0x4159c3) */
    for (int i = 0; i < m && mp > 0; ++i) {
        double prev[256], cur[256];
        for (int t = 0; t < mp; ++t) prev[t] = 0.0;      /* 0x415a21 memset; 0x415a74 see header */
        for (int l = 1; l <= mp; ++l) {
            double s = 1.0;
            for (int t = 0; t < l; ++t) {
                const int r = i + l - 1 - t;
                const double a = 1.0 - (r <= m ? mprob[r * P1 + t + 1] : 0.0);
                const double b = 1.0 - (t < l - 1 ? prev[t] : 0.0);
                cur[t] = 1.0 - a * b;
                s = s + cur[t];
            }
            cost[i * mp + l - 1] = s;
            memcpy(prev, cur, sizeof(double) * (size_t)l);
        }
    }
    const int K2 = k + 2;
    static double D[(256 + 1) * (PMN_MAXK + 2)];
    static int Wc[(256 + 1) * (PMN_MAXK + 2)];
    double best = 0.97;                                  /* 0x41d418 */
    int bestL = 0, offs[PMN_MAXK + 1];
    if (mp > 1 && !(1.0 / (double)mp > 0.97)) {          /* 0x415b29 */
        for (int L = mp;;) {                             /* 0x415d3f */
            for (int e = 0; e <= m; ++e) D[e * K2] = 0.0;
            for (int c = 1; c <= k + 1; ++c) D[m * K2 + c] = 1.0;
            for (int c = 1; c <= k + 1; ++c) {           /* 0x415ef0 */
                const int pmax = m - L - (c - 1) * L;
                for (int p = pmax; p >= 0; --p) {
                    const double x1 = cost[p * mp + L - 1];
                    double q;
                    if ((double)(L + 1) > x1) {
                        const double x = x1 / (((double)L - x1) + 1.0);
                        q = x <= 1.0 ? 1.0 - x : 0.0;
                    } else {
                        q = 0.0;
                    }
                    double val = 1.0 - q * (1.0 - D[(p + L) * K2 + c - 1]);
                    Wc[p * K2 + c] = p;
                    if (p < pmax && val > D[(p + 1) * K2 + c]) {
                        val = D[(p + 1) * K2 + c];
                        Wc[p * K2 + c] = Wc[(p + 1) * K2 + c];
                    }
                    D[p * K2 + c] = val;
                }
            }
            const double v = D[k + 1];                   /* 0x415ff4 */
            if (v < best) {
                int p = 0;
                for (int c = k + 1, idx = 0; c >= 1; --c, ++idx) {
                    p = Wc[p * K2 + c];
                    offs[idx] = p;
                    p = p + L;
                }
                best = v;
                bestL = L;
            }
            if (L - 1 <= 1) break;                       /* 0x41604a */
            const double inv = 1.0 / (double)(L - 1);
            --L;
            if (inv > best) break;
        }
    }
    int split = 0;
    if (0.97 > best && !(best >= (double)(k + 1) * prob) && bestL != 0) split = 1;   /* 0x4163c5 */
    if (split) {
        out[0] = 1; out[1] = bestL; out[2] = wbeg; out[3] = wend;
        for (int i = 0; i <= k; ++i) out[4 + i] = offs[i];
        return k + 1;
    }
    out[0] = fwd ? 2 : 3;                                /* 0x4162a6 */
    out[1] = 0; out[2] = wbeg; out[3] = wend;
    out[4] = fwd ? wbeg : wend;                          /* 0x416109 */
    return 1;
}

/* ------------------------------------------------------------------------
 * verification (checkMatch1 0x414190)
 * ---------------------------------------------------------------------- */

typedef struct {
    const uint8_t* t;
    int64_t n;
    const uint64_t* B;
    int m, k, errs, icase, mode;
    const int64_t* nl;        /* positions of every '\n' (sorted) */
    int64_t nnl;
    /* phase masks per (direction, left length), built on first use */
    int cached_L[2][PMN_MAXK + 1];
    uint64_t (*tab[2][PMN_MAXK + 1])[PMN_NW];
} ctx_t;

/* the phase table: bit r of tab[c] = pattern position p0 + dir * r accepts
 * byte c (simpleLoadVerif 0x4173f0 with start p0 and step dir) */
static const uint64_t (*phase_tab(ctx_t* x, int dir, int p0, int len))[PMN_NW] {
    const int d = dir > 0;
    const int L = d ? p0 : p0 + 1;
    int slot = -1;
    for (int i = 0; i <= PMN_MAXK; ++i) {
        if (x->tab[d][i] && x->cached_L[d][i] == L) return (const uint64_t (*)[PMN_NW])x->tab[d][i];
        if (!x->tab[d][i] && slot < 0) slot = i;
    }
    if (slot < 0) slot = 0;
    free(x->tab[d][slot]);
    uint64_t (*tab)[PMN_NW] = calloc(256, sizeof(*tab));
    for (int c = 0; c < 256; ++c) {
        const uint64_t* bc = cls(x->B, x->icase, (uint8_t)c);
        for (int r = 0; r < len; ++r)
            if (isset(bc, p0 + dir * r)) tab[c][r >> 6] |= 1ull << (r & 63);
    }
    x->tab[d][slot] = tab;
    x->cached_L[d][slot] = L;
    return (const uint64_t (*)[PMN_NW])tab;
}

/* recCheckLeftContext 0x402170 / recCheckRightContext 0x4021e0 (no -w) */
static int left_ok(const ctx_t* x, int64_t p, int64_t recbeg) {
    return !((x->mode & PMN_START) && p > recbeg && x->t[p - 1] != '\n');
}
static int right_ok(const ctx_t* x, int64_t q, int64_t recend) {
    return !((x->mode & PMN_END) && q < recend && x->t[q] != '\n');
}

/* one phase of checkMatch1: `len` pattern positions starting at pattern
 * position p0 and stepping `dir` (-1: the left part reversed, bit r =
 * position p0 - r, simpleLoadVerif(L, .., L-1, -1); +1: the right part,
 * bit r = position p0 + r); the text is read from pos leftwards (dir -1,
 * down to recbeg) or rightwards (dir +1, up to recend - 1).  Returns 1 and
 * the boundary (start for dir -1, end for dir +1) and its error count. */
static int phase(ctx_t* x, int64_t pos, int64_t recbeg, int64_t recend, int dir, int p0,
                 int len, int kmax, int64_t* bound, int* nerr) {
    const uint8_t* t = x->t;
    const int left = dir < 0;
    if (len == 0) {                                      /* 0x4141ef / 0x414eae */
        for (int e = 0; e <= kmax; ++e) {
            const int64_t b = left ? pos - e : pos + e;
            if (left ? left_ok(x, b, recbeg) : right_ok(x, b, recend)) { *bound = b; *nerr = e; return 1; }
            if (left ? b == recbeg : e == recend - pos) return 0;
            if (!(x->errs & PMN_INS)) return 0;
        }
        return 0;
    }
    const int W = (len + 63) >> 6, lw = W - 1;
    const uint64_t fin = 1ull << ((len - 1) & 63), alive_mask = fin * 2 - 1;
    uint64_t M[PMN_NW], R[PMN_MAXK + 1][PMN_NW], tmp0[PMN_NW], tmp1[PMN_NW];
    int maxk = kmax, best = kmax;
    int64_t found = -1;
    const uint64_t (*tab)[PMN_NW] = phase_tab(x, dir, p0, len);
    for (int j = 0; j <= maxk; ++j) {                    /* 0x414380 / 0x414958 */
        for (int w = 0; w < W; ++w) {
            uint64_t v = 0;
            if (x->errs & PMN_DEL) {
                if (j >= 64 * (w + 1)) v = ~0ull;
                else if (j > 64 * w) v = ~(~0ull << (j & 63));
            }
            R[j][w] = v;
        }
        if ((R[j][lw] & fin) && (left ? left_ok(x, pos, recbeg) : right_ok(x, pos, recend))) {
            best = j;
            maxk = j - 1;
            found = pos;
        }
    }
    if (left ? pos == recbeg : pos == recend) goto done;
    uint64_t inj = 1;
    for (int64_t p = pos;;) {
        int64_t cpos, b;
        if (left) { --p; cpos = p; b = p; } else { cpos = p; b = p + 1; ++p; }
        for (int w = 0; w < W; ++w) M[w] = tab[t[cpos]][w];
        uint64_t carry = inj;                            /* row 0: 0x41458a / 0x414b48 */
        for (int w = 0; w < W; ++w) {
            const uint64_t old = R[0][w];
            const uint64_t nv = ((old << 1) | carry) & M[w];
            tmp0[w] = old;
            tmp1[w] = nv;
            R[0][w] = nv;
            carry = old >> 63;
        }
        if ((R[0][lw] & fin) && (left ? left_ok(x, b, recbeg) : right_ok(x, b, recend))) {
            *bound = b;
            *nerr = 0;
            return 1;
        }
        for (int j = 1; j <= maxk; ++j) {                /* 0x414640 / 0x414c18 */
            uint64_t dc = 0, sc = inj, mc = inj;
            for (int w = 0; w < W; ++w) {
                uint64_t r10 = 0;
                if (x->errs & PMN_DEL) { r10 = (tmp1[w] << 1) | dc; dc = tmp1[w] >> 63; }
                if (x->errs & PMN_INS) r10 |= tmp0[w];
                if (x->errs & PMN_SUB) { r10 |= (tmp0[w] << 1) | sc; sc = tmp0[w] >> 63; }
                const uint64_t old = R[j][w];
                const uint64_t nv = (((old << 1) | mc) & M[w]) | r10;
                mc = old >> 63;
                tmp0[w] = old;
                tmp1[w] = nv;
                R[j][w] = nv;
            }
            if ((R[j][lw] & fin) && (left ? left_ok(x, b, recbeg) : right_ok(x, b, recend))) {
                int c = j;                               /* walk down 0x414834 / 0x414f7e */
                for (;;) {
                    const int d = c - 1;
                    if (d == -1) { *bound = b; *nerr = 0; return 1; }
                    if (!(R[d][lw] & fin)) { found = b; best = c; maxk = d; break; }
                    c = d;
                }
                break;
            }
        }
        int alive = 0;                                   /* 0x414de3 / 0x414fe3 */
        for (int w = 0; w < lw; ++w) alive |= R[maxk][w] != 0;
        alive |= (R[maxk][lw] & alive_mask) != 0;
        if (!alive) break;
        if (left ? p == recbeg : p == recend) break;
        inj = 0;
    }
done:
    if (found < 0) return 0;
    *bound = found;
    *nerr = best;
    return 1;
}

/* checkMatch 0x4151d0 + checkMatch1: verify piece/window `L` (left length)
 * at text position pos inside the region [R, n).  type 3 looks the record
 * up from pos - 1 (0x4152dc). */
static int verify(ctx_t* x, int type, int L, int64_t pos, int64_t R, int64_t* mb, int64_t* me) {
    const int64_t rp = type == 3 ? pos - 1 : pos;
    /* recGetRecord 0x402030: the last '\n' before rp (searched back to R
     * only), the first '\n' at/after rp */
    int64_t lo = 0, hi = x->nnl;                         /* first nl index with position >= rp */
    while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if (x->nl[mid] < rp) lo = mid + 1; else hi = mid;
    }
    int64_t recbeg = R;
    if (lo > 0 && x->nl[lo - 1] >= R) recbeg = x->nl[lo - 1] + 1;
    const int64_t recend = lo < x->nnl ? x->nl[lo] : x->n;
    if (rp < recbeg || rp >= recend) return 0;
    int64_t start, end;
    int eL, eR;
    if (!phase(x, pos, recbeg, recend, -1, L - 1, L, x->k, &start, &eL)) return 0;
    if (!phase(x, pos, recbeg, recend, +1, L, x->m - L, x->k - eL, &end, &eR)) return 0;
    *mb = start;
    *me = end;
    return 1;
}

/* ------------------------------------------------------------------------
 * scanners (esimpleScan 0x4136d0) over the region [R, n)
 * ---------------------------------------------------------------------- */

static int scan_pieces(ctx_t* x, const int* plan, int64_t R, int64_t* mb, int64_t* me) {
    const int mpc = plan[1], np = x->k + 1;
    const int* off = plan + 4;
    uint64_t T0[256], T2[256];                           /* esimpleLoadFast 0x4153fa */
    for (int c = 0; c < 256; ++c) {
        T0[c] = T2[c] = 0;
        const uint64_t* bc = cls(x->B, x->icase, (uint8_t)c);
        for (int r = 0; r < np; ++r)
            for (int pp = 0; pp < mpc; ++pp)
                if (isset(bc, off[r] + mpc - 1 - pp)) {
                    const uint64_t bit = 1ull << (r * mpc + pp);
                    T0[c] |= bit;
                    if (pp > 0) T2[c] |= bit;
                }
    }
    const uint8_t* t = x->t;
    int64_t r9 = R - 1;
    const int64_t limit = x->n - mpc;
    while (r9 < limit) {                                 /* 0x413780 */
        uint64_t D = T0[t[r9 + mpc]];
        if (!D) { r9 += mpc; continue; }
        int64_t a = r9 + mpc - 1;
        int e = mpc - 1;
        do {
            D = (D << 1) & T2[t[a]];
            --e;
            --a;
        } while (D && e);
        if (D) {
            for (int i = 0; i < np; ++i) {               /* 0x41384b: 32-bit shift */
                const int bit = i * mpc + mpc - 1;
                const uint64_t msk = (uint64_t)(int64_t)(int32_t)(1u << (bit & 31));
                if ((D & msk) && verify(x, 1, off[i], r9 + 1, R, mb, me)) return 1;
            }
        }
        r9 += e + 1;
    }
    return 0;
}

static int scan_backward(ctx_t* x, const int* plan, int64_t R, int64_t* mb, int64_t* me) {
    const int beg = plan[2], end = plan[3], Lw = end - beg, k = x->k;
    uint64_t T[256];                                     /* simpleLoadFast 0x417561 (backward) */
    for (int c = 0; c < 256; ++c) {
        T[c] = 0;
        const uint64_t* bc = cls(x->B, x->icase, (uint8_t)c);
        for (int r = 0; r < Lw; ++r)
            if (isset(bc, end - 1 - r)) T[c] |= 1ull << (64 - Lw + r);
    }
    const uint64_t top = ~0ull << (64 - Lw);
    const int W = Lw - k;
    const int64_t limit = x->n - (Lw - k - 1);
    uint64_t Rr[PMN_MAXK + 1], Tr[PMN_MAXK + 1];
    const uint8_t* t = x->t;
    for (int64_t s = R; s < limit;) {                    /* 0x413b6f */
        const uint64_t b0 = T[t[s + W - 1]];
        Rr[0] = b0;
        for (int j = 1; j <= k; ++j) { Rr[j] = top; Tr[j] = b0; }
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
            if (rb == 0) {                               /* 0x413ca1 */
                if ((Rr[k] >> 63) && verify(x, 2, plan[4], s, R, mb, me)) return 1;
                break;
            }
            if (!Rr[k] && !Tr[k]) break;
            --rb;
        }
        s += rb + 1;                                     /* 0x413cfa */
    }
    return 0;
}

static int scan_forward(ctx_t* x, const int* plan, int64_t R, int64_t* mb, int64_t* me) {
    const int Lw = plan[3], k = x->k;                    /* window [0, min(m,64)) */
    uint64_t T[256];                                     /* simpleLoadFast 0x417615 (forward) */
    const uint64_t full = Lw == 64 ? ~0ull : (1ull << Lw) - 1;
    for (int c = 0; c < 256; ++c) {
        T[c] = full;
        const uint64_t* bc = cls(x->B, x->icase, (uint8_t)c);
        for (int r = 0; r < Lw; ++r)
            if (isset(bc, r)) T[c] &= ~(1ull << r);
    }
    const uint64_t fin = 1ull << (Lw - 1);
    uint64_t Rr[PMN_MAXK + 1], Tr[PMN_MAXK + 1];
    for (int j = 0; j <= k; ++j) { Rr[j] = ~0ull << j; Tr[j] = ~0ull; }   /* 0x413905 */
    const uint8_t* t = x->t;
    for (int64_t p = R; p < x->n;) {                     /* 0x413932 */
        const uint64_t bc = T[t[p]];
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
        if (!(Rr[k] & fin) && verify(x, 3, plan[4], p, R, mb, me)) return 1;
    }
    return 0;
}

/* What nrgrep_coords prints for a class sequence at k > 0 (recSearchFile
 * 0x402250 over one buffer: region [R, n), print, R = match end, stop when
 * the match ends at n).  B: [256][4] position sets of the folded bytes.
 * Returns the number of matches (may exceed cap), -1 if out of range. */
int64_t pmn_esimple(const uint8_t* text, int64_t n, const uint64_t* B, int m, int k, int errs,
                    int icase, int mode, int64_t* out_beg, int64_t* out_end, int64_t cap) {
    int plan[4 + PMN_MAXK + 1];
    if (pmn_plan(B, m, k, icase, plan) < 0) return -1;
    ctx_t x;
    memset(&x, 0, sizeof(x));
    x.t = text; x.n = n; x.B = B; x.m = m; x.k = k; x.errs = errs; x.icase = icase; x.mode = mode;
    int64_t nnl = 0;
    for (int64_t p = 0; p < n; ++p) nnl += text[p] == '\n';
    int64_t* nl = malloc(sizeof(int64_t) * (size_t)(nnl + 1));
    nnl = 0;
    for (int64_t p = 0; p < n; ++p)
        if (text[p] == '\n') nl[nnl++] = p;
    x.nl = nl;
    x.nnl = nnl;
    int64_t count = 0, R = 0;
    while (R < n) {
        int64_t mb = 0, me = 0, ok;
        if (plan[0] == 1) ok = scan_pieces(&x, plan, R, &mb, &me);
        else if (plan[0] == 2) ok = scan_backward(&x, plan, R, &mb, &me);
        else ok = scan_forward(&x, plan, R, &mb, &me);
        if (!ok) break;
        if (count < cap) { out_beg[count] = mb; out_end[count] = me; }
        ++count;
        if (me == n) break;                              /* 0x4022eb */
        R = me;
    }
    free(nl);
    for (int d = 0; d < 2; ++d)
        for (int i = 0; i <= PMN_MAXK; ++i) free(x.tab[d][i]);
    return count;
}
