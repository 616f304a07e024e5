// pm_esimple.hip -- what nrgrep_coords reports for a class sequence at k > 0
// (nrgrep's "esimple" engine), on the GPU.
//
// The reference runs `nrgrep_coords -i -b 1600000 -k <k><ids> '<pattern>'`
// (www/FlaskApp/FlaskApp/patmatch.py:733-743).  For a plain class sequence
// with errors searchPreproc (0x402710) picks esimple; the binary's code
// (disassembled, never run; DESIGN.md §1, oracle/pm_nrgrep.c) does this:
//
//  * plan (esimplePreproc 0x415540): a cost model over letterProb (.data
//    0x621120) chooses one of three scanners (esimpleScan 0x4136d0):
//      1  k+1 pieces of one length at offsets L[0..k], found exactly by a
//         multi-piece BNDM; piece i at pos is tested with a 32-bit
//         `1 << bit` (0x41384b: shll + cltq), bit = i*len + len - 1;
//      2  one pattern window [wbeg, wend): ABNDM with k errors; a candidate
//         is a window start pos < n - (wend - wbeg - k - 1), L = wbeg;
//      3  the prefix [0, min(m, 64)): forward shift-or with k errors; a
//         candidate is a text position e (the window's end), L = wend, the
//         record is looked up from e - 1.
//  * verify (checkMatch 0x4151d0 -> checkMatch1 0x414190): inside the line
//    around the candidate (never before the search region start R), the
//    L pattern positions left of it are matched backward from pos and the
//    other m - L forward; each phase keeps the nearest boundary with the
//    fewest errors (row 0 ends it at once); the right phase gets what the
//    left phase left of k.
//  * report (recSearchFile 0x402250): the first verified candidate in scan
//    order is printed, R = its end, the scan restarts at R.
//
// GPU form.  The scan kernels (pm_linear / pm_ids / pm_nfa) produce every
// start of a match (oracle semantics).  Every start nrgrep can report is one
// of them, and a reported match starting at s ends before s + m + k, so the
// candidate list falls into independent clusters (consecutive starts more
// than 2(m + k) + 1 apart never interact: every phase reads at most
// m + k characters).  One thread per cluster then replays nrgrep's candidate
// order and verification over the cluster's text (k_es_walk); the matches
// it prints are written in place and compacted by the report pass's scatter.
#include "pm_internal.h"

#include <cmath>

namespace pm {

// ---------------------------------------------------------------------------
// plan (host): esimplePreproc's cost model, transpositions off (PatMatch's
// -k letters are i/d/s only, patmatch.py:299-314)
// ---------------------------------------------------------------------------
namespace {

// letterProb (.data 0x621120): the 73 non-zero entries
struct LP { uint8_t c; double p; };
const LP kLetterProb[] = {
    {9, 0.000344},  {10, 0.020793}, {32, 0.146588}, {33, 4.3e-05},  {34, 0.00046},  {35, 0.000398}, {36, 0.01143},
    {37, 0.003034}, {38, 0.001013}, {39, 0.001707}, {40, 0.004156}, {41, 0.004162}, {42, 0.000506}, {43, 0.000998},
    {44, 0.008441}, {45, 0.003342}, {46, 0.009616}, {47, 0.000903}, {48, 0.002255}, {49, 0.004002}, {50, 0.002441},
    {51, 0.001222}, {52, 0.000937}, {53, 0.001102}, {54, 0.000874}, {55, 0.000828}, {56, 0.00097},  {57, 0.00181},
    {58, 0.000679}, {59, 0.000168}, {60, 0.00019},  {61, 0.001562}, {62, 0.000143}, {63, 3.5e-05},  {64, 8.6e-05},
    {65, 0.002093}, {66, 0.001334}, {67, 0.00153},  {68, 0.000818}, {69, 0.000981}, {70, 0.001181}, {71, 0.000571},
    {72, 0.000754}, {73, 0.001534}, {74, 0.000156}, {75, 0.000228}, {76, 0.000656}, {77, 0.001308}, {78, 0.000922},
    {79, 0.001299}, {80, 0.001202}, {81, 0.000261}, {82, 0.000689}, {83, 0.001809}, {84, 0.003403}, {85, 0.000669},
    {86, 0.00034},  {87, 0.000961}, {88, 0.000158}, {89, 0.00039},  {90, 0.000234}, {91, 0.000847}, {92, 0.01584},
    {93, 0.000846}, {94, 0.001258}, {95, 0.001695}, {96, 0.000715}, {97, 0.053857}, {98, 0.011376}, {99, 0.0279},
    {100, 0.021596}, {101, 0.094887}, {102, 0.015707}, {103, 0.013246}, {104, 0.030408}, {105, 0.054368},
    {106, 0.000933}, {107, 0.003729}, {108, 0.028211}, {109, 0.020693}, {110, 0.048064}, {111, 0.047054},
    {112, 0.018812}, {113, 0.002436}, {114, 0.044806}, {115, 0.048118}, {116, 0.065831}, {117, 0.016154},
    {118, 0.006572}, {119, 0.008692}, {120, 0.005656}, {121, 0.007099}, {122, 0.001124}, {123, 0.008146},
    {124, 0.000445}, {125, 0.008146}, {126, 0.001852}, {160, 1e-06},  {225, 3.5e-05}, {233, 1.9e-05},
    {237, 3.2e-05}, {241, 9e-06},  {243, 4e-05},  {250, 2.7e-05},
};

#pragma clang fp contract(off)

inline bool bit_of(const uint64_t* B, int W, int c, int i) { return (B[(size_t)c * W + i / 64] >> (i % 64)) & 1; }

// simpleFindBest 0x416a10 with K errors: the cheapest window for a backward
// scan, or none (*fwd = 0, window = [0, min(m, 64)))
double find_best(const std::vector<double>& pr, int m, int K, int* fwd, int* beg, int* end) {
    const int M1 = m + 1;
    std::vector<double> mprob((size_t)M1 * M1, 0.0);
    mprob[(size_t)m * M1] = 1.0;
    for (int i = m - 1; i >= 0; --i) {
        mprob[(size_t)i * M1] = 1.0;
        for (int s = 0; s < m; ++s) mprob[(size_t)i * M1 + 1 + s] = pr[i] * mprob[(size_t)(i + 1) * M1 + s];
    }
    *beg = *end = 0;
    double best = 0.8;
    std::vector<double> pprob(m);
    std::vector<int> pos(m);
    for (int i = 0; i < m; ++i) {
        for (int d = 0; d < m; ++d) {
            pprob[d] = 0.0;
            pos[d] = i - 1 + d;
        }
        int j = K + 1 + i;
        if (m < j || j - i > 64) continue;
        for (int len = j - i;;) {
            const double k1 = (double)(K + 1);
            const int lk = len - K;
            const double lim = (double)(lk + 1);
            double sum = k1;
            if (len > 0 && !(k1 >= lim) && !(k1 / (((double)lk - k1) + 1.0) >= best)) {
                for (int t = 1;;) {
                    double v = pprob[t - 1];
                    for (int e = pos[t - 1] + 1; e <= j; ++e) {
                        const double a = 1.0 - mprob[(size_t)(e - t + 1) * M1 + t];
                        v = 1.0 - (1.0 - v) * a;
                        pprob[t - 1] = v;
                    }
                    pos[t - 1] = j;
                    sum = sum + v;
                    if (++t > len || sum >= lim || !(sum / (((double)lk - sum) + 1.0) < best)) break;
                }
            }
            if (lim > sum) {
                const double x = sum / (((double)lk - sum) + 1.0);
                if (best > x) {
                    best = x;
                    *beg = i;
                    *end = j;
                }
            }
            if (m < j + 1 || (len = ++j - i) > 64) break;
        }
    }
    if (*end - *beg <= K + 1) *beg = *end = 0;
    *fwd = *end != 0;
    if (!*end) *end = m >= 65 ? 64 : m;
    return best < 0.8 ? best : 1.0;
}

}  // namespace

EsPlan es_plan(const uint64_t* B, int W, int m, int k) {
    require(m >= 1 && m <= PM_MAX_POSITIONS && k >= 1 && k <= PM_MAX_K, "esimple plan: m or k out of range");
    // class probabilities, bytes in increasing order (0x4156b8); B holds the
    // folded byte's set, and with -i a class holds both cases (getAclass)
    std::vector<double> pr(m, 0.0);
    for (int i = 0; i < m; ++i) {
        double s = 0.0;
        for (const LP& e : kLetterProb)
            if (bit_of(B, W, fold(e.c), i)) s += e.p;
        pr[i] = s;
    }
    EsPlan P{};
    int fwd = 0, wbeg = 0, wend = 0;
    const double prob = find_best(pr, m, k, &fwd, &wbeg, &wend);
    const int ml = m > 64 ? 64 : m;
    const int mp = ml / (k + 1);
    const int P1 = mp + 1;
    std::vector<double> mprob((size_t)(m + 1) * P1, 0.0);
    mprob[(size_t)m * P1] = 1.0;
    for (int i = m - 1; i >= 0; --i) {
        mprob[(size_t)i * P1] = 1.0;
        for (int j = 1; j <= mp; ++j) mprob[(size_t)i * P1 + j] = pr[i] * mprob[(size_t)(i + 1) * P1 + j - 1];
    }
    // cost[i][l] = 1 + sum over t of P(a random (t+1)-gram is a factor of
    // pattern[i, i + l)) (0x4159c3; the never-written diagonal reads as 0)
    std::vector<double> cost((size_t)m * std::max(mp, 1), 0.0);
    for (int i = 0; i < m && mp > 0; ++i) {
        std::vector<double> prev(mp, 0.0), cur(mp, 0.0);
        for (int l = 1; l <= mp; ++l) {
            double s = 1.0;
            for (int t = 0; t < l; ++t) {
                const int r = i + l - 1 - t;
                const double a = 1.0 - (r <= m ? mprob[(size_t)r * P1 + t + 1] : 0.0);
                const double b = 1.0 - (t < l - 1 ? prev[t] : 0.0);
                cur[t] = 1.0 - a * b;
                s = s + cur[t];
            }
            cost[(size_t)i * mp + l - 1] = s;
            prev = cur;
        }
    }
    // the piece DP (0x415d3f): D[p][c] = the best "probability" of placing
    // c pieces of length L in [p, m); W records the placement
    const int K2 = k + 2;
    std::vector<double> D((size_t)(m + 1) * K2, 0.0);
    std::vector<int> Wc((size_t)(m + 1) * K2, 0);
    double best = 0.97;
    int bestL = 0;
    int offs[PM_MAX_K + 1] = {};
    if (mp > 1 && !(1.0 / (double)mp > 0.97)) {
        for (int L = mp;;) {
            for (int e = 0; e <= m; ++e) D[(size_t)e * K2] = 0.0;
            for (int c = 1; c <= k + 1; ++c) D[(size_t)m * K2 + c] = 1.0;
            for (int c = 1; c <= k + 1; ++c) {
                const int pmax = m - L - (c - 1) * L;
                for (int p = pmax; p >= 0; --p) {
                    const double x1 = cost[(size_t)p * mp + L - 1];
                    double q = 0.0;
                    if ((double)(L + 1) > x1) {
                        const double x = x1 / (((double)L - x1) + 1.0);
                        q = x <= 1.0 ? 1.0 - x : 0.0;
                    }
                    double val = 1.0 - q * (1.0 - D[(size_t)(p + L) * K2 + c - 1]);
                    Wc[(size_t)p * K2 + c] = p;
                    if (p < pmax && val > D[(size_t)(p + 1) * K2 + c]) {
                        val = D[(size_t)(p + 1) * K2 + c];
                        Wc[(size_t)p * K2 + c] = Wc[(size_t)(p + 1) * K2 + c];
                    }
                    D[(size_t)p * K2 + c] = val;
                }
            }
            if (D[k + 1] < best) {
                for (int c = k + 1, idx = 0, p = 0; c >= 1; --c, ++idx) {
                    p = Wc[(size_t)p * K2 + c];
                    offs[idx] = p;
                    p += L;
                }
                best = D[k + 1];
                bestL = L;
            }
            if (L - 1 <= 1) break;
            const double inv = 1.0 / (double)(L - 1);
            --L;
            if (inv > best) break;
        }
    }
    if (0.97 > best && !(best >= (double)(k + 1) * prob) && bestL != 0) {   // 0x4163c5
        P.type = 1;
        P.piece_len = bestL;
        P.npieces = k + 1;
        for (int i = 0; i <= k; ++i) P.L[i] = offs[i];
    } else {
        P.type = fwd ? 2 : 3;
        P.npieces = 1;
        P.L[0] = fwd ? wbeg : wend;
    }
    P.wbeg = wbeg;
    P.wend = wend;
    return P;
}

#pragma clang fp contract(on)

// ---------------------------------------------------------------------------
// per-pattern tables (host) and their device view
// ---------------------------------------------------------------------------
void es_add_slot(EsBuild& b, const uint64_t* B, int W, int m, int k, int errs, uint32_t flags, int32_t pid) {
    require(W >= 1 && W <= 4 && m <= 64 * W, "esimple: bad position words");
    const EsPlan P = es_plan(B, W, m, k);
    EsSlot s{};
    s.m = m;
    s.k = k;
    s.errs = errs;
    s.type = P.type;
    s.mpc = P.piece_len;
    s.wbeg = P.wbeg;
    s.wend = P.wend;
    s.W = W;
    s.np = P.npieces;
    s.anchors = (int32_t)(flags & (PM_ANCHOR_START | PM_ANCHOR_END));
    s.pid = pid;
    for (int i = 0; i < s.np; ++i) {
        s.L[i] = P.L[i];
        if (P.type == 1) {
            const int bit = i * P.piece_len + P.piece_len - 1;
            s.test[i] = (uint64_t)(int64_t)(int32_t)(1u << (bit & 31));
        }
    }
    // B | TL[np] | TR[np], each [256][W]: bit r of TL[i][c] = position
    // L_i - 1 - r accepts c (simpleLoadVerif(L, .., L-1, -1)); of TR[i][c]
    // = position L_i + r (simpleLoadVerif(m - L, .., L, +1))
    const size_t per = (size_t)256 * W;
    s.o_B = b.tab.size();
    b.tab.insert(b.tab.end(), B, B + per);
    s.o_TL = b.tab.size();
    b.tab.resize(b.tab.size() + per * s.np, 0);
    s.o_TR = b.tab.size();
    b.tab.resize(b.tab.size() + per * s.np, 0);
    for (int i = 0; i < s.np; ++i) {
        const int L = s.L[i];
        for (int c = 0; c < 256; ++c) {
            for (int r = 0; r < L; ++r)
                if (bit_of(B, W, c, L - 1 - r)) b.tab[s.o_TL + per * i + (size_t)c * W + r / 64] |= 1ull << (r % 64);
            for (int r = 0; r < m - L; ++r)
                if (bit_of(B, W, c, L + r)) b.tab[s.o_TR + per * i + (size_t)c * W + r / 64] |= 1ull << (r % 64);
        }
    }
    b.slots.push_back(s);
}

void es_upload(const EsBuild& b, Upload& up, EsUpload& u) {
    u.o_slots = up.add(b.slots.data(), b.slots.size() * sizeof(EsSlot));
    u.o_tab = up.add(b.tab.data(), b.tab.size() * sizeof(uint64_t));
    u.nslots = (int)b.slots.size();
    u.pid_base = b.slots.empty() ? 0 : b.slots[0].pid;
}

EsPrep es_bind(const EsUpload& u, const uint8_t* d_up, int32_t gap_max) {
    EsPrep p;
    p.slots = reinterpret_cast<const EsSlot*>(d_up + u.o_slots);
    p.tab = reinterpret_cast<const uint64_t*>(d_up + u.o_tab);
    p.nslots = u.nslots;
    p.pid_base = u.pid_base;
    p.gap_max = gap_max;
    return p;
}

int32_t es_gap(const EsBuild& b) {
    int32_t g = 0;
    for (const EsSlot& s : b.slots) g = std::max(g, 2 * (s.m + s.k) + 2);
    return g;
}

// ---------------------------------------------------------------------------
// device: the per-cluster replay
// ---------------------------------------------------------------------------
namespace {

constexpr uint64_t ES_POS_MASK = (1ull << 48) - 1;

struct EsText {
    TextView tv;
    uint64_t n;
    // a record break: '\n', a header-line byte, the end of the text
    __device__ bool brk(uint64_t p) const {
        if (p >= n) return true;
        if (tv.nuc_layout) {
            const Loc l = loc_of(p);
            return (tv.nuc.bo[l.word].x >> l.bit) & 1;
        }
        return tv.bytes[p] == (uint8_t)'\n';
    }
    // the (folded) byte inside a record
    __device__ uint8_t chr(uint64_t p) const { return tv.nuc_layout ? nuc_char_at(tv.nuc, p) : tv.bytes[p]; }
    // the file's own (folded) byte, header lines and '\n' included: what
    // the BNDM scanner reads
    __device__ uint8_t raw(uint64_t p) const { return tv.nuc_layout ? nuc_raw_at(tv.nuc, p) : tv.raw[p]; }
};

struct EsCtx {
    const EsSlot* S;
    const uint64_t* tab;
    EsText t;
    uint64_t R;   // the search region start
    // recCheckLeftContext 0x402170 / recCheckRightContext 0x4021e0; p ==
    // recbeg <=> p == R or p starts its line (a record holds no break)
    __device__ bool at_recbeg(uint64_t p) const { return p == R || p == 0 || t.brk(p - 1); }
    __device__ bool left_ok(uint64_t p) const { return !(S->anchors & PM_ANCHOR_START) || at_recbeg(p); }
    __device__ bool right_ok(uint64_t q) const { return !(S->anchors & PM_ANCHOR_END) || t.brk(q); }
};

// one phase of checkMatch1 (left: dir < 0, bit r = position L - 1 - r read
// backward from pos; right: bit r = position L + r read forward from pos).
// Returns the boundary (start / end) and its error count.
__device__ bool es_phase(const EsCtx& x, const uint64_t* T, uint64_t pos, bool left, int len, int kmax,
                         uint64_t& bound, int& nerr) {
    const int errs = x.S->errs;
    if (len == 0) {   // 0x4141ef / 0x414eae
        for (int e = 0; e <= kmax; ++e) {
            const uint64_t b = left ? pos - e : pos + e;
            if (left ? x.left_ok(b) : x.right_ok(b)) {
                bound = b;
                nerr = e;
                return true;
            }
            if (left ? x.at_recbeg(b) : x.t.brk(b)) return false;
            if (!(errs & PM_ERR_INS)) return false;
        }
        return false;
    }
    const int W = (len + 63) >> 6, lw = W - 1;
    const uint64_t fin = 1ull << ((len - 1) & 63), alive_mask = fin * 2 - 1;
    uint64_t Rw[PM_MAX_K + 1][4];
    int maxk = kmax, best = kmax;
    bool found = false;
    uint64_t fb = 0;
    for (int j = 0; j <= maxk; ++j) {   // 0x414380: deletions reach the first j positions
        for (int w = 0; w < W; ++w) {
            uint64_t v = 0;
            if (errs & PM_ERR_DEL) {
                if (j >= 64 * (w + 1)) v = ~0ull;
                else if (j > 64 * w) v = ~(~0ull << (j & 63));
            }
            Rw[j][w] = v;
        }
        if ((Rw[j][lw] & fin) && (left ? x.left_ok(pos) : x.right_ok(pos))) {
            best = j;
            maxk = j - 1;
            found = true;
            fb = pos;
        }
    }
    if (!(left ? x.at_recbeg(pos) : x.t.brk(pos))) {
        uint64_t inj = 1, p = pos;
        for (;;) {
            uint64_t b;
            uint8_t c;
            if (left) {
                --p;
                c = x.t.chr(p);
                b = p;
            } else {
                c = x.t.chr(p);
                b = ++p;
            }
            const uint64_t* M = T + (size_t)c * x.S->W;
            uint64_t t0[4], t1[4];
            uint64_t carry = inj;
            for (int w = 0; w < W; ++w) {   // row 0
                const uint64_t old = Rw[0][w];
                const uint64_t nv = ((old << 1) | carry) & M[w];
                t0[w] = old;
                t1[w] = nv;
                Rw[0][w] = nv;
                carry = old >> 63;
            }
            if ((Rw[0][lw] & fin) && (left ? x.left_ok(b) : x.right_ok(b))) {
                bound = b;
                nerr = 0;
                return true;
            }
            for (int j = 1; j <= maxk; ++j) {   // 0x414640: rows 1..maxk
                uint64_t dc = 0, sc = inj, mc = inj;
                for (int w = 0; w < W; ++w) {
                    uint64_t r = 0;
                    if (errs & PM_ERR_DEL) {
                        r = (t1[w] << 1) | dc;
                        dc = t1[w] >> 63;
                    }
                    if (errs & PM_ERR_INS) r |= t0[w];
                    if (errs & PM_ERR_SUB) {
                        r |= (t0[w] << 1) | sc;
                        sc = t0[w] >> 63;
                    }
                    const uint64_t old = Rw[j][w];
                    const uint64_t nv = (((old << 1) | mc) & M[w]) | r;
                    mc = old >> 63;
                    t0[w] = old;
                    t1[w] = nv;
                    Rw[j][w] = nv;
                }
                if ((Rw[j][lw] & fin) && (left ? x.left_ok(b) : x.right_ok(b))) {
                    // the rows below j do not reach the end here (else they
                    // had returned first): record, look for fewer errors
                    int c2 = j;
                    for (;;) {
                        const int d = c2 - 1;
                        if (d < 0) {
                            bound = b;
                            nerr = 0;
                            return true;
                        }
                        if (!(Rw[d][lw] & fin)) {
                            found = true;
                            fb = b;
                            best = c2;
                            maxk = d;
                            break;
                        }
                        c2 = d;
                    }
                    break;
                }
            }
            bool alive = false;   // 0x414de3: the highest live row
            for (int w = 0; w < lw; ++w) alive |= Rw[maxk][w] != 0;
            alive |= (Rw[maxk][lw] & alive_mask) != 0;
            if (!alive) break;
            if (left ? x.at_recbeg(p) : x.t.brk(p)) break;
            inj = 0;
        }
    }
    if (!found) return false;
    bound = fb;
    nerr = best;
    return true;
}

// checkMatch 0x4151d0 + checkMatch1 0x414190 for candidate (pos, piece i)
__device__ bool es_verify(const EsCtx& x, uint64_t pos, int i, uint64_t& mb, uint64_t& me) {
    const EsSlot& S = *x.S;
    const uint64_t rp = S.type == 3 ? pos - 1 : pos;   // 0x4152dc
    if (x.t.brk(rp)) return false;                      // the record ends at rp
    const size_t per = (size_t)256 * S.W;
    const int L = S.L[i];
    uint64_t start, end;
    int eL, eR;
    if (!es_phase(x, x.tab + S.o_TL + per * i, pos, true, L, S.k, start, eL)) return false;
    if (!es_phase(x, x.tab + S.o_TR + per * i, pos, false, S.m - L, S.k - eL, end, eR)) return false;
    mb = start;
    me = end;
    return true;
}

// the pieces that match exactly at pos, as BNDM's surviving bits
__device__ uint64_t es_pieces_at(const EsCtx& x, uint64_t pos) {
    const EsSlot& S = *x.S;
    const uint64_t* B = x.tab + S.o_B;
    uint64_t D = 0;
    for (int r = 0; r < S.np; ++r) {
        bool ok = true;
        for (int j = 0; j < S.mpc && ok; ++j) {
            const int q = S.L[r] + j;
            ok = (B[(size_t)x.t.raw(pos + j) * S.W + q / 64] >> (q % 64)) & 1;
        }
        if (ok) D |= 1ull << (r * S.mpc + S.mpc - 1);
    }
    return D;
}

__global__ void k_es_heads(const uint64_t* __restrict__ keys, const uint64_t* total_d, uint64_t total_h,
                           uint8_t* __restrict__ acc, uint32_t* __restrict__ bcnt, uint32_t G, int32_t gap) {
    const uint64_t total = total_d ? *total_d : total_h;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t b = tid; b < G; b += stride) bcnt[b] = 0u;
    for (uint64_t i = tid; i < total; i += stride) {
        // a new pattern (high key bits) or a gap wider than any phase reads
        const bool head = i == 0 || keys[i] - keys[i - 1] > (uint64_t)gap;
        acc[i] = head ? 2 : 0;
    }
}

__global__ void k_es_walk(EsPrep P, uint64_t* __restrict__ keys, uint32_t* __restrict__ lens, const uint64_t* total_d,
                          uint64_t total_h, uint8_t* __restrict__ acc, uint32_t* __restrict__ bcnt, uint32_t G,
                          TextView tv) {
    const uint64_t total = total_d ? *total_d : total_h;
    const uint64_t C = (total + G - 1) / G;   // the scatter's chunk
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        if (!(acc[i] & 2)) continue;
        uint64_t j = i + 1;   // the next cluster's head keeps bit 1 set whatever its owner writes
        while (j < total && !(acc[j] & 2)) ++j;
        const uint64_t lo = keys[i] & ES_POS_MASK, hi = keys[j - 1] & ES_POS_MASK;
        const uint64_t pid = keys[i] >> 48;
        const uint64_t nmax = j - i;
        uint64_t nout = 0;
        const int64_t slot = (int64_t)pid - P.pid_base;
        if (slot >= 0 && slot < P.nslots) {
            const EsSlot& S = P.slots[slot];
            EsCtx x{&S, P.tab, EsText{tv, tv.n}, 0};
            const uint64_t n = tv.n;
            const uint64_t pmax = umin64(n, hi + (uint64_t)(S.m + S.k));
            // type 2: ABNDM windows of wend - wbeg - k characters must fit (0x413a5b)
            const uint64_t wtail = (uint64_t)(S.wend - S.wbeg - S.k - 1);
            const uint64_t lim2 = S.type == 2 ? (n > wtail ? n - wtail : 0) : n + 1;
            uint64_t pos = S.type == 3 ? lo + 1 : lo;
            uint64_t guard = (pmax - lo + 2) * (uint64_t)(S.np + 2) * 4;
            while (pos <= pmax && guard--) {
                bool hit = false;
                uint64_t mb = 0, me = 0;
                if (S.type == 1) {
                    if (pos + (uint64_t)S.mpc <= n) {
                        const uint64_t D = es_pieces_at(x, pos);
                        for (int q = 0; q < S.np && !hit; ++q)
                            if (D & S.test[q]) hit = es_verify(x, pos, q, mb, me);
                    }
                } else if (pos < lim2) {
                    hit = es_verify(x, pos, 0, mb, me);
                }
                if (!hit) {
                    ++pos;
                    continue;
                }
                if (nout < nmax) {   // matches start at distinct candidates: never more than the cluster holds
                    keys[i + nout] = (pid << 48) | mb;
                    lens[i + nout] = (uint32_t)(me - mb);
                    acc[i + nout] = (nout == 0 ? 2 : 0) | 1;
                    atomicAdd(&bcnt[(i + nout) / C], 1u);
                    ++nout;
                }
                if (me >= n) break;   // 0x4022eb: a match that ends the region ends the search
                x.R = me;
                pos = S.type == 3 ? me + 1 : me;
            }
        }
        for (uint64_t q = i + nout; q < j; ++q) acc[q] = q == i ? 2 : 0;
    }
}

}  // namespace

void es_launch(const EsPrep& P, uint64_t* keys, uint32_t* lens, const uint64_t* total_d, uint64_t total_h,
               uint8_t* acc, uint32_t* bcnt, uint32_t G, const TextView& tv, hipStream_t s) {
    const uint32_t blocks = 1024;
    hipLaunchKernelGGL(k_es_heads, dim3(blocks), dim3(256), 0, s, keys, total_d, total_h, acc, bcnt, G, P.gap_max);
    hipLaunchKernelGGL(k_es_walk, dim3(blocks), dim3(64), 0, s, P, keys, lens, total_d, total_h, acc, bcnt, G, tv);
    HIPCHK(hipGetLastError());
}

}  // namespace pm

using namespace pm;

extern "C" int pm_esimple_plan(int m, int words, const uint64_t* byte_mask, int k, int32_t* out) {
    return guarded([&] {
        require(byte_mask != nullptr && out != nullptr, "null argument");
        require(words >= 1 && words <= 4 && m >= 1 && m <= 64 * words, "m / words out of range");
        const EsPlan P = es_plan(byte_mask, words, m, k);
        out[0] = P.type;
        out[1] = P.piece_len;
        out[2] = P.wbeg;
        out[3] = P.wend;
        out[4] = P.npieces;
        for (int i = 0; i < P.npieces; ++i) out[5 + i] = P.L[i];
    });
}
