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
#include <map>

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

void letter_probs(double out[256]) {
    for (int c = 0; c < 256; ++c) out[c] = 0.0;
    for (const LP& e : kLetterProb) out[e.c] = e.p;
}

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
    // lone starts need no walk (k_es_walk): substitutions only, no
    // anchors, and every piece test sees its own piece (the 32-bit shift
    // misses bits 32..63)
    s.lone = errs == PM_ERR_SUB && !s.anchors;
    for (int i = 0; i < s.np; ++i) {
        s.L[i] = P.L[i];
        if (P.type == 1) {
            const int bit = i * P.piece_len + P.piece_len - 1;
            s.test[i] = (uint64_t)(int64_t)(int32_t)(1u << (bit & 31));
            if (!((s.test[i] >> bit) & 1)) s.lone = 0;
        } else {
            s.test[i] = ~0ull;   // the one window / prefix candidate
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
    // type 1: the pieces packed as BNDM holds them (piece i in bits
    // [i * len, i * len + len)): bit i * len + j of P[c] = position L_i + j
    // accepts c.  A forward shift-and over P finds the pieces that match
    // exactly at a window start (its last bits) -- BNDM's D there.
    s.o_P = b.tab.size();
    if (s.type == 1) {
        require(s.np * s.mpc <= 64, "esimple: pieces exceed a word");
        b.tab.resize(b.tab.size() + 256, 0);
        for (int i = 0; i < s.np; ++i) {
            s.pstart |= 1ull << (i * s.mpc);
            s.pend |= 1ull << (i * s.mpc + s.mpc - 1);
            for (int j = 0; j < s.mpc; ++j)
                for (int c = 0; c < 256; ++c)
                    if (bit_of(B, W, c, s.L[i] + j)) b.tab[s.o_P + c] |= 1ull << (i * s.mpc + j);
        }
    }
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

// The walk's tables over a compact alphabet: bytes whose rows agree in every
// table of every slot share a code (a DNA query: A, C, G, T, '\n' and "the
// rest"), code 0 is '\n' alone (a break).  The tables then shrink from 256
// rows to a few and k_es_walk keeps them, and the byte -> code map, in LDS:
// its per-step lookups are LDS reads instead of a chain of global loads.
void es_upload(const EsBuild& b, Upload& up, EsUpload& u) {
    std::vector<std::vector<uint64_t>> sig(256);
    for (int c = 0; c < 256; ++c)
        for (const EsSlot& sl : b.slots) {
            const size_t W = sl.W, per = 256 * W;
            for (size_t w = 0; w < W; ++w) {
                sig[c].push_back(b.tab[sl.o_B + c * W + w]);
                for (int i = 0; i < sl.np; ++i) {
                    sig[c].push_back(b.tab[sl.o_TL + per * i + c * W + w]);
                    sig[c].push_back(b.tab[sl.o_TR + per * i + c * W + w]);
                }
            }
            if (sl.type == 1) sig[c].push_back(b.tab[sl.o_P + c]);
        }
    std::vector<uint8_t> cmap(256, 0);
    std::vector<int> rep{'\n'};   // the byte whose rows a code takes
    {
        std::map<std::vector<uint64_t>, int> code;
        for (int c = 0; c < 256; ++c) {
            if (c == '\n') continue;
            auto it = code.find(sig[c]);
            if (it == code.end()) {
                it = code.emplace(sig[c], (int)rep.size()).first;
                rep.push_back(c);
            }
            cmap[c] = (uint8_t)it->second;
        }
    }
    const int nc = (int)rep.size();
    std::vector<EsSlot> slots = b.slots;
    std::vector<uint64_t> ctab;
    auto rows = [&](uint64_t o, size_t W) {   // [nc][W] from [256][W] at o
        const uint64_t at = ctab.size();
        for (int q = 0; q < nc; ++q)
            for (size_t w = 0; w < W; ++w) ctab.push_back(b.tab[o + rep[q] * W + w]);
        return at;
    };
    for (size_t j = 0; j < slots.size(); ++j) {
        EsSlot& sl = slots[j];
        const EsSlot& src = b.slots[j];
        const size_t W = sl.W, per = 256 * W;
        sl.o_B = rows(src.o_B, W);
        sl.o_TL = ctab.size();
        for (int i = 0; i < sl.np; ++i) rows(src.o_TL + per * i, W);
        sl.o_TR = ctab.size();
        for (int i = 0; i < sl.np; ++i) rows(src.o_TR + per * i, W);
        sl.o_P = sl.type == 1 ? rows(src.o_P, 1) : 0;
    }
    u.o_slots = up.add(slots.data(), slots.size() * sizeof(EsSlot));
    u.o_tab = up.add(ctab.data(), ctab.size() * sizeof(uint64_t));
    u.o_map = up.add(cmap.data(), cmap.size());
    u.tab_words = (uint32_t)ctab.size();
    u.ncodes = nc;
    u.nslots = (int)b.slots.size();
    u.pid_base = b.slots.empty() ? 0 : b.slots[0].pid;
    u.wmax = 1;
    u.kmax = 1;
    for (const EsSlot& sl : b.slots) {
        u.wmax = std::max(u.wmax, (int)sl.W);
        u.kmax = std::max(u.kmax, (int)sl.k);
    }
}

EsPrep es_bind(const EsUpload& u, const uint8_t* d_up, int32_t gap_max) {
    EsPrep p;
    p.slots = reinterpret_cast<const EsSlot*>(d_up + u.o_slots);
    p.tab = reinterpret_cast<const uint64_t*>(d_up + u.o_tab);
    p.cmap = d_up + u.o_map;
    p.tab_words = u.tab_words;
    p.ncodes = u.ncodes;
    p.nslots = u.nslots;
    p.pid_base = u.pid_base;
    p.gap_max = gap_max;
    p.wmax = u.wmax;
    p.kmax = u.kmax;
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

constexpr int ES_CHUNK = 16;     // positions staged per refill of a thread's window
constexpr int ES_THREADS = 256;  // walk threads per block (4 waves: the block's tables in LDS serve them all)
constexpr int ES_SPAN = 16;      // window starts whose pieces one shift-and pass finds
constexpr size_t ES_TAB_LDS = 16 << 10;   // compact tables kept in LDS up to this size
constexpr size_t ES_SLOTS_LDS = 4 << 10;  // slots kept in LDS up to this size
static_assert(sizeof(EsSlot) % 8 == 0, "k_es_walk copies the slots in 8-byte words");

// A thread's text window: the codes (es_upload) of the line-bounded bytes of
// positions [lo, hi) in an LDS ring of win (a power of two) bytes.  The walk
// moves forward and every phase reads at most m + k + 1 positions on either
// side of the candidate; before each candidate the walk tops the ring up to
// pos + m + k + 2 (EsText::fill), so with win >= gap_max + ES_CHUNK every
// read hits it; a read outside it (a pattern wider than the ring was sized
// for) goes to memory.  A refill issues ES_CHUNK independent loads at once
// instead of one dependent load per step.
extern __shared__ uint8_t es_lds[];   // k_es_walk: win bytes per thread

struct EsRing {
    uint32_t base;   // the thread's ring in es_lds
    uint32_t mask;   // win - 1 (win = 0: no ring)
    uint64_t lo, hi; // valid positions [lo, hi)
};

struct EsText {
    TextView tv;
    uint64_t n;
    EsRing r;
    const uint8_t* cmap;   // byte -> code (LDS); code 0 = a break
    // the line-bounded byte's code from memory: 0 for breaks and past the end
    __device__ uint8_t load(uint64_t p) const {
        if (p >= n) return 0;
        return cmap[tv.nuc_layout ? nuc_char_at(tv.nuc, p) : tv.bytes[p]];
    }
    __device__ void restart(uint64_t p) { r.lo = r.hi = p; }
    // extend the ring to cover [.., upto).  NUC: one 16-byte load of the
    // position-contiguous planes (pm_db::lin) gives 32 positions; an
    // "other" byte (N, IUPAC letters) comes from the side tables (rare).
    // BYTE: ES_CHUNK bytes per round trip.
    __device__ void fill(uint64_t upto) {
        if (r.mask == ~0u) return;
        while (r.hi < upto) {
            const uint64_t b = r.hi;
            if (b >= n) {
                const uint32_t cnt = (uint32_t)umin64(ES_CHUNK, upto - b);
                for (uint32_t q = 0; q < cnt; ++q) es_lds[r.base + ((uint32_t)(b + q) & r.mask)] = 0;
                r.hi = b + cnt;
            } else if (tv.nuc_layout) {
                // the whole 32-position word, four codes per 32-bit LDS store
                // (a word's slots never wrap: win >= 64 is a power of two);
                // positions of the word before b get the codes they hold
                // already, or sit below the ring (round 6: one byte store
                // and a table read per position before)
                const uint64_t wb = b & ~31ull;
                const uint4 v = tv.nuc.lin[wb >> 5];
                const uint32_t acgt4 = (uint32_t)cmap['A'] | (uint32_t)cmap['C'] << 8 | (uint32_t)cmap['G'] << 16 |
                                       (uint32_t)cmap['T'] << 24;
                uint32_t* dst = reinterpret_cast<uint32_t*>(es_lds + r.base + ((uint32_t)wb & r.mask));
#pragma unroll
                for (uint32_t g = 0; g < 8; ++g) {
                    uint32_t o = 0;
#pragma unroll
                    for (uint32_t i = 0; i < 4; ++i) {
                        const uint32_t bit = 4 * g + i;
                        const uint32_t code = (((v.x >> bit) & 1) << 1) | ((v.y >> bit) & 1);
                        const uint32_t c = ((v.z >> bit) & 1) ? 0u : (acgt4 >> (8 * code)) & 0xffu;   // a break: 0
                        o |= c << (8 * i);
                    }
                    dst[g] = o;
                }
                // "other" bytes (N, IUPAC letters) from the side tables; past
                // the end of the text every position is a break (0)
                for (uint32_t ex = v.w & ~v.z; ex; ex &= ex - 1) {
                    const uint64_t p = wb + (uint32_t)__builtin_ctz(ex);
                    es_lds[r.base + ((uint32_t)p & r.mask)] = p < n ? cmap[nuc_char_at(tv.nuc, p)] : (uint8_t)0;
                }
                if (wb + 32 > n)
                    for (uint64_t p = umax64(wb, n); p < wb + 32; ++p) es_lds[r.base + ((uint32_t)p & r.mask)] = 0;
                r.hi = wb + 32;
            } else {
                const uint32_t cnt = (uint32_t)umin64(ES_CHUNK, upto - b);
                uint8_t c[ES_CHUNK];
#pragma unroll
                for (int q = 0; q < ES_CHUNK; ++q) c[q] = tv.bytes[umin64(b + q, n)];   // bytes[n..] pad with '\n'
#pragma unroll
                for (int q = 0; q < ES_CHUNK; ++q)
                    if ((uint32_t)q < cnt) es_lds[r.base + ((uint32_t)(b + q) & r.mask)] = b + q < n ? cmap[c[q]] : 0;
                r.hi = b + cnt;
            }
            if (r.hi - r.lo > r.mask + 1) r.lo = r.hi - (r.mask + 1);
        }
    }
    // a position known to be in the ring
    __device__ uint8_t ring(uint64_t p) const {
        return r.mask == ~0u ? load(p) : es_lds[r.base + ((uint32_t)p & r.mask)];   // (no ring: uniform)
    }
    // the line-bounded (folded) byte's code: 0 at every break
    __device__ uint8_t chr(uint64_t p) const {
        return p - r.lo < r.hi - r.lo ? es_lds[r.base + ((uint32_t)p & r.mask)] : load(p);
    }
    // a record break: '\n', a header-line byte, the end of the text
    __device__ bool brk(uint64_t p) const { return chr(p) == 0; }
    // the code of the file's byte at a break (a header byte or '\n'), p < n:
    // what the BNDM scanner reads there
    __device__ uint8_t raw_code(uint64_t p) const { return cmap[tv.nuc_layout ? nuc_raw_at(tv.nuc, p) : tv.raw[p]]; }
};

struct EsCtx {
    const EsSlot* S;
    const uint64_t* tab;
    EsText t;
    uint64_t R;   // the search region start
    int errs, W, anchors;   // S's fields read on every step
    int nc;                 // codes of the compact alphabet (rows per table)
    // recCheckLeftContext 0x402170 / recCheckRightContext 0x4021e0; p ==
    // recbeg <=> p == R or p starts its line (a record holds no break)
    __device__ bool at_recbeg(uint64_t p) const { return p == R || p == 0 || t.brk(p - 1); }
    __device__ bool left_ok(uint64_t p) const { return !(anchors & PM_ANCHOR_START) || at_recbeg(p); }
    __device__ bool right_ok(uint64_t q) const { return !(anchors & PM_ANCHOR_END) || t.brk(q); }
};

// one phase of checkMatch1 (left: dir < 0, bit r = position L - 1 - r read
// backward from pos; right: bit r = position L + r read forward from pos).
// Returns the boundary (start / end) and its error count.  WB: position
// words (len <= 64 WB); the rows are unrolled to PM_MAX_K so that the row
// vectors stay in registers.
template <int WB, int KR>
__device__ bool es_phase(const EsCtx& x, const uint64_t* T, uint64_t pos, bool left, int len, int kmax,
                         uint64_t& bound, int& nerr) {
    const int errs = x.errs;
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
    const int W = WB == 1 ? 1 : (len + 63) >> 6, lw = W - 1;
    const uint64_t fin = 1ull << ((len - 1) & 63), alive_mask = fin * 2 - 1;
    uint64_t Rw[KR + 1][WB];
    int maxk = kmax, best = kmax;
    bool found = false;
    uint64_t fb = 0;
#pragma unroll
    for (int j = 0; j <= KR; ++j) {   // 0x414380: deletions reach the first j positions
        if (j > maxk) break;
        uint64_t last = 0;
#pragma unroll
        for (int w = 0; w < WB; ++w) {
            uint64_t v = 0;
            if (errs & PM_ERR_DEL) {
                if (j >= 64 * (w + 1)) v = ~0ull;
                else if (j > 64 * w) v = ~(~0ull << (j & 63));
            }
            Rw[j][w] = v;
            if (w == lw) last = v;
        }
        if ((last & fin) && (left ? x.left_ok(pos) : x.right_ok(pos))) {
            best = j;
            maxk = j - 1;
            found = true;
            fb = pos;
        }
    }
    if (!(left ? x.at_recbeg(pos) : x.t.brk(pos))) {
        uint64_t inj = 1, p = pos;
        // a step's mask is loaded one step ahead (its latency overlaps the
        // step before)
        uint64_t Mn[WB];
        {
            const uint64_t* M = T + (size_t)x.t.chr(left ? p - 1 : p) * x.W;
#pragma unroll
            for (int w = 0; w < WB; ++w) Mn[w] = w < W ? M[w] : 0ull;
        }
        for (;;) {
            uint64_t b;
            if (left) {
                --p;
                b = p;
            } else {
                b = ++p;
            }
            uint64_t Mw[WB], t0[WB], t1[WB];
#pragma unroll
            for (int w = 0; w < WB; ++w) Mw[w] = Mn[w];
            {   // the next step reads p - 1 (left) or p (right)
                const uint8_t cn = left ? (p > 0 ? x.t.chr(p - 1) : (uint8_t)0) : x.t.chr(p);
                const uint64_t* M = T + (size_t)cn * x.W;
#pragma unroll
                for (int w = 0; w < WB; ++w) Mn[w] = w < W ? M[w] : 0ull;
            }
            uint64_t carry = inj, last = 0;
#pragma unroll
            for (int w = 0; w < WB; ++w) {   // row 0
                const uint64_t old = Rw[0][w];
                const uint64_t nv = ((old << 1) | carry) & Mw[w];
                t0[w] = old;
                t1[w] = nv;
                Rw[0][w] = nv;
                carry = old >> 63;
                if (w == lw) last = nv;
            }
            const bool ok = left ? x.left_ok(b) : x.right_ok(b);
            if ((last & fin) && ok) {
                bound = b;
                nerr = 0;
                return true;
            }
            uint64_t top = 0;   // 0x414de3: the highest live row
#pragma unroll
            for (int w = 0; w < WB; ++w)
                if (maxk == 0 && w < W) top |= w == lw ? t1[w] & alive_mask : t1[w];
#pragma unroll
            for (int j = 1; j <= KR; ++j) {   // 0x414640: rows 1..maxk
                if (j > maxk) break;
                uint64_t dc = 0, sc = inj, mc = inj;
                last = 0;
#pragma unroll
                for (int w = 0; w < WB; ++w) {
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
                    const uint64_t nv = (((old << 1) | mc) & Mw[w]) | r;
                    mc = old >> 63;
                    t0[w] = old;
                    t1[w] = nv;
                    Rw[j][w] = nv;
                    if (w == lw) last = nv;
                }
                if ((last & fin) && ok) {
                    // the rows below j do not reach the end here (they had
                    // returned or stopped here first): record, look for fewer
                    // errors with the rows below
                    found = true;
                    fb = b;
                    best = j;
                    maxk = j - 1;
                    top = 0;
#pragma unroll
                    for (int w = 0; w < WB; ++w)
                        if (w < W) top |= w == lw ? Rw[j - 1][w] & alive_mask : Rw[j - 1][w];
                    break;
                }
                if (j == maxk) {
#pragma unroll
                    for (int w = 0; w < WB; ++w)
                        if (w < W) top |= w == lw ? t1[w] & alive_mask : t1[w];
                }
            }
            if (!top) break;
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
template <int WB, int KR>
__device__ bool es_verify(EsCtx& x, uint64_t pos, int i, uint64_t& mb, uint64_t& me) {
    const EsSlot& S = *x.S;
    const uint64_t rp = S.type == 3 ? pos - 1 : pos;   // 0x4152dc
    const int L = S.L[i];
    // the ring covers what the phases can read: back from pos (a read
    // before the ring goes to memory) and m - L + k + 1 ahead
    x.t.fill(pos + (uint64_t)(S.m - L + S.k + 2));
    if (x.t.brk(rp)) return false;                      // the record ends at rp
    const size_t per = (size_t)x.nc * S.W;
    int kmax = S.k;
#pragma nounroll
    for (int ph = 0; ph < 2; ++ph) {   // left, then right with what the left left of k
        uint64_t bound;
        int e;
        if (!es_phase<WB, KR>(x, x.tab + (ph ? S.o_TR : S.o_TL) + per * i, pos, ph == 0, ph ? S.m - L : L, kmax, bound,
                          e))
            return false;
        kmax -= e;
        (ph ? me : mb) = bound;
    }
    return true;
}

// a record break before p (p > 0): '\n', a header byte
__device__ inline bool es_brk_before(const TextView& tv, uint64_t p) {
    if (tv.nuc_layout) {
        const uint4 v = tv.nuc.lin[(p - 1) >> 5];
        return (v.z >> ((uint32_t)(p - 1) & 31)) & 1;
    }
    return tv.bytes[p - 1] == (uint8_t)'\n';
}

// Cluster heads: a new pattern (high key bits) or a gap wider than any phase
// reads; with `lines` also every start of a line (records never interact).
// The search restarts at every region start (recSearchFile), so a cluster
// never spans one.
__device__ inline bool es_head(const uint64_t* keys, uint64_t i, int32_t gap, int lines, const TextView& tv) {
    if (i == 0 || keys[i] - keys[i - 1] > (uint64_t)gap) return true;
    const uint64_t p = keys[i] & ES_POS_MASK;
    if (region_near(tv.reg, p) && region_of(tv.reg, p) != region_of(tv.reg, keys[i - 1] & ES_POS_MASK)) return true;
    if (!lines) return false;
    return p > 0 && es_brk_before(tv, p);
}

// One thread per list entry: acc = 2 at a cluster head, else 0.  A lone
// start of a slot whose lone starts need no walk (EsSlot::lone) is settled
// here (acc = 3, its length m); every other head goes to the walk list
// (one atomic per block and pass: the list length is one counter, and
// thousands of waves' atomics on it serialize -- ~0.1 ms with one per wave).
constexpr uint32_t ES_HEADS_T = 1024;
__global__ __launch_bounds__(ES_HEADS_T) void k_es_heads(EsPrep P, const uint64_t* __restrict__ keys,
                                                         uint32_t* __restrict__ lens, const uint64_t* total_d,
                                                         uint64_t total_h, uint8_t* __restrict__ acc,
                                                         uint32_t* __restrict__ wlist, uint32_t* __restrict__ wcount,
                                                         TextView tv) {
    __shared__ uint32_t s_wc[ES_HEADS_T / 64];
    __shared__ uint32_t s_base;
    const uint64_t total = total_d ? *total_d : total_h;
    const uint64_t stride = (uint64_t)gridDim.x * ES_HEADS_T;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint64_t b0 = (uint64_t)blockIdx.x * ES_HEADS_T; b0 < total; b0 += stride) {   // block-uniform
        const uint64_t i = b0 + threadIdx.x;
        bool walk = false;
        if (i < total) {
            uint8_t a = 0;
            if (es_head(keys, i, P.gap_max, P.lines, tv)) {
                a = 2;
                walk = true;
                const int64_t slot = (int64_t)(keys[i] >> 48) - P.pid_base;
                if (!P.lines && slot >= 0 && slot < P.nslots && (i + 1 == total || es_head(keys, i + 1, P.gap_max, 0, tv))) {
                    const EsSlot& S = P.slots[slot];
                    if (S.lone && (!region_near(tv.reg, keys[i] & ES_POS_MASK) ||
                                   (keys[i] & ES_POS_MASK) + (uint64_t)S.m <= tv.reg.e[region_of(tv.reg, keys[i] & ES_POS_MASK)])) {
                        // A lone start with substitutions only is what nrgrep
                        // prints: a verification from any candidate returns
                        // the window [pos - L, pos - L + m) (no indels: both
                        // phases have fixed lengths), i.e. one of the
                        // cluster's starts, so only this one; and some
                        // candidate leads to it (k + 1 pieces, at most k
                        // errors: one piece of the window is exact and its
                        // test bit is right (es_add_slot); the window and
                        // prefix scanners stop at every start of a match).
                        // No text is read.
                        lens[i] = (uint32_t)S.m;
                        a = 3;
                        walk = false;
                    }
                }
            }
            acc[i] = a;
        }
        const uint64_t m = __builtin_amdgcn_ballot_w64(walk);
        if (lane == 0) s_wc[wv] = (uint32_t)__builtin_popcountll(m);
        __syncthreads();
        if (threadIdx.x == 0) {   // the waves' offsets, then one reservation for the block
            uint32_t run = 0;
            for (uint32_t w = 0; w < ES_HEADS_T / 64; ++w) {
                const uint32_t c = s_wc[w];
                s_wc[w] = run;
                run += c;
            }
            s_base = run ? atomicAdd(wcount, run) : 0u;
        }
        __syncthreads();
        if (walk)
            wlist[s_base + s_wc[wv] + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
                (uint32_t)i;
        __syncthreads();   // s_wc / s_base are rewritten by the next pass
    }
}

__global__ void k_es_iota(uint64_t* __restrict__ keys, uint64_t n, uint64_t pid) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i < n) keys[i] = (pid << 48) | i;
}

// One thread per cluster of the walk list (grid-stride): nrgrep's candidate
// order over the cluster's text; the printed matches are written in place
// from the head on (acc bit 0), every other entry of the cluster is cleared.
// (capping the registers for 3 blocks per CU -- 168 VGPRs, 68-190 B of
// spills -- measured slower: -k 2ids 5.02 vs 4.86 ms per step, r05k)
template <int WB, int KR>
__global__ __launch_bounds__(ES_THREADS) void k_es_walk(EsPrep P, uint64_t* __restrict__ keys, uint32_t* __restrict__ lens,
                                                        const uint64_t* total_d, uint64_t total_h,
                                                        uint8_t* __restrict__ acc, const uint32_t* __restrict__ wlist,
                                                        const uint32_t* __restrict__ wcount, TextView tv) {
    const uint64_t total = total_d ? *total_d : total_h;
    const uint32_t nw = *wcount;
    const uint32_t stride = gridDim.x * blockDim.x;
    // list entry t goes to block t % gridDim.x, thread rank t / gridDim.x
    // (below): a short list is spread one cluster per wave (a wave runs its
    // lanes' divergent walks one after the other)
    if (blockIdx.x >= nw) return;   // (block-uniform) nothing to walk
    // the compact tables (when they fit) and the byte -> code map in LDS
    uint8_t* cmap = es_lds + P.map_off;
    for (uint32_t c = threadIdx.x; c < 256; c += blockDim.x) cmap[c] = P.cmap[c];
    const uint64_t* tab = P.tab;
    if (P.tab_lds) {
        uint64_t* lt = reinterpret_cast<uint64_t*>(es_lds + P.tab_off);
        for (uint32_t q = threadIdx.x; q < P.tab_words; q += blockDim.x) lt[q] = P.tab[q];
        tab = lt;
    }
    // the slots too (a few hundred bytes each): every cluster's walk reads
    // its slot's fields, a chain of global loads otherwise
    const EsSlot* slots = P.slots;
    if (P.slots_lds) {
        uint64_t* ls = reinterpret_cast<uint64_t*>(es_lds + P.slots_off);
        const uint64_t* gs = reinterpret_cast<const uint64_t*>(P.slots);
        for (uint32_t q = threadIdx.x; q < (uint32_t)P.nslots * (uint32_t)(sizeof(EsSlot) / 8); q += blockDim.x) ls[q] = gs[q];
        slots = reinterpret_cast<const EsSlot*>(ls);
    }
    __syncthreads();
    // the thread's rank lane * waves + wave: consecutive entries of a block
    // go to different waves
    const uint32_t rank = (threadIdx.x & 63u) * (ES_THREADS / 64) + (threadIdx.x >> 6);
    for (uint32_t t = rank * gridDim.x + blockIdx.x; t < nw; t += stride) {
        const uint64_t i = wlist[t];
        uint64_t j = i + 1;   // the next cluster's head keeps bit 1 set whatever its owner writes
        while (j < total && !(acc[j] & 2)) ++j;
        const uint64_t lo = keys[i] & ES_POS_MASK, hi = keys[j - 1] & ES_POS_MASK;
        const uint64_t pid = keys[i] >> 48;
        const uint64_t nmax = j - i;
        uint64_t nout = 0;
        const int64_t slot = (int64_t)pid - P.pid_base;
        if (slot >= 0 && slot < P.nslots) {
            const EsSlot& S = slots[slot];
            // the cluster's region [R0, n): its search starts at R0 and the
            // text ends at n for it (reads past it see a break)
            uint64_t R0 = 0, n = tv.n;
            if (tv.reg.n > 1) {
                const uint32_t r = region_of(tv.reg, lo);
                R0 = tv.reg.t[r];
                n = tv.reg.e[r];
            }
            EsCtx x{&S, tab, EsText{tv, n, EsRing{threadIdx.x * P.win, P.win - 1u, 0, 0}, cmap}, R0, S.errs, S.W,
                    S.anchors, P.ncodes};
            const int type = S.type, m = S.m, k = S.k, mpc = S.mpc, np = S.np;
            if (S.lone) {
                // Substitutions only, no anchors: a verification from (pos,
                // piece q) succeeds exactly when the window pos - L_q is one
                // of the cluster's starts (both phases have fixed lengths)
                // and it returns that window.  So nrgrep prints, from R on,
                // the start s >= R discovered first: type 1 at its smallest
                // (s + L_q, q) with piece q exact there (every test bit is
                // right, es_add_slot), types 2 and 3 at s itself; R = s + m.
                // The walk needs only the cluster's starts and their pieces:
                // a start s is discovered at or before s + L_max (one of its
                // k + 1 pieces is exact), so none after the first start
                // s_f >= R plus L_max can come first -- each round looks at
                // the starts in [s_f, s_f + L_max] only.
                x.t.restart(lo);
                const uint64_t lim = type == 2 ? (n > (uint64_t)(S.wend - S.wbeg - k - 1) ? n - (uint64_t)(S.wend - S.wbeg - k - 1) : 0) : n + 1;
                const uint64_t last = n >= (uint64_t)mpc ? n - (uint64_t)mpc : 0;
                const uint64_t lmax = (uint64_t)S.L[np - 1];
                const size_t W = (size_t)S.W;
                uint64_t R = 0, f = i;
                for (;;) {
                    while (f < j && (keys[f] & ES_POS_MASK) < R) ++f;
                    if (f == j) break;
                    const uint64_t sf = keys[f] & ES_POS_MASK;
                    if (sf + (uint64_t)m > n) break;   // (and every later start): past the region end
                    uint64_t best = ~0ull, bs = 0;
                    if (type != 1) {
                        if (sf + (uint64_t)S.L[0] >= lim) break;   // (and every later start)
                        best = bs = sf;
                    }
                    for (uint64_t q2 = f; type == 1 && q2 < j; ++q2) {
                        const uint64_t sj = keys[q2] & ES_POS_MASK;
                        if (sj > sf + lmax || sj + (uint64_t)m > n) break;
                        x.t.fill(umin64(sj + (uint64_t)m, n) + 1);
                        for (int q = 0; q < np; ++q) {   // L_q increases with q: the first exact piece
                            const uint64_t pp = sj + (uint64_t)S.L[q];
                            bool exact = pp <= last;
                            for (int t = 0; t < mpc && exact; ++t) {
                                const int bpos = S.L[q] + t;
                                exact = (tab[S.o_B + (size_t)x.t.chr(pp + t) * W + (bpos >> 6)] >> (bpos & 63)) & 1;
                            }
                            if (exact) {
                                if (pp * 64 + (uint64_t)q < best) {
                                    best = pp * 64 + (uint64_t)q;
                                    bs = sj;
                                }
                                break;
                            }
                        }
                    }
                    if (best == ~0ull) break;
                    // the entries below f are < R: overwriting them is safe
                    keys[i + nout] = (pid << 48) | bs;
                    lens[i + nout] = (uint32_t)m;
                    acc[i + nout] = (nout == 0 ? 2 : 0) | 1;
                    ++nout;
                    R = bs + (uint64_t)m;
                }
                for (uint64_t q = i + nout; q < j; ++q) acc[q] = q == i ? 2 : 0;
                continue;
            }
            // A verification from (pos, piece q) returns a start within k of
            // pos - L_q, and every start nrgrep can print is one of the
            // cluster's, so candidates with pos + k < lo + L_q cannot print
            // (skipped: a failed verification changes nothing).  The left
            // phase of the others reads back to lo - 2k - 2: the ring starts
            // there (an earlier read goes to memory) and is filled only as
            // far as the piece pass and each verification need.
            x.t.restart(lo > (uint64_t)(2 * k + 3) ? lo - (uint64_t)(2 * k + 3) : 0);
            // lines (every position is a key): the cluster is one line and
            // its break, the next line is another cluster's
            const uint64_t pmax = P.lines ? hi : umin64(n, hi + (uint64_t)(m + k));
            // type 2: ABNDM windows of wend - wbeg - k characters must fit (0x413a5b)
            const uint64_t wtail = (uint64_t)(S.wend - S.wbeg - k - 1);
            const uint64_t lim2 = type == 2 ? (n > wtail ? n - wtail : 0) : n + 1;
            // type 1: the packed shift-and over the window starts (see
            // es_add_slot); flags bit d = the pieces' last bits survive at
            // start fb + d.  Every start < n - mpc + 1 is tested (0x4137f2).
            const uint64_t* Pt = tab + S.o_P;
            const uint64_t pstart = S.pstart, pend = S.pend;
            const uint64_t last_start = n >= (uint64_t)mpc ? n - (uint64_t)mpc : 0;   // starts <= this fit
            uint64_t* dl = reinterpret_cast<uint64_t*>(es_lds + P.dl_off) + threadIdx.x * ES_SPAN;   // D per span start
            uint64_t fb = 0;
            uint32_t flags = 0;
            bool fvalid = false;
            uint64_t pos = type == 3 ? lo + 1 : lo;
            uint64_t guard = (pmax - lo + 2) * (uint64_t)(np + 2) * 4;
            uint32_t cand = 0;   // the pieces still to try at pos, in order
            // Each round first moves every lane to its next (position, piece)
            // candidate (the inner loop: cheap, divergent), then verifies them
            // together, so a wave runs one verification chain per round, not
            // one per lane or per piece.
            for (;;) {
                while (!cand && pos <= pmax && guard) {   // the next candidate position at or after pos
                    --guard;
                    if (type != 1) {
                        // every start is the window / prefix candidate
                        if (pos < lim2 && pos + (uint64_t)k >= lo + (uint64_t)S.L[0]) cand = 1u;
                        else ++pos;
                        continue;
                    }
                    if (!fvalid || pos < fb || pos >= fb + ES_SPAN) {
                        // the next ES_SPAN starts: feed characters pos ..
                        // pos + ES_SPAN + mpc - 2 from a fresh state
                        uint64_t st = 0, tfeed = pos;
                        fb = pos;
                        flags = 0;
                        fvalid = true;
                        const uint64_t tend = umin64(pos + ES_SPAN, pmax + 1) + (uint64_t)mpc - 1;
                        x.t.fill(tend);
                        while (tfeed < tend) {
                            // 8 characters from the ring, their 8 masks in one
                            // round trip; a break's mask comes from the file's
                            // own byte (a header line: rare)
                            uint8_t cc[8];
                            uint64_t mk[8];
#pragma unroll
                            for (int q = 0; q < 8; ++q) cc[q] = tfeed + q < tend ? x.t.ring(tfeed + q) : (uint8_t)0;
#pragma unroll
                            for (int q = 0; q < 8; ++q) mk[q] = Pt[cc[q]];
#pragma unroll
                            for (int q = 0; q < 8; ++q) {
                                const uint64_t t = tfeed + q;
                                if (cc[q] == 0 && t < n) mk[q] = Pt[x.t.raw_code(t)];
                                if (t >= tend) mk[q] = 0ull;
                            }
#pragma unroll
                            for (int q = 0; q < 8; ++q) {
                                st = ((st << 1) | pstart) & mk[q];
                                const uint64_t t = tfeed + q + 1 - (uint64_t)mpc;   // the start whose window ends here
                                if ((st & pend) && tfeed + q + 1 >= fb + (uint64_t)mpc && t < fb + ES_SPAN) {
                                    flags |= 1u << (uint32_t)(t - fb);
                                    dl[t - fb] = st & pend;
                                }
                            }
                            tfeed += 8;
                        }
                    }
                    const uint32_t f = flags >> (uint32_t)(pos - fb);
                    if (!f) {   // no piece before the span's end
                        pos = fb + ES_SPAN;
                        continue;
                    }
                    pos += (uint64_t)__builtin_ctz(f);
                    if (pos > pmax) break;
                    if (pos <= last_start) {
                        // BNDM's surviving bits at pos, then the pieces
                        // checkMatch is called for, in order (0x41384b)
                        const uint64_t D = dl[pos - fb];
                        for (int q = 0; q < np; ++q)
                            if ((D & S.test[q]) && pos + (uint64_t)k >= lo + (uint64_t)S.L[q]) cand |= 1u << q;
                    }
                    if (!cand) ++pos;
                }
                if (!cand) break;
                const int q = __builtin_ctz(cand);
                cand &= cand - 1;
                uint64_t mb = 0, me = 0;
                if (!es_verify<WB, KR>(x, pos, q, mb, me)) {
                    if (!cand) ++pos;
                    continue;
                }
                cand = 0;
                if (nout < nmax) {   // matches start at distinct candidates: never more than the cluster holds
                    keys[i + nout] = (pid << 48) | mb;
                    lens[i + nout] = (uint32_t)(me - mb);
                    acc[i + nout] = (nout == 0 ? 2 : 0) | 1;
                    ++nout;
                }
                if (me >= n) break;   // 0x4022eb: a match that ends the region ends the search
                x.R = me;
                pos = type == 3 ? me + 1 : me;
            }
        }
        for (uint64_t q = i + nout; q < j; ++q) acc[q] = q == i ? 2 : 0;
    }
}

// kept entries (acc bit 0) per chunk of C = ceil(total / G) entries, for
// k_rep_scatter
__global__ __launch_bounds__(256) void k_es_count(const uint64_t* total_d, uint64_t total_h,
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

void es_launch(const EsPrep& P0, uint64_t* keys, uint32_t* lens, const uint64_t* total_d, uint64_t total_h,
               uint8_t* acc, uint32_t* wlist, uint32_t* wcount, uint32_t* bcnt, uint32_t G, const TextView& tv,
               hipStream_t s) {
    // a device-side total comes from the speculative sort, which zeroed
    // wcount too (report_ws puts it right after the total)
    if (!total_d) HIPCHK(hipMemsetAsync(wcount, 0, sizeof(uint32_t), s));
    hipLaunchKernelGGL(k_es_heads, dim3(256), dim3(ES_HEADS_T), 0, s, P0, keys, lens, total_d, total_h, acc, wlist, wcount,
                       tv);
    EsPrep P = P0;
    // a candidate's phases reach m + k + 1 back and forth, the piece pass
    // ES_SPAN + mpc ahead, a refill to the end of a 32-position word; the
    // ring keeps the last win positions (a read before them goes to memory)
    uint32_t win = 64;
    while (win < (uint32_t)P.gap_max + ES_SPAN + 32) win <<= 1;
    // wider patterns read memory directly (a block's rings, piece words and
    // tables stay within the CU's LDS)
    P.win = (size_t)ES_THREADS * win + (size_t)ES_THREADS * ES_SPAN * 8 + ES_TAB_LDS + 256 + ES_SLOTS_LDS <= (160u << 10) ? win : 0;
    P.dl_off = ES_THREADS * P.win;  // then ES_SPAN piece words per thread
    // then the compact tables (up to ES_TAB_LDS bytes) and the code map
    P.tab_off = P.dl_off + ES_THREADS * ES_SPAN * 8;
    P.tab_lds = (size_t)P.tab_words * 8 <= ES_TAB_LDS ? 1 : 0;
    P.map_off = P.tab_off + (P.tab_lds ? P.tab_words * 8 : 0);
    // then the slots, when they are few (PM_ES_SLOTS_LDS=0: global, A/B)
    static const bool slots_env = !(getenv("PM_ES_SLOTS_LDS") && getenv("PM_ES_SLOTS_LDS")[0] == '0');
    P.slots_off = P.map_off + 256;
    P.slots_lds = slots_env && (size_t)P.nslots * sizeof(EsSlot) <= ES_SLOTS_LDS ? 1 : 0;
    const size_t lds = P.slots_off + (P.slots_lds ? (size_t)P.nslots * sizeof(EsSlot) : 0);
    // a cluster's walk is a chain of dependent steps, so as many waves as
    // the registers allow: blocks of ES_THREADS share the tables in LDS, all
    // resident, striding over the walk list (its length is on the device)
    int dev = 0, ncu = 0;
    HIPCHK(hipGetDevice(&dev));
    HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const uint32_t per_cu = (uint32_t)std::max<size_t>(1, std::min<size_t>(8, (160u << 10) / lds));
    const uint32_t blocks = (uint32_t)std::max(1, ncu) * per_cu;
    // WB: position words; KR: the rows unrolled (k <= 3, the common case,
    // keeps the row vectors in few registers: k itself)
    auto by_w = [&](auto kr) {
        constexpr int KR = decltype(kr)::value;
        return P.wmax <= 1 ? k_es_walk<1, KR> : P.wmax == 2 ? k_es_walk<2, KR> : k_es_walk<4, KR>;
    };
    auto kern = P.kmax <= 1   ? by_w(std::integral_constant<int, 1>{})
                : P.kmax == 2 ? by_w(std::integral_constant<int, 2>{})
                : P.kmax == 3 ? by_w(std::integral_constant<int, 3>{})
                              : by_w(std::integral_constant<int, PM_MAX_K>{});
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(ES_THREADS), lds, s, P, keys,
                       lens, total_d, total_h, acc, wlist, wcount, tv);
    hipLaunchKernelGGL(k_es_count, dim3(G), dim3(256), 0, s, total_d, total_h, acc, bcnt);
    HIPCHK(hipGetLastError());
}

}  // namespace pm

using namespace pm;

namespace pm {

pm_hits* es_all_positions(pm_db* db, int32_t pattern_id) {
    require(db->n <= ES_ALL_MAX, "deletions with k >= the pattern length: the file is too large for the GPU walk",
            PM_E_UNSUPPORTED);
    pm_hits* h = new pm_hits();
    h->device = db->device;
    h->count = db->n;
    try {
        h->keys = static_cast<uint64_t*>(pool_get(db->device, std::max<uint64_t>(db->n, 1) * 8, &h->keys_cap));
        h->lens = static_cast<uint32_t*>(pool_get(db->device, std::max<uint64_t>(db->n, 1) * 4, &h->lens_cap));
        if (db->n) {
            hipLaunchKernelGGL(k_es_iota, dim3(blocks_for(db->n, 256)), dim3(256), 0, db->stream, h->keys, db->n,
                               (uint64_t)pattern_id);
            HIPCHK(hipGetLastError());
        }
    } catch (...) {
        pool_put(h->device, h->keys, h->keys_cap);
        pool_put(h->device, h->lens, h->lens_cap);
        delete h;
        throw;
    }
    return h;
}

}  // namespace pm

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
