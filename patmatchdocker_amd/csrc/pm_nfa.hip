// pm_nfa.hip -- general patterns: bit-parallel Glushkov automaton scan.
//
// Everything that is not a fixed-length class sequence on a nucleotide file
// (PROSITE-style peptide patterns such as C-x(2,4)-C-x(3)-[LIVMFYWC],
// {m,n} ranges, groups, alternation; www/bin/patmatch_to_nrgrep.pl output)
// runs here.  k_nfa_rev scans each lane's chunk right to left with the
// reversed automaton (one 64-bit state word per error row, transitions by
// 8-position table lookups in LDS) and emits every start that has a match;
// k_nfa_verify runs the forward automaton from each start and records the
// shortest end -- the hit nrgrep_coords prints for that start (oracle/
// pm_oracle.c).
//
// Error model: `-k <k><ids>` (patmatch.py:299-314; the web form's default
// when mismatches > 0 is all three).  Row j holds the positions reached with
// j errors; substitution (any non-break char consumes a position), insertion
// (a text char consumed, the state kept) and deletion (a position skipped
// without text: a closure over the rows after every step) are each enabled by
// a bit of `errs`.  The reverse scan is the forward recurrence of
// pm_oracle.c:55-94 mirrored (prec for follow, last for first) in search
// mode: a fresh start config -- init row 0, insertion rows when INS, and its
// deletion closure, precomputed on the host as rev_pre[j] / rev_ins[j] -- is
// injected before every character.
#include "pm_internal.h"

namespace pm {
namespace {

constexpr int NFA_MAXW = PM_MAX_POSITIONS / 64;   // state words
constexpr int NFA_MAXR = PM_MAX_K + 1;             // error rows

struct NfaArgs {
    NucView nuc;
    const uint8_t* bytes;       // BYTE alphabet (headers stored as '\n')
    const uint8_t* bytes_raw;   // BYTE alphabet, the file's own bytes (cross mode)
    const uint32_t* p5;         // BYTE alphabet: the 5-bit residue planes (p5[q * nw5 + w], pm_db.hip)
    uint64_t nw5;
    const uint64_t* bmask5;     // [32][W]: positions accepting each residue code (0 header, 1 '\n': none)
    const uint64_t* prec;       // [nt][2^S][W] positions preceding a slice value
    const uint64_t* follow;     // [nt][2^S][W] positions following it
    const uint64_t* bmask;      // [256][W]
    uint64_t first[NFA_MAXW], last[NFA_MAXW], mmask[NFA_MAXW];
    int nt;                     // slices of S = 8 (W = 1) or 4 (W > 1) positions
    int halo;
    int chunk;                  // positions per lane
    uint64_t n;
    uint64_t nchunks;
    int pattern_id;
    int end_anchor;             // '$': the verify's end must be a line end
    int cross;                  // nrgrep's simple engine (k = 0 class sequence): windows span lines
    int k;                      // errors (<= the kernel's row count - 1)
    Sink sink;
    int errs;                   // PM_ERR_INS | PM_ERR_DEL | PM_ERR_SUB
    uint64_t rev_pre[NFA_MAXR][NFA_MAXW];   // reverse: prec(S[j]) | (I[j] ? last : 0) for the injected start config
    uint64_t rev_ins[NFA_MAXR][NFA_MAXW];   // reverse: S[j] (insertion source rows of the injected config)
    uint64_t fwd_del[NFA_MAXR][NFA_MAXW];   // forward: deletion closure of the start config (rows of R)
    // unbounded patterns: reverse state entering each chunk from the right
    // ((k+1) * W words per chunk), found by k_nfa_carry; null = start from the halo
    const uint64_t* in_state;
    int st_stride;
    // a plain class sequence (follow(i) = {i+1}): transitions are shifts
    // instead of table lookups
    int shift_only;
    // verify
    const uint64_t* starts;
    uint64_t nstarts;
    uint32_t* lens;
    int max_len;
};

// A set of automaton positions: W 64-bit words (position i = bit i % 64 of
// word i / 64).
template <int W>
struct Bits {
    uint64_t w[W];
};
template <int W>
__device__ inline Bits<W> bits_zero() {
    Bits<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = 0;
    return r;
}
template <int W>
__device__ inline Bits<W> bits_of(const uint64_t* p) {
    Bits<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = p[i];
    return r;
}
template <int W>
__device__ inline Bits<W> operator|(const Bits<W>& a, const Bits<W>& b) {
    Bits<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = a.w[i] | b.w[i];
    return r;
}
template <int W>
__device__ inline Bits<W> operator&(const Bits<W>& a, const Bits<W>& b) {
    Bits<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = a.w[i] & b.w[i];
    return r;
}
template <int W>
__device__ inline Bits<W> mask_if(const Bits<W>& a, bool keep) {
    Bits<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = keep ? a.w[i] : 0ull;
    return r;
}
template <int W>
__device__ inline bool any_of(const Bits<W>& a) {
    uint64_t x = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) x |= a.w[i];
    return x != 0;
}
template <int W>
__device__ inline bool meets(const Bits<W>& a, const uint64_t* m) {
    uint64_t x = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) x |= a.w[i] & m[i];
    return x != 0;
}

// transitions of a set: OR of per-slice table rows
template <int W>
__device__ inline Bits<W> table_or(const uint64_t* __restrict__ tab, const Bits<W>& set, int nt) {
    Bits<W> acc = bits_zero<W>();
    if constexpr (W == 1) {
        for (int t = 0; t < nt; ++t) acc.w[0] |= tab[t * 256 + ((set.w[0] >> (8 * t)) & 255)];
    } else {
        // 4-position slices, only the non-empty ones (states are sparse)
#pragma unroll
        for (int i = 0; i < W; ++i) {
            uint64_t x = set.w[i];
            while (x) {
                const int t = i * 16 + (__builtin_ctzll(x) >> 2);
                const uint64_t* row = tab + ((uint64_t)t * 16 + ((set.w[i] >> ((t & 15) * 4)) & 15)) * W;
#pragma unroll
                for (int q = 0; q < W; ++q) acc.w[q] |= row[q];
                x &= ~(15ull << ((t & 15) * 4));
            }
        }
    }
    return acc;
}
// positions preceding / following a set (reverse / forward transitions)
template <int W>
__device__ inline Bits<W> prec_of(const NfaArgs& a, const uint64_t* __restrict__ s_prec, const Bits<W>& set) {
    if (!a.shift_only) return table_or<W>(s_prec, set, a.nt);
    Bits<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = (set.w[i] >> 1) | (i + 1 < W ? set.w[i + 1] << 63 : 0ull);
    return r;
}
template <int W>
__device__ inline Bits<W> fol_of(const NfaArgs& a, const uint64_t* __restrict__ s_fol, const Bits<W>& set) {
    if (!a.shift_only) return table_or<W>(s_fol, set, a.nt);
    Bits<W> r;
#pragma unroll
    for (int i = 0; i < W; ++i) r.w[i] = ((set.w[i] << 1) | (i > 0 ? set.w[i - 1] >> 63 : 0ull)) & a.mmask[i];
    return r;
}

// One character of the reverse search (right to left).  Substitution-only
// patterns (the common case) take the short form.  Rows above a.k stay empty.
template <int K, int W>
__device__ inline void nfa_rev_step(Bits<W> (&R)[K + 1], const Bits<W>& bc, bool nb,
                                    const uint64_t* __restrict__ s_prec, const NfaArgs& a) {
    Bits<W> A[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j) A[j] = prec_of<W>(a, s_prec, R[j]) | bits_of<W>(a.rev_pre[j]);
    if (a.errs == PM_ERR_SUB) {
#pragma unroll
        for (int j = K; j >= 0; --j)
            R[j] = mask_if<W>((A[j] & bc) | (j > 0 ? mask_if<W>(A[j - 1], nb) : bits_zero<W>()), j <= a.k);
        return;
    }
    Bits<W> N[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j) {
        N[j] = A[j] & bc;
        if (j > 0) {
            if (a.errs & PM_ERR_SUB) N[j] = N[j] | mask_if<W>(A[j - 1], nb);
            if (a.errs & PM_ERR_INS) N[j] = N[j] | mask_if<W>(R[j - 1] | bits_of<W>(a.rev_ins[j - 1]), nb);
        }
    }
    if (a.errs & PM_ERR_DEL) {
        // ninit[j] (j >= 1) = an insertion-kept start; row 0's init is consumed
#pragma unroll
        for (int j = 0; j < K; ++j)
            N[j + 1] = N[j + 1] | prec_of<W>(a, s_prec, N[j]) |
                       mask_if<W>(bits_of<W>(a.last), j >= 1 && (a.errs & PM_ERR_INS) && nb);
    }
#pragma unroll
    for (int j = 0; j <= K; ++j) R[j] = mask_if<W>(N[j], j <= a.k);
}

// Text byte at p and whether it ends every partial match: past the end of
// the file always; a line break unless nrgrep's simple engine runs (cross:
// the file's own bytes, header lines included).
template <bool NUC>
__device__ inline uint8_t char_at(const NfaArgs& a, uint64_t p, bool& kill) {
    if (p >= a.n) {
        kill = true;
        return (uint8_t)'\n';
    }
    uint8_t ch;
    if constexpr (NUC) ch = a.cross ? nuc_raw_at(a.nuc, p) : nuc_char_at(a.nuc, p);
    else ch = a.cross ? a.bytes_raw[p] : a.bytes[p];
    kill = !a.cross && ch == (uint8_t)'\n';
    return ch;
}

template <int W>
__device__ inline void load_tables(uint64_t* s_tab, uint64_t* s_b, const uint64_t* tab, const uint64_t* bmask, int nt) {
    const int rows = W == 1 ? 256 : 16;
    for (int i = threadIdx.x; i < nt * rows * W; i += blockDim.x) s_tab[i] = tab[i];
    for (int i = threadIdx.x; i < 256 * W; i += blockDim.x) s_b[i] = bmask[i];
    __syncthreads();
}
// LDS words of the transition tables: 8 slices x 256 (W = 1), 16 * W
// slices x 16 x W words otherwise
template <int W>
constexpr int tab_words() { return W == 1 ? 8 * 256 : 16 * W * 16 * W; }

// The text a start pass reads: the nucleotide planes, the byte copy, or
// (a BYTE database with residue planes, line-bounded scans) the 5-bit
// residue codes -- north_star's 5-bit-packed database: 0.625 B per residue
// instead of 1 (round 6; PM_SCAN_BYTES keeps the byte copy, A/B)
constexpr int SRC_NUC = 0, SRC_BYTE = 1, SRC_P5 = 2;

// the residue code of position p (< n): bit q from plane q
__device__ inline uint32_t p5_code(const NfaArgs& a, uint64_t p) {
    const uint64_t w = p >> 5;
    const uint32_t i = (uint32_t)p & 31u;
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < 5; ++q) c |= ((a.p5[(uint64_t)q * a.nw5 + w] >> i) & 1u) << q;
    return c;
}

template <int K, int W, int SRC>
__global__ __launch_bounds__(256) void k_nfa_rev(NfaArgs a) {
    constexpr bool NUC = SRC == SRC_NUC;
    __shared__ uint64_t s_prec[tab_words<W>()];
    __shared__ uint64_t s_b[256 * W];
    load_tables<W>(s_prec, s_b, a.prec, SRC == SRC_P5 ? a.bmask5 : a.bmask, a.nt);
    const uint64_t gid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const bool live = gid < a.nchunks;
    const uint64_t chunk_id = live ? gid : a.nchunks - 1;
    const uint64_t c0 = chunk_id * a.chunk;
    const uint64_t c1 = c0 + a.chunk;           // emit for [c0, c1) ∩ [0, n)
    const uint64_t top = c1 + a.halo;           // process (top .. c0]
    Bits<W> R[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j) {
        R[j] = bits_zero<W>();
        if (a.in_state && chunk_id + 1 < a.nchunks && j <= a.k)
            R[j] = bits_of<W>(a.in_state + (chunk_id + 1) * a.st_stride + j * W);
    }
    auto step = [&](uint64_t p, uint8_t ch, bool kill) {
        nfa_rev_step<K, W>(R, bits_of<W>(s_b + ch * W), !kill, s_prec, a);
        Bits<W> any = bits_zero<W>();
#pragma unroll
        for (int j = 0; j <= K; ++j) any = any | R[j];
        if (live && p < c1 && p < a.n && meets<W>(any, a.first))
            a.sink.push(a.sink.bin_of(0, p), ((uint64_t)a.pattern_id << 48) | p);
    };
    if constexpr (NUC) {
        for (uint64_t p = top; p-- > c0;) {
            bool kill;
            const uint8_t ch = char_at<NUC>(a, p, kill);
            step(p, ch, kill);
        }
    } else if constexpr (SRC == SRC_P5) {
        // 32 positions per word of each plane: the word's five plane words
        // are loaded when p enters it, the word below's are in flight; a
        // code <= 1 (a header byte, '\n') or a position past the file kills
        auto load = [&](uint64_t w, uint32_t (&v)[5]) {
#pragma unroll
            for (int q = 0; q < 5; ++q) v[q] = w < a.nw5 ? a.p5[(uint64_t)q * a.nw5 + w] : 0u;
        };
        uint64_t w = (top - 1) >> 5;
        uint32_t cur[5], nxt[5];
        load(w, cur);
        load(w - 1, nxt);   // (w = 0: wraps past nw5, reads nothing)
        for (uint64_t p = top; p-- > c0;) {
            if ((p >> 5) != w) {
                --w;
#pragma unroll
                for (int q = 0; q < 5; ++q) cur[q] = nxt[q];
                load(w - 1, nxt);
            }
            const uint32_t i = (uint32_t)p & 31u;
            uint32_t c = 0;
#pragma unroll
            for (int q = 0; q < 5; ++q) c |= ((cur[q] >> i) & 1u) << q;
            const bool kill = p >= a.n || c <= P5_NL;
            step(p, (uint8_t)c, kill);
        }
    } else {
        // the lane's bytes arrive 16 at a time (aligned uint4 loads), the
        // next group in flight while this one is stepped: the text reads no
        // longer sit on the state chain
        const uint8_t* src = a.cross ? a.bytes_raw : a.bytes;
        auto group = [&](uint64_t g) {
            return g + 16 <= a.n ? *reinterpret_cast<const uint4*>(src + g) : make_uint4(0, 0, 0, 0);
        };
        uint64_t g = (top - 1) & ~15ull;
        uint4 cur = group(g), nxt = g >= 16 ? group(g - 16) : make_uint4(0, 0, 0, 0);
        for (uint64_t p = top; p-- > c0;) {
            if ((p & ~15ull) != g) {   // p moved into the group below
                g -= 16;
                cur = nxt;
                nxt = g >= 16 ? group(g - 16) : make_uint4(0, 0, 0, 0);
            }
            bool kill;
            uint8_t ch;
            if (g + 16 <= a.n) {
                const uint32_t i = (uint32_t)(p & 15);
                const uint32_t wv = i < 8 ? (i < 4 ? cur.x : cur.y) : (i < 12 ? cur.z : cur.w);
                ch = (uint8_t)(wv >> (8 * (i & 3)));
                kill = !a.cross && ch == (uint8_t)'\n';
            } else {
                ch = char_at<NUC>(a, p, kill);   // the file's last partial group and past it
            }
            step(p, ch, kill);
        }
    }
}

// Unbounded patterns (`*`, `+`: a match may run to the end of its record):
// chunk i's reverse scan must start from the true state entering it from the
// right, which is chunk i+1's state after its leftmost position.  One
// relaxation round: every chunk rescans itself from its right neighbour's
// state of the previous round (from zero initially); the transfer is
// monotone, so the states only grow and the rounds stop when none changed
// (at most the chunks per record; a record break kills every state, so
// patterns that die quickly converge in 1-2 rounds).  Chunks whose input did
// not change since the previous round copy their old output.
template <int K, int W, int SRC>
__global__ __launch_bounds__(256) void k_nfa_carry(NfaArgs a, const uint64_t* __restrict__ st_old,
                                                   uint64_t* __restrict__ st_new, const uint64_t* __restrict__ in_seen,
                                                   uint64_t* __restrict__ in_now, uint32_t* changed) {
    constexpr bool NUC = SRC == SRC_NUC;
    __shared__ uint64_t s_prec[tab_words<W>()];
    __shared__ uint64_t s_b[256 * W];
    load_tables<W>(s_prec, s_b, a.prec, SRC == SRC_P5 ? a.bmask5 : a.bmask, a.nt);
    const uint64_t gid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (gid >= a.nchunks) return;
    const uint64_t c0 = gid * a.chunk, c1 = c0 + a.chunk;
    const int words = (a.k + 1) * W;
    Bits<W> R[K + 1];
    bool same = true;
#pragma unroll
    for (int j = 0; j <= K; ++j) R[j] = bits_zero<W>();
    for (int i = 0; i < words; ++i) {
        const uint64_t v = gid + 1 < a.nchunks ? st_old[(gid + 1) * a.st_stride + i] : 0ull;
        same &= v == in_seen[gid * a.st_stride + i];
        in_now[gid * a.st_stride + i] = v;
    }
#pragma unroll
    for (int j = 0; j <= K; ++j)
        if (j <= a.k && gid + 1 < a.nchunks) R[j] = bits_of<W>(st_old + (gid + 1) * a.st_stride + j * W);
    if (same) {   // input unchanged: output unchanged
        for (int i = 0; i < words; ++i) st_new[gid * a.st_stride + i] = st_old[gid * a.st_stride + i];
        return;
    }
    for (uint64_t p = c1; p-- > c0;) {
        bool kill;
        uint8_t ch;
        if constexpr (SRC == SRC_P5) {
            ch = p < a.n ? (uint8_t)p5_code(a, p) : 0;
            kill = ch <= P5_NL;
        } else {
            ch = char_at<NUC>(a, p, kill);
        }
        nfa_rev_step<K, W>(R, bits_of<W>(s_b + ch * W), !kill, s_prec, a);
    }
    bool diff = false;
#pragma unroll
    for (int j = 0; j <= K; ++j) {
        if (j > a.k) continue;
#pragma unroll
        for (int q = 0; q < W; ++q) {
            diff |= R[j].w[q] != st_old[gid * a.st_stride + j * W + q];
            st_new[gid * a.st_stride + j * W + q] = R[j].w[q];
        }
    }
    if (diff) atomicOr(changed, 1u);
}

// k_nfa_verify: one lane per start, forward automaton -> shortest end.
template <int K, int W, bool NUC>
__global__ __launch_bounds__(256) void k_nfa_verify(NfaArgs a) {
    __shared__ uint64_t s_fol[tab_words<W>()];
    __shared__ uint64_t s_b[256 * W];
    load_tables<W>(s_fol, s_b, a.follow, a.bmask, a.nt);
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= a.nstarts) return;
    const uint64_t s = a.starts[i] & ((1ull << 48) - 1);
    // pm_oracle.c match_from(): rows R[j] and the "before the first position"
    // state init[j] (kept alive by insertions), deletion closures after every
    // step; the first accepting step gives the shortest end
    Bits<W> R[K + 1];
    bool init[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j) {
        R[j] = bits_of<W>(a.fwd_del[j]);
        init[j] = j == 0;
    }
    const Bits<W> first = bits_of<W>(a.first);
    uint32_t len = 0;
    // max_len == 0: unbounded pattern; every start came with a match inside
    // its record, and the record break ('\n', also the end of the file) kills
    // every state, so the loop ends at the shortest end
    const uint64_t steps = a.max_len ? (uint64_t)a.max_len : a.n - s + 1;
    for (uint64_t d = 0; d < steps; ++d) {
        bool kill;
        const uint8_t ch = char_at<NUC>(a, s + d, kill);
        const Bits<W> bc = bits_of<W>(s_b + ch * W);
        const bool nb = !kill;
        Bits<W> A[K + 1], N[K + 1];
        bool ninit[K + 1];
#pragma unroll
        for (int j = 0; j <= K; ++j) A[j] = fol_of<W>(a, s_fol, R[j]) | mask_if<W>(first, init[j]);
#pragma unroll
        for (int j = 0; j <= K; ++j) {
            N[j] = mask_if<W>(A[j] & bc, !kill);
            ninit[j] = false;
            if (j > 0) {
                if (a.errs & PM_ERR_SUB) N[j] = N[j] | mask_if<W>(A[j - 1], nb);
                if (a.errs & PM_ERR_INS) {
                    N[j] = N[j] | mask_if<W>(R[j - 1], nb);
                    ninit[j] = init[j - 1] && nb;
                }
            }
        }
        if (a.errs & PM_ERR_DEL) {
#pragma unroll
            for (int j = 0; j < K; ++j) N[j + 1] = N[j + 1] | fol_of<W>(a, s_fol, N[j]) | mask_if<W>(first, ninit[j]);
        }
        Bits<W> any = bits_zero<W>();
        bool alive = false;
#pragma unroll
        for (int j = 0; j <= K; ++j) {
            R[j] = mask_if<W>(N[j], j <= a.k);
            init[j] = ninit[j] && j <= a.k;
            any = any | R[j];
            alive |= init[j];
        }
        if (meets<W>(any, a.last)) {
            // '$': nrgrep's forward verification keeps extending while the
            // right context fails (extended checkMatch 0x411eb0), i.e. the
            // match must end at the line end
            bool k2;
            if (!a.end_anchor || char_at<NUC>(a, s + d + 1, k2) == (uint8_t)'\n') { len = (uint32_t)(d + 1); break; }
        }
        if (!any_of<W>(any) && !alive) break;
    }
    a.lens[i] = len;   // 0 = no match (cannot happen for a start found by k_nfa_rev)
}

// kernels instantiated per (error rows K + 1, state words W, layout); the
// runtime k runs on the smallest K >= k
#define PM_NFA_KW(X) X(0, 1) X(1, 1) X(2, 1) X(3, 1) X(7, 1) X(15, 1) \
                     X(0, 2) X(1, 2) X(2, 2) X(3, 2) X(7, 2) X(15, 2) \
                     X(0, 4) X(1, 4) X(2, 4) X(3, 4) X(7, 4)

// PM_IDS_JIT: "0" never, "1" always, default: databases of >= 64 Mi
// positions (below, the hipRTC compile would dominate the scan)
bool use_ids_kernel(const pm_db* db) {
    const char* e = getenv("PM_IDS_JIT");
    if (e) return e[0] != '0';
    return db->n >= (64ull << 20);
}

int kernel_rows(int k) { return k <= 3 ? k : k <= 7 ? 7 : 15; }
int kernel_words(int m) { return m <= 64 ? 1 : m <= 128 ? 2 : 4; }
bool nfa_supported(int k, int m) { return k <= PM_MAX_K && m <= PM_MAX_POSITIONS && !(kernel_words(m) == 4 && k > 7); }

template <int SRC>
void launch_nfa_rev(int K, int W, const NfaArgs& a, uint32_t blocks, hipStream_t s) {
#define PM_X(KK, WW) \
    if (K == KK && W == WW) { hipLaunchKernelGGL((k_nfa_rev<KK, WW, SRC>), dim3(blocks), dim3(256), 0, s, a); return; }
    PM_NFA_KW(PM_X)
#undef PM_X
    throw failure(PM_E_UNSUPPORTED, "no NFA kernel for these rows/words");
}

template <int SRC>
void launch_nfa_carry(int K, int W, const NfaArgs& a, uint32_t blocks, hipStream_t s, const uint64_t* o, uint64_t* n,
                      const uint64_t* seen, uint64_t* now, uint32_t* changed) {
#define PM_X(KK, WW)                                                                                          \
    if (K == KK && W == WW) {                                                                                 \
        hipLaunchKernelGGL((k_nfa_carry<KK, WW, SRC>), dim3(blocks), dim3(256), 0, s, a, o, n, seen, now, changed); \
        return;                                                                                               \
    }
    PM_NFA_KW(PM_X)
#undef PM_X
    throw failure(PM_E_UNSUPPORTED, "no NFA kernel for these rows/words");
}

template <bool NUC>
void launch_nfa_verify(int K, int W, const NfaArgs& a, uint32_t blocks, hipStream_t s) {
#define PM_X(KK, WW) \
    if (K == KK && W == WW) { hipLaunchKernelGGL((k_nfa_verify<KK, WW, NUC>), dim3(blocks), dim3(256), 0, s, a); return; }
    PM_NFA_KW(PM_X)
#undef PM_X
    throw failure(PM_E_UNSUPPORTED, "no NFA kernel for these rows/words");
}

}  // namespace
}  // namespace pm

namespace pm {
namespace {

// a plain class sequence: first = {0}, last = {m-1}, follow(i) = {i+1}
bool a_shift_only(int m, int W, const uint64_t* first, const uint64_t* last, const uint64_t* follow) {
    bool ok = true;
    for (int q = 0; q < W; ++q) {
        ok = ok && first[q] == (q == 0 ? 1ull : 0ull);
        ok = ok && last[q] == (q == (m - 1) / 64 ? 1ull << ((m - 1) % 64) : 0ull);
    }
    for (int i = 0; i < m && ok; ++i)
        for (int q = 0; q < W; ++q)
            ok = ok && follow[(size_t)i * W + q] == ((i + 1 < m && (i + 1) / 64 == q) ? 1ull << ((i + 1) % 64) : 0ull);
    return ok;
}

// PM_EXTENDED: the automaton of a sequence of classes each with an optional
// '?', '*' or '+' (nrgrep's detClass() == 2).  Its optional / repeatable
// positions are read off the automaton (position i is optional iff the
// position before it -- or the start -- may skip to i + 1; repeatable iff it
// follows itself) and the automaton is rebuilt from them to check the shape.
bool extended_shape(int m, int W, const uint64_t* first, const uint64_t* last, const uint64_t* follow,
                    uint64_t* opt, uint64_t* rep) {
    auto bit = [&](const uint64_t* set, int i) { return ((set[i >> 6] >> (i & 63)) & 1) != 0; };
    for (int q = 0; q < 4; ++q) opt[q] = rep[q] = 0;
    for (int i = 0; i < m; ++i) {
        if (bit(follow + (size_t)i * W, i)) rep[i >> 6] |= 1ull << (i & 63);
        const bool o = i + 1 < m ? (i == 0 ? bit(first, 1) : bit(follow + (size_t)(i - 1) * W, i + 1))
                                 : (m > 1 && bit(last, m - 2));
        if (o) opt[i >> 6] |= 1ull << (i & 63);
    }
    auto is_opt = [&](int i) { return bit(opt, i); };
    std::vector<uint64_t> f2(W, 0), l2(W, 0), fo2((size_t)m * W, 0);
    auto put = [&](uint64_t* set, int i) { set[i >> 6] |= 1ull << (i & 63); };
    for (int j = 0; j < m; ++j) {
        put(f2.data(), j);
        if (!is_opt(j)) break;
    }
    for (int j = m - 1; j >= 0; --j) {
        put(l2.data(), j);
        if (!is_opt(j)) break;
    }
    for (int i = 0; i < m; ++i) {
        if (bit(rep, i)) put(fo2.data() + (size_t)i * W, i);
        for (int j = i + 1; j < m; ++j) {
            put(fo2.data() + (size_t)i * W, j);
            if (!is_opt(j)) break;
        }
    }
    for (int q = 0; q < W; ++q)
        if (f2[q] != first[q] || l2[q] != last[q]) return false;
    for (size_t q = 0; q < (size_t)m * W; ++q)
        if (fo2[q] != follow[q]) return false;
    return true;
}

// The scan behind pm_scan_nfa_errs / pm_scan_nfa_wide: position sets of W
// words (W = ceil(m / 64)).
void scan_nfa(pm_db* db, int m, int W, const uint64_t* byte_mask, const uint64_t* follow, const uint64_t* first,
              const uint64_t* last, int max_len, int min_len, int k, int errs, int pattern_id, int flags,
              pm_hits** out, const RgTree* rgt = nullptr) {
    require((flags & ~(PM_REPORT_NRGREP | PM_ANCHOR_START | PM_ANCHOR_END | PM_KEEP_HEADERS | PM_CROSS_LINES |
                       PM_ESIMPLE | PM_EXTENDED | PM_REGULAR | PM_SCAN_BYTES | PM_PIPELINED)) == 0,
            "bad flags");
    // PM_PIPELINED: the report pass is queued and the count resolves on
    // first use (hits_finalize); the report kernels never see the bit
    const bool pipelined = (flags & PM_PIPELINED) != 0;
    flags &= ~PM_PIPELINED;
    require(!(flags & PM_REGULAR) || rgt != nullptr, "PM_REGULAR needs nrgrep's tree (pm_scan_nfa_tree)");
    require(db != nullptr, "db is NULL");
    std::lock_guard<std::recursive_mutex> lk(db->mu);
    DeviceGuard pj(db->device);
    post_join(db);   // a pipelined scan's post-processing may still read the workspaces
    require(out != nullptr && byte_mask && follow && first && last, "null argument");
    require(m >= 1 && m <= PM_MAX_POSITIONS, "m out of range", PM_E_UNSUPPORTED);
    require(W == kernel_words(m), "words must be ceil(m / 64), at most 4");
    require(max_len >= 0, "max_len < 0");
    const bool unbounded = max_len == 0;   // '*' / '+': matches may run to the record end
    require(k >= 0 && nfa_supported(k, m), "k out of range for the GPU kernels", PM_E_UNSUPPORTED);
    require(pattern_id >= 0 && pattern_id < 65536, "pattern_id out of range");
    bool nonempty_first = false, nonempty_last = false;
    for (int q = 0; q < W; ++q) {
        nonempty_first |= first[q] != 0;
        nonempty_last |= last[q] != 0;
    }
    require(nonempty_first && nonempty_last, "empty automaton");
    require((errs & ~(PM_ERR_INS | PM_ERR_DEL | PM_ERR_SUB)) == 0, "bad error-type mask");
    if (k == 0) errs = PM_ERR_SUB;   // no errors: the type letters are irrelevant
    const bool cross = (flags & PM_CROSS_LINES) != 0;
    require(!cross || (k == 0 && !unbounded), "PM_CROSS_LINES is nrgrep's simple engine: k = 0, bounded");
    // PM_ESIMPLE: a class sequence at k > 0 reported as nrgrep's esimple
    // engine does (pm_esimple.hip); its walk computes the ends itself
    const bool esimple = (flags & PM_ESIMPLE) && k > 0 && (flags & PM_REPORT_NRGREP);
    // PM_EXTENDED: an extended pattern reported as nrgrep's extended engine
    // (k = 0, pm_extended.hip) or eextended engine (k > 0, pm_eextended.hip)
    // does; its walk computes the ends
    const bool extended = (flags & PM_EXTENDED) && (flags & PM_REPORT_NRGREP);
    // PM_REGULAR: a regular pattern reported as nrgrep's regular engine
    // (k = 0) or eregular engine (k > 0) does (pm_regular.hip); its walk
    // computes the ends
    const bool regular = (flags & PM_REGULAR) && (flags & PM_REPORT_NRGREP) && !extended;
    uint64_t xopt[4] = {}, xrep[4] = {};
    require(!(flags & PM_EXTENDED) || extended_shape(m, W, first, last, follow, xopt, xrep),
            "PM_EXTENDED needs a sequence of classes with '?', '*', '+'");
    // a match must consume a pattern position (pm_oracle.c reports
    // non-empty matches only): with deletions that needs min_len > k --
    // except for nrgrep's esimple report, whose walk takes every position
    // of every line (es_all_positions; nrgrep then prints empty matches too)
    const bool all_pos = esimple && (errs & PM_ERR_DEL) && min_len <= k;
    // ... and for nrgrep's eextended report, whose walk then takes every
    // line (every position a key): the automaton scan is skipped
    const bool ee_all = extended && k > 0 && (errs & PM_ERR_DEL) && min_len <= k;
    // ... and for nrgrep's eregular report (every line a cluster)
    const bool rg_all = regular && k > 0 && (errs & PM_ERR_DEL) && min_len <= k;
    require(!(errs & PM_ERR_DEL) || min_len > k || all_pos || ee_all || rg_all,
            "deletions with k >= the shortest match length are not supported by the GPU scan", PM_E_UNSUPPORTED);
    const int ins_extra = (errs & PM_ERR_INS) ? k : 0;   // insertions lengthen a match
    require((uint64_t)max_len + ins_extra < (1ull << 31), "max_len out of range");
    DeviceGuard g(db->device);
    lane_begin(db);
    hipStream_t s = db->stream;
    const int K = kernel_rows(k);
    // Glushkov transition tables per slice of S positions (S = 8 for one
    // word, 4 above: nt * 2^S * W words of LDS)
    const int S = W == 1 ? 8 : 4, V = 1 << S;
    const int nt = (m + S - 1) / S;
    std::vector<uint64_t> prec((size_t)m * W, 0);
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < m; ++j)
            if ((follow[(size_t)i * W + j / 64] >> (j % 64)) & 1) prec[(size_t)j * W + i / 64] |= 1ull << (i % 64);
    std::vector<uint64_t> tf((size_t)nt * V * W, 0), tp((size_t)nt * V * W, 0);
    for (int t = 0; t < nt; ++t)
        for (int v = 0; v < V; ++v)
            for (int b = 0; b < S; ++b)
                if (((v >> b) & 1) && t * S + b < m)
                    for (int q = 0; q < W; ++q) {
                        tf[((size_t)t * V + v) * W + q] |= follow[(size_t)(t * S + b) * W + q];
                        tp[((size_t)t * V + v) * W + q] |= prec[(size_t)(t * S + b) * W + q];
                    }
    // start configurations (see the kernel comment): forward deletion
    // closure of the start, and the reverse search's injected config
    using Set = std::vector<uint64_t>;
    auto set_or = [&](const std::vector<uint64_t>& per_pos, const Set& set) {
        Set acc(W, 0);
        for (int i = 0; i < m; ++i)
            if ((set[i / 64] >> (i % 64)) & 1)
                for (int q = 0; q < W; ++q) acc[q] |= per_pos[(size_t)i * W + q];
        return acc;
    };
    auto set_union = [&](Set a2, const uint64_t* b2, bool on) {
        if (on)
            for (int q = 0; q < W; ++q) a2[q] |= b2[q];
        return a2;
    };
    const std::vector<uint64_t> fol_v(follow, follow + (size_t)m * W);
    std::vector<Set> fwd_del(k + 1, Set(W, 0)), rev_pre(k + 1, Set(W, 0)), rev_ins(k + 1, Set(W, 0)),
        S_rows(k + 1, Set(W, 0));
    {
        const bool del = errs & PM_ERR_DEL, ins = errs & PM_ERR_INS;
        for (int j = 0; j < k && del; ++j) {
            fwd_del[j + 1] = set_union(set_or(fol_v, fwd_del[j]), first, j == 0);
            S_rows[j + 1] = set_union(set_or(prec, S_rows[j]), last, j == 0 || ins);
        }
        for (int j = 0; j <= k; ++j) {
            rev_ins[j] = S_rows[j];
            rev_pre[j] = set_union(set_or(prec, S_rows[j]), last, j == 0 || ins);
        }
    }
    std::vector<uint64_t> bm(byte_mask, byte_mask + 256 * W);
    if (!cross)
        for (int q = 0; q < W; ++q) bm['\n' * W + q] = 0;   // records never span the delimiter
    Upload up;
    const size_t o_f = up.add(tf.data(), tf.size() * 8);
    const size_t o_p = up.add(tp.data(), tp.size() * 8);
    const size_t o_b = up.add(bm.data(), bm.size() * 8);
    // residue code -> positions (the byte copy's folded byte of the code; 0
    // a header byte or padding, 1 '\n': none)
    std::vector<uint64_t> bm5((size_t)32 * W, 0);
    if (db->alphabet == PM_ALPHA_BYTE && db->n_codes > 0)
        for (int b = 0; b < 256; ++b)
            if (db->code_of[b] > P5_NL)
                for (int q = 0; q < W; ++q) bm5[(size_t)db->code_of[b] * W + q] = bm[(size_t)b * W + q];
    const size_t o_b5 = up.add(bm5.data(), bm5.size() * 8);
    EsBuild esb;
    EsUpload esu;
    if (esimple) {
        require(a_shift_only(m, W, first, last, follow), "PM_ESIMPLE needs a class sequence");
        es_add_slot(esb, byte_mask, W, m, k, errs, (uint32_t)flags, pattern_id);
        es_upload(esb, up, esu);
    }
    size_t o_xslot = 0, o_xtab = 0;
    if (extended && k == 0)
        xt_build(byte_mask, W, m, xopt, xrep, max_len == 0 ? -1 : (int64_t)max_len, (uint32_t)flags, pattern_id, up,
                 o_xslot, o_xtab);
    bool ee_lines = false;
    if (extended && k > 0)
        ee_lines = ee_build(byte_mask, W, m, xopt, xrep, k, errs,
                            unbounded ? -1 : (int64_t)max_len + ((errs & PM_ERR_INS) ? k : 0), (uint32_t)flags,
                            pattern_id, ee_all, up, o_xslot, o_xtab);
    bool rg_prints = false;
    if (regular) {
        rg_prints = rg_build(*rgt, byte_mask, W, m, unbounded ? -1 : (int64_t)max_len, k, errs, (uint32_t)flags,
                             pattern_id, up, o_xslot, o_xtab);
        if (!rg_prints) {
            // k = 0: the window is a class / extended sequence, simpleScan /
            // extendedScan never set the state word checkMatch reads; k > 0:
            // detClass 2, eregularPreproc dies -- nrgrep_coords prints no
            // match (pm_regular.hip); no scan runs
            pm_hits* h = new pm_hits();
            h->device = db->device;
            h->keys = static_cast<uint64_t*>(pool_get(db->device, 8, &h->keys_cap));
            h->lens = static_cast<uint32_t*>(pool_get(db->device, 4, &h->lens_cap));
            hits_ready(db, h);
            *out = h;
            return;
        }
    }
    // the walk tables are the last upload of their build (xt / ee / rg)
    const uint32_t walk_tab_words = (extended || regular) ? (uint32_t)((up.blob.size() - o_xtab) / 8) : 0u;
    uint8_t* d_up = up.commit(db);
    EsPrep esp = esimple ? es_bind(esu, d_up, es_gap(esb)) : EsPrep{};
    XtPrep xtp;
    if (regular) {
        xtp.rg = reinterpret_cast<const RgSlot*>(d_up + o_xslot);
        xtp.tab = reinterpret_cast<const uint64_t*>(d_up + o_xtab);
        xtp.pid = pattern_id;
        xtp.words = m + 1 <= 64 ? 1 : RG_NW;
        xtp.eregular = k > 0 ? 1 : 0;
        xtp.k = k;
        if (k > 0) xtp.scanner = erg_scanner(up, o_xslot);
        xtp.tab_words = walk_tab_words;
    }
    if (extended) {
        if (k == 0) xtp.slot = reinterpret_cast<const XtSlot*>(d_up + o_xslot);
        if (k == 0) xtp.scanner = xt_scanner(up, o_xslot);
        else xtp.ee = reinterpret_cast<const EeSlot*>(d_up + o_xslot);
        if (k > 0) xtp.scanner = ee_scanner(up, o_xslot);
        xtp.tab = reinterpret_cast<const uint64_t*>(d_up + o_xtab);
        xtp.pid = pattern_id;
        xtp.words = W;
        xtp.k = k;
        xtp.tab_words = walk_tab_words;
    }
    esp.lines = all_pos ? 1 : 0;

    NfaArgs a{};
    a.nuc = nuc_view(db);
    a.bytes = db->bytes;
    a.bytes_raw = db->bytes_raw;
    a.follow = reinterpret_cast<const uint64_t*>(d_up + o_f);
    a.prec = reinterpret_cast<const uint64_t*>(d_up + o_p);
    a.bmask = reinterpret_cast<const uint64_t*>(d_up + o_b);
    for (int q = 0; q < W; ++q) {
        a.first[q] = first[q];
        a.last[q] = last[q];
        const int bits = std::min(64, m - 64 * q);
        a.mmask[q] = bits >= 64 ? ~0ull : bits <= 0 ? 0ull : ((1ull << bits) - 1);
    }
    a.nt = nt;
    a.halo = unbounded ? 0 : max_len + ins_extra - 1;
    a.shift_only = a_shift_only(m, W, first, last, follow);
    a.errs = errs;
    a.k = k;
    for (int j = 0; j <= k; ++j)
        for (int q = 0; q < W; ++q) {
            a.rev_pre[j][q] = rev_pre[j][q];
            a.rev_ins[j][q] = rev_ins[j][q];
            a.fwd_del[j][q] = fwd_del[j][q];
        }
    a.n = db->n;
    a.pattern_id = pattern_id;
    a.end_anchor = (flags & PM_ANCHOR_END) ? 1 : 0;
    a.cross = cross ? 1 : 0;
    require(!cross || db->alphabet == PM_ALPHA_NUC || db->bytes_raw, "internal: no raw bytes for a cross-line scan");
    // chunk per lane: a power of two (so that on the nucleotide layout
    // the lanes of a wave walk the streams of one tile in lock step and
    // their loads coincide), enough lanes to fill the chip; reads stop at
    // the end of the file (char_at), so the halo needs no padding.  A small
    // file gets chunks down to 16 positions: a lane's scan is a chain of
    // dependent steps, so lanes (not the halo's re-read) set the time
    // (configs[3], 3.5 MB at k = 1: 64-position chunks left < 1 wave per
    // SIMD).  Unbounded patterns keep 64 (their carry rounds grow with the
    // chunks per record).  The short chunks start at the halo's size (a
    // lane re-reads halo positions per chunk, so a 200-position pattern in
    // 16-position chunks would step ~14x per emitted position).
    uint64_t chunk = unbounded ? 64 : 16;
    if (!unbounded)
        while (chunk < 64 && chunk < (uint64_t)a.halo) chunk *= 2;
    while (chunk < (uint64_t)MAX_NFA_CHUNK && db->n / (chunk * 2) >= 256ull * 4 * 64 * 2) chunk *= 2;
    if (db->alphabet == PM_ALPHA_NUC) chunk = std::min<uint64_t>(chunk, STREAM);
    a.chunk = (int)chunk;
    a.nchunks = std::max<uint64_t>(1, (db->n + chunk - 1) / chunk);
    a.st_stride = (k + 1) * W;
    const bool nuc = db->alphabet == PM_ALPHA_NUC;
    // a peptide file's start pass reads the 5-bit residue planes (0.625 B per
    // residue) when it has them and the scan is line-bounded
    const bool p5 = !nuc && db->p5 && db->n_codes > 0 && !cross && !(flags & PM_SCAN_BYTES);
    if (p5) {
        a.p5 = db->p5;
        a.nw5 = db->nw5;
        a.bmask5 = reinterpret_cast<const uint64_t*>(d_up + o_b5);
    }

    uint64_t expected = std::max<uint64_t>(db->n / 64, 1 << 16);
    SinkBuffers sb;
    std::vector<uint32_t> counts;
    uint64_t total = 0;
    EventPair ev;
    const uint32_t blocks = blocks_for(a.nchunks, 256);
    double carry_ms = 0.0;
    if (unbounded) {
        // relaxation rounds (k_nfa_carry) until no chunk's state changes
        Carve c;
        const size_t st_bytes = a.nchunks * (size_t)a.st_stride * sizeof(uint64_t);
        const size_t o_a = c.take(st_bytes), o_b2 = c.take(st_bytes), o_s = c.take(st_bytes),
                     o_n = c.take(st_bytes), o_f2 = c.take(sizeof(uint32_t));
        uint8_t* base = static_cast<uint8_t*>(reserve(db, db->ws_rec, c.off));
        uint64_t* st[2] = {reinterpret_cast<uint64_t*>(base + o_a), reinterpret_cast<uint64_t*>(base + o_b2)};
        uint64_t* in_seen = reinterpret_cast<uint64_t*>(base + o_s);
        uint64_t* in_now = reinterpret_cast<uint64_t*>(base + o_n);
        uint32_t* changed = reinterpret_cast<uint32_t*>(base + o_f2);
        HIPCHK(hipMemsetAsync(st[0], 0, st_bytes, s));
        HIPCHK(hipMemsetAsync(in_seen, 0xff, st_bytes, s));   // no chunk has been scanned yet
        uint32_t* h_changed = static_cast<uint32_t*>(reserve_host(db, db->pin_slots, 64));
        int cur = 0;
        EventPair cev;
        HIPCHK(hipEventRecord(cev.a, s));
        for (uint64_t round = 0; round <= a.nchunks; ++round) {
            HIPCHK(hipMemsetAsync(changed, 0, sizeof(uint32_t), s));
            if (nuc) launch_nfa_carry<SRC_NUC>(K, W, a, blocks, s, st[cur], st[cur ^ 1], in_seen, in_now, changed);
            else if (p5) launch_nfa_carry<SRC_P5>(K, W, a, blocks, s, st[cur], st[cur ^ 1], in_seen, in_now, changed);
            else launch_nfa_carry<SRC_BYTE>(K, W, a, blocks, s, st[cur], st[cur ^ 1], in_seen, in_now, changed);
            HIPCHK(hipGetLastError());
            std::swap(in_seen, in_now);
            cur ^= 1;
            HIPCHK(hipMemcpyAsync(h_changed, changed, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            if (!*h_changed) break;
        }
        HIPCHK(hipEventRecord(cev.b, s));
        HIPCHK(hipEventSynchronize(cev.b));
        carry_ms = cev.ms();
        a.in_state = st[cur];
    }
    // a class sequence on the nucleotide planes: the bit-sliced start pass
    // (pm_ids.hip), 32 streams per lane instead of one
    const bool ids = nuc && W == 1 && a.shift_only && !cross && !unbounded && use_ids_kernel(db);
    for (int attempt = 0; attempt < 2 && !all_pos && !ee_lines && !rg_all; ++attempt) {
        sb = make_sink(db, 1, db->n, expected);
        a.sink = sb.sink();
        bool launched = false;
        if (ids) {
            IdsSpec sp{m, k, errs, bm.data(), a.bmask, {}, {}, pattern_id};
            for (int j = 0; j <= k; ++j) {
                sp.rev_pre[j] = rev_pre[j][0];
                sp.rev_ins[j] = rev_ins[j][0];
            }
            launched = ids_rev_scan(db, sp, a.sink, s, ev.a, ev.b);
        }
        if (!launched) {
            HIPCHK(hipEventRecord(ev.a, s));
            if (nuc) launch_nfa_rev<SRC_NUC>(K, W, a, blocks, s);
            else if (p5) launch_nfa_rev<SRC_P5>(K, W, a, blocks, s);
            else launch_nfa_rev<SRC_BYTE>(K, W, a, blocks, s);
            HIPCHK(hipEventRecord(ev.b, s));
        }
        HIPCHK(hipGetLastError());
        bool overflow = false;
        total = sink_total(db, sb, counts, overflow);
        if (!overflow) break;
        require(attempt == 0, "internal: hit bins overflowed twice");
        expected = (uint64_t)(*std::max_element(counts.begin(), counts.end())) * sb.nbins + sb.nbins;
    }
    // eextended walking every line (EeSlot::lines): every position is a key,
    // the lines are its clusters
    const bool every_pos = all_pos || ee_lines || rg_all;
    double kms = every_pos ? 0.0 : ev.ms() + carry_ms;
    if (every_pos) total = db->n;
    pm_hits* h = every_pos ? es_all_positions(db, pattern_id) : sink_to_hits(db, sb, counts, total);
    // eextended: an alignment starting a header line prints one position
    // before it (pm_eextended.hip): every header line starts a cluster
    if (extended && k > 0 && !ee_lines) total = ee_add_headers(db, h, total, pattern_id);
    if (total && !esimple && !extended && !regular) {
        a.starts = h->keys;
        a.nstarts = total;
        a.lens = h->lens;
        a.max_len = unbounded ? 0 : max_len + ins_extra;
        EventPair ev2;
        HIPCHK(hipEventRecord(ev2.a, s));
        if (nuc) launch_nfa_verify<true>(K, W, a, blocks_for(total, 256), s);
        else launch_nfa_verify<false>(K, W, a, blocks_for(total, 256), s);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ev2.b, s));
        HIPCHK(hipStreamSynchronize(s));
        kms += ev2.ms();
    }
    h->kernel_ms = kms;
    // line-bounded engines (nrgrep's extended/regular/e* verify inside the
    // record, e.g. extended checkMatch 0x411b1d): no candidate starts on a
    // header line, the pass only selects what nrgrep reports; the simple
    // engine (cross) also drops the windows starting on a header line
    // (esimple: the walk replaces the lengths; until it runs they are unset)
    const bool walk = esimple || extended || regular;
    const bool rep = walk || report_needed(db, (uint32_t)flags, cross);
    const EsPrep* rep_es = esimple ? &esp : nullptr;
    const XtPrep* rep_xt = (extended || regular) ? &xtp : nullptr;
    if (pipelined && rep && total && !every_pos) {
        // the report pass is queued behind the scan and its kept count lands
        // in pinned memory with the pass's last dispatch: the caller launches
        // its next scan (the other strand) while this one's walk runs --
        // between the two strands of a `-k 2ids` query the GPU idled ~0.1 ms
        // for the host's wait, copy and next launch (round 6)
        std::unique_ptr<pm_pending> pd(new pm_pending());
        pd->db = db;
        pd->count_only = true;
        pd->counts_h = static_cast<uint32_t*>(pinned_get(8, &pd->counts_cap));
        pd->counts_h[0] = 0u;
        const ReportWs ws = report_ws(db, h->keys_cap / 8);
        if (!h->ready) HIPCHK(hipEventCreate(&h->ready));
        report_enqueue_ws(db, h, (uint32_t)flags, ws, false, total, pd->counts_h, s, h->ready, !walk && cross, rep_es,
                          rep_xt);
        lane_end(db, s);
        h->pending = pd.release();
        db->pending.insert(h);
        *out = h;
        return;
    }
    if (rep) report_sync(db, h, (uint32_t)flags, total, !walk && cross, rep_es, rep_xt);
    HIPCHK(hipStreamSynchronize(s));
    hits_ready(db, h);
    *out = h;
}

}  // namespace
}  // namespace pm

using namespace pm;

extern "C" int pm_scan_nfa(pm_db* db, int m, const uint64_t* byte_mask, const uint64_t* follow, uint64_t first,
                           uint64_t last, int max_len, int k, int pattern_id, pm_hits** out) {
    return pm_scan_nfa_errs(db, m, byte_mask, follow, first, last, max_len, 0, k, PM_ERR_SUB, pattern_id,
                            PM_REPORT_NRGREP, out);
}

extern "C" int pm_scan_nfa_errs(pm_db* db, int m, const uint64_t* byte_mask, const uint64_t* follow, uint64_t first,
                                uint64_t last, int max_len, int min_len, int k, int errs, int pattern_id,
                                int flags, pm_hits** out) {
    return guarded([&] {
        require(m >= 1 && m <= 64, "m out of range (pm_scan_nfa_wide takes longer automata)");
        require(!(flags & PM_CROSS_LINES), "bad flags");
        scan_nfa(db, m, 1, byte_mask, follow, &first, &last, max_len, min_len, k, errs, pattern_id, flags, out);
    });
}

extern "C" int pm_scan_nfa_tree(pm_db* db, int m, int words, const uint64_t* byte_mask, const uint64_t* follow,
                                const uint64_t* first, const uint64_t* last, int max_len, int min_len, int k,
                                int errs, int pattern_id, int flags, int nodes, const int32_t* tree,
                                const int32_t* tree_nullable, pm_hits** out) {
    return guarded([&] {
        require(nodes >= 1 && tree != nullptr && tree_nullable != nullptr, "null tree");
        const RgTree t{nodes, tree, tree_nullable};
        scan_nfa(db, m, words, byte_mask, follow, first, last, max_len, min_len, k, errs, pattern_id, flags, out, &t);
    });
}

extern "C" int pm_scan_nfa_wide(pm_db* db, int m, int words, const uint64_t* byte_mask, const uint64_t* follow,
                                const uint64_t* first, const uint64_t* last, int max_len, int min_len, int k,
                                int errs, int pattern_id, int flags, pm_hits** out) {
    return guarded([&] {
        scan_nfa(db, m, words, byte_mask, follow, first, last, max_len, min_len, k, errs, pattern_id, flags, out);
    });
}
