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

struct NfaArgs {
    NucView nuc;
    const uint8_t* bytes;
    const uint64_t* prec;     // [nt][256]   positions preceding the set
    const uint64_t* follow;   // [nt][256]   positions following the set
    const uint64_t* bmask;    // [256]
    uint64_t first, last;
    int nt;
    int halo;
    int chunk;                // positions per lane
    uint64_t n;
    uint64_t nchunks;
    int pattern_id;
    int end_anchor;           // '$': the verify's end must be a line end
    Sink sink;
    int errs;                 // PM_ERR_INS | PM_ERR_DEL | PM_ERR_SUB
    uint64_t rev_pre[4];      // reverse: prec(S[j]) | (I[j] ? last : 0) for the injected start config
    uint64_t rev_ins[4];      // reverse: S[j] (insertion source rows of the injected config)
    uint64_t fwd_del[4];      // forward: deletion closure of the start config (rows of R)
    // unbounded patterns: reverse state entering each chunk from the right
    // (rows at stride 4), found by k_nfa_carry; null = start from the halo
    const uint64_t* in_state;
    // a plain class sequence (follow(i) = {i+1}): transitions are shifts
    // instead of table lookups; mmask = the m position bits
    int shift_only;
    uint64_t mmask;
    // verify
    const uint64_t* starts;
    uint64_t nstarts;
    uint32_t* lens;
    int max_len;
};

__device__ inline uint64_t table_or(const uint64_t* __restrict__ tab, uint64_t set, int nt) {
    uint64_t acc = 0;
    for (int t = 0; t < nt; ++t) acc |= tab[t * 256 + ((set >> (8 * t)) & 255)];
    return acc;
}
// positions preceding / following a set (reverse / forward transitions)
__device__ inline uint64_t prec_of(const NfaArgs& a, const uint64_t* __restrict__ s_prec, uint64_t set) {
    return a.shift_only ? set >> 1 : table_or(s_prec, set, a.nt);
}
__device__ inline uint64_t fol_of(const NfaArgs& a, const uint64_t* __restrict__ s_fol, uint64_t set) {
    return a.shift_only ? (set << 1) & a.mmask : table_or(s_fol, set, a.nt);
}

// One character of the reverse search (right to left).  Substitution-only
// patterns (the common case) take the short form.
template <int K>
__device__ inline void nfa_rev_step(uint64_t (&R)[K + 1], uint64_t bc, uint64_t nb,
                                    const uint64_t* __restrict__ s_prec, const NfaArgs& a) {
    uint64_t A[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j) A[j] = prec_of(a, s_prec, R[j]) | a.rev_pre[j];
    if (a.errs == PM_ERR_SUB) {
#pragma unroll
        for (int j = K; j >= 0; --j) R[j] = (A[j] & bc) | (j > 0 ? (A[j - 1] & nb) : 0ull);
        return;
    }
    uint64_t N[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j) {
        N[j] = A[j] & bc;
        if (j > 0) {
            if (a.errs & PM_ERR_SUB) N[j] |= A[j - 1] & nb;
            if (a.errs & PM_ERR_INS) N[j] |= (R[j - 1] | a.rev_ins[j - 1]) & nb;
        }
    }
    if (a.errs & PM_ERR_DEL) {
        // ninit[j] (j >= 1) = an insertion-kept start; row 0's init is consumed
#pragma unroll
        for (int j = 0; j < K; ++j)
            N[j + 1] |= prec_of(a, s_prec, N[j]) | ((j >= 1 && (a.errs & PM_ERR_INS) && nb) ? a.last : 0ull);
    }
#pragma unroll
    for (int j = 0; j <= K; ++j) R[j] = N[j];
}

template <bool NUC>
__device__ inline uint8_t char_at(const NfaArgs& a, uint64_t p) {
    if constexpr (NUC) return nuc_char_at(a.nuc, p);
    else return a.bytes[p];
}

template <int K, bool NUC>
__global__ __launch_bounds__(256) void k_nfa_rev(NfaArgs a) {
    __shared__ uint64_t s_prec[8 * 256];
    __shared__ uint64_t s_b[256];
    for (int i = threadIdx.x; i < a.nt * 256; i += blockDim.x) s_prec[i] = a.prec[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s_b[i] = a.bmask[i];
    __syncthreads();
    const uint64_t gid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const bool live = gid < a.nchunks;
    const uint64_t chunk_id = live ? gid : a.nchunks - 1;
    const uint64_t c0 = chunk_id * a.chunk;
    const uint64_t c1 = c0 + a.chunk;           // emit for [c0, c1) ∩ [0, n)
    const uint64_t top = c1 + a.halo;           // process (top .. c0], padded storage
    uint64_t R[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j)
        R[j] = (a.in_state && chunk_id + 1 < a.nchunks) ? a.in_state[(chunk_id + 1) * 4 + j] : 0ull;
    for (uint64_t p = top; p-- > c0;) {
        const uint8_t ch = char_at<NUC>(a, p);
        const uint64_t bc = s_b[ch];
        const uint64_t nb = ch == '\n' ? 0ull : ~0ull;
        nfa_rev_step<K>(R, bc, nb, s_prec, a);
        uint64_t any = 0;
#pragma unroll
        for (int j = 0; j <= K; ++j) any |= R[j];
        if (live && p < c1 && p < a.n && (any & a.first))
            a.sink.push(a.sink.bin_of(0, p), ((uint64_t)a.pattern_id << 48) | p);
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
template <int K, bool NUC>
__global__ __launch_bounds__(256) void k_nfa_carry(NfaArgs a, const uint64_t* __restrict__ st_old,
                                                   uint64_t* __restrict__ st_new, const uint64_t* __restrict__ in_seen,
                                                   uint64_t* __restrict__ in_now, uint32_t* changed) {
    __shared__ uint64_t s_prec[8 * 256];
    __shared__ uint64_t s_b[256];
    for (int i = threadIdx.x; i < a.nt * 256; i += blockDim.x) s_prec[i] = a.prec[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s_b[i] = a.bmask[i];
    __syncthreads();
    const uint64_t gid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (gid >= a.nchunks) return;
    const uint64_t c0 = gid * a.chunk, c1 = c0 + a.chunk;
    uint64_t R[K + 1];
    bool same = true;
#pragma unroll
    for (int j = 0; j <= K; ++j) {
        R[j] = gid + 1 < a.nchunks ? st_old[(gid + 1) * 4 + j] : 0ull;
        same &= R[j] == in_seen[gid * 4 + j];
        in_now[gid * 4 + j] = R[j];
    }
    if (same) {   // input unchanged: output unchanged
#pragma unroll
        for (int j = 0; j <= K; ++j) st_new[gid * 4 + j] = st_old[gid * 4 + j];
        return;
    }
    for (uint64_t p = c1; p-- > c0;) {
        const uint8_t ch = char_at<NUC>(a, p);
        nfa_rev_step<K>(R, s_b[ch], ch == '\n' ? 0ull : ~0ull, s_prec, a);
    }
    bool diff = false;
#pragma unroll
    for (int j = 0; j <= K; ++j) {
        diff |= R[j] != st_old[gid * 4 + j];
        st_new[gid * 4 + j] = R[j];
    }
    if (diff) atomicOr(changed, 1u);
}

// k_nfa_verify: one lane per start, forward automaton -> shortest end.
template <int K, bool NUC>
__global__ __launch_bounds__(256) void k_nfa_verify(NfaArgs a) {
    __shared__ uint64_t s_fol[8 * 256];
    __shared__ uint64_t s_b[256];
    for (int i = threadIdx.x; i < a.nt * 256; i += blockDim.x) s_fol[i] = a.follow[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s_b[i] = a.bmask[i];
    __syncthreads();
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= a.nstarts) return;
    const uint64_t s = a.starts[i] & ((1ull << 48) - 1);
    // pm_oracle.c match_from(): rows R[j] and the "before the first position"
    // state init[j] (kept alive by insertions), deletion closures after every
    // step; the first accepting step gives the shortest end
    uint64_t R[K + 1];
    bool init[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j) {
        R[j] = a.fwd_del[j];
        init[j] = j == 0;
    }
    uint32_t len = 0;
    // max_len == 0: unbounded pattern; every start came with a match inside
    // its record, and the record break ('\n', also the tail padding) kills
    // every state, so the loop ends at the shortest end
    const uint64_t steps = a.max_len ? (uint64_t)a.max_len : a.n - s + 1;
    for (uint64_t d = 0; d < steps; ++d) {
        const uint8_t ch = char_at<NUC>(a, s + d);
        const uint64_t bc = s_b[ch];
        const uint64_t nb = ch == '\n' ? 0ull : ~0ull;
        uint64_t A[K + 1], N[K + 1];
        bool ninit[K + 1];
#pragma unroll
        for (int j = 0; j <= K; ++j) A[j] = fol_of(a, s_fol, R[j]) | (init[j] ? a.first : 0ull);
#pragma unroll
        for (int j = 0; j <= K; ++j) {
            N[j] = A[j] & bc;
            ninit[j] = false;
            if (j > 0) {
                if (a.errs & PM_ERR_SUB) N[j] |= A[j - 1] & nb;
                if (a.errs & PM_ERR_INS) {
                    N[j] |= R[j - 1] & nb;
                    ninit[j] = init[j - 1] && nb;
                }
            }
        }
        if (a.errs & PM_ERR_DEL) {
#pragma unroll
            for (int j = 0; j < K; ++j) N[j + 1] |= fol_of(a, s_fol, N[j]) | (ninit[j] ? a.first : 0ull);
        }
        uint64_t any = 0;
        bool alive = false;
#pragma unroll
        for (int j = 0; j <= K; ++j) {
            R[j] = N[j];
            init[j] = ninit[j];
            any |= R[j];
            alive |= init[j];
        }
        if (any & a.last) {
            // '$': nrgrep's forward verification keeps extending while the
            // right context fails (extended checkMatch 0x411eb0), i.e. the
            // match must end at the line end
            if (!a.end_anchor || char_at<NUC>(a, s + d + 1) == (uint8_t)'\n') { len = (uint32_t)(d + 1); break; }
        }
        if (!any && !alive) break;
    }
    a.lens[i] = len;   // 0 = no match (cannot happen for a start found by k_nfa_rev)
}

template <bool NUC>
void launch_nfa_rev(int k, const NfaArgs& a, uint32_t blocks, hipStream_t s) {
    switch (k) {
        case 0: hipLaunchKernelGGL((k_nfa_rev<0, NUC>), dim3(blocks), dim3(256), 0, s, a); break;
        case 1: hipLaunchKernelGGL((k_nfa_rev<1, NUC>), dim3(blocks), dim3(256), 0, s, a); break;
        case 2: hipLaunchKernelGGL((k_nfa_rev<2, NUC>), dim3(blocks), dim3(256), 0, s, a); break;
        default: hipLaunchKernelGGL((k_nfa_rev<3, NUC>), dim3(blocks), dim3(256), 0, s, a); break;
    }
}

template <bool NUC>
void launch_nfa_carry(int k, const NfaArgs& a, uint32_t blocks, hipStream_t s, const uint64_t* o, uint64_t* n,
                      const uint64_t* seen, uint64_t* now, uint32_t* changed) {
    switch (k) {
        case 0: hipLaunchKernelGGL((k_nfa_carry<0, NUC>), dim3(blocks), dim3(256), 0, s, a, o, n, seen, now, changed); break;
        case 1: hipLaunchKernelGGL((k_nfa_carry<1, NUC>), dim3(blocks), dim3(256), 0, s, a, o, n, seen, now, changed); break;
        case 2: hipLaunchKernelGGL((k_nfa_carry<2, NUC>), dim3(blocks), dim3(256), 0, s, a, o, n, seen, now, changed); break;
        default: hipLaunchKernelGGL((k_nfa_carry<3, NUC>), dim3(blocks), dim3(256), 0, s, a, o, n, seen, now, changed); break;
    }
}

template <bool NUC>
void launch_nfa_verify(int k, const NfaArgs& a, uint32_t blocks, hipStream_t s) {
    switch (k) {
        case 0: hipLaunchKernelGGL((k_nfa_verify<0, NUC>), dim3(blocks), dim3(256), 0, s, a); break;
        case 1: hipLaunchKernelGGL((k_nfa_verify<1, NUC>), dim3(blocks), dim3(256), 0, s, a); break;
        case 2: hipLaunchKernelGGL((k_nfa_verify<2, NUC>), dim3(blocks), dim3(256), 0, s, a); break;
        default: hipLaunchKernelGGL((k_nfa_verify<3, NUC>), dim3(blocks), dim3(256), 0, s, a); break;
    }
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
        require((flags & ~(PM_REPORT_NRGREP | PM_ANCHOR_START | PM_ANCHOR_END | PM_KEEP_HEADERS)) == 0, "bad flags");
        require(db != nullptr, "db is NULL");
        std::lock_guard<std::recursive_mutex> lk(db->mu);
        require(db != nullptr && out != nullptr && byte_mask && follow, "null argument");
        require(m >= 1 && m <= PM_MAX_POSITIONS, "m out of range");
        require(max_len >= 0, "max_len < 0");
        const bool unbounded = max_len == 0;   // '*' / '+': matches may run to the record end
        require(max_len <= 1024, "max_len above 1024", PM_E_UNSUPPORTED);
        require(k >= 0 && k <= PM_MAX_K, "k out of range for the GPU kernels", PM_E_UNSUPPORTED);
        require(pattern_id >= 0 && pattern_id < 65536, "pattern_id out of range");
        require(first != 0 && last != 0, "empty automaton");
        require((errs & ~(PM_ERR_INS | PM_ERR_DEL | PM_ERR_SUB)) == 0, "bad error-type mask");
        if (k == 0) errs = PM_ERR_SUB;   // no errors: the type letters are irrelevant
        // a match must consume a pattern position (pm_oracle.c reports
        // non-empty matches only): with deletions that needs min_len > k
        require(!(errs & PM_ERR_DEL) || min_len > k,
                "deletions with k >= the shortest match length are not supported by the GPU scan",
                PM_E_UNSUPPORTED);
        const int ins_extra = (errs & PM_ERR_INS) ? k : 0;   // insertions lengthen a match
        require(max_len + ins_extra <= 1024 + PM_MAX_K, "max_len above 1024", PM_E_UNSUPPORTED);
        DeviceGuard g(db->device);
        lane_begin(db);
        hipStream_t s = db->stream;
        const int nt = (m + 7) / 8;
        // Glushkov transition tables per 8-position slice: follow / precede
        std::vector<uint64_t> tf(nt * 256, 0), tp(nt * 256, 0), prec(m, 0);
        for (int i = 0; i < m; ++i)
            for (int j = 0; j < m; ++j)
                if ((follow[i] >> j) & 1) prec[j] |= 1ull << i;
        for (int t = 0; t < nt; ++t)
            for (int v = 0; v < 256; ++v)
                for (int b = 0; b < 8; ++b)
                    if (((v >> b) & 1) && t * 8 + b < m) {
                        tf[t * 256 + v] |= follow[t * 8 + b];
                        tp[t * 256 + v] |= prec[t * 8 + b];
                    }
        // start configurations (see the kernel comment): forward deletion
        // closure of the start, and the reverse search's injected config
        auto set_or = [&](const std::vector<uint64_t>& per_pos, uint64_t set) {
            uint64_t acc = 0;
            for (int i = 0; i < m; ++i)
                if ((set >> i) & 1) acc |= per_pos[i];
            return acc;
        };
        const std::vector<uint64_t> fol_v(follow, follow + m);
        uint64_t fwd_del[4] = {0, 0, 0, 0}, rev_pre[4] = {0, 0, 0, 0}, rev_ins[4] = {0, 0, 0, 0};
        {
            uint64_t S[4] = {0, 0, 0, 0};
            const bool del = errs & PM_ERR_DEL, ins = errs & PM_ERR_INS;
            for (int j = 0; j < k && del; ++j) {
                fwd_del[j + 1] = set_or(fol_v, fwd_del[j]) | (j == 0 ? first : 0);
                S[j + 1] = set_or(prec, S[j]) | ((j == 0 || ins) ? last : 0);
            }
            for (int j = 0; j <= k; ++j) {
                rev_ins[j] = S[j];
                rev_pre[j] = set_or(prec, S[j]) | ((j == 0 || ins) ? last : 0);
            }
        }
        std::vector<uint64_t> bm(byte_mask, byte_mask + 256);
        bm['\n'] = 0;   // records never span the delimiter
        Upload up;
        const size_t o_f = up.add(tf.data(), tf.size() * 8);
        const size_t o_p = up.add(tp.data(), tp.size() * 8);
        const size_t o_b = up.add(bm.data(), 256 * 8);
        uint8_t* d_up = up.commit(db);

        NfaArgs a{};
        a.nuc = nuc_view(db);
        a.bytes = db->bytes;
        a.follow = reinterpret_cast<const uint64_t*>(d_up + o_f);
        a.prec = reinterpret_cast<const uint64_t*>(d_up + o_p);
        a.bmask = reinterpret_cast<const uint64_t*>(d_up + o_b);
        a.first = first;
        a.last = last;
        a.nt = nt;
        a.halo = unbounded ? 0 : max_len + ins_extra - 1;
        a.mmask = m == 64 ? ~0ull : ((1ull << m) - 1);
        a.shift_only = first == 1 && last == (1ull << (m - 1));
        for (int i = 0; i < m && a.shift_only; ++i)
            a.shift_only = follow[i] == (i + 1 < m ? (1ull << (i + 1)) : 0ull);
        a.errs = errs;
        for (int j = 0; j < 4; ++j) {
            a.rev_pre[j] = rev_pre[j];
            a.rev_ins[j] = rev_ins[j];
            a.fwd_del[j] = fwd_del[j];
        }
        a.n = db->n;
        a.pattern_id = pattern_id;
        a.end_anchor = (flags & PM_ANCHOR_END) ? 1 : 0;
        // chunk per lane: a power of two (so that on the nucleotide layout
        // the lanes of a wave walk the streams of one tile in lock step and
        // their loads coincide), enough lanes to fill the chip
        uint64_t chunk = 64;
        while (chunk < (uint64_t)MAX_NFA_CHUNK && db->n / (chunk * 2) >= 256ull * 4 * 64 * 2) chunk *= 2;
        if (db->alphabet == PM_ALPHA_NUC) chunk = std::min<uint64_t>(chunk, STREAM);
        a.chunk = (int)chunk;
        a.nchunks = std::max<uint64_t>(1, (db->n + chunk - 1) / chunk);
        const bool nuc = db->alphabet == PM_ALPHA_NUC;
        const uint64_t need = a.nchunks * chunk + a.halo + 64;   // storage must cover the last halo
        if (nuc) require(need <= db->ntiles * TILE_POS, "internal: NUC padding too small");
        else require(need <= db->nbytes_alloc, "internal: byte padding too small");

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
            const size_t st_bytes = a.nchunks * 4 * sizeof(uint64_t);
            const size_t o_a = c.take(st_bytes), o_b = c.take(st_bytes), o_s = c.take(st_bytes),
                         o_n = c.take(st_bytes), o_f = c.take(sizeof(uint32_t));
            uint8_t* base = static_cast<uint8_t*>(reserve(db, db->ws_rec, c.off));
            uint64_t* st[2] = {reinterpret_cast<uint64_t*>(base + o_a), reinterpret_cast<uint64_t*>(base + o_b)};
            uint64_t* in_seen = reinterpret_cast<uint64_t*>(base + o_s);
            uint64_t* in_now = reinterpret_cast<uint64_t*>(base + o_n);
            uint32_t* changed = reinterpret_cast<uint32_t*>(base + o_f);
            HIPCHK(hipMemsetAsync(st[0], 0, st_bytes, s));
            HIPCHK(hipMemsetAsync(in_seen, 0xff, st_bytes, s));   // no chunk has been scanned yet
            uint32_t* h_changed = static_cast<uint32_t*>(reserve_host(db, db->pin_slots, 64));
            int cur = 0;
            EventPair cev;
            HIPCHK(hipEventRecord(cev.a, s));
            for (uint64_t round = 0; round <= a.nchunks; ++round) {
                HIPCHK(hipMemsetAsync(changed, 0, sizeof(uint32_t), s));
                if (nuc) launch_nfa_carry<true>(k, a, blocks, s, st[cur], st[cur ^ 1], in_seen, in_now, changed);
                else launch_nfa_carry<false>(k, a, blocks, s, st[cur], st[cur ^ 1], in_seen, in_now, changed);
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
        for (int attempt = 0; attempt < 2; ++attempt) {
            sb = make_sink(db, 1, db->n, expected);
            a.sink = sb.sink();
            HIPCHK(hipEventRecord(ev.a, s));
            if (nuc) launch_nfa_rev<true>(k, a, blocks, s);
            else launch_nfa_rev<false>(k, a, blocks, s);
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventRecord(ev.b, s));
            bool overflow = false;
            total = sink_total(db, sb, counts, overflow);
            if (!overflow) break;
            require(attempt == 0, "internal: hit bins overflowed twice");
            expected = (uint64_t)(*std::max_element(counts.begin(), counts.end())) * sb.nbins + sb.nbins;
        }
        double kms = ev.ms() + carry_ms;
        pm_hits* h = sink_to_hits(db, sb, counts, total);
        if (total) {
            a.starts = h->keys;
            a.nstarts = total;
            a.lens = h->lens;
            a.max_len = unbounded ? 0 : max_len + ins_extra;
            EventPair ev2;
            HIPCHK(hipEventRecord(ev2.a, s));
            if (nuc) launch_nfa_verify<true>(k, a, blocks_for(total, 256), s);
            else launch_nfa_verify<false>(k, a, blocks_for(total, 256), s);
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventRecord(ev2.b, s));
            HIPCHK(hipStreamSynchronize(s));
            kms += ev2.ms();
        }
        h->kernel_ms = kms;
        // line-bounded engines (nrgrep's extended/regular/e* verify inside the
        // record, e.g. extended checkMatch 0x411b1d): no candidate starts on a
        // header line, the pass only selects what nrgrep reports
        if (report_needed((uint32_t)flags, false)) report_sync(db, h, (uint32_t)flags, total, false);
        HIPCHK(hipStreamSynchronize(s));
        hits_ready(db, h);
        *out = h;
    });
}
