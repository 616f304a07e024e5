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
    Sink sink;
    // verify
    const uint64_t* starts;
    uint64_t nstarts;
    uint32_t* lens;
    int max_len;
};

template <int K>
__device__ inline void nfa_rev_step(uint64_t (&R)[K + 1], uint64_t bc, uint64_t nb,
                                    const uint64_t* __restrict__ s_prec, int nt, uint64_t last) {
    uint64_t A[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j) {
        uint64_t acc = last;
        const uint64_t d = R[j];
        for (int t = 0; t < nt; ++t) acc |= s_prec[t * 256 + ((d >> (8 * t)) & 255)];
        A[j] = acc;
    }
#pragma unroll
    for (int j = K; j >= 0; --j) R[j] = (A[j] & bc) | (j > 0 ? (A[j - 1] & nb) : 0ull);
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
    for (int j = 0; j <= K; ++j) R[j] = 0;
    for (uint64_t p = top; p-- > c0;) {
        const uint8_t ch = char_at<NUC>(a, p);
        const uint64_t bc = s_b[ch];
        const uint64_t nb = ch == '\n' ? 0ull : ~0ull;
        nfa_rev_step<K>(R, bc, nb, s_prec, a.nt, a.last);
        uint64_t any = 0;
#pragma unroll
        for (int j = 0; j <= K; ++j) any |= R[j];
        if (live && p < c1 && p < a.n && (any & a.first))
            a.sink.push(a.sink.bin_of(0, p), ((uint64_t)a.pattern_id << 48) | p);
    }
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
    uint64_t R[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j) R[j] = 0;
    uint32_t len = 0;
    for (int d = 0; d < a.max_len; ++d) {
        const uint8_t ch = char_at<NUC>(a, s + d);
        const uint64_t bc = s_b[ch];
        const uint64_t nb = ch == '\n' ? 0ull : ~0ull;
        uint64_t A[K + 1];
#pragma unroll
        for (int j = 0; j <= K; ++j) {
            uint64_t acc = (d == 0 && j == 0) ? a.first : 0ull;
            const uint64_t v = R[j];
            for (int t = 0; t < a.nt; ++t) acc |= s_fol[t * 256 + ((v >> (8 * t)) & 255)];
            A[j] = acc;
        }
        uint64_t any = 0;
#pragma unroll
        for (int j = K; j >= 0; --j) {
            R[j] = (A[j] & bc) | (j > 0 ? (A[j - 1] & nb) : 0ull);
            any |= R[j];
        }
        if (any & a.last) { len = d + 1; break; }
        if (!any) break;
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
    return guarded([&] {
        require(db != nullptr && out != nullptr && byte_mask && follow, "null argument");
        require(m >= 1 && m <= PM_MAX_POSITIONS, "m out of range");
        require(max_len >= 1, "unbounded patterns (*, +) are not supported by the GPU scan yet", PM_E_UNSUPPORTED);
        require(max_len <= 1024, "max_len above 1024", PM_E_UNSUPPORTED);
        require(k >= 0 && k <= PM_MAX_K, "k out of range for the GPU kernels", PM_E_UNSUPPORTED);
        require(pattern_id >= 0 && pattern_id < 65536, "pattern_id out of range");
        require(first != 0 && last != 0, "empty automaton");
        DeviceGuard g(db->device);
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
        a.halo = max_len - 1;
        a.n = db->n;
        a.pattern_id = pattern_id;
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
        double kms = ev.ms();
        pm_hits* h = sink_to_hits(db, sb, counts, total);
        if (total) {
            a.starts = h->keys;
            a.nstarts = total;
            a.lens = h->lens;
            a.max_len = max_len;
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
        HIPCHK(hipStreamSynchronize(s));
        hits_ready(db, h);
        *out = h;
    });
}
