// pm_batch.hip -- a large batch of fixed-length patterns at k = 0 in ONE pass
// over the nucleotide planes (BASELINE configs[4]: 256 degenerate motifs).
//
// The reference answers a batch with one nrgrep_coords process per pattern
// (www/FlaskApp/FlaskApp/patmatch.py:733-743), i.e. one scan of the file per
// pattern.  The bit-sliced kernel (pm_linear_jit) answers <= 8 patterns per
// HBM pass at ~9 VALU ops per (pattern, 32 windows); for hundreds of patterns
// that is 30+ passes and VALU-bound.  Here the work per position does not
// grow with the batch: a q-gram filter.
//
//  * Index (host, build_batch_index): per pattern the 10-position piece
//    (offset o_p <= L - 10) with the fewest ACGT expansions; every expansion
//    is a 20-bit code (2 bits per base, A=00 C=01 G=10 T=11, base i at bits
//    2i..2i+1).  A 2^20-bit table (128 KB) marks the codes present; per code
//    a list of (pattern, o_p).
//  * k_batch_scan: one 1024-thread workgroup per CU holds the table in LDS.
//    A wave takes one tile at a time: each lane loads its 32 words of both
//    planes (coalesced rows) and transposes them in registers (two 32x32 bit
//    transposes of the interleaved lo/hi words), which yields, per stream,
//    the 2-bit codes of 32 consecutive positions as two 32-bit words; the
//    next 32 positions come from the next lane (ds_bpermute; lane 63 from
//    lane 0's next stream, the tile's last stream from the halo).  Each
//    position then costs one table probe: two v_alignbit for the code and
//    the LDS byte address, one ds_read_b32, a shift and an alignbit into the
//    candidate mask -- ~5 VALU + 1 LDS read per position, whatever the batch
//    size.  Candidates (~1 % of positions at configs[4]) leave as 16-byte
//    entries with the 32 bases around them.
//  * k_batch_verify: one block per output segment checks every candidate
//    against the patterns listed for its code (bit-parallel class test over
//    the 16-base window), drops windows that overlap an exception (lane
//    flags, like k_linear_expand) and writes (pattern, segment) hit lists.
//  * k_batch_fixup: keys that landed in the next segment, and the file's
//    first starts (their probe position lies before the first probe).
// Windows with an exception byte are the exception pass's (k_linear_others,
// class-id form), exactly as for the bit-sliced kernel.
#include <hip/hip_ext.h>

#include "pm_internal.h"

namespace pm {
namespace {

__device__ __forceinline__ uint32_t alignb(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbit(hi, lo, s);
}

// one level of the 32x32 bit transpose: swaps the (rows r, columns c + J)
// block with the (rows r + J, columns c) block, r and c with bit J clear
template <int J, uint32_t M>
__device__ __forceinline__ void tr_level(uint32_t (&a)[32]) {
#pragma unroll
    for (int r = 0; r < 32; ++r) {
        if (r & J) continue;
        const uint32_t t = ((a[r] >> J) ^ a[r + J]) & M;
        a[r + J] ^= t;
        a[r] ^= t << J;
    }
}

// a[r] bit c  ->  a[c] bit r
__device__ __forceinline__ void transpose32(uint32_t (&a)[32]) {
    tr_level<16, 0x0000FFFFu>(a);
    tr_level<8, 0x00FF00FFu>(a);
    tr_level<4, 0x0F0F0F0Fu>(a);
    tr_level<2, 0x33333333u>(a);
    tr_level<1, 0x55555555u>(a);
}

// bits 0..15 of x to the even bits
__device__ __forceinline__ uint32_t spread16(uint32_t x) {
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}

// Every position is probed.  (Probing every other position with two
// consecutive pieces per pattern measured: scan 3.0 -> 2.16 ms, but the two
// pieces' expansions raise the candidates and verify 2.08 -> 2.74 ms, 10.6
// vs 9.9 ms per configs[4] step; round 2.)
__global__ __launch_bounds__(BATCH_THREADS) void k_batch_scan(BatchScanArgs a) {
    __shared__ uint32_t s_tab[BQ_TABLE_WORDS];   // 128 KB: one workgroup per CU
    for (uint32_t i = threadIdx.x; i < BQ_TABLE_WORDS; i += BATCH_THREADS) s_tab[i] = a.table[i];
    if (blockIdx.x == 0 && threadIdx.x == 0) {   // read by the later kernels
        *a.zero_a = 0u;
        *a.zero_b = 0u;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * BATCH_WAVES + (threadIdx.x >> 6);
    if (wave >= a.nwaves) return;   // no barrier below
    const uint64_t t0 = (uint64_t)wave * a.tiles_per_wave;
    const uint64_t t1 = umin64(t0 + a.tiles_per_wave, a.ntiles);
    uint4* cseg = a.cand + (uint64_t)wave * a.ccap;
    uint32_t ccnt = 0;   // wave-uniform
    const uint32_t sh = 2u * a.omax;
    const uint32_t src = (uint32_t)((lane + 1) & 63) << 2;   // ds_bpermute byte address of the next lane
    for (uint64_t tile = t0; tile < t1; ++tile) {
        const uint2* tb = a.hl + tile * TILE_WORDS;
        // A: positions 0..15 of the lane's block, B: 16..31, as the words
        // (lo_0, hi_0, lo_1, hi_1, ...): after the transpose A[s] holds the
        // interleaved 2-bit codes of stream s (base i at bits 2i, 2i + 1)
        uint32_t A[32], B[32];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint2 v = tb[i * 64 + lane];
            A[2 * i] = v.y;
            A[2 * i + 1] = v.x;
            const uint2 u = tb[(16 + i) * 64 + lane];
            B[2 * i] = u.y;
            B[2 * i + 1] = u.x;
        }
        // lane 63 / stream 31 continues in the next tile's stream 0: bit 31
        // of halo words 2048..2079
        const uint2 hv = lane < 32 ? tb[STREAM + lane] : make_uint2(0u, 0u);
        const uint64_t bh = __builtin_amdgcn_ballot_w64((hv.x >> 31) & 1u);
        const uint64_t bl = __builtin_amdgcn_ballot_w64((hv.y >> 31) & 1u);
        transpose32(A);
        transpose32(B);
        const uint32_t h0 = (spread16((uint32_t)bh) << 1) | spread16((uint32_t)bl);
        const uint32_t h1 = (spread16((uint32_t)bh >> 16) << 1) | spread16((uint32_t)bl >> 16);
#pragma unroll
        for (int s = 0; s < 32; ++s) {
            const uint32_t c0 = A[s], c1 = B[s];
            // the next 32 positions of stream s: the next lane's block; lane
            // 63 continues in stream s + 1 of lane 0 (the tile's last stream
            // in the halo)
            const int sn = s < 31 ? s + 1 : s;
            const uint32_t p0 = lane == 0 ? A[sn] : c0;
            const uint32_t p1 = lane == 0 ? B[sn] : c1;
            uint32_t c2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)p0);
            uint32_t c3 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)p1);
            if (s == 31 && lane == 63) {
                c2 = h0;
                c3 = h1;
            }
            // probe positions o_max + i (i < 32): the bases from o_max on
            const uint32_t d[3] = {alignb(c1, c0, sh), alignb(c2, c1, sh), alignb(c3, c2, sh)};
            uint32_t acc = 0;
#pragma unroll
            for (int i = 0; i < 32; ++i) {
                const int b0 = 2 * i, b3 = 2 * i + 3;
                const uint32_t code = (b0 & 31) ? alignb(d[(b0 >> 5) + 1], d[b0 >> 5], b0 & 31) : d[b0 >> 5];
                // code bits 5..19 (the table word) at bits 2..16: its LDS byte address
                const uint32_t a3 = (b3 >> 5) < 2 ? alignb(d[(b3 >> 5) + 1], d[b3 >> 5], b3 & 31) : d[2] >> (b3 & 31);
                const uint32_t tw =
                    *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(s_tab) + (a3 & 0x1FFFCu));
                // bit (code & 31) of the word into bit 31, the earlier probes down by one
                acc = alignb(tw >> (code & 31u), acc, 1u);
            }
            // candidates: probe i -> 16-byte entry {tile, lane << 11 | s << 6
            // | i, the 32 bases from position i of the block}, written in
            // position order (stream, then lane, then i): each lane's at its
            // exclusive prefix of the wave's counts, so the verify's ordered
            // form reads every segment's candidates in increasing position.
            // The prefix is bit-sliced: per bit b of the counts a ballot and
            // mbcnt (VALU/SALU; a shuffle scan is 7 ds_bpermute per stream in
            // this LDS-bound kernel, measured 3.0 -> 3.48 ms; an LDS staging
            // of the entries 3.67 ms), a round or two at ~0.26 per lane
            uint32_t m = acc;
            if (__builtin_amdgcn_ballot_w64(m != 0u)) {   // wave-uniform
                const uint32_t cnt = (uint32_t)__builtin_popcount(m);
                uint32_t q = 0, tot = 0;
                for (uint32_t b = 0; __builtin_amdgcn_ballot_w64((cnt >> b) != 0u); ++b) {
                    const uint64_t bb = __builtin_amdgcn_ballot_w64((cnt >> b) & 1u);
                    q += __builtin_amdgcn_mbcnt_hi((uint32_t)(bb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bb, 0u)) << b;
                    tot += (uint32_t)__builtin_popcountll(bb) << b;
                }
                while (m) {
                    const uint32_t i = (uint32_t)__builtin_ctz(m);
                    m &= m - 1u;
                    const bool up = i >= 16u;
                    const uint32_t r = (2u * i) & 31u;
                    const uint32_t w0 = up ? c1 : c0, w1 = up ? c2 : c1, w2 = up ? c3 : c2;
                    const uint4 e = make_uint4((uint32_t)tile, ((uint32_t)lane << 11) | ((uint32_t)s << 6) | i,
                                               alignb(w1, w0, r), alignb(w2, w1, r));
                    if (ccnt + q < a.ccap) cseg[ccnt + q] = e;
                    ++q;
                }
                ccnt += tot;
            }
        }
    }
    if (lane == 0) a.cand_cnt[wave] = ccnt;
}

// Slot tables of the block's hit lists, staged in LDS.
struct VerifySlots {
    uint64_t* base;   // [P] this segment's list of pattern p: out + slot_base[p] + og * slot_cap[p]
    uint32_t* cap;    // [P]
    uint32_t* cnt;    // [P] keys so far
};

// One entry (h, mk) of a candidate: 0 no match, 1 a match of this segment
// (its key in `key`), 2 a match whose start lies in the next segment (its key
// already in xkeys).  lf: the lane flags of the candidate's tile (prefetched).
// tend: the segment's end tile (a start never lies before its candidate's
// segment, so tile < tend is this segment -- no 64-bit division)
__device__ __forceinline__ int verify_key(const BatchVerifyArgs& a, uint64_t tend, uint4 e, uint64_t lf, uint4 h,
                                          uint4 mk, uint64_t& key) {
    const uint32_t x0 = e.z, x1 = e.w;
    const uint32_t i = e.y & 63u, st0 = (e.y >> 6) & 31u, bl = e.y >> 11;
    const uint32_t p = h.x & 0xFFFFu, op = (h.x >> 16) & 255u;
    const int len = (int)(h.x >> 24);
    // the window's 16 bases; per position the class's bit for its base
    // (A/C by lo, G/T by lo, then by hi), at odd bits
    const uint32_t wc = alignb(x1, x0, 2u * (a.omax - op));
    const uint32_t lsh = wc << 1;
    const uint32_t s1 = (lsh & mk.y) | (~lsh & mk.x);
    const uint32_t s2 = (lsh & mk.w) | (~lsh & mk.z);
    const uint32_t res = (wc & s2) | (~wc & s1);
    if ((res & h.y) != h.y) return 0;
    uint64_t tile = e.x;
    uint32_t w = 32u * bl + a.omax + i - op, st = st0;
    if (w >= STREAM) {   // the start lies in the next stream (or tile)
        w -= (uint32_t)STREAM;
        if (++st == 32) {
            st = 0;
            ++tile;
            if (tile < a.ntiles) lf = a.lflag[tile];
        }
    }
    const uint64_t pos = pos_of(tile, w, st);
    if (tile >= a.ntiles || pos + (uint64_t)len > a.n) return 0;
    if ((lf >> (w >> 5)) & 1) {   // an exception near: windows over it are the others pass's
        // the window's break | other bits from the position-contiguous
        // planes: 1-2 words (round 6; a load per position before)
        const uint64_t q = pos >> 5;
        const uint4 v0 = a.lin[q], v1 = a.lin[q + 1];   // (lin has a word past every position)
        const uint64_t ex = ((uint64_t)(v1.z | v1.w) << 32 | (v0.z | v0.w)) >> (pos & 31);
        if (ex & ((1ull << len) - 1)) return 0;
    }
    key = ((uint64_t)p << 48) | pos;
    if (tile < tend) return 1;
    const uint32_t o = atomicAdd(a.xcnt, 1u);
    if (o < a.xcap) a.xkeys[o] = key;
    return 2;
}
// the unordered form: a match of this segment into its (pattern, segment)
// list by an LDS counter
__device__ __forceinline__ void verify_entry(const BatchVerifyArgs& a, uint64_t tend, const VerifySlots& vs, uint4 e,
                                             uint64_t lf, uint4 h, uint4 mk) {
    uint64_t key;
    if (verify_key(a, tend, e, lf, h, mk, key) == 1) {
        const uint32_t p = (uint32_t)(key >> 48);
        const uint32_t o = atomicAdd(&vs.cnt[p], 1u);
        if (o < vs.cap[p]) a.out[vs.base[p] + o] = key;
    }
}

// One block per output segment (wpo scan waves).  A thread takes VU
// candidates at a time, and every dependent load of them is issued for all
// VU together: the candidates, then their code -> entry offsets and tiles'
// lane flags, then their first entries (a candidate code lists ~1 entry;
// further ones are loaded as needed).  The slot tables are staged in LDS.
// (6 candidates per thread measured no faster: 8.46 vs 8.39 ms per
// configs[4] step, round 5)
constexpr int VU = 4;
// HASH: the codes' first entry and count from an LDS hash table (one global
// stage less per candidate than the 4 MB code_off array)
template <bool HASH>
__global__ __launch_bounds__(1024) void k_batch_verify(BatchVerifyArgs a) {
    __shared__ uint64_t s_hash[HASH ? BQ_HASH_SLOTS : 1];
    __shared__ uint32_t cnt_p[BATCH_MAX_P];
    __shared__ uint32_t cap_p[BATCH_MAX_P];
    __shared__ uint64_t base_p[BATCH_MAX_P];
    __shared__ uint32_t s_n[BATCH_MAX_WPO + 1];   // prefix of the waves' candidate counts
    const uint32_t og = blockIdx.x;
    for (int p = threadIdx.x; p < a.P; p += blockDim.x) {
        cnt_p[p] = 0;
        cap_p[p] = a.slot_cap[p];
        base_p[p] = a.slot_base[p] + (uint64_t)og * a.slot_cap[p];
    }
    if constexpr (HASH)
        for (uint32_t i = threadIdx.x; i < BQ_HASH_SLOTS; i += blockDim.x) s_hash[i] = a.hash[i];
    const uint32_t w0 = og * a.wpo, nw = min(a.nwaves, w0 + a.wpo) - w0;
    const uint64_t tend = (uint64_t)(w0 + a.wpo) * a.tiles_per_wave;
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (uint32_t k = 0; k < nw; ++k) {
            uint32_t c = a.cand_cnt[w0 + k];
            if (c > a.ccap) {
                atomicMax(a.aux, c);
                c = a.ccap;
            }
            s_n[k] = run;
            run += c;
        }
        s_n[nw] = run;
    }
    __syncthreads();
    const VerifySlots vs{base_p, cap_p, cnt_p};
    const uint32_t total = s_n[nw];
    // candidate q of the segment: wave k with s_n[k] <= q < s_n[k + 1]
    auto at = [&](uint32_t q) {
        uint32_t k = 0;
        while (q >= s_n[k + 1]) ++k;
        return a.cand + (uint64_t)(w0 + k) * a.ccap + (q - s_n[k]);
    };
    // candidate base + u * blockDim + thread: a wave's loads are 64
    // consecutive 16-byte entries
    for (uint32_t base = 0; base < total; base += blockDim.x * VU) {
        uint4 e[VU], h[VU], mk[VU];
        uint32_t co[VU];
        uint64_t lf[VU];
#pragma unroll
        for (int u = 0; u < VU; ++u) {
            const uint32_t q = base + u * blockDim.x + threadIdx.x;
            e[u] = q < total ? *at(q) : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int u = 0; u < VU; ++u) {
            const bool ok = base + u * blockDim.x + threadIdx.x < total;
            const uint32_t code = alignb(e[u].w, e[u].z, 2u * a.omax) & ((1u << (2 * BQ)) - 1u);
            co[u] = 0u;
            if constexpr (HASH) {
                if (ok)   // a candidate's code is present: the probe ends there (an empty slot: none)
                    for (uint32_t h = bq_hash(code);; h = (h + 1) & (BQ_HASH_SLOTS - 1)) {
                        const uint64_t sl = s_hash[h];
                        if (sl == ~0ull) break;
                        if ((uint32_t)(sl & 0xFFFFFu) == code) {
                            co[u] = bq_slot_entry(sl);
                            break;
                        }
                    }
            } else {
                co[u] = ok ? a.code_off[code] : 0u;
            }
            lf[u] = ok && e[u].x < a.ntiles ? a.lflag[e[u].x] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < VU; ++u) {
            const uint32_t lo = co[u] >> 8;
            if (co[u] & BQ_CO_ONE) {   // a one-entry code: the entry from the slot, the masks by pattern
                const uint32_t w0 = co[u] & ~BQ_CO_ONE;
                h[u] = make_uint4(w0, bq_len_mask(w0 >> 24), 0u, 0u);
                mk[u] = a.pmask[w0 & 0xFFFFu];
            } else {
                h[u] = co[u] ? a.ents[2 * lo] : make_uint4(0u, 0u, 0u, 0u);
                mk[u] = co[u] ? a.ents[2 * lo + 1] : make_uint4(0u, 0u, 0u, 0u);
            }
        }
#pragma unroll
        for (int u = 0; u < VU; ++u) {
            if (!co[u]) continue;
            verify_entry(a, tend, vs, e[u], lf[u], h[u], mk[u]);
            if (co[u] & BQ_CO_ONE) continue;   // its one entry came from the slot
            const uint32_t lo = co[u] >> 8, hi = lo + (co[u] & 255u);
            for (uint32_t t = lo + 1; t < hi; ++t) verify_entry(a, tend, vs, e[u], lf[u], a.ents[2 * t], a.ents[2 * t + 1]);
        }
    }
    __syncthreads();
    for (int p = threadIdx.x; p < a.P; p += blockDim.x) a.seg_cnt[(uint64_t)p * a.nout + og] = cnt_p[p];
}

// The ordered form (BatchVerifyArgs::ord set): a segment's matches leave in
// position order, so no sort by position follows, only a stable one by
// pattern (pm_hits.hip ordered_to_hits).  Wave wv of the segment's block
// takes the contiguous wv-th sixteenth of its candidates (the scan writes
// them in position order), VU * 64 per round; each candidate's matches go to
// the wave's own list at the lanes' exclusive prefix (no barrier).  A
// candidate with more than VH matches sets ord_bad (the host then runs the
// unordered form); matches of the next segment go to xkeys and those keys,
// like the exception pass's, to the (pattern, segment) bins.
constexpr int VH = 4;
// HIST: each wave also counts its list's keys per pattern (LDS), stored as
// ord_hist[p][list]: the host's stable scatter by pattern needs no
// histogram pass (patterns <= ORD_HIST_MAX_P).
template <bool HASH, bool HIST>
__global__ __launch_bounds__(1024) void k_batch_verify_ord(BatchVerifyArgs a) {
    __shared__ uint64_t s_hash[HASH ? BQ_HASH_SLOTS : 1];
    __shared__ uint32_t s_n[BATCH_MAX_WPO + 1];   // prefix of the waves' candidate counts
    __shared__ uint32_t s_hist[HIST ? BATCH_VERIFY_WAVES : 1][HIST ? ORD_HIST_MAX_P : 1];
    // HIST (<= ORD_HIST_MAX_P patterns): the patterns' class masks in LDS too,
    // so a one-entry code (the slot holds its entry) is verified with no
    // global load after the candidate's (round 6)
    __shared__ uint4 s_pmask[HASH && HIST ? ORD_HIST_MAX_P : 1];
    const uint32_t og = blockIdx.x;
    if constexpr (HIST)
        for (uint32_t i = threadIdx.x; i < BATCH_VERIFY_WAVES * ORD_HIST_MAX_P; i += blockDim.x) (&s_hist[0][0])[i] = 0u;
    if constexpr (HASH && HIST)
        for (uint32_t p = threadIdx.x; p < (uint32_t)a.P; p += blockDim.x) s_pmask[p] = a.pmask[p];
    if constexpr (HASH)
        for (uint32_t i = threadIdx.x; i < BQ_HASH_SLOTS; i += blockDim.x) s_hash[i] = a.hash[i];
    // (the bins of the exception pass, xkeys and first starts are zeroed by
    // the host: the exception pass may run concurrently)
    const uint32_t w0 = og * a.wpo, nw = min(a.nwaves, w0 + a.wpo) - w0;
    const uint64_t tend = (uint64_t)(w0 + a.wpo) * a.tiles_per_wave;
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (uint32_t k = 0; k < nw; ++k) {
            uint32_t c = a.cand_cnt[w0 + k];
            if (c > a.ccap) {
                atomicMax(a.aux, c);
                c = a.ccap;
            }
            s_n[k] = run;
            run += c;
        }
        s_n[nw] = run;
    }
    __syncthreads();
    const uint32_t total = s_n[nw];
    auto at = [&](uint32_t q) {
        uint32_t k = 0;
        while (q >= s_n[k + 1]) ++k;
        return a.cand + (uint64_t)(w0 + k) * a.ccap + (q - s_n[k]);
    };
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr uint32_t NWV = BATCH_VERIFY_WAVES;
    static_assert(NWV * 64 == 1024, "one verify block: 1024 threads");
    const uint32_t per = (total + NWV - 1) / NWV;
    const uint32_t q0 = min(total, wv * per), q1 = min(total, q0 + per);
    const uint64_t list = (uint64_t)og * NWV + wv;
    uint64_t* out = a.ord_out + list * a.ord_cap;
    uint32_t wcnt = 0;   // wave-uniform
    // the scan wave a lane's next candidate lies in (its candidates increase)
    uint32_t kk = 0;
    auto at_k = [&](uint32_t q) {
        while (q >= s_n[kk + 1]) ++kk;
        return a.cand + (uint64_t)(w0 + kk) * a.ccap + (q - s_n[kk]);
    };
    (void)at;
    // a round: candidate base + u * 64 + lane (coalesced loads); its matches
    // leave per u, in (u, lane) order = position order.  The next round's
    // candidates are loaded while this round's lookups run (verify 2.14 ->
    // 2.00 ms on configs[4]).
    uint4 ne[VU];
#pragma unroll
    for (int u = 0; u < VU; ++u) {
        const uint32_t q = q0 + u * 64 + lane;
        ne[u] = q < q1 ? *at_k(q) : make_uint4(0u, 0u, 0u, 0u);
    }
    for (uint32_t base = q0; base < q1; base += 64 * VU) {
        uint4 e[VU], h[VU], mk[VU];
        uint32_t co[VU];
        uint64_t lf[VU];
#pragma unroll
        for (int u = 0; u < VU; ++u) {
            e[u] = ne[u];
            const uint32_t q = base + 64 * VU + u * 64 + lane;
            ne[u] = q < q1 ? *at_k(q) : make_uint4(0u, 0u, 0u, 0u);
        }
        // the candidates' first hash slots read together (their tiles' lane
        // flags in flight meanwhile), then the rare further probes
        uint32_t hh[VU], code[VU];
        uint64_t sl[VU];
#pragma unroll
        for (int u = 0; u < VU; ++u) {
            const bool ok = base + u * 64 + lane < q1;
            code[u] = alignb(e[u].w, e[u].z, 2u * a.omax) & ((1u << (2 * BQ)) - 1u);
            co[u] = 0u;
            if constexpr (HASH) {
                hh[u] = bq_hash(code[u]);
                sl[u] = ok ? s_hash[hh[u]] : ~0ull;
            } else {
                co[u] = ok ? a.code_off[code[u]] : 0u;
            }
            lf[u] = ok && e[u].x < a.ntiles ? a.lflag[e[u].x] : 0ull;
        }
        if constexpr (HASH) {
#pragma unroll
            for (int u = 0; u < VU; ++u) {
                // a candidate's code is present: the probe ends there (an empty slot: none)
                while (sl[u] != ~0ull && (uint32_t)(sl[u] & 0xFFFFFu) != code[u]) {
                    hh[u] = (hh[u] + 1) & (BQ_HASH_SLOTS - 1);
                    sl[u] = s_hash[hh[u]];
                }
                if (sl[u] != ~0ull) co[u] = bq_slot_entry(sl[u]);
            }
        }
        // HASH && HIST: a one-entry code's entry is its slot's and its masks
        // are in LDS, so nothing is loaded ahead (and no h / mk registers are
        // held across the round); a code with more entries (rare) loads them
        // where it is verified.  Otherwise the entries load here, together.
        constexpr bool LATE = HASH && HIST;
        if constexpr (!LATE) {
#pragma unroll
            for (int u = 0; u < VU; ++u) {
                const uint32_t lo = co[u] >> 8;
                if (co[u] & BQ_CO_ONE) {   // a one-entry code: the entry from the slot, the masks by pattern
                    const uint32_t w0 = co[u] & ~BQ_CO_ONE;
                    h[u] = make_uint4(w0, bq_len_mask(w0 >> 24), 0u, 0u);
                    mk[u] = a.pmask[w0 & 0xFFFFu];
                } else {
                    h[u] = co[u] ? a.ents[2 * lo] : make_uint4(0u, 0u, 0u, 0u);
                    mk[u] = co[u] ? a.ents[2 * lo + 1] : make_uint4(0u, 0u, 0u, 0u);
                }
            }
        }
        // LATE: when every candidate of the round has one entry or none
        // (wave-uniform; a batch of distinct motifs almost always), each has
        // at most one match, and a single ballot places them -- no match
        // list, no bit-sliced prefix
        bool fast = false;
        if constexpr (LATE) {
            bool multi = false;
#pragma unroll
            for (int u = 0; u < VU; ++u) multi |= co[u] != 0u && !(co[u] & BQ_CO_ONE);
            fast = __builtin_amdgcn_ballot_w64(multi) == 0;
        }
        if (fast) {
#pragma unroll
            for (int u = 0; u < VU; ++u) {
                uint64_t key = 0;
                bool hit = false;
                if (co[u]) {
                    const uint32_t w0 = co[u] & ~BQ_CO_ONE;
                    hit = verify_key(a, tend, e[u], lf[u], make_uint4(w0, bq_len_mask(w0 >> 24), 0u, 0u),
                                     s_pmask[w0 & 0xFFFFu], key) == 1;
                }
                const uint64_t bb = __builtin_amdgcn_ballot_w64(hit);
                if (bb) {   // wave-uniform
                    const uint32_t at0 =
                        wcnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(bb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bb, 0u));
                    if (hit) {
                        if (at0 < a.ord_cap) out[at0] = key;
                        if constexpr (HIST) atomicAdd(&s_hist[wv][(uint32_t)(key >> 48)], 1u);
                    }
                    wcnt += (uint32_t)__builtin_popcountll(bb);
                }
            }
            continue;
        }
#pragma unroll
        for (int u = 0; u < VU; ++u) {
            uint64_t hk[VH];
            uint32_t nh = 0;
            bool bad = false;
            auto take = [&](uint4 h1, uint4 m1) {
                uint64_t key;
                if (verify_key(a, tend, e[u], lf[u], h1, m1, key) == 1) {
#pragma unroll
                    for (int t = 0; t < VH; ++t)
                        if (t == (int)nh) hk[t] = key;
                    if (nh < VH) ++nh;
                    else bad = true;
                }
            };
            if (co[u]) {
                const uint32_t lo = co[u] >> 8, hi = (co[u] & BQ_CO_ONE) ? 0u : lo + (co[u] & 255u);
                if constexpr (LATE) {
                    if (co[u] & BQ_CO_ONE) {
                        const uint32_t w0 = co[u] & ~BQ_CO_ONE;
                        take(make_uint4(w0, bq_len_mask(w0 >> 24), 0u, 0u), s_pmask[w0 & 0xFFFFu]);
                    } else {
                        take(a.ents[2 * lo], a.ents[2 * lo + 1]);
                    }
                } else {
                    take(h[u], mk[u]);
                }
                for (uint32_t t = lo + 1; t < hi; ++t) take(a.ents[2 * t], a.ents[2 * t + 1]);
            }
            if (bad) atomicOr(a.ord_bad, 1u);
            // the lanes' exclusive prefix of their match counts, bit-sliced
            // (ballot + mbcnt per bit, as in k_batch_scan)
            uint32_t at0 = wcnt, tot = 0;
            for (uint32_t b = 0; __builtin_amdgcn_ballot_w64((nh >> b) != 0u); ++b) {
                const uint64_t bb = __builtin_amdgcn_ballot_w64((nh >> b) & 1u);
                at0 += __builtin_amdgcn_mbcnt_hi((uint32_t)(bb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bb, 0u)) << b;
                tot += (uint32_t)__builtin_popcountll(bb) << b;
            }
#pragma unroll
            for (int t = 0; t < VH; ++t)
                if ((uint32_t)t < nh && at0 + t < a.ord_cap) out[at0 + t] = hk[t];
            if constexpr (HIST) {
#pragma unroll
                for (int t = 0; t < VH; ++t)
                    if ((uint32_t)t < nh) atomicAdd(&s_hist[wv][(uint32_t)(hk[t] >> 48)], 1u);
            }
            wcnt += tot;
        }
    }
    if (lane == 0) a.ord_cnt[list] = wcnt;
    if constexpr (HIST) {
        const uint64_t nl = (uint64_t)a.nout * NWV;
        for (uint32_t p = lane; p < (uint32_t)a.P; p += 64) a.ord_hist[p * nl + list] = s_hist[wv][p];
    }
}

__global__ __launch_bounds__(256) void k_batch_fixup(BatchVerifyArgs a) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
    // keys whose start fell into the next segment (the next tile's first positions)
    const uint32_t nx = min(*a.xcnt, a.xcap);
    const uint32_t ns = a.sink_segs ? a.sink_segs : a.nout;
    for (uint32_t q = tid; q < nx; q += nth) {
        const uint64_t key = a.xkeys[q];
        const uint32_t p = (uint32_t)(key >> 48);
        const uint64_t tile = (key & 0xFFFFFFFFFFFFull) / TILE_POS;
        const uint32_t ogr = ns == 1 ? 0u : (uint32_t)tile / a.tiles_per_wave / a.wpo;   // 32-bit division
        const uint32_t o = atomicAdd(&a.seg_cnt[(uint64_t)p * ns + ogr], 1u);
        if (o < a.slot_cap[p]) a.out[a.slot_base[p] + (uint64_t)ogr * a.slot_cap[p] + o] = key;
    }
    // the file's first starts st < o_max - o_p: probed by no block
    for (uint32_t q = tid; q < (uint32_t)a.P * a.omax; q += nth) {
        const uint32_t p = q / a.omax, st = q % a.omax;
        // the position this start is probed at; probes start at o_max
        const uint32_t y = st + a.popt[p];
        if (y >= a.omax) continue;
        const int len = a.lengths[p];
        if ((uint64_t)st + len > a.n) continue;
        const uint4 mk = a.pmask[p];
        bool ok = true;
        for (int j = 0; j < len && ok; ++j) {
            const Loc l = loc_of(st + j);
            const uint2 b = a.bo[l.word];
            if (((b.x | b.y) >> l.bit) & 1u) {
                ok = false;   // an exception: the others pass's window
                break;
            }
            const uint2 v = a.hl[l.word];
            const uint32_t base = (((v.x >> l.bit) & 1u) << 1) | ((v.y >> l.bit) & 1u);
            const uint32_t m = base == 0 ? mk.x : base == 1 ? mk.y : base == 2 ? mk.z : mk.w;
            ok = (m >> (2 * j + 1)) & 1u;
        }
        if (!ok) continue;
        const uint32_t o = atomicAdd(&a.seg_cnt[(uint64_t)p * ns], 1u);
        if (o < a.slot_cap[p]) a.out[a.slot_base[p] + o] = ((uint64_t)p << 48) | st;
    }
}

}  // namespace

bool build_batch_index(int P, const int32_t* lengths, const uint8_t* pos_class, const uint8_t* class_acgt,
                       const uint8_t* class_is_any, BatchIndex& bi) {
    bi = BatchIndex();
    if (P < 1 || P > BATCH_MAX_P) return false;
    for (int p = 0; p < P; ++p)
        if (lengths[p] < BQ || lengths[p] > BATCH_MAX_LEN) return false;
    struct Ent {
        uint32_t code, p, op;
    };
    const int npieces = 1;   // one indexed piece per pattern
    std::vector<Ent> ents;
    std::vector<uint32_t> plen(P, 0);
    bi.popt.assign(P, 0);
    bi.pmask.assign((size_t)4 * P, 0);
    for (int p = 0; p < P; ++p) {
        const int L = lengths[p];
        uint32_t sub[BATCH_MAX_LEN];
        for (int j = 0; j < L; ++j) {
            const int c = pos_class[64 * p + j];
            sub[j] = class_is_any[c] ? 15u : (class_acgt[c] & 15u);
            for (int b = 0; b < 4; ++b) bi.pmask[(size_t)4 * p + b] |= ((sub[j] >> b) & 1u) << (2 * j + 1);
            plen[p] |= 1u << (2 * j + 1);
        }
        // the piece with the fewest expansions (0: the pattern matches no
        // ACGT-only window, nothing to index)
        uint64_t best = ~0ull;
        int bo = 0;
        auto expansions = [&](int o) {
            uint64_t prod = 1;
            for (int i = 0; i < BQ; ++i) prod *= (uint64_t)__builtin_popcount(sub[o + i]);
            return prod;
        };
        for (int o = 0; o + BQ + npieces - 1 <= L; ++o) {
            uint64_t tot = 0;
            for (int q = 0; q < npieces; ++q) tot += expansions(o + q);
            if (tot < best) {
                best = tot;
                bo = o;
            }
        }
        bi.popt[p] = (uint32_t)bo;
        bi.omax = std::max(bi.omax, (uint32_t)(bo + npieces - 1));
        bi.expansions += best;
        if (bi.expansions > BATCH_MAX_EXPANSIONS) return false;
        for (int q = 0; q < npieces; ++q) {
            if (!expansions(bo + q)) continue;   // the pattern matches no ACGT-only window
            std::vector<uint32_t> codes(1, 0u);
            for (int i = 0; i < BQ; ++i) {
                std::vector<uint32_t> nx;
                nx.reserve(codes.size() * 4);
                for (uint32_t c : codes)
                    for (uint32_t b = 0; b < 4; ++b)
                        if ((sub[bo + q + i] >> b) & 1u) nx.push_back(c | (b << (2 * i)));
                codes.swap(nx);
            }
            for (uint32_t c : codes) ents.push_back({c, (uint32_t)p, (uint32_t)(bo + q)});
        }
    }
    std::sort(ents.begin(), ents.end(), [](const Ent& x, const Ent& y) {
        return x.code != y.code ? x.code < y.code : x.p != y.p ? x.p < y.p : x.op < y.op;
    });
    bi.table.assign(BQ_TABLE_WORDS, 0u);
    bi.code_off.assign((size_t)1 << (2 * BQ), 0u);
    bi.ents.assign(ents.size() * BATCH_ENT_WORDS, 0u);
    for (size_t i = 0; i < ents.size(); ++i) {
        const uint32_t c = ents[i].code, p = ents[i].p, op = ents[i].op;
        if (i == 0 || c != ents[i - 1].code) {
            bi.table[c >> 5] |= 1u << (c & 31);
            bi.code_off[c] = (uint32_t)i << 8;
        }
        if ((bi.code_off[c] & 255u) == 255u || i >= (1u << 23)) return false;
        ++bi.code_off[c];
        uint32_t* e = &bi.ents[i * BATCH_ENT_WORDS];
        e[0] = p | op << 16 | (uint32_t)lengths[p] << 24;
        e[1] = plen[p];
        for (int b = 0; b < 4; ++b) e[4 + b] = bi.pmask[(size_t)4 * p + b];   // the second uint4
    }
    // the verify's hash table of the codes present (LDS): first entry and
    // count per code, open addressing
    {
        std::vector<std::pair<uint32_t, uint32_t>> codes;   // (code, first entry)
        for (size_t i = 0; i < ents.size(); ++i)
            if (i == 0 || ents[i].code != ents[i - 1].code) codes.push_back({ents[i].code, (uint32_t)i});
        if (codes.size() <= BQ_HASH_MAX_CODES && ents.size() < (1u << 24)) {
            bi.hash.assign(BQ_HASH_SLOTS, ~0ull);
            for (const auto& cf : codes) {
                uint32_t h = bq_hash(cf.first);
                while (bi.hash[h] != ~0ull) h = (h + 1) & (BQ_HASH_SLOTS - 1);
                // a code with one entry carries the entry's first word in
                // the slot (the verify then needs no entry load: pattern,
                // offset and length from the slot, the class masks per
                // pattern), else its first entry's index
                const uint64_t cnt = bi.code_off[cf.first] & 255u;
                const uint64_t mid = cnt == 1 ? (uint64_t)bi.ents[(size_t)cf.second * BATCH_ENT_WORDS]
                                              : (uint64_t)cf.second;
                bi.hash[h] = (uint64_t)cf.first | mid << 20 | cnt << 52;
            }
        }
    }
    Carve cv;
    bi.o_table = cv.take(bi.table.size() * 4);
    bi.o_code = cv.take(bi.code_off.size() * 4);
    bi.o_ents = cv.take(std::max<size_t>(bi.ents.size(), BATCH_ENT_WORDS) * 4);
    bi.o_pmask = cv.take(bi.pmask.size() * 4);
    bi.o_popt = cv.take(bi.popt.size() * 4);
    bi.o_hash = cv.take(bi.hash.size() * 8);
    bi.bytes = cv.off;
    return true;
}

void batch_launch(const BatchScanArgs& sa, const BatchVerifyArgs& va, uint32_t nblocks, hipStream_t s,
                  hipEvent_t ev_a, hipEvent_t ev_b) {
    // the kernel's own dispatch timestamps (no marker packets)
    hipExtLaunchKernelGGL(k_batch_scan, dim3(nblocks), dim3(BATCH_THREADS), 0, s, ev_a, ev_b, 0u, sa);
    HIPCHK(hipGetLastError());
    // PM_BATCH_HASH=0: the code_off array (A/B)
    static const bool hash_on = !(getenv("PM_BATCH_HASH") && getenv("PM_BATCH_HASH")[0] == '0');
    const bool hash = va.hash && hash_on;
    if (va.ord_out) {
        const bool hist = va.ord_hist != nullptr;
        auto kern = hash ? (hist ? k_batch_verify_ord<true, true> : k_batch_verify_ord<true, false>)
                         : (hist ? k_batch_verify_ord<false, true> : k_batch_verify_ord<false, false>);
        hipLaunchKernelGGL(kern, dim3(va.nout), dim3(1024), 0, s, va);
    } else
        hipLaunchKernelGGL(hash ? k_batch_verify<true> : k_batch_verify<false>, dim3(va.nout), dim3(1024), 0, s, va);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_batch_fixup, dim3(64), dim3(256), 0, s, va);
    HIPCHK(hipGetLastError());
}

}  // namespace pm
