// pm_linear.hip -- fixed-length patterns on the nucleotide planes, <= k
// substitutions (pm_scan_linear).
//
// The common PatMatch DNA query: a class sequence (IUPAC codes, '.' for N)
// from patmatch_to_nrgrep.pl, forward and reverse-complement strand
// (www/FlaskApp/FlaskApp/patmatch.py:270-314 builds both, :733-743 runs
// nrgrep_coords once per strand).  Both strands -- and up to four patterns
// -- are answered in ONE pass over the HBM-resident planes.
//
// Bit-slicing over window starts: thanks to the stream-tile layout
// (pm_internal.h) bit b of logical word w is the window starting at stream
// position w of stream b, and its j-th base is bit b of word w + j.  For a
// class c the mismatch word X_c(w) is one v_bitop3 of the (hi, lo) pair, and
// a window's mismatch count is a bit-sliced adder over X_{c_j}(w + j) --
// no shifts.  Two kernels:
//  * pm_linear_jit: the batch is compiled into the kernel with hipRTC (class
//    words kept in a register ring, the count a carry-save Wallace tree that
//    only resolves "count > k"), used for large databases;
//  * k_linear_generic: pattern tables read at run time, one word load per
//    (position, window word); for small databases (no compile latency).
// Windows touching an exception (break, N, other letter) are handled
// exactly: breaks kill, other bytes are tested against the class's 256-bit
// byte table.  The specialized kernel runs the exception-blind fast path on
// every tile, drops the (rare) emitted windows that overlap an exception, and
// k_linear_others evaluates exactly the windows whose first exception is an
// "other" byte (windows with a break are dead).
#include <hip/hiprtc.h>

#include <deque>
#include <memory>
#include <set>
#include <map>
#include <tuple>
#include <mutex>
#include <sstream>

#include <hip/hip_ext.h>

#include "pm_internal.h"

namespace pm {
namespace {

// ---------------------------------------------------------------------------
// generic kernel
// ---------------------------------------------------------------------------
struct LinearArgs {
    NucView nuc;
    const uint64_t* lflag;
    uint64_t ntiles, n;
    const uint8_t* pos_class;     // [P][64] class of each pattern position (chunk)
    const int32_t* lengths;       // [P]
    const uint8_t* class_acgt;    // [nc] subset of {A,C,G,T}
    const uint8_t* class_any;     // [nc] '.'
    const uint32_t* class_bytes;  // [nc][8] membership over folded bytes
    int k;
    int pattern_base;
    int cross;                    // k = 0 simple engine: windows may span breaks (k_linear_others)
    Sink sink;
};

constexpr int GEN_SPLIT = 4;   // waves per tile in the generic kernel (8 words each)

// mismatch word of ACGT subset s against planes (h, l): A=00 C=01 G=10 T=11
__device__ inline uint32_t subset_mismatch(uint32_t s, uint32_t h, uint32_t l) {
    const uint32_t sA = (s & 1) ? ~0u : 0u, sC = (s & 2) ? ~0u : 0u;
    const uint32_t sG = (s & 4) ? ~0u : 0u, sT = (s & 8) ? ~0u : 0u;
    const uint32_t m_hi = (l & sT) | (~l & sG);
    const uint32_t m_lo = (l & sC) | (~l & sA);
    return ~((h & m_hi) | (~h & m_lo));
}

template <int P>
__global__ __launch_bounds__(256) void k_linear_generic(LinearArgs a) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = (gridDim.x * (uint64_t)blockDim.x) >> 6;
    for (uint64_t item = wave; item < a.ntiles * GEN_SPLIT; item += nwaves) {
        const uint64_t tile = item / GEN_SPLIT;
        const int part = (int)(item % GEN_SPLIT);
        const bool flagged = (a.lflag[tile] >> lane) & 1;
        for (int t = part * (LANE_WORDS / GEN_SPLIT); t < (part + 1) * (LANE_WORDS / GEN_SPLIT); ++t) {
            const uint32_t w0 = (uint32_t)lane * LANE_WORDS + t;
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const int len = a.lengths[p];
                uint32_t c0 = 0, c1 = 0, d = 0, kill = 0;
                for (int j = 0; j < len; ++j) {
                    const uint64_t pw = phys_word(tile, w0 + j);
                    const int cls = a.pos_class[p * 64 + j];
                    uint2 e = make_uint2(0u, 0u);
                    if (flagged) {
                        e = a.nuc.bo[pw];
                        if (!a.cross) kill |= e.x;   // line-bounded: a break kills (see k_linear_others)
                    }
                    if (a.class_any[cls]) continue;
                    const uint2 v = a.nuc.hl[pw];
                    uint32_t x = subset_mismatch(a.class_acgt[cls], v.x, v.y);
                    const uint32_t exc = e.y | (a.cross ? e.x : 0u);
                    if (exc) {
                        const uint32_t idx = exception_index(a.nuc.sbflag, a.nuc.sbbase, pw);
                        uint32_t o = exc;
                        while (o) {
                            const int b = __builtin_ctz(o);
                            o &= o - 1;
                            const uint8_t ch = a.nuc.xbytes[(uint64_t)idx * 32 + b];
                            const bool member = (a.class_bytes[cls * 8 + (ch >> 5)] >> (ch & 31)) & 1;
                            x = member ? (x & ~(1u << b)) : (x | (1u << b));
                        }
                    }
                    const uint32_t cy0 = c0 & x;
                    c0 ^= x;
                    const uint32_t cy1 = c1 & cy0;
                    c1 ^= cy0;
                    d |= cy1;
                }
                uint32_t dead;
                switch (a.k) {
                    case 0: dead = c0 | c1 | d; break;
                    case 1: dead = c1 | d; break;
                    case 2: dead = (c1 & c0) | d; break;
                    default: dead = d; break;
                }
                uint32_t live = ~dead & ~kill;
                while (live) {
                    const uint32_t b = __builtin_ctz(live);
                    live &= live - 1;
                    const uint64_t pos = pos_of(tile, w0, b);
                    if (pos + (uint64_t)len <= a.n) {
                        const uint32_t slot = (uint32_t)(a.pattern_base + p);
                        a.sink.push(a.sink.bin_of(slot, pos), ((uint64_t)slot << 48) | pos);
                    }
                }
            }
        }
    }
}

void launch_generic(int P, const LinearArgs& a, hipStream_t s) {
    const uint64_t items = a.ntiles * GEN_SPLIT;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((items + 3) / 4, 256 * 32);
    switch (P) {
        case 1: hipLaunchKernelGGL(k_linear_generic<1>, dim3(blocks), dim3(256), 0, s, a); break;
        case 2: hipLaunchKernelGGL(k_linear_generic<2>, dim3(blocks), dim3(256), 0, s, a); break;
        case 4: hipLaunchKernelGGL(k_linear_generic<4>, dim3(blocks), dim3(256), 0, s, a); break;
        default: hipLaunchKernelGGL(k_linear_generic<8>, dim3(blocks), dim3(256), 0, s, a); break;
    }
}

// Windows of a specialized scan that overlap an exception, evaluated exactly.
// One wave per flagged word; a window is owned by the first position it
// contains that this pass evaluates, so each is evaluated once.  The fast
// path drops every window that overlaps any exception.
//  * line-bounded (k > 0: nrgrep's esimple verifies inside the record found
//    by recGetRecord, 0x41522d; or no class accepts '\n'): windows with a
//    break are dead, the pass owns windows by their first "other" byte;
//  * cross (k = 0 and some class accepts '\n'): nrgrep's simple engine
//    checks a window against the region, not the record (simplePreproc sets
//    the flag at 0x417f73, checkMatch 0x4167c7 then skips recGetRecord), so a
//    match may span '\n' and header bytes; every exception byte is compared
//    with its raw value and windows past the end of the file are dead.
struct OtherSel {
    uint64_t word;   // physical word
    uint32_t bits;   // its exception bits that can own a live window
    uint32_t pad;
};

struct OthersArgs {
    NucView nuc;
    const uint32_t* xoth;
    const uint32_t* xbrk;
    const uint64_t* xword;
    uint64_t nflag, n;
    const uint8_t* pos_class;
    const int32_t* lengths;
    const uint8_t* class_any;
    const uint32_t* class_bytes;
    int P, k, pattern_base, cross;
    int skip_ok;         // every pattern has k+1 positions whose class accepts only A/C/G/T
    const uint8_t* jsel; // [P][4]: the first k+1 such positions of each pattern
    int maxlen;          // longest pattern of the chunk
    int use_edge;        // skip_ok and every jsel <= RUN_SKIP: iterate the edge words only
    const uint32_t* xint;
    const uint32_t* xedge;   // the edge words (cross: any exception; else: "other" bytes)
    uint64_t nedge;
    OtherSel* sel;       // k_others_select -> k_linear_others
    uint32_t* nsel;
    uint64_t* out;       // the specialized kernel's (pattern, segment) hit lists
    uint32_t* seg_cnt;
    const uint64_t* slot_base;
    const uint32_t* slot_cap;
    uint32_t nwg, tiles_per_wg;
    int items_per_wave;  // k_linear_others: 1, 2 or 4 (2 * maxlen - 1 <= 64 / items_per_wave)
    int n_classes;       // k_linear_others<true>: classes staged in LDS (<= 256)
    uint64_t jall;       // skip_ok: bit j = some pattern's jsel entry is j (j >= 1)
};

// Phase 1, one thread per candidate word: the exception bits that can own a
// live window, compacted into `sel`.
// The exception bits of candidate word t that can own a live window (0:
// none), and the word's physical index.
__device__ inline uint32_t select_bits(const OthersArgs& a, uint64_t t, uint64_t* word) {
    const uint64_t idx = a.use_edge ? a.xedge[t] : t;   // run interiors removed at build (k_run_interior)
    uint32_t ot = a.xoth[idx] | (a.cross ? a.xbrk[idx] : 0u);
    if (a.use_edge) ot &= ~a.xint[idx];
    if (!ot) return 0u;
    const uint64_t w = a.xword[idx];
    *word = w;
    const uint64_t tile = w / TILE_WORDS;
    const uint32_t lw = logical_word((uint32_t)(w % TILE_WORDS));
    if (lw >= STREAM) return 0u;   // halo copy of a main word
    if (lw >= 1 && a.skip_ok) {
        // exceptions right before each bit's position (bit b of word lw - 1
        // is position e - 1)
        const uint2 pv = a.nuc.bo[phys_word(tile, lw - 1)];
        const uint32_t prev = pv.x | pv.y;
        // Runs of N, all 32 streams at once: a position e whose predecessor
        // is an exception owns only the window starting at e; that window is
        // dead when, for every pattern, the bytes at e + j are "other" for
        // the first k+1 positions j whose class accepts only A/C/G/T (jsel:
        // k+1 mismatches).  Bit b of logical word lw + j is position e + j.
        // The build-time index (xint/xedge) drops the run interiors for
        // any jsel <= RUN_SKIP; this query's jsel also drops most of the
        // RUN_SKIP edge words at a run's end.
        // Dead for every pattern of the chunk: the AND over the patterns p
        // of (m0 & the "other" words at p's jsel positions) is m0 & the AND
        // of those words over the DISTINCT positions of all patterns (`jall`,
        // a few for any batch): one load per distinct position instead of
        // one per (pattern, jsel) entry -- 256 patterns at configs[4] made
        // this pass 2.0 ms beside the scan (round 6)
        const uint32_t m0 = prev & a.xoth[idx];
        if (m0) {
            uint32_t m = m0;
            for (uint64_t jm = a.jall; jm; jm &= jm - 1)
                m &= a.nuc.bo[phys_word(tile, lw + (uint32_t)__builtin_ctzll(jm))].y;
            ot &= ~m;
        }
    }
    return ot;
}

constexpr uint32_t OTH_SELECT_T = 1024;
__global__ __launch_bounds__(OTH_SELECT_T) void k_others_select(OthersArgs a) {
    __shared__ uint32_t s_wc[OTH_SELECT_T / 64];
    __shared__ uint32_t s_base;
    const uint64_t t = blockIdx.x * (uint64_t)OTH_SELECT_T + threadIdx.x;
    uint64_t w = 0;
    const uint32_t ot = t < (a.use_edge ? a.nedge : a.nflag) ? select_bits(a, t, &w) : 0u;
    // one atomic per block on the list length (a single counter: the
    // atomics of many waves serialize on it)
    const uint64_t m = __builtin_amdgcn_ballot_w64(ot != 0u);
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) s_wc[wv] = (uint32_t)__builtin_popcountll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (uint32_t q = 0; q < OTH_SELECT_T / 64; ++q) {
            const uint32_t c = s_wc[q];
            s_wc[q] = run;
            run += c;
        }
        s_base = run ? atomicAdd(a.nsel, run) : 0u;
    }
    __syncthreads();
    if (ot)
        a.sel[s_base + s_wc[wv] + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
            OtherSel{w, ot, 0u};
}

constexpr int OTH_MAX_POS = 8 * 64;   // (pattern, position) entries of a chunk (JIT_MAX_P x 64)
constexpr uint32_t OTH_BLOCKS = 2048;   // phase 2: persistent blocks (8 per CU)

// The windows owned by the exception bits `ot` of logical word lw of a tile
// (one wave; a window is owned by the first exception it holds).
// class membership of byte ch at (pattern p, position j), entry p * maxlen + j:
// a table per entry (batches of <= 8 patterns) or a class id per entry and a
// table per class (large batches, k_linear_others<true>)
struct MembDirect {
    const uint32_t (*t)[8];
    __device__ bool operator()(int e, uint8_t ch) const { return (t[e][ch >> 5] >> (ch & 31)) & 1; }
};
struct MembClass {
    const uint8_t* cls;
    const uint32_t (*cm)[8];
    __device__ bool operator()(int e, uint8_t ch) const { return (cm[cls[e]][ch >> 5] >> (ch & 31)) & 1; }
};

template <class Memb>
__device__ inline void other_windows(const OthersArgs& a, const Memb& memb, uint64_t tile, uint32_t lw,
                                     uint32_t ot, int lane, int lanes, int slice) {
    // per exception bit e: the bytes of every window holding e --
    // positions e - maxlen + 1 .. e + maxlen - 1 -- are gathered once, one
    // position per lane (a few independent loads instead of one dependent
    // chain per window), into this wave's LDS slice; the lanes then test
    // (pattern, start offset) windows from LDS
    __shared__ uint8_t s_ch[4][128];
    __shared__ uint8_t s_fl[4][128];   // bit 0: break or other, bit 1: break
    uint8_t* const wch = &s_ch[threadIdx.x >> 6][slice * lanes];   // this item's part of the wave's slice
    uint8_t* const wfl = &s_fl[threadIdx.x >> 6][slice * lanes];
    const int span = 2 * a.maxlen - 1;
    const int per_bit = a.P * a.maxlen;
    uint32_t rest = ot;
    while (rest) {
        const uint32_t b = __builtin_ctz(rest);
        rest &= rest - 1;
        const uint64_t e = pos_of(tile, lw, b);
        if (e >= a.n) continue;
        const int64_t q0 = (int64_t)e - (a.maxlen - 1);
        wave_lds_sync();   // the previous bit's reads are done
        for (int i = lane; i < span; i += lanes) {
            const int64_t q = q0 + i;
            uint8_t c = 0, f = 0;
            if (q >= 0 && (uint64_t)q < a.n) {
                // the span is 1-2 words of the position-contiguous planes
                // (the lanes share their lines); an exception's byte comes
                // from the side tables
                const uint4 v = a.nuc.lin[(uint64_t)q >> 5];
                const uint32_t i5 = (uint32_t)q & 31;
                const uint32_t brk = (v.z >> i5) & 1, oth = (v.w >> i5) & 1;
                f = (uint8_t)((brk | oth) | (brk << 1));
                if (brk | oth) {
                    const Loc l = loc_of((uint64_t)q);
                    c = a.nuc.xbytes[(uint64_t)exception_index(a.nuc.sbflag, a.nuc.sbbase, l.word) * 32 + l.bit];
                } else {
                    c = (uint8_t)((0x54474341u >> (8 * ((((v.x >> i5) & 1) << 1) | ((v.y >> i5) & 1)))) & 0xff);
                }
            }
            wch[i] = c;
            wfl[i] = f;
        }
        wave_lds_sync();
        // a window that also holds position e - 1 is owned by an earlier
        // exception (or killed by a break) when e - 1 is one
        const bool prev_exc = a.maxlen >= 2 && (wfl[a.maxlen - 2] & 1);
        for (int c = lane; c < per_bit; c += lanes) {
            const int p = c / a.maxlen, d = c % a.maxlen;
            const int len = a.lengths[p];
            if (d >= len || (uint64_t)d > e || (prev_exc && d > 0)) continue;
            const uint64_t s = e - d;
            if (s + len > a.n) continue;
            const int i0 = a.maxlen - 1 - d;   // LDS index of position s
            int mm = 0;
            bool ok = true;
            for (int j = 0; j < len; ++j) {
                const uint8_t f = wfl[i0 + j];
                if ((f & 2) && !a.cross) { ok = false; break; }
                if ((f & 1) && j < d) { ok = false; break; }   // owned by an earlier exception
                const uint8_t ch = wch[i0 + j];
                if (!memb(p * a.maxlen + j, ch) && ++mm > a.k) { ok = false; break; }
            }
            if (ok) {
                const uint32_t slot = (uint32_t)(a.pattern_base + p);
                const uint64_t og = (uint32_t)(s / TILE_POS) / (uint32_t)a.tiles_per_wg;   // 32-bit division
                const uint32_t o = atomicAdd(&a.seg_cnt[(uint64_t)slot * a.nwg + og], 1u);
                if (o < a.slot_cap[slot]) a.out[a.slot_base[slot] + og * a.slot_cap[slot] + o] = ((uint64_t)slot << 48) | s;
            }
        }
    }
}

constexpr int JIT_MAX_P_ = 8;         // = JIT_MAX_P (declared further down)
constexpr int OTH_CLS_MAX_POS = BATCH_MAX_P * BATCH_MAX_LEN;   // (pattern, position) entries of a q-gram batch

// bit vectors over a window span: the mismatch of an ACGT subset, and a
// bit-sliced add into a count (c0, c1; ge4 = count >= 4)
__device__ inline uint64_t vec_mismatch(uint64_t H, uint64_t L, uint32_t sub) {
    const uint64_t sA = (sub & 1) ? ~0ull : 0ull, sC = (sub & 2) ? ~0ull : 0ull;
    const uint64_t sG = (sub & 4) ? ~0ull : 0ull, sT = (sub & 8) ? ~0ull : 0ull;
    const uint64_t match = (~H & ((~L & sA) | (L & sC))) | (H & ((~L & sG) | (L & sT)));
    return ~match;
}

__device__ inline void vec_add(uint64_t x, uint64_t& c0, uint64_t& c1, uint64_t& ge4) {
    const uint64_t cy0 = c0 & x;
    c0 ^= x;
    const uint64_t cy1 = c1 & cy0;
    c1 ^= cy0;
    ge4 |= cy1;
}
// The lane form of the exception pass (line-bounded scans whose classes are
// all A/C/G/T-only or '.'): one LANE per entry of the database's
// "other"-position list (pm_db::xlist, built at load time), so no selection
// pass and no byte gathers.  An "other" byte then mismatches every A/C/G/T
// class and matches '.', and a break kills, so the planes decide every
// window: the lane loads the position-contiguous planes (pm_db::lin) of the
// 2 maxlen - 1 positions around e as 64-bit vectors (three 16-byte loads)
// and tests the windows owned by e (no exception between their start and e)
// bit-parallel over their starts, the count bit-sliced.  A run tail whose
// window at e starts with `jdead` exception bytes (k + 1 mismatches for
// every pattern) is skipped from the list entry alone.
struct LaneArgs {
    const uint64_t* list;
    uint64_t nlist;
    const uint4* lin;
    uint64_t nlin, n;
    const uint8_t* csub;      // chunk: [P][64] A/C/G/T subset of each position's class, | 16 for '.'
    const int32_t* lengths;   // chunk
    int P, k, pattern_base, maxlen, jdead;
    uint64_t* out;
    uint32_t* seg_cnt;
    const uint64_t* slot_base;
    const uint32_t* slot_cap;
    uint32_t nout, tiles_per_out;
};

__device__ inline uint4 lin_word(const LaneArgs& a, int64_t w) {
    return (w < 0 || (uint64_t)w >= a.nlin) ? make_uint4(0u, 0u, ~0u, 0u) : a.lin[w];   // outside: breaks
}
__device__ inline uint64_t span64(uint32_t v0, uint32_t v1, uint32_t v2, uint32_t off) {
    const uint64_t lo = ((uint64_t)v1 << 32) | v0;
    return off ? (lo >> off) | ((uint64_t)v2 << (64 - off)) : lo;
}

__global__ __launch_bounds__(256) void k_others_lane(LaneArgs a) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < a.nlist; t += stride) {
        const uint64_t it = a.list[t];
        const uint64_t e = it & XL_POS_MASK;
        const int ahead = (int)((it >> XL_AHEAD_SHIFT) & 255), prev = (int)((it >> XL_PREV_SHIFT) & 1);
        // e - 1 an exception: e owns only the window starting at e
        if ((prev && ahead >= a.jdead) || e >= a.n) continue;
        const int c = a.maxlen - 1;                 // span index of e
        const int64_t q0 = (int64_t)e - c;          // span: positions q0 .. q0 + 63
        const int64_t w0 = q0 >> 5;                 // (floor)
        const uint32_t off = (uint32_t)(q0 & 31);
        const uint4 v0 = lin_word(a, w0), v1 = lin_word(a, w0 + 1), v2 = lin_word(a, w0 + 2);
        const uint64_t H = span64(v0.x, v1.x, v2.x, off), L = span64(v0.y, v1.y, v2.y, off);
        const uint64_t B = span64(v0.z, v1.z, v2.z, off), O = span64(v0.w, v1.w, v2.w, off);
        // windows starting after the last exception before e (those before
        // are owned by it, or killed)
        const uint64_t Eb = (B | O) & ((1ull << c) - 1);
        const int own = Eb ? 64 - __builtin_clzll(Eb) : 0;
        for (int p = 0; p < a.P; ++p) {
            const int len = a.lengths[p];
            const int ulo = own > c - len + 1 ? own : c - len + 1;
            if (ulo > c) continue;
            const uint8_t* cs = a.csub + p * 64;
            uint64_t c0 = 0, c1 = 0, ge4 = 0, kill = 0;
            for (int j = 0; j < len; ++j) {
                kill |= B >> j;
                const uint32_t sub = cs[j];
                if (sub & 16) continue;   // '.': every byte
                vec_add((vec_mismatch(H, L, sub) | O) >> j, c0, c1, ge4);
            }
            uint64_t dead = ge4 | kill;
            switch (a.k) {
                case 0: dead |= c0 | c1; break;
                case 1: dead |= c1; break;
                case 2: dead |= c1 & c0; break;
                default: break;
            }
            uint64_t live = ~dead & (((2ull << c) - 1) & ~((1ull << ulo) - 1));
            for (; live; live &= live - 1) {
                const uint64_t s = (uint64_t)(q0 + __builtin_ctzll(live));
                const uint32_t slot = (uint32_t)(a.pattern_base + p);
                const uint64_t og = (uint32_t)(s / TILE_POS) / (uint32_t)a.tiles_per_out;   // 32-bit division
                const uint32_t o = atomicAdd(&a.seg_cnt[(uint64_t)slot * a.nout + og], 1u);
                if (o < a.slot_cap[slot]) a.out[a.slot_base[slot] + og * a.slot_cap[slot] + o] = ((uint64_t)slot << 48) | s;
            }
        }
    }
}

// Phase 2 for large batches (k_batch_scan's exception windows), one WAVE per
// exception bit e, with the work split per CLASS: a batch of hundreds of
// IUPAC motifs uses a handful of classes (A, C, G, T, the two-base codes,
// '.').  Lane i gathers position e - maxlen + 1 + i (one round trip for the
// whole window span); ballots turn the lanes' bits into 64-bit span vectors
// (planes, breaks, "other" bytes, off-file); the match vector of every class
// over the span (bit i = position i accepted: ACGT from the planes, N from
// its mark, other bytes by value) is one ballot per class, kept in LDS.
// Then lane l takes patterns l, l + 64, ...: one LDS read, a 64-bit shift and
// two ANDs per position give the windows of every start u holding e, alive
// iff every position accepts its byte (k > 0: mismatches counted
// bit-sliced).  A window is evaluated by the first exception it holds,
// breaks kill it unless the simple engine runs (cross), and windows off the
// file are dead -- the same verdicts as the wave form below.
constexpr int OTH_BATCH_THREADS = 256;
constexpr int OTH_BATCH_MAX_CLASSES = 32;

// TWO (spans of <= 32 positions: every q-gram batch, patterns <= 16): the
// wave takes two selected words at a time, one per 32-lane half -- lane
// 32 h + i gathers position i of half h's span, the ballots carry both
// spans side by side (half h at bits 32 h ..), and the class vectors and
// the per-pattern window tests run on both at once: a window of half 0
// reads bits < 31 and one of half 1 bits 32 .. 62, so the shifts that carry
// bits across the halves only reach bits no window start of the other half
// uses.  Half as many serial (gather, ballots, tests) rounds per exception
// (round 6).
template <bool TWO>
__global__ __launch_bounds__(OTH_BATCH_THREADS) void k_others_batch(OthersArgs a) {
    __shared__ uint4 s_cls[BATCH_MAX_P];                          // 16 class ids per pattern
    __shared__ uint32_t s_cm[OTH_BATCH_MAX_CLASSES][8];           // byte membership per class
    __shared__ uint8_t s_csub[OTH_BATCH_MAX_CLASSES];             // A/C/G/T subset + 16: accepts N
    __shared__ uint64_t s_mv[OTH_BATCH_THREADS / 64][OTH_BATCH_MAX_CLASSES];   // per wave: match vector per class
    const int nc = a.n_classes;
    for (int i = threadIdx.x; i < nc * 8; i += blockDim.x) {
        const int c = i >> 3;
        s_cm[c][i & 7] = a.class_any[c] ? ~0u : a.class_bytes[c * 8 + (i & 7)];
    }
    uint8_t* cls8 = reinterpret_cast<uint8_t*>(s_cls);
    for (int e = threadIdx.x; e < a.P * 16; e += blockDim.x) {
        const int p = e >> 4, j = e & 15;
        cls8[e] = j < a.lengths[p] ? a.pos_class[p * 64 + j] : 0;
    }
    __syncthreads();
    for (int c = threadIdx.x; c < nc; c += blockDim.x) {
        uint32_t sub = 0;
        const char* acgt = "ACGT";
        for (int x = 0; x < 4; ++x) {
            const uint8_t ch = (uint8_t)acgt[x];
            if ((s_cm[c][ch >> 5] >> (ch & 31)) & 1) sub |= 1u << x;
        }
        if ((s_cm[c]['N' >> 5] >> ('N' & 31)) & 1) sub |= 16;
        s_csub[c] = (uint8_t)sub;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int half = TWO ? lane >> 5 : 0, hl = TWO ? lane & 31 : lane;   // this lane's half, its lane in it
    uint64_t* const mv = s_mv[wid];
    const int ML = a.maxlen, span = 2 * ML - 1;
    const uint32_t nsel = *a.nsel;
    constexpr uint32_t WPI = TWO ? 2 : 1;   // selected words per wave round
    for (uint32_t it = (blockIdx.x * (OTH_BATCH_THREADS / 64) + wid) * WPI; it < nsel;
         it += gridDim.x * (OTH_BATCH_THREADS / 64) * WPI) {
        OtherSel sv[2];
        uint32_t bits[2], lw[2];
        uint64_t tile[2];
#pragma unroll
        for (uint32_t h = 0; h < WPI; ++h) {
            sv[h] = it + h < nsel ? a.sel[it + h] : OtherSel{0, 0u, 0u};
            bits[h] = sv[h].bits;
            tile[h] = sv[h].word / TILE_WORDS;
            lw[h] = logical_word((uint32_t)(sv[h].word % TILE_WORDS));
        }
        while (bits[0] | (TWO ? bits[1] : 0u)) {   // wave-uniform
            // each half's next exception bit (a half without one idles: e = n)
            uint64_t eh[2] = {a.n, a.n};
#pragma unroll
            for (uint32_t h = 0; h < WPI; ++h)
                if (bits[h]) {
                    eh[h] = pos_of(tile[h], lw[h], __builtin_ctz(bits[h]));
                    bits[h] &= bits[h] - 1;
                }
            const bool live0 = eh[0] < a.n, live1 = TWO && eh[1] < a.n;
            if (!live0 && !live1) continue;   // wave-uniform
            const uint64_t e = TWO && half ? eh[1] : eh[0];
            const bool live = TWO && half ? live1 : live0;
            const int64_t q0 = (int64_t)e - (ML - 1);
            const int64_t q = q0 + hl;
            const bool in_span = live && hl < span, in_file = in_span && q >= 0 && (uint64_t)q < a.n;
            uint32_t h = 0, l = 0, br = 0, ot = 0;
            if (in_file) {   // 1-2 words of the position-contiguous planes for the whole span
                const uint4 v = a.nuc.lin[(uint64_t)q >> 5];
                const uint32_t i5 = (uint32_t)q & 31;
                h = (v.x >> i5) & 1;
                l = (v.y >> i5) & 1;
                br = (v.z >> i5) & 1;
                ot = (v.w >> i5) & 1;
            }
            const uint64_t H = __builtin_amdgcn_ballot_w64(h != 0), L = __builtin_amdgcn_ballot_w64(l != 0);
            const uint64_t BR = __builtin_amdgcn_ballot_w64(br != 0), OT = __builtin_amdgcn_ballot_w64(ot != 0);
            const uint64_t OUT = __builtin_amdgcn_ballot_w64(in_span && !in_file);
            const uint64_t EX = OT | (a.cross ? BR : 0ull);
            const uint64_t EXN = OT & ~BR & H;   // N (NUC_N_MARK)
            const uint64_t EXL = EX & ~EXN;       // bytes compared by value
            const uint64_t KILL = OUT | (a.cross ? 0ull : BR);
            // windows that also hold an earlier exception of the span are its
            // (per half: below the last exception before e)
            const uint64_t bm = (1ull << (ML - 1)) - 1;
            const uint64_t before = (OT | BR) & (TWO ? (bm | bm << 32) : bm);
            uint64_t owned;
            if constexpr (TWO) {
                const uint32_t b0 = (uint32_t)before, b1 = (uint32_t)(before >> 32);
                owned = (b0 ? 0xFFFFFFFFull >> __builtin_clz(b0) : 0ull) |
                        ((b1 ? 0xFFFFFFFFull >> __builtin_clz(b1) : 0ull) << 32);
            } else {
                owned = before ? ~0ull >> __builtin_clzll(before) : 0ull;
            }
            // the lane's byte when it is compared by value (N: its mark)
            uint8_t ch = 'N';
            const bool byval = ((EXN | EXL) >> lane) & 1;
            if ((EXL >> lane) & 1) {
                const Loc lc = loc_of((uint64_t)q);
                ch = a.nuc.xbytes[(uint64_t)exception_index(a.nuc.sbflag, a.nuc.sbbase, lc.word) * 32 + lc.bit];
            }
            for (int c = 0; c < nc; ++c) {
                const uint64_t vb = __builtin_amdgcn_ballot_w64(byval && ((s_cm[c][ch >> 5] >> (ch & 31)) & 1));
                if (lane == c) mv[c] = (~vec_mismatch(H, L, s_csub[c]) & ~EX) | vb;
            }
            wave_lds_sync();
            const int64_t q00 = (int64_t)eh[0] - (ML - 1), q01 = (int64_t)eh[1] - (ML - 1);
            for (int p = lane; p < a.P; p += 64) {
                const int len = a.lengths[p];
                const uint4 cl = s_cls[p];
                const uint32_t cw[4] = {cl.x, cl.y, cl.z, cl.w};
                // starts u whose window holds e: u in [ML - len, ML - 1] (per half)
                const uint64_t r = ((1ull << len) - 1) << (ML - len);
                uint64_t alive = ((live0 ? r : 0ull) | (TWO && live1 ? r << 32 : 0ull)) & ~owned;
                if (KILL) {   // wave-uniform; rare with the simple engine (off-file positions only)
                    uint64_t kw = 0;
                    for (int j = 0; j < len; ++j) kw |= KILL >> j;
                    alive &= ~kw;
                }
                uint64_t c0 = 0, c1 = 0, ge4 = 0;
                for (int j = 0; j < len; ++j) {   // (not unrolled: dead windows leave early)
                    const uint64_t m = mv[(cw[j >> 2] >> (8 * (j & 3))) & 255u] >> j;
                    if (a.k == 0) {
                        alive &= m;
                        if (!alive) break;   // most windows around an exception die within a few positions
                    } else {
                        vec_add(~m, c0, c1, ge4);
                    }
                }
                if (a.k) {
                    uint64_t dead;
                    switch (a.k) {
                        case 1: dead = c1 | ge4; break;
                        case 2: dead = (c1 & c0) | ge4; break;
                        default: dead = ge4; break;
                    }
                    alive &= ~dead;
                }
                for (; alive; alive &= alive - 1) {
                    const int b = __builtin_ctzll(alive);
                    const uint64_t s0 = TWO && b >= 32 ? (uint64_t)(q01 + (b - 32)) : (uint64_t)(q00 + b);
                    const uint32_t slot = (uint32_t)(a.pattern_base + p);
                    const uint64_t og = (uint32_t)(s0 / TILE_POS) / (uint32_t)a.tiles_per_wg;   // 32-bit division
                    const uint32_t o = atomicAdd(&a.seg_cnt[(uint64_t)slot * a.nwg + og], 1u);
                    if (o < a.slot_cap[slot]) a.out[a.slot_base[slot] + og * a.slot_cap[slot] + o] = ((uint64_t)slot << 48) | s0;
                }
            }
            wave_lds_sync();   // mv is rewritten for the next bit
        }
    }
}

// Phase 2: one wave per selected word, waves loop over the list (its length
// is on the device), so every wave reaches the end of the list and exits.
// CLS: large batches (more than OTH_MAX_POS (pattern, position) entries) stage
// a class id per entry and one membership table per class instead.
template <bool CLS>
__global__ __launch_bounds__(256) void k_linear_others(OthersArgs a) {
    // membership of every byte in the class of (pattern p, position j), at
    // p * maxlen + j ('.' all ones), staged in LDS once per block: the window
    // tests below then touch no global table
    __shared__ uint32_t s_memb[CLS ? 256 : OTH_MAX_POS][8];
    __shared__ uint8_t s_cls[CLS ? OTH_CLS_MAX_POS : 1];
    if (CLS) {
        for (int i = threadIdx.x; i < 256 * 8; i += blockDim.x) {
            const int c = i >> 3;
            s_memb[c][i & 7] = c < a.n_classes ? (a.class_any[c] ? ~0u : a.class_bytes[c * 8 + (i & 7)]) : 0u;
        }
        for (int e = threadIdx.x; e < a.P * a.maxlen; e += blockDim.x) {
            const int p = e / a.maxlen, j = e % a.maxlen;
            s_cls[e] = j < a.lengths[p] ? a.pos_class[p * 64 + j] : 0;
        }
    } else {
        for (int i = threadIdx.x; i < a.P * a.maxlen * 8; i += blockDim.x) {
            const int e = i >> 3, p = e / a.maxlen, j = e % a.maxlen;
            uint32_t m = 0;
            if (j < a.lengths[p]) {
                const int cl = a.pos_class[p * 64 + j];
                m = a.class_any[cl] ? ~0u : a.class_bytes[cl * 8 + (i & 7)];
            }
            s_memb[e][i & 7] = m;
        }
    }
    __syncthreads();
    // items_per_wave (1, 2 or 4) items share a wave, 64 / items_per_wave
    // lanes each (an item's window span fits them): more gathers in flight
    const int G = a.items_per_wave, lanes = 64 / G;
    const int lane = (threadIdx.x & 63) % lanes, slice = (threadIdx.x & 63) / lanes;
    const uint64_t nsel = *a.nsel;
    const uint32_t nitems = gridDim.x * (blockDim.x >> 6) * G;
    for (uint64_t it = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * G + slice; it < nsel; it += nitems) {
        const OtherSel sv = a.sel[it];
        const uint64_t tile = sv.word / TILE_WORDS;
        const uint32_t lw = logical_word((uint32_t)(sv.word % TILE_WORDS));
        if (CLS)
            other_windows(a, MembClass{s_cls, s_memb}, tile, lw, sv.bits, lane, lanes, slice);
        else
            other_windows(a, MembDirect{s_memb}, tile, lw, sv.bits, lane, lanes, slice);
    }
}

// Fixed-length patterns on the byte layout (peptides): one thread per window
// start, every pattern of the batch; the file is small next to a genome
// (a proteome is a few MB), so a plain exact check per window suffices.
// Line-bounded (k > 0, or no class accepts '\n'): the folded bytes with
// header lines stored as '\n' -- a window holding one is dead.  Cross (k = 0
// and a class accepts '\n', nrgrep's simple engine): the file's own bytes.
struct ByteLinArgs {
    const uint8_t* bytes;
    const uint8_t* raw;
    uint64_t n;
    const uint8_t* pos_class;
    const int32_t* lengths;
    const uint8_t* class_any;
    const uint32_t* class_bytes;
    int P, k, cross;
    Sink sink;
};

__global__ __launch_bounds__(256) void k_bytes_linear(ByteLinArgs a) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint8_t* text = a.cross ? a.raw : a.bytes;
    for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < a.n; s += stride) {
        for (int p = 0; p < a.P; ++p) {
            const int len = a.lengths[p];
            if (s + (uint64_t)len > a.n) continue;
            int mm = 0;
            bool ok = true;
            for (int j = 0; j < len && ok; ++j) {
                const uint8_t ch = text[s + j];
                if (!a.cross && ch == (uint8_t)'\n') { ok = false; break; }
                const int c = a.pos_class[p * 64 + j];
                if (a.class_any[c]) continue;
                if (!((a.class_bytes[c * 8 + (ch >> 5)] >> (ch & 31)) & 1) && ++mm > a.k) ok = false;
            }
            if (ok) a.sink.push(a.sink.bin_of((uint32_t)p, s), ((uint64_t)p << 48) | s);
        }
    }
}

// BYTE databases on the 5-bit residue planes (pm_db::p5; north_star's
// 5-bit packing).  One lane per 32-position word w = the 32 window starts
// 32 w .. 32 w + 31: it loads W words of the five planes (coalesced: lane
// after lane), turns them into one membership word per distinct class of
// the batch (bit i: the residue at 32 w' + i is in the class) -- an OR of
// per-code equality words, each five XORs against the code's bits, over the
// class's codes or, when shorter, the codes it lacks -- staged in LDS, then
// counts every pattern's mismatches bit-parallel over its 32 windows:
// position j's word is the class word shifted by j (alignbit of two staged
// words), a code-0 residue (a line break or header byte) kills the window
// whatever k is, as it does in k_bytes_linear.  HBM: 0.625 byte per residue
// instead of the byte copy's 1.
constexpr int P5_MAX_CLS = 16;   // distinct classes of one scan
constexpr int P5_LIST = 16;      // codes listed per class (the shorter of the class and its complement)
constexpr int P5_T = 128;        // threads per block
struct P5Args {
    const uint32_t* p5;
    uint64_t nw;          // words per plane
    uint64_t nwords;      // words holding window starts
    const uint8_t* cls;   // [C][2 + P5_LIST]: count, complement flag, codes
    int C;
    const uint8_t* pidx;  // [P][64]: class index of each position, 255 = '.' (every residue but code 0)
    const int32_t* lengths;
    int P, k;
    Sink sink;
};

// CROSS (nrgrep's simple engine at k = 0 with a class that takes '\n'):
// windows span lines, '\n' (code 1) is a residue like any other and only
// header bytes (code 0) kill; the windows they kill are k_p5_cross_fix's.
template <int W, bool CROSS>
__global__ __launch_bounds__(P5_T) void k_p5_linear(P5Args a) {
    __shared__ uint32_t s_m[P5_MAX_CLS * W][P5_T];   // membership words, lane-contiguous (no bank conflicts)
    __shared__ uint8_t s_cls[P5_MAX_CLS][2 + P5_LIST];
    for (int i = threadIdx.x; i < a.C * (2 + P5_LIST); i += P5_T)
        s_cls[i / (2 + P5_LIST)][i % (2 + P5_LIST)] = a.cls[i];
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * P5_T;
    for (uint64_t w = blockIdx.x * (uint64_t)P5_T + threadIdx.x; w < a.nwords; w += stride) {
        uint32_t pl[W][5];
#pragma unroll
        for (int i = 0; i < W; ++i)
#pragma unroll
            for (int q = 0; q < 5; ++q) pl[i][q] = a.p5[(uint64_t)q * a.nw + w + i];   // zero-padded past the end
        uint32_t brk[W];   // code 0 (header bytes, padding), and '\n' unless CROSS
#pragma unroll
        for (int i = 0; i < W; ++i)
            brk[i] = CROSS ? ~(pl[i][0] | pl[i][1] | pl[i][2] | pl[i][3] | pl[i][4]) : ~(pl[i][1] | pl[i][2] | pl[i][3] | pl[i][4]);
        for (int c = 0; c < a.C; ++c) {
            const int cnt = s_cls[c][0];
            uint32_t m[W];
#pragma unroll
            for (int i = 0; i < W; ++i) m[i] = 0u;
            for (int e = 0; e < cnt; ++e) {
                const uint32_t x = s_cls[c][2 + e];
#pragma unroll
                for (int i = 0; i < W; ++i) {
                    uint32_t d = 0u;
#pragma unroll
                    for (int q = 0; q < 5; ++q) d |= pl[i][q] ^ (((x >> q) & 1u) ? ~0u : 0u);
                    m[i] |= ~d;
                }
            }
            const bool comp = s_cls[c][1] != 0;
#pragma unroll
            for (int i = 0; i < W; ++i) s_m[c * W + i][threadIdx.x] = comp ? ~m[i] : m[i];
        }
        for (int p = 0; p < a.P; ++p) {
            const int len = a.lengths[p];
            const uint8_t* pi = a.pidx + p * 64;
            uint32_t c0 = 0u, c1 = 0u, ge4 = 0u, kill = 0u;
            for (int j = 0; j < len; ++j) {
                const int i = j >> 5, sh = j & 31;
                const uint32_t b0 = i == 0 ? brk[0] : brk[W - 2], b1 = i == 0 ? brk[1] : brk[W - 1];
                kill |= __builtin_amdgcn_alignbit(b1, b0, sh);
                const int c = pi[j];
                if (c == 255) continue;
                const uint32_t m0 = s_m[c * W + i][threadIdx.x], m1 = s_m[c * W + i + 1][threadIdx.x];
                const uint32_t x = ~__builtin_amdgcn_alignbit(m1, m0, sh);
                const uint32_t cy0 = c0 & x;
                c0 ^= x;
                const uint32_t cy1 = c1 & cy0;
                c1 ^= cy0;
                ge4 |= cy1;
            }
            uint32_t dead = ge4 | kill;
            switch (a.k) {
                case 0: dead |= c0 | c1; break;
                case 1: dead |= c1; break;
                case 2: dead |= c1 & c0; break;
                default: break;
            }
            // one counter reservation per wave when its 64 words fall in
            // one bin (dense hits would serialize on the bin's counter)
            uint32_t live = ~dead;
            const uint64_t w0 = __builtin_amdgcn_readfirstlane((uint32_t)(w & 0xFFFFFFFFu)) |
                                ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(w >> 32)) << 32);
            const uint32_t bin0 = a.sink.bin_of((uint32_t)p, w0 * 32), bin1 = a.sink.bin_of((uint32_t)p, w0 * 32 + 64 * 32 - 1);
            if (bin0 == bin1 && __builtin_amdgcn_ballot_w64(true) == ~0ull) {
                const uint32_t cnt = __builtin_popcount(live);
                uint32_t incl = cnt;   // inclusive prefix over the wave
                const int lane = threadIdx.x & 63;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t o = __shfl_up(incl, d, 64);
                    if (lane >= d) incl += o;
                }
                const uint32_t tot = __shfl(incl, 63, 64);
                uint32_t base = 0;
                if (tot) {
                    if (lane == 0) base = atomicAdd(&a.sink.bin_cnt[bin0], tot);
                    base = __shfl(base, 0, 64);
                }
                uint32_t o = base + incl - cnt;
                for (; live; live &= live - 1u, ++o) {
                    const uint64_t st = w * 32 + (uint64_t)__builtin_ctz(live);
                    if (o < a.sink.cap) a.sink.out[(uint64_t)bin0 * a.sink.cap + o] = ((uint64_t)p << 48) | st;
                }
            } else {
                for (; live; live &= live - 1u) {
                    const uint64_t st = w * 32 + (uint64_t)__builtin_ctz(live);
                    a.sink.push(a.sink.bin_of((uint32_t)p, st), ((uint64_t)p << 48) | st);
                }
            }
        }
    }
}

// The windows k_p5_linear<W, true> killed on header bytes, checked against
// the file's own bytes as k_bytes_linear does: a wave per header line r
// (a header line and a pattern give ~60-100 windows), the windows that
// overlap it and no earlier header line.
struct P5FixArgs {
    const uint8_t* raw;
    uint64_t n;
    const uint64_t* hdr;
    const uint64_t* hdr_end;
    uint64_t nhdr;
    const uint8_t* pos_class;
    const int32_t* lengths;
    const uint8_t* class_any;
    const uint32_t* class_bytes;
    int P, k;
    Sink sink;
};

__global__ __launch_bounds__(64) void k_p5_cross_fix(P5FixArgs a) {   // one wave per header line
    for (uint64_t r = blockIdx.x; r < a.nhdr; r += gridDim.x) {
        const int64_t hb = (int64_t)a.hdr[r], he = (int64_t)a.hdr_end[r];
        const int64_t prev = r ? (int64_t)a.hdr_end[r - 1] : 0;
        for (int p = 0; p < a.P; ++p) {
            const int len = a.lengths[p];
            int64_t lo = hb - len + 1;
            if (lo < prev) lo = prev;
            if (lo < 0) lo = 0;
            for (int64_t s = lo + threadIdx.x; s < he; s += blockDim.x) {
                if ((uint64_t)s + (uint64_t)len > a.n) continue;
                int mm = 0;
                bool ok = true;
                for (int j = 0; j < len && ok; ++j) {
                    const uint8_t ch = a.raw[s + j];
                    const int c = a.pos_class[p * 64 + j];
                    if (a.class_any[c]) continue;
                    if (!((a.class_bytes[c * 8 + (ch >> 5)] >> (ch & 31)) & 1) && ++mm > a.k) ok = false;
                }
                if (ok) a.sink.push(a.sink.bin_of((uint32_t)p, (uint64_t)s), ((uint64_t)p << 48) | (uint64_t)s);
            }
        }
    }
}

// waves per workgroup = parts of a lane's 32 window words; each wave scans
// 32 / parts consecutive words of every lane column of the tile.  Two waves
// of 16 words (12 % fewer VALU instructions per tile: the Lmax - 1 halo words
// and the strands' shared blocks are paid per wave) measured slower, 0.500 vs
// 0.464 ms: the LDS ring then allows only 2 waves per SIMD (r04b A/B).  A
// wave per whole tile reading the rows straight from global memory (19 %
// fewer VALU instructions, no LDS) measured slower still, 0.546 vs 0.473 ms:
// each row load's latency is exposed at 3 waves per SIMD (r04w A/B).
// waves per workgroup = parts of a tile's 32 window words (PM_JIT_PARTS, A/B:
// 1, 2 or 4; default 4).  Each wave derives the class words of its steps'
// rows plus the Lmax - 1 rows its last windows reach into: fewer parts
// derive fewer rows twice, more parts keep more waves per SIMD
int jit_parts() {
    static const int v = [] {
        const char* e = getenv("PM_JIT_PARTS");
        const int p = e ? atoi(e) : 4;
        return p == 1 || p == 2 || p == 4 ? p : 4;
    }();
    return v;
}
// the graded tail (scan_linear), on unless PM_JIT_GRADED=0: kernel -1.4 %
// at 10 Gbp (frac 0.704 vs 0.694) with the same step time, -3 % kernel and
// step at 100 Gbp (round 4, gpu_envab.sh; tests/test_gpu_graded.py checks
// both partitions against each other)
bool jit_graded() {
    const char* e = getenv("PM_JIT_GRADED");
    return !e || atoi(e) != 0;
}
constexpr int JIT_MAX_P = 8;   // patterns per specialized kernel
static_assert(JIT_MAX_P * 64 <= OTH_MAX_POS, "k_linear_others stages a chunk's classes in LDS");

// Hit records of pm_linear_jit -> hit keys.  A record is (tile, lane, step,
// pattern) and the live mask of that window word, exact for the ACGT fast
// path; windows overlapping an exception are dropped here (breaks kill,
// windows with an "other" byte belong to k_linear_others), which needs the
// exception planes only for lanes the tile's lane flags mark.  One
// 1024-thread block per output segment (`group` consecutive pm_linear_jit
// workgroups, a contiguous tile range); its 16 waves take the (workgroup,
// wave) record lists in turn, reserve slots of the (pattern, segment) hit
// lists with LDS atomics and write the segment counts once at the end
// (k_linear_others, launched after, appends with global atomics).
struct ExpandArgs {
    const uint2* bo;
    const uint64_t* lflag;
    const uint2* rec;
    const uint32_t* rec_cnt;
    uint32_t* rec_over;   // max record count seen above rcap (0: none)
    uint32_t rcap;
    uint64_t ntiles, n;
    const int32_t* lengths;
    int P, pattern_base;
    uint64_t* out;
    uint32_t* seg_cnt;
    const uint64_t* slot_base;
    const uint32_t* slot_cap;
    uint32_t nwg, nout, group, tiles_per_wg;
    uint32_t parts;   // waves per pm_linear_jit workgroup (32 / parts words each)
    // graded tail (JArgs): segments ogA.. hold groupB workgroups of tpwB tiles
    uint32_t nA, tpwB, ogA, groupB, tpo;
    uint64_t tilesA;
};

// One block per output segment (`group` workgroups x 4 wave segments); each
// wave segment is expanded by SEG_LANES lanes (a segment holds a few records:
// ~7 at the bench's density), so all 32 segments of a block are in flight at
// once and 4 blocks fit a CU -- the whole grid is resident in one round and a
// block's latency is one chain of loads (count, records, lane flags).
constexpr int EXPAND_THREADS = 512;
constexpr uint32_t SEG_LANES = 16;

__global__ __launch_bounds__(EXPAND_THREADS) void k_linear_expand(ExpandArgs a) {
    __shared__ uint32_t cnt_p[JIT_MAX_P];
    // a graded-tail segment holds groupB short workgroups (a quarter of the
    // records per wave segment): 2 lanes per wave segment, so its ~150 wave
    // segments are all in flight at once
    const uint32_t og = blockIdx.x, seg_lanes = og < a.ogA ? SEG_LANES : SEG_LANES / 8;
    const uint32_t sub = threadIdx.x / seg_lanes, lane_t = threadIdx.x % seg_lanes;
    if (threadIdx.x < JIT_MAX_P) cnt_p[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t wg0 = og < a.ogA ? og * a.group : a.nA + (og - a.ogA) * a.groupB;
    const uint32_t pairs = (min(a.nwg, wg0 + (og < a.ogA ? a.group : a.groupB)) - wg0) * a.parts;
    for (uint32_t q = sub; q < pairs; q += EXPAND_THREADS / seg_lanes) {
        const uint32_t wg = wg0 + q / a.parts, part = q % a.parts;
        const uint32_t seg = wg * a.parts + part;
        uint32_t cnt = a.rec_cnt[seg];
        if (cnt > a.rcap) {
            if (lane_t == 0) atomicMax(a.rec_over, cnt);
            cnt = a.rcap;
        }
        for (uint32_t i = lane_t; i < cnt; i += seg_lanes) {
            const uint2 r = a.rec[(uint64_t)seg * a.rcap + i];
            uint64_t t0 = (uint64_t)wg * a.tiles_per_wg;
            if (wg >= a.nA) {
                const uint32_t j = wg - a.nA, sg = j / a.groupB;
                t0 = a.tilesA + (uint64_t)sg * a.tpo + (uint64_t)(j - sg * a.groupB) * a.tpwB;
            }
            const uint64_t tile = t0 + (r.x >> 15);
            const uint32_t lane = (r.x >> 9) & 63, s = (r.x >> 3) & 63, p = r.x & 7;   // s up to 31 + a shift
            if (tile >= a.ntiles) continue;
            const uint32_t w0 = 32u * lane + s;
            uint32_t live = r.y;
            if ((a.lflag[tile] >> lane) & 1) {
                uint32_t kill = 0;
                const int len = a.lengths[p];
                for (int j = 0; j < len; ++j) {
                    const uint2 e = a.bo[phys_word(tile, w0 + j)];
                    kill |= e.x | e.y;
                }
                live &= ~kill;
            }
            const uint32_t slot = (uint32_t)a.pattern_base + p;
            const uint32_t cap = a.slot_cap[slot];
            uint64_t* dst = a.out + a.slot_base[slot] + (uint64_t)og * cap;
            for (; live; live &= live - 1) {
                const uint64_t pos = pos_of(tile, w0, __builtin_ctz(live));
                if (pos >= a.n) continue;
                const uint32_t o = atomicAdd(&cnt_p[p], 1u);
                if (o < cap) dst[o] = ((uint64_t)slot << 48) | pos;
            }
        }
    }
    __syncthreads();
    // k_linear_others (launched after) appends to the same counters
    if ((int)threadIdx.x < a.P)
        a.seg_cnt[(uint64_t)(a.pattern_base + threadIdx.x) * a.nout + og] = cnt_p[threadIdx.x];
}

__global__ void k_linear_lens(const uint64_t* __restrict__ keys, uint64_t n, const int32_t* __restrict__ lengths,
                              uint32_t* __restrict__ lens) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    lens[i] = (uint32_t)lengths[(int)(keys[i] >> 48)];
}

// ---------------------------------------------------------------------------
// runtime-specialized kernel (hipRTC)
// ---------------------------------------------------------------------------
const char* kJitCommon = R"JIT(
typedef unsigned int u32;
typedef unsigned long long u64;
typedef unsigned char u8;
// Hit records: one uint2 per (tile, lane, step, pattern) with a live window:
// x = (tile - first tile of the workgroup) << 15 | lane << 9 | word << 3 |
// pattern, y = the live mask (bit b = the window of stream b).  Staged per
// wave in LDS and flushed to the wave's global segment, so the scan loop
// never waits on a global store; k_linear_expand turns records into keys.
struct JArgs {
    const uint2* hl;
    uint2* rec;             // [nwg * NW][rcap]
    u32* rec_cnt;           // [nwg * NW]
    u32* aux_zero;          // the sink's record-overflow counter, zeroed by the first launch of a scan (or null)
    u64 ntiles;
    u32 rcap, tiles_per_wg;
    // graded tail: from tile tilesA on, each output segment's tpo tiles go
    // to groupB workgroups (nA, nA + 1, ...) of tpwB tiles (the last fewer)
    u32 nA, tpwB, groupB, tpo;
    u64 tilesA;
    u64* clk;               // PM_JIT_CLOCK builds: per workgroup {shader cycles, 100 MHz ticks, start tick}
};
#define STREAM 2048u
#define TILE_POS 65536ull
#define TILE_WORDS 2112ull
#define B3(a, b, c, t) ((u32)__builtin_amdgcn_bitop3_b32((a), (b), (c), (t)))
// pins a class word in a register: the compiler would otherwise re-derive it
// from the plane words at every step that uses it
#define PIN(x) asm("" : "+v"(x))
typedef __attribute__((address_space(1))) uint2 glb_uint2;
typedef __attribute__((address_space(3))) uint2 lds_uint2;
)JIT";

struct JitKernel {
    hipModule_t module = nullptr;
    hipFunction_t fn = nullptr;
};

std::mutex g_jit_mu;
std::map<std::pair<int, std::string>, JitKernel> g_jit_cache;

struct JArgsHost {           // must match JArgs in kJitCommon
    const uint2* hl;
    uint2* rec;
    uint32_t* rec_cnt;
    uint32_t* aux_zero;
    uint64_t ntiles;
    uint32_t rcap, tiles_per_wg;
    uint32_t nA, tpwB, groupB, tpo;
    uint64_t tilesA;
    uint64_t* clk = nullptr;
};
constexpr int JIT_REC_LDS = 96;       // hit records staged per wave in LDS (3 workgroups per CU)
// workgroups resident per CU (4: two 16.5 KiB tile slots each fit the LDS)
constexpr int JIT_WG_PER_CU = 4;

// mismatch of an ACGT subset as an expression of the plane words h, l.
// Forms with an inverted plane are one explicit v_bitop3 (truth table over
// (h, l, l)): written as C, the compiler splits them into a NOT (shared or
// not) plus an OR/AND -- measured 16 extra ops per wave-tile.
std::string subset_expr(int subset, const std::string& h, const std::string& l) {
    auto b3 = [&](int (*f)(int, int)) {
        int tt = 0;
        for (int idx = 0; idx < 8; ++idx) tt |= f((idx >> 2) & 1, (idx >> 1) & 1) << idx;   // idx = 4h + 2l + l
        char buf[8];
        snprintf(buf, sizeof buf, "0x%02X", tt);
        return "B3(" + h + ", " + l + ", " + l + ", " + buf + ")";
    };
    switch (subset & 15) {
        case 0x2: return b3([](int a, int b) { return a | (b ^ 1); });
        case 0x4: return b3([](int a, int b) { return (a ^ 1) | b; });
        case 0x8: return b3([](int a, int b) { return (a ^ 1) | (b ^ 1); });
        case 0xB: return b3([](int a, int b) { return a & (b ^ 1); });
        case 0xD: return b3([](int a, int b) { return (a ^ 1) & b; });
        case 0xE: return b3([](int a, int b) { return (a ^ 1) & (b ^ 1); });
        default: break;
    }
    switch (subset & 15) {
        case 0x0: return "~0u";
        case 0x1: return "(" + h + " | " + l + ")";
        case 0x2: return "(" + h + " | ~" + l + ")";
        case 0x4: return "(~" + h + " | " + l + ")";
        case 0x8: return "(~" + h + " | ~" + l + ")";
        case 0x3: return h;
        case 0x5: return l;
        case 0x9: return "(" + h + " ^ " + l + ")";
        case 0x6: return "~(" + h + " ^ " + l + ")";
        case 0xA: return "~" + l;
        case 0xC: return "~" + h;
        case 0x7: return "(" + h + " & " + l + ")";
        case 0xB: return "(" + h + " & ~" + l + ")";
        case 0xD: return "(~" + h + " & " + l + ")";
        case 0xE: return "(~" + h + " & ~" + l + ")";
        default: return "0u";
    }
}

// Carry-save state of a partial mismatch count: column 0 (weight 1) and, for
// K >= 2, column 1 (weight 2); every carry whose weight exceeds K is a dead
// term (the window is dead whatever the other inputs are).
struct CountNet {
    std::deque<std::string> col[2];
    std::vector<std::string> dead;
};

// ORs `terms` into one word (three-way ORs as v_bitop3 0xFE: v_or3_b32
// issues ~1.5x slower on gfx950, profiles/r01c_valu_rates.txt).
std::string emit_or(std::ostringstream& o, const std::vector<std::string>& terms, int& uid, const std::string& ind) {
    if (terms.empty()) return "0u";
    std::string acc = terms[0];
    size_t i = 1;
    for (; i + 1 < terms.size(); i += 2) {
        const std::string v = "d" + std::to_string(uid++);
        o << ind << "const u32 " << v << " = B3(" << acc << ", " << terms[i] << ", " << terms[i + 1] << ", 0xFE);\n";
        acc = v;
    }
    if (i < terms.size()) {
        const std::string v = "d" + std::to_string(uid++);
        o << ind << "const u32 " << v << " = " << acc << " | " << terms[i] << ";\n";
        acc = v;
    }
    return acc;
}

// Adds mismatch words to a count and compresses every column to at most 2
// bits with full adders (xor3 + majority, one v_bitop3 each); carries of
// weight > K go straight into the dead terms.  K = 0: every input is dead.
void net_add(std::ostringstream& o, CountNet& n, const std::vector<std::string>& in, int K, int& uid,
             const std::string& ind) {
    if (K == 0) {
        n.dead.insert(n.dead.end(), in.begin(), in.end());
        return;
    }
    n.col[0].insert(n.col[0].end(), in.begin(), in.end());
    const int lmax = K >= 2 ? 1 : 0;   // highest column whose weight is <= K
    for (int L = 0; L <= lmax; ++L) {
        auto& c = n.col[L];
        while (c.size() > 2) {
            const std::string a = c.front(); c.pop_front();
            const std::string b = c.front(); c.pop_front();
            const std::string d = c.front(); c.pop_front();
            const std::string s = "s" + std::to_string(uid), cy = "c" + std::to_string(uid);
            ++uid;
            o << ind << "const u32 " << s << " = B3(" << a << ", " << b << ", " << d << ", 0x96);\n";
            o << ind << "const u32 " << cy << " = B3(" << a << ", " << b << ", " << d << ", 0xE8);\n";
            c.push_back(s);
            if (L < lmax) n.col[L + 1].push_back(cy);
            else n.dead.push_back(cy);
        }
    }
}

// "count > K" of a compressed count: the dead terms OR the comparison of
// what is left -- a, b (weight 1) and, for K >= 2, c, d (weight 2).
std::string net_dead(std::ostringstream& o, const CountNet& n, int K, int& uid, const std::string& ind) {
    std::vector<std::string> terms = n.dead;
    auto at = [&](int L, size_t i) { return i < n.col[L].size() ? n.col[L][i] : std::string("0u"); };
    if (K == 1) {
        if (n.col[0].size() == 2) terms.push_back("(" + at(0, 0) + " & " + at(0, 1) + ")");
    } else if (K >= 2 && !n.col[1].empty()) {
        // count = a + b + 2 (c + d) (+ 4 per dead carry):
        //   K = 2: dead iff c & d, or (c | d) & (a | b)  = maj(c, d, a | b)
        //   K = 3: dead iff c & d, or (c | d) & a & b    = maj(c, d, a & b)
        const std::string ab = n.col[0].size() < 2 ? at(0, 0)
                               : "(" + at(0, 0) + (K == 2 ? " | " : " & ") + at(0, 1) + ")";
        if (K == 3 && n.col[0].size() < 2) terms.push_back("(" + at(1, 0) + " & " + at(1, 1) + ")");
        else terms.push_back("B3(" + at(1, 0) + ", " + at(1, 1) + ", " + ab + ", 0xE8)");
    }
    return emit_or(o, terms, uid, ind);
}

// Shared blocks.  Two patterns whose class sequences agree on a run of
// positions at some offset -- the strands of a (near-)palindromic motif:
// TGCTGA[GC]TCAGCA.[AT] and its reverse complement agree on 13 positions
// at offset 2, restriction sites on all of them -- read the same
// (row, class) words for those positions at steps `off` apart, so the
// carry-save count of the block is built once per row and both windows
// only add their own positions (a 13-position block at k = 2: 17 ops
// once, then 3 per window, instead of 19 per window).  Greedy pairing,
// each pattern in at most one pair; a pair pays when the block is large
// and the offset small against the wave's `steps` window words.
// shift[p]: the pair's member whose block rows sit `off` words later is
// scanned `off` steps later (its windows at words t + off read the rows
// its partner's windows at t read): each block is built once per step
// instead of twice at the wave's right edge (see gen_linear_source).
std::vector<std::vector<int>> shared_blocks(int P, const int32_t* lengths, const uint8_t* pos_class,
                                            const uint8_t* class_acgt, const uint8_t* class_is_any, int steps,
                                            std::vector<int>* shift = nullptr) {
    const int JIT_STEPS = steps;
    if (shift) shift->assign(P, 0);
    std::vector<std::vector<int>> block(P);   // positions of pattern p in its shared block
    {
        std::vector<bool> used(P, false);
        auto cls = [&](int p, int j) { return class_is_any[pos_class[64 * p + j]] ? -1 : class_acgt[pos_class[64 * p + j]] & 15; };
        for (;;) {
            int bp = -1, bq = -1, boff = 0, best = 0;
            for (int p = 0; p < P; ++p)
                for (int q = p + 1; q < P; ++q) {
                    if (used[p] || used[q]) continue;
                    for (int off = -(JIT_STEPS / 2); off <= JIT_STEPS / 2; ++off) {
                        // position j of p meets position j - off of q
                        int n = 0;
                        for (int j = 0; j < lengths[p]; ++j)
                            n += j - off >= 0 && j - off < lengths[q] && cls(p, j) >= 0 && cls(p, j) == cls(q, j - off);
                        // ops saved ~ 1.3 per shared input and shared step, a block per extra step
                        const int gain = n * (JIT_STEPS - 2 * std::abs(off));
                        if (n >= 6 && gain > best) { best = gain; bp = p; bq = q; boff = off; }
                    }
                }
            if (bp < 0) break;
            used[bp] = used[bq] = true;
            // position j of bp meets j - boff of bq: bq's block at step t + boff
            // reads bp's rows at step t
            if (shift) (*shift)[boff > 0 ? bq : bp] = boff > 0 ? boff : -boff;
            for (int j = 0; j < lengths[bp]; ++j)
                if (j - boff >= 0 && j - boff < lengths[bq] && cls(bp, j) >= 0 && cls(bp, j) == cls(bq, j - boff)) {
                    block[bp].push_back(j);
                    block[bq].push_back(j - boff);
                }
        }
    }
    return block;
}

// Source of the specialized kernel for a batch of P <= 8 patterns.
//
// Workgroup = 4 waves = one tile at a time: wave w scans steps
// [8 w, 8 w + 8) of the tile for EVERY pattern of the batch, so the class
// words X_c(word) of a word are derived once and shared by both strands
// (they are pinned in registers: one VALU op per (word, class)).  Tiles
// arrive in a 3-deep LDS ring by global_load_lds_dwordx4 (LDS-DMA, no
// VGPRs, 1 KiB per wave-instruction): while the workgroup computes tile i
// the DMAs of tiles i+1 and i+2 are in flight (~100 KB per CU at 3
// workgroups/CU), so HBM latency is off the critical path and every tile is
// read from HBM once however many waves scan it.  Each step is a
// straight-line Wallace tree per pattern ending in a "dead" word; the fast
// path only ANDs them.  When some lane has a live window (rare: the branch
// is wave-uniform), every (step, pattern) with live windows leaves an 8-byte
// record with its live mask (wave ballot + mbcnt into an LDS stage, flushed
// rarely); k_linear_expand turns records into hit keys.
// PM_JIT_ROTATE=0: every wave keeps its part (the round-4 form, for A/B
// measurements); default: the parts rotate from tile to tile
bool jit_rotate() {
    const char* e = getenv("PM_JIT_ROTATE");
    return !(e && e[0] == '0');
}

// PM_JIT_M0=0 (A/B): the tile DMAs save and restore m0 around themselves
// (the round-5 form); default: m0 is a declared clobber of the DMA's asm
bool jit_m0() {
    static const bool on = !(getenv("PM_JIT_M0") && getenv("PM_JIT_M0")[0] == '0');
    return on;
}

// PM_JIT_CLOCK=1 (measurement only): every workgroup of pm_linear_jit reads
// the shader clock counter (s_memtime) and the 100 MHz real-time counter
// (s_memrealtime) at its start and end, and the library prints per launch
// the effective shader clock of the launch (cycles / real time over the
// workgroups) on stderr -- whether a slower dispatch ran at a lower clock
// (tools/clock_trace.py)
bool jit_clock() {
    static const bool on = [] {
        const char* e = getenv("PM_JIT_CLOCK");
        return e && e[0] == '1';
    }();
    return on;
}

// PM_JIT_PREFETCH=<bytes> (A/B): besides the LDS DMA of the next tile, each
// workgroup touches the tile after it -- one 4-byte read per `bytes` of it
// (64 or 128), landing in a 256-byte dummy LDS row -- so two tiles per
// workgroup are in flight from HBM instead of one, with no extra LDS ring
// slot; the DMA of that tile an iteration later then hits L2 / MALL.  0: off
int jit_prefetch() {
    static const int v = [] {
        const char* e = getenv("PM_JIT_PREFETCH");
        const int b = e ? atoi(e) : 0;
        return b == 64 || b == 128 || b == 256 ? b : 0;
    }();
    return v;
}

// PM_JIT_CLOCK: a ring of per-launch sample buffers (a pipelined query is
// resolved after the next one launched), and the report of one launch
uint64_t* clock_buffer(int device, uint64_t nwg) {
    static std::mutex mu;
    static std::map<int, std::pair<std::vector<uint64_t*>, size_t>> rings;   // device -> (buffers, next)
    std::lock_guard<std::mutex> lk(mu);
    auto& r = rings[device];
    constexpr size_t N = 16, CAP = 3 * 65536;   // workgroups per launch at most (nwg <= 256 CUs x 4 x 8 x ...)
    require(nwg <= 65536, "PM_JIT_CLOCK: too many workgroups");
    if (r.first.empty()) {
        r.first.resize(N);
        for (auto& p : r.first) HIPCHK(hipMalloc(&p, CAP * sizeof(uint64_t)));
    }
    uint64_t* p = r.first[r.second];
    r.second = (r.second + 1) % N;
    return p;
}

void clock_report(const uint64_t* d, uint64_t nwg, double kms) {
    std::vector<uint64_t> h(3 * nwg);
    HIPCHK(hipMemcpy(h.data(), d, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    double cyc = 0, ticks = 0, lo = 1e9, hi = 0;
    uint64_t t_first = ~0ull, t_last = 0;
    for (uint64_t i = 0; i < nwg; ++i) {
        if (!h[3 * i + 1]) continue;
        cyc += (double)h[3 * i];
        ticks += (double)h[3 * i + 1];
        const double g = (double)h[3 * i] / (double)h[3 * i + 1] * 0.1;   // 100 MHz ticks -> GHz
        lo = std::min(lo, g);
        hi = std::max(hi, g);
        t_first = std::min(t_first, h[3 * i + 2]);
        t_last = std::max(t_last, h[3 * i + 2] + h[3 * i + 1]);
    }
    fprintf(stderr, "PM_JIT_CLOCK nwg=%llu kernel_ms=%.4f clock_ghz=%.4f min=%.3f max=%.3f span_ms=%.4f t0_tick=%llu\n",
            (unsigned long long)nwg, kms, ticks > 0 ? cyc / ticks * 0.1 : 0.0, lo, hi,
            (double)(t_last - t_first) * 1e-5, (unsigned long long)t_first);
}

std::string gen_linear_source(int P, int K, const int32_t* lengths, const uint8_t* pos_class,
                              const uint8_t* class_acgt, const uint8_t* class_is_any, int waves, int parts) {
    const int PARTS = parts;                     // waves per workgroup
    const int JIT_STEPS = LANE_WORDS / parts;    // window words per lane and wave
    // LDS tile buffers: 2 (the next tile streams in while this one is
    // scanned) leave room for 4 workgroups per CU, which measured 10 %
    // faster than 3 buffers at 3 workgroups per CU (profiles/r01c_ring_sweep.txt)
    constexpr int RING = 2;
    const int TILE_BYTES = (int)(TILE_WORDS * 8);         // 16896: 16.5 KiB
    const int DMA_PIECES = (TILE_BYTES + 1023) / 1024;   // 1 KiB per glds wave-instruction (last one half)
    const int LDS_TILE = TILE_BYTES;
    std::ostringstream o;
    o << kJitCommon;
    o << "#define P " << P << "\n#define K " << K << "\n#define REC_LDS " << JIT_REC_LDS << "\n#define STEPS "
      << JIT_STEPS << "\n#define NW " << PARTS << "\n#define JIT_CLOCK " << (jit_clock() ? 1 : 0)
      << "\n#define JIT_M0_CLOBBER " << (jit_m0() ? 1 : 0) << "\n";
    auto word_off = [&](int i) {   // physical word of logical word 32 lane + i, relative to the tile
        std::ostringstream s;
        if (i < LANE_WORDS) s << (i * 64) << " + lane";
        else if (i < 2 * LANE_WORDS) s << "hb1 + " << (i - 32) << " * hs1";
        else s << "hb2 + " << (i - 64) << " * hs2";
        return s.str();
    };
    int Lmax = 0;
    for (int p = 0; p < P; ++p) Lmax = std::max(Lmax, (int)lengths[p]);
    // Class words are pinned in registers (derived once per row); unpinned,
    // the compiler re-derives them per use and keeps the plane words of every
    // row alive instead, which measured worse for every shape (round 1).
    // Shared blocks.  Two patterns whose class sequences agree on a run of
    // positions at some offset -- the strands of a (near-)palindromic motif:
    // TGCTGA[GC]TCAGCA.[AT] and its reverse complement agree on 13 positions
    // at offset 2, restriction sites on all of them -- read the same
    // (row, class) words for those positions at steps `off` apart, so the
    // carry-save count of the block is built once per row and both windows
    // only add their own positions (a 13-position block at k = 2: 17 ops
    // once, then 3 per window, instead of 19 per window).  Greedy pairing,
    // each pattern in at most one pair; a pair pays when the block is large
    // and the offset small against the wave's 8 steps.
    std::vector<int> shift;
    const std::vector<std::vector<int>> block =
        shared_blocks(P, lengths, pos_class, class_acgt, class_is_any, JIT_STEPS, &shift);
    // Shifted members (shift[p] > 0) are scanned at steps [t0 + shift,
    // t1 + shift) so their blocks coincide with the partner's.  The last
    // wave's steps past 31 are the next lane's first words (for lane 63 the
    // next stream's; bit 31 -- the next tile -- is left to that tile); the
    // first wave adds the words [0, shift) of lane 0, bit 0 only (the
    // tile's own stream 0).  dd[STEPS + e] holds those extras.
    int XS = 0;
    for (int p = 0; p < P; ++p) XS = std::max(XS, shift[p]);
    // a shifted window reads logical words up to LANE_WORDS + XS + Lmax - 2;
    // k_lane_flags (pm_db.hip) flags a lane for exceptions in words
    // [32 l, 32 l + LANE_WORDS + HALO - 1) only, and the expansion's break /
    // other kill runs only for flagged lanes, so a window must stay inside
    // that span (a 61-64-mer shifted pair would read word 95): no shifts
    if (LANE_WORDS + XS + Lmax - 1 > LANE_WORDS + HALO - 1) {
        shift.assign(P, 0);
        XS = 0;
    }
    o << "#define XS " << std::max(XS, 1) << "\n";
    o << "__device__ constexpr int SHIFT[P] = {";
    for (int p = 0; p < P; ++p) o << (p ? ", " : "") << shift[p];
    o << "};\n";
    for (int part = 0; part < PARTS; ++part) {
        const int t0 = part * JIT_STEPS, t1 = t0 + JIT_STEPS;
        const int wend = t1 + XS + Lmax - 1;   // words [0, wend)
        o << "__device__ __forceinline__ void tile_body" << part
          << "(const uint2* __restrict__ sw, int lane, u32 hb1, u32 hs1, u32 hb2, u32 hs2, u32 (&dd)[STEPS + XS][P]) {\n";
        std::vector<bool> loaded(wend, false);
        std::map<std::pair<int, int>, std::string> cw;   // (word, ACGT subset) -> class word
        auto class_word = [&](int i, int subset) {
            const auto key = std::make_pair(i, subset);
            auto it = cw.find(key);
            if (it != cw.end()) return it->second;
            if (!loaded[i]) {
                loaded[i] = true;
                o << "  const uint2 v" << i << " = sw[" << word_off(i) << "];\n";
            }
            const std::string nm = "x" + std::to_string(subset) + "_" + std::to_string(i);
            o << "  u32 " << nm << " = "
              << subset_expr(subset, "v" + std::to_string(i) + ".x", "v" + std::to_string(i) + ".y") << ";"
              << " PIN(" + nm + ");" << "\n";
            cw[key] = nm;
            return nm;
        };
        int uid = 0;
        std::map<std::vector<std::string>, CountNet> blocks;   // block inputs -> its compressed count
        // (slot, word) of every window word this wave evaluates, per pattern
        std::vector<std::tuple<int, int, int>> work;   // (dd slot, pattern, word)
        for (int s = 0; s < JIT_STEPS; ++s)
            for (int p = 0; p < P; ++p) work.emplace_back(s, p, t0 + s + shift[p]);
        if (part == 0)
            for (int p = 0; p < P; ++p)
                for (int e = 0; e < shift[p]; ++e) work.emplace_back(JIT_STEPS + e, p, e);
        std::vector<std::vector<bool>> set(JIT_STEPS + std::max(XS, 1), std::vector<bool>(P, false));
        for (const auto& wk : work) {
            {
                const int slot = std::get<0>(wk), p = std::get<1>(wk), t = std::get<2>(wk);
                set[slot][p] = true;
                const uint8_t* pc = pos_class + 64 * p;
                std::vector<std::string> in, bin;
                for (int j = 0, b = 0; j < lengths[p]; ++j) {
                    if (class_is_any[pc[j]]) continue;
                    const bool shared = b < (int)block[p].size() && block[p][b] == j;
                    b += shared;
                    (shared ? bin : in).push_back(class_word(t + j, class_acgt[pc[j]] & 15));
                }
                CountNet n;
                if (!bin.empty()) {   // the block's count, at function scope (the partner reuses it)
                    auto it = blocks.find(bin);
                    if (it == blocks.end()) {
                        o << "  // shared block, rows " << t + block[p].front() << ".." << t + block[p].back() << "\n";
                        CountNet b;
                        net_add(o, b, bin, K, uid, "  ");
                        if (b.dead.size() > 1) b.dead = {emit_or(o, b.dead, uid, "  ")};
                        it = blocks.emplace(bin, b).first;
                    }
                    n = it->second;
                }
                o << "  {  // step " << t << ", pattern " << p << "\n";
                net_add(o, n, in, K, uid, "    ");
                const std::string d = net_dead(o, n, K, uid, "    ");
                std::string mask;
                if (slot >= JIT_STEPS) mask = " | (lane == 0 ? 0xFFFFFFFEu : 0xFFFFFFFFu)";   // lane 0, bit 0 only
                else if (t >= LANE_WORDS) mask = " | (lane == 63 ? 0x80000000u : 0u)";     // the next tile's: its own
                o << "    dd[" << slot << "][" << p << "] = " << d << mask << ";\n  }\n";
            }
        }
        for (size_t slot = 0; slot < set.size(); ++slot)
            for (int p = 0; p < P; ++p)
                if (!set[slot][p]) o << "  dd[" << slot << "][" << p << "] = ~0u;\n";
        o << "}\n";
    }
    // `waves`: __launch_bounds__ minimum workgroups per CU (4 -> at most
    // 128 VGPRs; jit_function falls back to 3 when that would spill)
    // bytes DMA'd per tile: the 2048 words and only the halo words a window
    // reads (Lmax - 1 of the 64) -- ~2 % fewer HBM lines per tile for a
    // 15-mer (round 2: 1.036 -> 1.012 x algorithmic traffic)
    int XSh = 0;   // (the generator's shift, recomputed: the halo words the shifted windows read)
    {
        std::vector<int> sh;
        shared_blocks(P, lengths, pos_class, class_acgt, class_is_any, JIT_STEPS, &sh);
        for (int v : sh) XSh = std::max(XSh, v);
        if (LANE_WORDS + XSh + Lmax - 1 > 3 * LANE_WORDS) XSh = 0;
    }
    const int halo_used = std::min(HALO, std::max(1, Lmax - 1 + XSh));
    const int LOAD_BYTES = std::min(TILE_BYTES, (int)(((STREAM + halo_used) * 8 + 15) / 16 * 16));
    const int LOAD_PIECES = (LOAD_BYTES + 1023) / 1024;
    (void)DMA_PIECES;
    o << "#define RING " << RING << "\n#define LDS_TILE " << LDS_TILE << "\n#define DMA_PIECES " << LOAD_PIECES
      << "\n#define LOAD_BYTES " << LOAD_BYTES << "\n#define PF_STRIDE " << jit_prefetch() << "\n";
    o << R"JIT(// Raw barrier: __syncthreads()'s release fence would wait vmcnt(0) and
// drain the tile prefetch in flight.  LDS writes are complete at
// lgkmcnt(0); the empty asm statements keep the compiler from moving memory
// accesses across.
#define BARRIER()                                                   \
  do {                                                              \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");              \
    __builtin_amdgcn_s_barrier();                                   \
    asm volatile("" ::: "memory");                                  \
  } while (0)
// DMA tile t into the ring slot at LDS byte address `dst0`: DMA_PIECES 1-KiB
// pieces, piece q issued by wave q % NW (lane-linear LDS image of the tile).
// Inline asm so that the compiler's wait bookkeeping does not drain it
// before the ds_reads of the slot being computed; waited for explicitly.
__device__ __forceinline__ void stage(const JArgs& a, u32 dst0, u64 tile, u64 tend, u32 wid, int lane) {
  if (tile >= tend) return;
  // scalar base (SGPR pair, SALU arithmetic) + the lane's constant 16-byte
  // offset: no VALU address math per piece
  const unsigned char* tb = reinterpret_cast<const unsigned char*>(a.hl + tile * TILE_WORDS);
  const u32 voff = (u32)lane * 16u;
#pragma unroll
  for (int q = 0; q < DMA_PIECES; q += NW) {
    if (q + (int)wid >= DMA_PIECES) break;
    if ((q + (int)wid + 1) * 1024 > LOAD_BYTES && lane * 16 >= LOAD_BYTES % 1024) continue;   // partial last piece
    const u32 dst = __builtin_amdgcn_readfirstlane(dst0 + (q + wid) * 1024);
    const unsigned char* pb = tb + (q + wid) * 1024;
#if JIT_M0_CLOBBER   // m0 a declared clobber: no save / restore around the DMA
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" : : "v"(voff), "s"(pb), "s"(dst)
                 : "memory", "m0");
#else
    u32 keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(pb), "s"(dst) : "memory");
#endif
  }
}
#if PF_STRIDE
// PM_JIT_PREFETCH: one dword per PF_STRIDE bytes of tile t into the dummy
// row at LDS byte address `dst` (no VGPR destination; waited for with the
// DMAs by the loop's vmcnt(0))
__device__ __forceinline__ void prefetch(const JArgs& a, u32 dst, u64 tile, u64 tend, u32 wid, int lane) {
  if (tile >= tend) return;
  const unsigned char* tb = reinterpret_cast<const unsigned char*>(a.hl + tile * TILE_WORDS);
  constexpr int LINES = (LOAD_BYTES + PF_STRIDE - 1) / PF_STRIDE;
  const u32 d = __builtin_amdgcn_readfirstlane(dst);
#pragma unroll
  for (int q = 0; q * 64 < LINES; q += NW) {
    if ((q + (int)wid) * 64 >= LINES) break;
    if ((q + (int)wid) * 64 + lane >= LINES) continue;
    const u32 voff = (u32)(((q + (int)wid) * 64 + lane) * PF_STRIDE);
    u32 keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(tb), "s"(d) : "memory");
  }
}
#endif
// Moves the wave's staged records to its global segment.  Rare; ends with
// vmcnt(0), so the DMA wait arithmetic of the main loop stays exact whatever
// order stores and loads retire in.
__device__ __noinline__ void flush_records(const lds_uint2* st, u32 n, glb_uint2* g,
                                           u32 gcnt, u32 rcap, int lane) {
  for (u32 r = lane; r < n; r += 64)
    if (gcnt + r < rcap) g[gcnt + r] = st[r];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
)JIT";
    o << "extern \"C\" __global__ __launch_bounds__(" << 64 * PARTS << ", " << std::max(1, waves * PARTS / 4)
      << ") void pm_linear_jit(JArgs a) {\n"
         "  __shared__ __attribute__((aligned(1024))) unsigned char lds[RING * LDS_TILE];\n"
         "  __shared__ uint2 rst[NW][REC_LDS];\n"
         "  const int lane = threadIdx.x & 63;\n"
         "  const u32 wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n"
         "#if JIT_CLOCK\n"
         "  const u64 clk_c0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();\n"
         "#endif\n"
         "  // halo word offsets (logical words 32 lane + 32 g + r, r < 32)\n"
         "  const u32 hb1 = lane + 1 < 64 ? lane + 1 : 32u * lane + 32u, hs1 = lane + 1 < 64 ? 64u : 1u;\n"
         "  const u32 hb2 = lane + 2 < 64 ? lane + 2 : 32u * lane + 64u, hs2 = lane + 2 < 64 ? 64u : 1u;\n"
         "  const u32 lds_base = (u32)reinterpret_cast<u64>(lds);   // LDS byte address (low bits of the flat address)\n"
         "  // this workgroup's contiguous tile range (the graded tail's are shorter)\n"
         "  u64 t0, tlim;\n"
         "  if (blockIdx.x < a.nA) {\n"
         "    t0 = (u64)blockIdx.x * a.tiles_per_wg;\n"
         "    tlim = t0 + a.tiles_per_wg;\n"
         "  } else {\n"
         "    const u32 j = blockIdx.x - a.nA, sg = j / a.groupB;\n"
         "    const u64 s0 = a.tilesA + (u64)sg * a.tpo;\n"
         "    t0 = s0 + (u64)(j - sg * a.groupB) * a.tpwB;\n"
         "    tlim = t0 + a.tpwB < s0 + a.tpo ? t0 + a.tpwB : s0 + a.tpo;\n"
         "  }\n"
         "  const u64 tend = tlim < a.ntiles ? tlim : a.ntiles;   // empty for a last segment's spare workgroups\n"
         "  glb_uint2* grec = (glb_uint2*)(a.rec + ((u64)blockIdx.x * NW + wid) * a.rcap);\n"
         "  lds_uint2* st = (lds_uint2*)(size_t)(u32)reinterpret_cast<u64>(&rst[wid][0]);\n"
         "  u32 scnt = 0, gcnt = 0;   // staged / flushed records (wave-uniform)\n"
         "  if (a.aux_zero && blockIdx.x == 0 && threadIdx.x == 0) *a.aux_zero = 0u;   // read by k_linear_expand (after)\n"
         "  stage(a, lds_base, t0, tend, wid, lane);\n"
         "  stage(a, lds_base + LDS_TILE, t0 + 1, tend, wid, lane);\n"
         "#if PF_STRIDE\n"
         "  __shared__ u32 pfd[64];\n"
         "  const u32 pf_base = (u32)reinterpret_cast<u64>(pfd);\n"
         "  prefetch(a, pf_base, t0 + RING, tend, wid, lane);\n"
         "#endif\n"
         "  u32 slot = 0;\n"
         "  for (u64 tile = t0; tile < tend; ++tile) {\n"
         "    // wait for this tile's pieces (own DMAs), then the barrier makes\n"
         "    // everyone's pieces visible and frees the previous tile's slot\n"
         "    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n"
         "    BARRIER();\n"
         "    stage(a, lds_base + (slot == 0 ? RING - 1 : slot - 1) * LDS_TILE, tile + RING - 1, tend, wid, lane);\n"
         "#if PF_STRIDE\n"
         "    prefetch(a, pf_base, tile + RING, tend, wid, lane);\n"
         "#endif\n"
         "    const uint2* sw = reinterpret_cast<const uint2*>(lds + slot * LDS_TILE);\n"
         "    u32 dd[STEPS + XS][P];   // dead windows per slot and pattern (every path writes all of them)\n";
    // The parts rotate over the waves from tile to tile: part 0 (the words
    // the shifted partner adds) is the longest, and a workgroup's waves sit
    // on different SIMDs -- a fixed part 0 would load one SIMD more than the
    // others, which then idle at the tile barrier.  b < PARTS: the last part
    // is the plain else (no ~0 initialization of dd).
    o << (jit_rotate() ? "    const u32 b = (wid + (u32)tile) % NW;   // this tile's part for the wave (wave-uniform)\n"
                       : "    const u32 b = wid;\n");
    for (int part = 0; part < PARTS; ++part)
        o << "    " << (part ? "else " : "") << (part + 1 < PARTS ? "if (b == " + std::to_string(part) + ") " : "")
          << "tile_body" << part << "(sw, lane, hb1, hs1, hb2, hs2, dd);\n";
    o << "    const u32 S0 = b * STEPS;   // the part's first window word\n"
         "    u32 all = ~0u;\n"
         "#pragma unroll\n    for (int s = 0; s < STEPS + XS; ++s)\n#pragma unroll\n      for (int p = 0; p < P; ++p) all &= dd[s][p];\n"
         "    if (__builtin_expect(__builtin_amdgcn_ballot_w64(all != ~0u) != 0, 0)) {   // wave-uniform, rare\n"
         "#pragma unroll\n"
         "      for (int s = 0; s < STEPS + XS; ++s) {\n"
         "#pragma unroll\n"
         "        for (int p = 0; p < P; ++p) {\n"
         "          const u32 lv = ~dd[s][p];\n"
         "          const u64 m = __builtin_amdgcn_ballot_w64(lv != 0u);\n"
         "          if (m) {\n"
         "            const u32 below = __builtin_amdgcn_mbcnt_hi((u32)(m >> 32), __builtin_amdgcn_mbcnt_lo((u32)m, 0u));\n"
         "            const u32 word = s < STEPS ? S0 + s + SHIFT[p] : s - STEPS;   // the window word (may pass 31)\n"
         "            if (lv) st[scnt + below] = make_uint2((u32)(tile - t0) << 15 | (u32)lane << 9 | word << 3 | (u32)p, lv);\n"
         "            scnt += (u32)__builtin_popcountll(m);\n"
         "            if (scnt > REC_LDS - 64) {\n"
         "              flush_records(st, scnt, grec, gcnt, a.rcap, lane);\n"
         "              gcnt += scnt;\n"
         "              scnt = 0;\n"
         "            }\n"
         "          }\n"
         "        }\n"
         "      }\n"
         "    }\n"
         "    slot = slot == RING - 1 ? 0 : slot + 1;\n  }\n"
         "  if (scnt) flush_records(st, scnt, grec, gcnt, a.rcap, lane);\n"
         "  if (lane == 0) a.rec_cnt[(u64)blockIdx.x * NW + wid] = gcnt + scnt;\n"
         "#if JIT_CLOCK\n"
         "  if (threadIdx.x == 0 && a.clk) {\n"
         "    const u64 c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();\n"
         "    a.clk[3 * (u64)blockIdx.x] = c1 - clk_c0;\n"
         "    a.clk[3 * (u64)blockIdx.x + 1] = r1 - clk_r0;\n"
         "    a.clk[3 * (u64)blockIdx.x + 2] = clk_r0;\n"
         "  }\n"
         "#endif\n"
         "}\n";
    return o.str();
}

#define RTCCHK(expr)                                                                      \
    do {                                                                                  \
        hiprtcResult r_ = (expr);                                                         \
        if (r_ != HIPRTC_SUCCESS)                                                         \
            throw failure(PM_E_HIP, std::string(#expr) + ": " + hiprtcGetErrorString(r_)); \
    } while (0)

std::vector<char> jit_compile(const std::string& src) {
    if (const char* dump = getenv("PM_JIT_DUMP")) {      // debugging: keep the generated source
        if (FILE* f = fopen(dump, "w")) {
            fwrite(src.data(), 1, src.size(), f);
            fclose(f);
        }
    }
    hiprtcProgram prog;
    RTCCHK(hiprtcCreateProgram(&prog, src.c_str(), "pm_linear_jit.hip", 0, nullptr, nullptr));
    const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
    hiprtcResult rc = hiprtcCompileProgram(prog, 3, opts);
    if (rc != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n, '\0');
        if (n) hiprtcGetProgramLog(prog, &log[0]);
        hiprtcDestroyProgram(&prog);
        throw failure(PM_E_HIP, "hipRTC compile failed: " + log.substr(0, 2000));
    }
    size_t n = 0;
    RTCCHK(hiprtcGetCodeSize(prog, &n));
    std::vector<char> code(n);
    RTCCHK(hiprtcGetCode(prog, code.data()));
    hiprtcDestroyProgram(&prog);
    if (const char* dump = getenv("PM_JIT_DUMP_CO")) {   // debugging: keep the code object
        if (FILE* f = fopen(dump, "wb")) {
            fwrite(code.data(), 1, code.size(), f);
            fclose(f);
        }
    }
    return code;
}

// Specialized kernels, cached per device by the batch's signature (pattern
// lengths, class subsets and '.' flags per position, k, and the PM_JIT_*
// experiment knobs): the generated source (~100 KB) is built and compiled
// only on a miss.
std::string jit_signature(int P, int K, const int32_t* lengths, const uint8_t* pos_class, const uint8_t* class_acgt,
                          const uint8_t* class_is_any) {
    std::string sig = std::to_string(P) + ":" + std::to_string(K) + ":";
    for (int p = 0; p < P; ++p) {
        sig += std::to_string(lengths[p]) + "[";
        for (int j = 0; j < lengths[p]; ++j) {
            const int c = pos_class[64 * p + j];
            sig += class_is_any[c] ? '.' : (char)('a' + (class_acgt[c] & 15));
        }
        sig += "]";
    }
    return sig;
}

hipFunction_t jit_function(int device, int P, int K, const int32_t* lengths, const uint8_t* pos_class,
                           const uint8_t* class_acgt, const uint8_t* class_is_any) {
    const int parts = jit_parts();
    const auto key = std::make_pair(device, std::to_string(parts) + (jit_rotate() ? "r/" : "f/") +
                                                (jit_clock() ? "c/" : "") + (jit_m0() ? "" : "m0s/") + "pf" + std::to_string(jit_prefetch()) + "/" +
                                                jit_signature(P, K, lengths, pos_class, class_acgt, class_is_any));
    std::lock_guard<std::mutex> lk(g_jit_mu);
    auto it = g_jit_cache.find(key);
    if (it != g_jit_cache.end()) return it->second.fn;
    // 4 workgroups per CU when the kernel fits 128 VGPRs without spilling,
    // else 3 (up to 168 VGPRs)
    JitKernel jk;
    for (int waves = JIT_WG_PER_CU; waves >= 1; --waves) {
        std::vector<char> code =
            jit_compile(gen_linear_source(P, K, lengths, pos_class, class_acgt, class_is_any, waves, parts));
        if (jk.module) HIPCHK(hipModuleUnload(jk.module));
        HIPCHK(hipModuleLoadData(&jk.module, code.data()));
        HIPCHK(hipModuleGetFunction(&jk.fn, jk.module, "pm_linear_jit"));
        int scratch = 0;
        HIPCHK(hipFuncGetAttribute(&scratch, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, jk.fn));
        if (scratch == 0 || waves <= 3) break;
    }
    g_jit_cache[key] = jk;
    return jk.fn;
}

// Segment / record capacities per (database, batch) that held all hits
// last time.
std::mutex g_cap_mu;
std::map<std::pair<const pm_db*, std::string>, std::pair<std::vector<uint32_t>, uint32_t>> g_cap_hint;
std::map<std::pair<const pm_db*, std::string>, uint32_t> g_ord_hint;   // the ordered batch verify's list capacity

// PM_JIT: "0" never, "1" always, default: databases of >= 64 Mi positions
bool use_jit(const pm_db* db) {
    const char* e = getenv("PM_JIT");
    if (e && e[0] == '0') return false;
    if (e && e[0] == '1') return true;
    return db->n >= (64ull << 20);
}

}  // namespace
}  // namespace pm

using namespace pm;

namespace {

// (database, batch) whose hit bins outgrew the LDS sort: pipelined scans of
// it run synchronously (the speculative list would be re-done every time)
std::mutex g_nospec_mu;
std::set<std::pair<const pm_db*, std::string>> g_nospec;

// q-gram batch indexes by batch signature (host), and the device image of
// the last one per database (ws_batch): a repeated batch rebuilds and
// uploads nothing
std::mutex g_bidx_mu;
std::map<std::string, std::shared_ptr<const BatchIndex>> g_bidx;   // null: not for the filter

std::shared_ptr<const BatchIndex> batch_index_cached(const std::string& sig, int P, const int32_t* lengths,
                                                     const uint8_t* pos_class, const uint8_t* class_acgt,
                                                     const uint8_t* class_is_any) {
    {
        std::lock_guard<std::mutex> lk(g_bidx_mu);
        auto it = g_bidx.find(sig);
        if (it != g_bidx.end()) return it->second;
    }
    auto bi = std::make_shared<BatchIndex>();
    std::shared_ptr<const BatchIndex> r;
    if (build_batch_index(P, lengths, pos_class, class_acgt, class_is_any, *bi)) r = bi;
    std::lock_guard<std::mutex> lk(g_bidx_mu);
    if (g_bidx.size() > 64) g_bidx.clear();
    g_bidx[sig] = r;
    return r;
}

uint8_t* batch_tables(pm_db* db, const BatchIndex& bi, const std::string& sig) {
    if (db->batch_sig == sig && db->ws_batch.p) return static_cast<uint8_t*>(db->ws_batch.p);
    // queued scans may still read the old tables
    HIPCHK(hipStreamSynchronize(db->stream));
    if (db->post) HIPCHK(hipStreamSynchronize(db->post));
    uint8_t* d = static_cast<uint8_t*>(reserve(db, db->ws_batch, bi.bytes));
    std::vector<uint8_t> img(bi.bytes, 0);
    memcpy(img.data() + bi.o_table, bi.table.data(), bi.table.size() * 4);
    memcpy(img.data() + bi.o_code, bi.code_off.data(), bi.code_off.size() * 4);
    memcpy(img.data() + bi.o_ents, bi.ents.data(), bi.ents.size() * 4);
    memcpy(img.data() + bi.o_pmask, bi.pmask.data(), bi.pmask.size() * 4);
    memcpy(img.data() + bi.o_popt, bi.popt.data(), bi.popt.size() * 4);
    if (!bi.hash.empty()) memcpy(img.data() + bi.o_hash, bi.hash.data(), bi.hash.size() * 8);
    HIPCHK(hipMemcpyAsync(d, img.data(), img.size(), hipMemcpyHostToDevice, db->stream));
    HIPCHK(hipStreamSynchronize(db->stream));
    db->batch_sig = sig;
    return d;
}

// k > 0 with nrgrep's report: every pattern of the batch is a class
// sequence searched by nrgrep's esimple engine; its plan and tables
bool linear_esimple(int n_patterns, const int32_t* lengths, const uint8_t* pos_class, const uint32_t* class_bytes,
                    int k, uint32_t flags, EsBuild& esb) {
    if (k == 0 || !(flags & PM_REPORT_NRGREP)) return false;
    std::vector<uint64_t> B(256);
    for (int p = 0; p < n_patterns; ++p) {
        std::fill(B.begin(), B.end(), 0ull);
        for (int j = 0; j < lengths[p]; ++j) {
            const uint32_t* cb = class_bytes + 8 * pos_class[64 * p + j];
            for (int c = 0; c < 256; ++c)
                if ((cb[c >> 5] >> (c & 31)) & 1) B[c] |= 1ull << j;
        }
        es_add_slot(esb, B.data(), 1, lengths[p], k, PM_ERR_SUB, flags, p);
    }
    return true;
}

// pm_scan_linear on the byte layout (synchronous; the pipelined entry point
// runs it too)
void scan_linear_bytes(pm_db* db, int n_patterns, const int32_t* lengths, const uint8_t* pos_class, int n_classes,
                       const uint32_t* class_bytes, const uint8_t* class_is_any, int k, uint32_t flags, bool cross,
                       pm_hits** out) {
    require(n_patterns <= (int)MAX_BINS, "too many patterns for one byte-layout scan", PM_E_UNSUPPORTED);
    hipStream_t s = db->stream;
    lane_begin(db);
    Upload up;
    const size_t o_cb = up.add(class_bytes, (size_t)n_classes * 32);
    const size_t o_len = up.add(lengths, (size_t)n_patterns * 4);
    const size_t o_pc = up.add(pos_class, (size_t)n_patterns * 64);
    const size_t o_any = up.add(class_is_any, (size_t)n_classes);
    EsBuild esb;
    EsUpload esu;
    const bool esimple = linear_esimple(n_patterns, lengths, pos_class, class_bytes, k, flags, esb);
    if (esimple) es_upload(esb, up, esu);
    // the 5-bit residue planes when the batch's classes fit the kernel
    P5Args pa{};
    const int maxlen = *std::max_element(lengths, lengths + n_patterns);
    bool p5 = db->p5 && !(flags & PM_SCAN_BYTES) && k <= 3 && maxlen <= 64;
    std::vector<uint8_t> cls, pidx((size_t)n_patterns * 64, 255);
    if (p5) {
        std::map<int, int> idx;   // class id -> distinct index
        for (int q = 0; q < n_patterns && p5; ++q)
            for (int j = 0; j < lengths[q] && p5; ++j) {
                const int c = pos_class[64 * q + j];
                if (class_is_any[c]) continue;   // every residue but code 0
                auto it = idx.find(c);
                if (it == idx.end()) {
                    if ((int)idx.size() == P5_MAX_CLS) {
                        p5 = false;
                        break;
                    }
                    it = idx.emplace(c, (int)idx.size()).first;
                }
                pidx[(size_t)64 * q + j] = (uint8_t)it->second;
            }
        if (p5) {
            cls.assign(idx.size() * (2 + P5_LIST), 0);
            for (const auto& kv : idx) {
                uint32_t in = 0;   // the class's codes (bytes absent from the file have none)
                for (int b = 0; b < 256; ++b)
                    if (((class_bytes[8 * kv.first + b / 32] >> (b % 32)) & 1) && db->code_of[b]) in |= 1u << db->code_of[b];
                const uint32_t uni = db->n_codes >= 31 ? ~0u : (2u << db->n_codes) - 1u;   // codes 0..n_codes occur
                const bool comp = __builtin_popcount(in) > __builtin_popcount(uni & ~in);
                const uint32_t list = comp ? uni & ~in : in;
                uint8_t* e = &cls[(size_t)kv.second * (2 + P5_LIST)];
                e[0] = (uint8_t)__builtin_popcount(list);
                e[1] = comp ? 1 : 0;
                int t = 0;
                for (int x = 0; x < 32; ++x)
                    if ((list >> x) & 1) e[2 + t++] = (uint8_t)x;
            }
            pa.C = (int)idx.size();
        }
    }
    size_t o_cls = 0, o_pidx = 0;
    if (p5) {
        o_cls = up.add(cls.data(), std::max<size_t>(cls.size(), 1));
        o_pidx = up.add(pidx.data(), pidx.size());
    }

    uint8_t* d_up = up.commit(db);
    const EsPrep esp = esimple ? es_bind(esu, d_up, es_gap(esb)) : EsPrep{};
    ByteLinArgs a{db->bytes, db->bytes_raw, db->n, d_up + o_pc, reinterpret_cast<const int32_t*>(d_up + o_len),
                  d_up + o_any, reinterpret_cast<const uint32_t*>(d_up + o_cb), n_patterns, k, cross ? 1 : 0, Sink{}};
    if (p5) {
        pa.p5 = db->p5;
        pa.nw = db->nw5;
        pa.nwords = (db->n + 31) / 32;
        pa.cls = d_up + o_cls;
        pa.pidx = d_up + o_pidx;
        pa.lengths = reinterpret_cast<const int32_t*>(d_up + o_len);
        pa.P = n_patterns;
        pa.k = k;
    }
    uint64_t expected = std::max<uint64_t>(db->n / 64, 1 << 16);
    SinkBuffers sb;
    std::vector<uint32_t> counts;
    uint64_t total = 0;
    EventPair ev;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(blocks_for(db->n, 256), 256 * 64);
    for (int attempt = 0; attempt < 2; ++attempt) {
        sb = make_sink(db, n_patterns, db->n, expected);
        a.sink = sb.sink();
        pa.sink = sb.sink();
        HIPCHK(hipEventRecord(ev.a, s));
        if (p5) {
            const uint32_t b5 = (uint32_t)std::min<uint64_t>(blocks_for(pa.nwords, P5_T), 256 * 16);
            auto kern = maxlen <= 32 ? (cross ? k_p5_linear<2, true> : k_p5_linear<2, false>)
                                     : (cross ? k_p5_linear<3, true> : k_p5_linear<3, false>);
            hipLaunchKernelGGL(kern, dim3(b5), dim3(P5_T), 0, s, pa);
            if (cross && db->nhdr) {
                HIPCHK(hipGetLastError());
                P5FixArgs fa{db->bytes_raw, db->n, db->hdr, db->hdr_end, db->nhdr, d_up + o_pc,
                             reinterpret_cast<const int32_t*>(d_up + o_len), d_up + o_any,
                             reinterpret_cast<const uint32_t*>(d_up + o_cb), n_patterns, k, pa.sink};
                hipLaunchKernelGGL(k_p5_cross_fix, dim3((uint32_t)std::min<uint64_t>(db->nhdr, 65536)), dim3(64), 0, s, fa);
            }
        } else {
            hipLaunchKernelGGL(k_bytes_linear, dim3(blocks), dim3(256), 0, s, a);
        }
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ev.b, s));
        bool overflow = false;
        total = sink_total(db, sb, counts, overflow);
        if (!overflow) break;
        require(attempt == 0, "internal: hit bins overflowed twice");
        expected = (uint64_t)(*std::max_element(counts.begin(), counts.end())) * sb.nbins + sb.nbins;
    }
    bool lens_done = false;
    pm_hits* h = sink_to_hits(db, sb, counts, total, reinterpret_cast<const int32_t*>(d_up + o_len), &lens_done);
    h->kernel_ms = ev.ms();
    if (total && !lens_done) {
        hipLaunchKernelGGL(k_linear_lens, dim3(blocks_for(total, 256)), dim3(256), 0, s, h->keys, total,
                           reinterpret_cast<const int32_t*>(d_up + o_len), h->lens);
        HIPCHK(hipGetLastError());
    }
    if (report_needed(db, flags, cross)) report_sync(db, h, flags, total, cross, esimple ? &esp : nullptr);
    hits_ready(db, h);
    *out = h;
}

// pm_scan_linear (async = false) and pm_scan_linear_async: the specialized
// path launches the scan, record expansion, the speculative sort and the
// count readback, and returns a pending hit list without a host sync.
void scan_linear_impl(pm_db* db, int n_patterns, const int32_t* lengths, const uint8_t* pos_class, int n_classes,
                      const uint8_t* class_acgt, const uint32_t* class_bytes, const uint8_t* class_is_any, int k,
                      uint32_t flags, pm_hits** out, bool async) {
    {
        require(db != nullptr && out != nullptr && lengths && pos_class && class_acgt && class_bytes && class_is_any,
                "null argument");
        require(n_patterns >= 1 && n_patterns <= 4096, "n_patterns out of range");
        require(n_classes >= 1 && n_classes <= 256, "n_classes out of range");
        require(k >= 0 && k <= PM_MAX_LINEAR_K, "k out of range for the GPU kernels", PM_E_UNSUPPORTED);
        for (int p = 0; p < n_patterns; ++p) {
            require(lengths[p] >= 1 && lengths[p] <= PM_MAX_LINEAR_POSITIONS, "pattern length out of range");
            for (int j = 0; j < lengths[p]; ++j) require(pos_class[64 * p + j] < n_classes, "class id out of range");
        }
        require((flags & ~(uint32_t)(PM_REPORT_NRGREP | PM_ANCHOR_START | PM_ANCHOR_END | PM_KEEP_HEADERS | PM_ESIMPLE | PM_SCAN_BYTES)) ==
                    0,
                "bad flags");
        DeviceGuard g(db->device);
        hipStream_t s = db->stream;
        const bool jit = use_jit(db);
        // k = 0: nrgrep's simple engine, whose windows may span lines when a
        // class accepts the delimiter (k_linear_others)
        bool cross = false;
        if (k == 0)
            for (int c = 0; c < n_classes; ++c) cross |= ((class_bytes[8 * c] >> '\n') & 1) != 0;
        const bool report = report_needed(db, flags, cross);
        // k_linear_others' run skip: per pattern, the first k+1 positions
        // whose class accepts only A/C/G/T (an "other" byte there is a
        // mismatch); jsel_ok[p]: the pattern has k+1 of them
        std::vector<uint8_t> jsel((size_t)n_patterns * 4, 0), jsel_ok(n_patterns, 0);
        for (int p = 0; p < n_patterns; ++p) {
            int t = 0;
            for (int j = 0; j < lengths[p] && t <= k; ++j) {
                const uint32_t* cb = class_bytes + 8 * pos_class[64 * p + j];
                bool acgt_only = true;
                for (int w = 0; w < 8 && acgt_only; ++w) {
                    uint32_t bits = cb[w];
                    if (w == 2) bits &= ~((1u << ('A' - 64)) | (1u << ('C' - 64)) | (1u << ('G' - 64)) | (1u << ('T' - 64)));
                    acgt_only = bits == 0;
                }
                if (acgt_only) jsel[(size_t)p * 4 + t++] = (uint8_t)j;
            }
            jsel_ok[p] = t == k + 1;
        }
        auto skip_ok = [&](int base, int P) {
            for (int p = base; p < base + P; ++p)
                if (!jsel_ok[p]) return false;
            return true;
        };
        auto edge_ok = [&](int base, int P) {   // every jsel within the build-time lookahead
            if (!skip_ok(base, P)) return false;
            for (int p = base; p < base + P; ++p)
                for (int t = 0; t <= k; ++t)
                    if (jsel[(size_t)p * 4 + t] > RUN_SKIP) return false;
            return true;
        };
        if (db->alphabet == PM_ALPHA_BYTE) {
            scan_linear_bytes(db, n_patterns, lengths, pos_class, n_classes, class_bytes, class_is_any, k, flags,
                              cross, out);
            return;
        }

        Upload up;
        const size_t o_cb = up.add(class_bytes, (size_t)n_classes * 32);
        const size_t o_len = up.add(lengths, (size_t)n_patterns * 4);
        const size_t o_pc = up.add(pos_class, (size_t)n_patterns * 64);
        const size_t o_acgt = up.add(class_acgt, (size_t)n_classes);
        const size_t o_any = up.add(class_is_any, (size_t)n_classes);
        const size_t o_jsel = up.add(jsel.data(), jsel.size());
        // k_others_lane: per (pattern, position) the class's A/C/G/T subset,
        // | 16 for '.'; lane_cls[p]: every class of pattern p is A/C/G/T-only
        // or '.' (an "other" byte is then a mismatch or a match without
        // looking at its value)
        std::vector<uint8_t> csub((size_t)n_patterns * 64, 0), lane_cls(n_patterns, 1);
        for (int p = 0; p < n_patterns; ++p)
            for (int j = 0; j < lengths[p]; ++j) {
                const int c = pos_class[64 * p + j];
                const uint32_t* cb = class_bytes + 8 * c;
                bool acgt_only = true;
                for (int w = 0; w < 8 && acgt_only; ++w) {
                    uint32_t bits = cb[w];
                    if (w == 2) bits &= ~((1u << ('A' - 64)) | (1u << ('C' - 64)) | (1u << ('G' - 64)) | (1u << ('T' - 64)));
                    acgt_only = bits == 0;
                }
                if (!acgt_only && !class_is_any[c]) lane_cls[p] = 0;
                csub[(size_t)64 * p + j] = (uint8_t)((class_acgt[c] & 15) | (class_is_any[c] ? 16 : 0));
            }
        const size_t o_csub = up.add(csub.data(), csub.size());
        // k > 0: nrgrep's esimple engine decides which overlapping window
        // is printed (pm_esimple.hip)
        EsBuild esb;
        EsUpload esu;
        const bool esimple = linear_esimple(n_patterns, lengths, pos_class, class_bytes, k, flags, esb);
        if (esimple) es_upload(esb, up, esu);
        // a large k = 0 batch: the q-gram filter (pm_batch.hip), one pass for
        // the whole batch (PM_BATCH=0 off; PM_BATCH_MIN: smallest batch, 16)
        static const int batch_min = getenv("PM_BATCH_MIN") ? std::max(1, atoi(getenv("PM_BATCH_MIN"))) : 16;
        std::shared_ptr<const BatchIndex> bip;
        std::string batch_sig;
        if (jit && k == 0 && n_patterns >= batch_min && env_flag("PM_BATCH", true)) {
            batch_sig = jit_signature(n_patterns, k, lengths, pos_class, class_acgt, class_is_any);
            bip = batch_index_cached(batch_sig, n_patterns, lengths, pos_class, class_acgt, class_is_any);
        }
        const bool batch = bip != nullptr;
        uint8_t* d_batch = nullptr;
        if (batch) d_batch = batch_tables(db, *bip, batch_sig);
        struct Chunk { int base, P; hipFunction_t jit; };
        std::vector<Chunk> chunks;
        if (batch) chunks.push_back({0, n_patterns, nullptr});
        for (int base = batch ? n_patterns : 0; base < n_patterns;) {
            const int rem = n_patterns - base;
            // instantiated widths; a specialized kernel takes up to 8 (class
            // words shared by more patterns, one pass over HBM for all of them)
            int P = (jit && rem >= 8) ? 8 : rem >= 4 ? 4 : (rem >= 2 ? 2 : 1);
            hipFunction_t fn = nullptr;
            if (jit) {
                // halve the width while the compiled kernel spills registers
                // to scratch (long patterns at high k with many patterns)
                for (;;) {
                    fn = jit_function(db->device, P, k, lengths + base, pos_class + 64 * base, class_acgt, class_is_any);
                    int scratch = 0;
                    HIPCHK(hipFuncGetAttribute(&scratch, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, fn));
                    if (scratch == 0 || P == 1) break;
                    P /= 2;
                }
            }
            chunks.push_back({base, P, fn});
            base += P;
        }
        // PM_POST_STREAM (A/B): a pipelined single-launch scan post-processes
        // on `post` in its own workspace lane (alternating), everything else
        // waits for `post` first
        const bool post2 = async && jit && !batch && chunks.size() == 1 && post_mode() > 0;
        struct LaneBack {
            pm_db* db;
            bool on;
            ~LaneBack() {
                if (on) switch_lane(db);
            }
        } lane_back{db, false};
        if (post2) {
            post_stream(db);
            if (db->lane_flip) {
                switch_lane(db);
                lane_back.on = true;
            }
            db->lane_flip = !db->lane_flip;
        } else {
            post_join(db);
        }
        lane_begin(db);
        uint8_t* d_up = up.commit(db);
        const EsPrep esp = esimple ? es_bind(esu, d_up, es_gap(esb)) : EsPrep{};
        const EsPrep* es = esimple ? &esp : nullptr;

        SinkBuffers sb;
        std::vector<uint32_t> counts;
        uint64_t total = 0;
        EventPair ev;
        std::vector<std::unique_ptr<EventPair>> jev;   // per specialized launch
        pm_hits* spec = nullptr;       // speculatively sorted hit list
        pm_hits* hit_list = nullptr;   // accepted speculative list
        bool done = false;
        // the exception pass for the patterns of chunk `ch`, appending to the hit
        // lists of `sb` (nout segments per pattern, tiles_per_out tiles each)
        auto launch_others = [&](const Chunk& ch, hipStream_t os, const SinkBuffers& sb, uint64_t nout,
                                 uint64_t tiles_per_out) {
            const bool use_edge = edge_ok(ch.base, ch.P);
            const int maxlen = *std::max_element(lengths + ch.base, lengths + ch.base + ch.P);
            bool lane = !cross && use_edge && 2 * maxlen - 1 <= 64;
            for (int p = ch.base; p < ch.base + ch.P && lane; ++p) lane = lane_cls[p] != 0;
            if (lane) {
                // the lane form over the database's "other"-position list
                if (!db->nxlist) return;
                int jdead = 0;   // a run tail's window at e with this many exceptions first is dead
                for (int p = ch.base; p < ch.base + ch.P; ++p) jdead = std::max(jdead, (int)jsel[(size_t)p * 4 + k] + 1);
                LaneArgs la{db->xlist, db->nxlist, db->lin, db->ntiles * STREAM, db->n, d_up + o_csub + 64 * ch.base,
                            reinterpret_cast<const int32_t*>(d_up + o_len) + ch.base, ch.P, k, ch.base, maxlen, jdead,
                            sb.out, sb.cnt, sb.slot_base, sb.slot_cap, (uint32_t)nout, (uint32_t)tiles_per_out};
                hipLaunchKernelGGL(k_others_lane, dim3((uint32_t)std::min<uint64_t>(8192, blocks_for(db->nxlist, 256))),
                                   dim3(256), 0, os, la);
                HIPCHK(hipGetLastError());
                return;
            }
            // line-bounded: only words with an "other" byte can own a window
            const uint32_t* edge = cross ? db->xedge : db->xedge_oth;
            const uint64_t nedge = cross ? db->nedge : db->nedge_oth;
            const uint64_t words = use_edge ? nedge : db->nflag;
            if (!words) return;
            uint8_t* ws = static_cast<uint8_t*>(reserve(db, db->ws_oth, 256 + words * sizeof(OtherSel)));
            OthersArgs oa{nuc_view(db), db->xoth, db->xbrk, db->xword, db->nflag, db->n,
                          d_up + o_pc + 64 * ch.base, reinterpret_cast<const int32_t*>(d_up + o_len) + ch.base,
                          d_up + o_any, reinterpret_cast<const uint32_t*>(d_up + o_cb), ch.P, k, ch.base,
                          cross ? 1 : 0, skip_ok(ch.base, ch.P) ? 1 : 0, d_up + o_jsel + 4 * ch.base,
                          *std::max_element(lengths + ch.base, lengths + ch.base + ch.P),
                          use_edge ? 1 : 0, db->xint, edge, nedge,
                          reinterpret_cast<OtherSel*>(ws + 256), reinterpret_cast<uint32_t*>(ws),
                          sb.out, sb.cnt, sb.slot_base, sb.slot_cap, (uint32_t)nout, (uint32_t)(tiles_per_out), 1,
                          n_classes};
            oa.jall = 0;
            for (int p = ch.base; p < ch.base + ch.P; ++p)
                for (int t = 0; t <= k; ++t)
                    if (const int j = jsel[(size_t)p * 4 + t]) oa.jall |= 1ull << j;
            const int span = 2 * oa.maxlen - 1;
            oa.items_per_wave = span <= 16 ? 4 : span <= 32 ? 2 : 1;
            // phase 1: one thread per candidate word selects the
            // exception bits that can own a live window; phase 2:
            // persistent waves evaluate them
            const bool cls = ch.P * oa.maxlen > OTH_MAX_POS;
            require(!cls || ch.P * oa.maxlen <= OTH_CLS_MAX_POS, "internal: batch too large for the exception pass");
            // the per-class wave form for large batches (class-id staging)
            const bool batch_form = cls && n_classes <= OTH_BATCH_MAX_CLASSES && oa.maxlen <= BATCH_MAX_LEN &&
                                    ch.P <= BATCH_MAX_P;
            // a selection pass compacts the words first (an inline selection
            // in the waves measured slower, 0.231 vs 0.138 + 0.046 ms on
            // configs[2]: the persistent waves then wait on the selection
            // loads of every filtered-out word; a lane-per-bit form measured
            // 0.20 vs 0.18 ms -- both are bound by ~58 gathered cache lines
            // per exception bit)
            HIPCHK(hipMemsetAsync(oa.nsel, 0, sizeof(uint32_t), os));
            hipLaunchKernelGGL(k_others_select, dim3(blocks_for(words, OTH_SELECT_T)), dim3(OTH_SELECT_T), 0, os, oa);
            HIPCHK(hipGetLastError());
            // PM_OTH_TWO=0: one exception per wave round (A/B)
            static const bool two_env = !(getenv("PM_OTH_TWO") && getenv("PM_OTH_TWO")[0] == '0');
            if (batch_form)
                hipLaunchKernelGGL(two_env && span <= 32 ? k_others_batch<true> : k_others_batch<false>,
                                   dim3((uint32_t)std::min<uint64_t>(OTH_BLOCKS, blocks_for(words * 64, OTH_BATCH_THREADS))),
                                   dim3(OTH_BATCH_THREADS), 0, os, oa);
            else
                hipLaunchKernelGGL(cls ? k_linear_others<true> : k_linear_others<false>,
                                   dim3((uint32_t)std::min<uint64_t>(OTH_BLOCKS, blocks_for(words * 64, 256))),
                                   dim3(256), 0, os, oa);
            HIPCHK(hipGetLastError());
        };
        if (jit && batch) {
            // k_batch_scan: one workgroup of BATCH_WAVES waves per CU, each
            // wave a contiguous tile range; an output segment = wpo waves
            int ncu = 0;
            HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, db->device));
            uint64_t nwaves = std::min<uint64_t>(db->ntiles, (uint64_t)std::max(ncu, 1) * BATCH_WAVES);
            const uint64_t tpw = (db->ntiles + nwaves - 1) / nwaves;
            nwaves = (db->ntiles + tpw - 1) / tpw;
            const uint32_t nblocks = (uint32_t)((nwaves + BATCH_WAVES - 1) / BATCH_WAVES);
            // scan waves per output segment: segments of ~750 tiles (~49 Mbp;
            // configs[4] at 12.5 Gbp: 16 waves, 256 segments -- one round of
            // verify blocks and 64 Ki (pattern, segment) bins; measured 9.25,
            // 8.73, 10.6 ms per step at 8, 16, 32 waves)
            // (round 5: ~376-tile segments, two verify blocks per CU,
            // measured the same, 8.67 vs 8.69 ms)
            const uint64_t wpo = std::min<uint64_t>(BATCH_MAX_WPO, std::max<uint64_t>(1, (752 + tpw / 2) / tpw));
            const uint64_t nout = (nwaves + wpo - 1) / wpo;
            std::vector<uint32_t> slot_caps(n_patterns, 64);
            // candidates per wave: ~1 % of the positions at configs[4]
            uint32_t ccap = (uint32_t)std::min<uint64_t>(tpw * 16384, std::max<uint64_t>(4096, tpw * 512));
            const std::string cap_key =
                "batch|" + jit_signature(n_patterns, k, lengths, pos_class, class_acgt, class_is_any);
            {
                std::lock_guard<std::mutex> lk(g_cap_mu);
                auto it = g_cap_hint.find({db, cap_key});
                if (it != g_cap_hint.end() && it->second.first.size() == slot_caps.size()) {
                    slot_caps = it->second.first;
                    ccap = std::max(ccap, it->second.second);
                }
            }
            // keys whose start lies past a segment's last tile: at most o_max
            // starts per pattern and segment boundary
            const uint64_t xcap = std::max<uint64_t>(4096, nout * n_patterns * (bip->omax + 1));
            const bool exc = db->nflag && (db->n_oth_words || cross);
            // the ordered verify (PM_BATCH_ORDERED=0: off, A/B): per (segment,
            // verify wave) a position-ordered list of ord_cap keys
            const bool ord_env = !(getenv("PM_BATCH_ORDERED") && getenv("PM_BATCH_ORDERED")[0] == '0');
            const bool exc_conc = !(getenv("PM_BATCH_EXC_CONC") && getenv("PM_BATCH_EXC_CONC")[0] == '0');
            const bool scatter_env = !(getenv("PM_BATCH_SCATTER") && getenv("PM_BATCH_SCATTER")[0] == '0');
            bool ordered = ord_env;
            const uint32_t nlists = (uint32_t)nout * BATCH_VERIFY_WAVES;
            // (PM_BATCH_ORD_CAP: a smaller first capacity, for the tests of the
            // grow-and-retry path)
            uint32_t ord_cap = getenv("PM_BATCH_ORD_CAP") ? std::max(1, atoi(getenv("PM_BATCH_ORD_CAP"))) : 1024;
            {
                std::lock_guard<std::mutex> lk(g_cap_mu);
                auto it = g_ord_hint.find({db, cap_key});
                if (it != g_ord_hint.end()) ord_cap = it->second;
            }
            const uint32_t* ord_h = nullptr;   // the lists' counts (pinned)
            // the ordered form's bins (exception pass, next-segment keys,
            // first starts) are one per pattern: a few keys each, so the
            // host's per-bin work after the sync is 256 bins, not 64 Ki
            std::vector<uint32_t> caps_ord(n_patterns, 256);
            {
                std::lock_guard<std::mutex> lk(g_cap_mu);
                auto it = g_cap_hint.find({db, cap_key + "|ord"});
                if (it != g_cap_hint.end() && it->second.first.size() == caps_ord.size()) {
                    caps_ord = it->second.first;
                    ccap = std::max(ccap, it->second.second);
                }
            }
            for (int attempt = 0; attempt < 6 && !done; ++attempt) {
                const uint64_t snout = ordered ? 1 : nout;   // sink segments per pattern
                std::vector<uint32_t>& caps = ordered ? caps_ord : slot_caps;
                Carve cv;
                const size_t o_cand = cv.take(nwaves * ccap * sizeof(uint4));
                const size_t o_ccnt = cv.take(nwaves * sizeof(uint32_t));
                const size_t o_xcnt = cv.take(sizeof(uint32_t));
                const size_t o_x = cv.take(xcap * sizeof(uint64_t));
                const size_t o_ocnt = cv.take((nlists + 1) * sizeof(uint32_t));   // + the overflow flag
                const size_t o_ord = cv.take(ordered ? (uint64_t)nlists * ord_cap * sizeof(uint64_t) : 0);
                // keys per (pattern, list): the stable scatter instead of a radix sort
                // (PM_BATCH_SCATTER=0: the radix sort, A/B)
                const bool hist = ordered && n_patterns <= (int)ORD_HIST_MAX_P && scatter_env;
                const size_t o_hist = cv.take(hist ? (uint64_t)n_patterns * nlists * sizeof(uint32_t) : 0);
                uint8_t* rbase = static_cast<uint8_t*>(reserve(db, db->ws_rec, cv.off));
                // k_batch_verify stores every (pattern, segment) count; the
                // ordered form only adds to the bins (zeroed here)
                sb = make_sink_segments(db, n_patterns, (uint32_t)snout, caps, /*zero_counts=*/ordered);
                const BatchIndex& bi = *bip;
                const uint32_t* d_tab = reinterpret_cast<const uint32_t*>(d_batch + bi.o_table);
                BatchScanArgs sa{db->hl, db->ntiles, d_tab, bi.omax, (uint32_t)tpw, (uint32_t)nwaves, ccap,
                                 reinterpret_cast<uint4*>(rbase + o_cand), reinterpret_cast<uint32_t*>(rbase + o_ccnt),
                                 sb.cnt + sb.nbins, reinterpret_cast<uint32_t*>(rbase + o_xcnt)};
                BatchVerifyArgs va{reinterpret_cast<const uint4*>(rbase + o_cand),
                                   reinterpret_cast<const uint32_t*>(rbase + o_ccnt), ccap, sb.cnt + sb.nbins,
                                   reinterpret_cast<const uint32_t*>(d_batch + bi.o_code),
                                   bi.hash.empty() ? nullptr : reinterpret_cast<const uint64_t*>(d_batch + bi.o_hash),
                                   reinterpret_cast<const uint4*>(d_batch + bi.o_ents),
                                   reinterpret_cast<const uint4*>(d_batch + bi.o_pmask),
                                   reinterpret_cast<const uint32_t*>(d_batch + bi.o_popt),
                                   reinterpret_cast<const int32_t*>(d_up + o_len), bi.omax, (uint32_t)tpw,
                                   (uint32_t)wpo, (uint32_t)nwaves, (uint32_t)nout, n_patterns, db->hl, db->bo,
                                   db->lflag, db->ntiles, db->n, sb.out, sb.cnt, sb.slot_base, sb.slot_cap,
                                   reinterpret_cast<uint64_t*>(rbase + o_x), reinterpret_cast<uint32_t*>(rbase + o_xcnt),
                                   (uint32_t)xcap};
                uint32_t* d_ocnt = reinterpret_cast<uint32_t*>(rbase + o_ocnt);
                va.sink_segs = (uint32_t)snout;
                va.lin = db->lin;
                // the exception pass's segment of a start: all in one with snout 1
                const uint64_t oth_tiles = ordered ? (uint64_t)UINT32_MAX : tpw * wpo;
                if (ordered) {
                    va.ord_out = reinterpret_cast<uint64_t*>(rbase + o_ord);
                    va.ord_cnt = d_ocnt;
                    va.ord_bad = d_ocnt + nlists;
                    va.ord_cap = ord_cap;
                    if (hist) va.ord_hist = reinterpret_cast<uint32_t*>(rbase + o_hist);
                    HIPCHK(hipMemsetAsync(va.ord_bad, 0, sizeof(uint32_t), s));
                }
                jev.clear();
                jev.emplace_back(new EventPair());
                // the ordered form's exception pass runs on its own stream,
                // beside the scan and verify (its bins are atomic adds;
                // PM_BATCH_EXC_CONC=0: after them, A/B)
                const bool conc = exc && ordered && exc_conc;
                if (conc) {
                    hipStream_t es2 = exc_stream(db);
                    HIPCHK(hipEventRecord(db->exc_fork, s));
                    HIPCHK(hipStreamWaitEvent(es2, db->exc_fork, 0));
                }
                batch_launch(sa, va, nblocks, s, jev.back()->a, jev.back()->b);
                if (conc) {
                    launch_others(chunks[0], db->exc, sb, snout, oth_tiles);
                    HIPCHK(hipEventRecord(db->exc_join, db->exc));
                    HIPCHK(hipStreamWaitEvent(s, db->exc_join, 0));
                } else if (exc) {
                    launch_others(chunks[0], s, sb, snout, oth_tiles);
                }
                if (ordered) {
                    uint32_t* hp = static_cast<uint32_t*>(reserve_host(db, db->pin_ord, (nlists + 1) * sizeof(uint32_t)));
                    HIPCHK(hipMemcpyAsync(hp, d_ocnt, (nlists + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
                    ord_h = hp;
                }
                bool overflow = false;
                total = sink_total(db, sb, counts, overflow);   // synchronizes the stream
                const uint32_t cneed = sb.aux;
                bool ord_retry = false;
                if (ordered) {
                    if (ord_h[nlists]) {   // a lane's round held more matches than it keeps
                        ordered = false;
                        ord_retry = true;
                    } else {
                        const uint32_t m = *std::max_element(ord_h, ord_h + nlists);
                        if (m > ord_cap) {
                            while (ord_cap < m) ord_cap *= 2;
                            ord_retry = true;
                        }
                    }
                }
                if (!overflow && cneed == 0 && !ord_retry) {
                    done = true;
                    std::lock_guard<std::mutex> lk(g_cap_mu);
                    if (g_cap_hint.size() > 256) g_cap_hint.clear();
                    g_cap_hint[{db, ordered ? cap_key + "|ord" : cap_key}] = {caps, ccap};
                    if (g_ord_hint.size() > 256) g_ord_hint.clear();
                    g_ord_hint[{db, cap_key}] = ord_cap;
                    if (ordered) {
                        hit_list = ordered_to_hits(db, sb, counts, total, va.ord_out, ord_cap, d_ocnt, ord_h, nlists,
                                                   n_patterns, va.ord_hist);
                        total = hit_list->count;
                        if (report) {
                            // the report pass reads each key's length by pattern
                            // and writes the kept ones' (no lens pass)
                            hit_list->plen = reinterpret_cast<const int32_t*>(d_up + o_len);
                        } else if (total) {
                            hipLaunchKernelGGL(k_linear_lens, dim3(blocks_for(total, 256)), dim3(256), 0, s,
                                               hit_list->keys, total, reinterpret_cast<const int32_t*>(d_up + o_len),
                                               hit_list->lens);
                            HIPCHK(hipGetLastError());
                        }
                    }
                    break;
                }
                if (cneed) ccap = std::max<uint32_t>(ccap, cneed + cneed / 8 + 64);
                if (overflow) {
                    uint64_t keys_total = 0;
                    for (int p = 0; p < n_patterns; ++p) {
                        const uint32_t* c = counts.data() + (uint64_t)p * snout;
                        const uint32_t m = *std::max_element(c, c + snout);
                        while (caps[p] < m) caps[p] *= 2;
                        keys_total += (uint64_t)caps[p] * snout;
                    }
                    require(keys_total * 8 <= (16ull << 30), "hit list larger than 16 GB of segments",
                            PM_E_UNSUPPORTED);
                }
            }
            require(done, "internal: batch scan capacities did not converge");
        } else if (jit) {
            // one output segment per (pattern, workgroup); workgroups own
            // contiguous tile ranges (3 per CU resident)
            // 8x more workgroups than resident slots: the dispatcher hands the
            // next one to whichever CU frees a slot, so an unevenly loaded CU
            // does not hold up the whole launch (4, 6, 12 within the noise,
            // 16 and 32 slower: profiles/r02k_bench_spread.txt)
            const uint64_t split = 8;
            uint64_t nwg = std::min<uint64_t>(db->ntiles, 256ull * JIT_WG_PER_CU * split);
            const uint64_t tpw = (db->ntiles + nwg - 1) / nwg;
            nwg = (db->ntiles + tpw - 1) / tpw;
            require(tpw < (1ull << 17), "database too large for the record encoding", PM_E_UNSUPPORTED);
            // output segments: `split` consecutive workgroups share one
            // (pattern, segment) hit list, so the sort sees ~1024 segments
            const uint64_t group = split;
            const uint64_t nout = (nwg + group - 1) / group;
            // graded tail: the last segments' tiles (about one round of the
            // resident workgroups) go to workgroups of tpwB < tpw tiles, so
            // the CUs run out of work closer together
            const uint64_t tpo = tpw * group;   // tiles per output segment
            uint64_t tpwB = tpw, ogA = nout, nA = nwg, tilesA = db->ntiles, groupB = group;
            const uint64_t ogB = (256ull * JIT_WG_PER_CU * tpw + tpo - 1) / tpo;
            if (jit_graded() && tpw >= 4 && ogB < nout) {
                tpwB = tpw / 4;
                ogA = nout - ogB;
                nA = ogA * group;
                tilesA = ogA * tpo;
                groupB = (tpo + tpwB - 1) / tpwB;
                nwg = nA + ogB * groupB;
            }
            const uint64_t parts = (uint64_t)jit_parts();
            const uint64_t nseg = nwg * parts;   // one lane-record segment per wave
            // segment capacities scale with the tiles a workgroup owns (a
            // random 15-mer at k = 2 leaves ~1.4 hits per tile and strand);
            // an overflow re-runs with the counts seen
            uint32_t cap = 256;
            while (cap < 4096 && cap < 16 * tpw * group) cap *= 2;
            while (cap > 256 && (uint64_t)n_patterns * nout * cap * 8 > (1ull << 30)) cap /= 2;
            // per-pattern capacities: a dense pattern (many hits) gets its own
            // larger segments on the retry, the others keep theirs
            std::vector<uint32_t> slot_caps(n_patterns, cap);
            // records per wave: at most tiles_per_wg * 64 lanes * steps * patterns
            const uint64_t rec_max = tpw * 64 * (LANE_WORDS / parts) * JIT_MAX_P;
            uint32_t rcap = (uint32_t)std::min<uint64_t>(rec_max, std::max<uint64_t>(128, 8 * tpw));
            // capacities that sufficed for the same batch on this database
            // last time (a repeated query does not pay the overflow retry)
            std::string cap_key;
            for (const Chunk& ch : chunks)
                cap_key += jit_signature(ch.P, k, lengths + ch.base, pos_class + 64 * ch.base, class_acgt, class_is_any) + "|";
            {
                std::lock_guard<std::mutex> lk(g_cap_mu);
                auto it = g_cap_hint.find({db, cap_key});
                if (it != g_cap_hint.end() && it->second.first.size() == slot_caps.size()) {
                    slot_caps = it->second.first;
                    rcap = std::max(rcap, it->second.second);
                }
            }
            for (int attempt = 0; attempt < 4 && !done; ++attempt) {
                Carve cv;
                const size_t o_rec = cv.take(nseg * rcap * sizeof(uint2));
                const size_t o_rcnt = cv.take(nseg * sizeof(uint32_t));
                const size_t o_over = cv.take(sizeof(uint32_t));
                uint8_t* rbase = static_cast<uint8_t*>(reserve(db, db->ws_rec, cv.off));
                uint2* d_rec = reinterpret_cast<uint2*>(rbase + o_rec);
                uint32_t* d_rcnt = reinterpret_cast<uint32_t*>(rbase + o_rcnt);
                (void)o_over;
                // no counter memset: k_linear_expand stores every (pattern,
                // segment) count, the first launch zeroes the aux counter.
                // The exception pass runs after the expansion on the same
                // stream (run concurrently with the scan it measured no
                // faster: the two contend for the CUs)
                const bool exc = db->nflag && (db->n_oth_words || cross);
                sb = make_sink_segments(db, n_patterns, (uint32_t)nout, slot_caps, /*zero_counts=*/false);
                uint32_t* d_over = sb.cnt + sb.nbins;   // the sink's aux counter
                // kernel_ms = the scan passes over the database (pm_linear_jit
                // launches); record expansion and the rest are not included
                jev.clear();
                bool nospec = false;
                if (async && sb.nbins <= 4096 && attempt == 0) {
                    std::lock_guard<std::mutex> lk(g_nospec_mu);
                    nospec = g_nospec.count({db, cap_key}) != 0;
                }
                const bool spec_async = async && sb.nbins <= 4096 && attempt == 0 && !nospec;
                uint64_t* clk = nullptr;   // PM_JIT_CLOCK samples of the launch
                // expansion, exception pass and sort run on the scan's stream
                // (overlapping them with the next scan on a second stream
                // measured no faster in round 4: the chip is at its power
                // limit; PM_POST_STREAM re-measures it, round 6)
                const hipStream_t xs = post2 && spec_async ? db->post : s;
                for (const Chunk& ch : chunks) {
                    JArgsHost ja{db->hl, d_rec, d_rcnt, ch.base == 0 ? d_over : nullptr, db->ntiles, rcap, (uint32_t)tpw,
                                 (uint32_t)nA, (uint32_t)tpwB, (uint32_t)groupB, (uint32_t)tpo, tilesA};
                    if (jit_clock() && chunks.size() == 1) {
                        ja.clk = clock_buffer(db->device, nwg);
                        clk = ja.clk;
                    }
                    void* params[] = {&ja};
                    jev.emplace_back(new EventPair());
                    // the events take the dispatch's own start/end timestamps
                    // (no marker packets around the launch; sizes in threads)
                    HIPCHK(hipExtModuleLaunchKernel(ch.jit, (uint32_t)(nwg * 64 * parts), 1, 1, (uint32_t)(64 * parts), 1, 1, 0, s, params,
                                                    nullptr, jev.back()->a, jev.back()->b, 0));
                    if (xs != s) {   // the post stream starts where the scan ends
                        HIPCHK(hipEventRecord(db->scan_ev, s));
                        HIPCHK(hipStreamWaitEvent(xs, db->scan_ev, 0));
                    }
                    ExpandArgs xa{db->bo, db->lflag, d_rec, d_rcnt, d_over, rcap, db->ntiles, db->n,
                                  reinterpret_cast<const int32_t*>(d_up + o_len) + ch.base, ch.P, ch.base, sb.out, sb.cnt,
                                  sb.slot_base, sb.slot_cap, (uint32_t)nwg, (uint32_t)nout, (uint32_t)group,
                                  (uint32_t)tpw, (uint32_t)parts, (uint32_t)nA, (uint32_t)tpwB, (uint32_t)ogA,
                                  (uint32_t)groupB, (uint32_t)tpo, tilesA};
                    hipLaunchKernelGGL(k_linear_expand, dim3((uint32_t)nout), dim3(EXPAND_THREADS), 0, xs, xa);
                    HIPCHK(hipGetLastError());
                    if (exc) launch_others(ch, xs, sb, nout, tpw * group);
                }
                if (spec_async) {
                    // pipelined: the speculative sort also writes the bin
                    // counts into mapped pinned memory (no copy), an event
                    // follows; the list resolves on first use (hits_finalize)
                    std::unique_ptr<pm_pending> pd(new pm_pending());
                    pd->db = db;
                    pd->nbins = sb.nbins;
                    pd->bins_per_pattern = sb.bins_per_pattern;
                    pd->slot_cap_h = sb.slot_cap_h;
                    pd->counts_h = static_cast<uint32_t*>(pinned_get((sb.nbins + 2) * 4, &pd->counts_cap));
                    pd->flags = flags;
                    if (report) {
                        // the report pass runs behind the sort, driven by the
                        // sort's device-side list length; the list's ready
                        // event is bound to the pass's last dispatch
                        uint64_t cap_total = 0;
                        for (uint32_t c : sb.slot_cap_h) cap_total += (uint64_t)c * sb.bins_per_pattern;
                        const ReportWs ws = report_ws(db, cap_total);
                        spec = sink_sort_speculative(db, sb, reinterpret_cast<const int32_t*>(d_up + o_len),
                                                     pd->counts_h, xs, ws.total, /*bind_ready=*/false);
                        HIPCHK(hipEventCreate(&spec->ready));
                        report_enqueue_ws(db, spec, flags, ws, true, 0, pd->counts_h + sb.nbins + 1, xs, spec->ready,
                                          cross, es);
                        pd->reported = true;
                    } else {
                        spec = sink_sort_speculative(db, sb, reinterpret_cast<const int32_t*>(d_up + o_len),
                                                     pd->counts_h, xs);
                    }
                    // on the db stream the list's own ready event (bound to
                    // the sort's dispatch) marks the same point
                    if (xs != s) {
                        HIPCHK(hipEventCreateWithFlags(&pd->counted, hipEventDisableTiming));
                        HIPCHK(hipEventRecord(pd->counted, xs));
                    }
                    pd->jev = std::move(jev);
                    pd->clk = clk;
                    pd->clk_nwg = nwg;
                    pd->hint_key = cap_key;
                    pd->slot_caps = slot_caps;
                    pd->rcap = rcap;
                    pd->n_patterns = n_patterns;
                    pd->n_classes = n_classes;
                    pd->k = k;
                    pd->lengths.assign(lengths, lengths + n_patterns);
                    pd->pos_class.assign(pos_class, pos_class + (size_t)64 * n_patterns);
                    pd->class_acgt.assign(class_acgt, class_acgt + n_classes);
                    pd->class_is_any.assign(class_is_any, class_is_any + n_classes);
                    pd->class_bytes.assign(class_bytes, class_bytes + (size_t)8 * n_classes);
                    // spec->ready is bound to the sort's dispatch on xs (the
                    // lane's last reader too)
                    lane_end(db, xs);
                    spec->pending = pd.release();
                    db->pending.insert(spec);
                    *out = spec;
                    return;
                }
                if (sb.nbins <= 4096)   // sort before the host sees the counts (one sync per scan)
                    spec = sink_sort_speculative(db, sb, reinterpret_cast<const int32_t*>(d_up + o_len), nullptr, s);
                bool overflow = false;
                total = sink_total(db, sb, counts, overflow);   // synchronizes the stream
                if (clk) clock_report(clk, nwg, jev.empty() ? 0.0 : jev[0]->ms());
                const uint32_t rec_need = sb.aux;
                if (!overflow && rec_need == 0) {
                    done = true;
                    if (spec && total && *std::max_element(counts.begin(), counts.end()) <= LDS_SORT_CAP_MAX) {
                        spec->count = total;
                        hit_list = spec;
                    } else {
                        discard_hits(spec);
                    }
                    spec = nullptr;
                    std::lock_guard<std::mutex> lk(g_cap_mu);
                    if (g_cap_hint.size() > 256) g_cap_hint.clear();
                    g_cap_hint[{db, cap_key}] = {slot_caps, rcap};
                    break;
                }
                discard_hits(spec);
                spec = nullptr;
                if (rec_need) rcap = std::max<uint32_t>(rcap, rec_need);
                if (overflow) {
                    uint64_t keys_total = 0;
                    for (int p = 0; p < n_patterns; ++p) {
                        const uint32_t* c = counts.data() + (uint64_t)p * nout;
                        const uint32_t m = *std::max_element(c, c + nout);
                        while (slot_caps[p] < m) slot_caps[p] *= 2;
                        keys_total += (uint64_t)slot_caps[p] * nout;
                    }
                    require(keys_total * 8 <= (16ull << 30), "hit list larger than 16 GB of segments",
                            PM_E_UNSUPPORTED);
                }
            }
        }
        if (!done) {
            uint64_t expected = std::max<uint64_t>(db->n / 64, 1 << 16);
            for (int attempt = 0; attempt < 2; ++attempt) {
                sb = make_sink(db, n_patterns, db->n, expected);
                HIPCHK(hipEventRecord(ev.a, s));
                for (const Chunk& ch : chunks) {
                    LinearArgs a{};
                    a.nuc = nuc_view(db);
                    a.lflag = db->lflag;
                    a.ntiles = db->ntiles;
                    a.n = db->n;
                    a.pos_class = d_up + o_pc + 64 * ch.base;
                    a.lengths = reinterpret_cast<const int32_t*>(d_up + o_len) + ch.base;
                    a.class_acgt = d_up + o_acgt;
                    a.class_any = d_up + o_any;
                    a.class_bytes = reinterpret_cast<const uint32_t*>(d_up + o_cb);
                    a.k = k;
                    a.pattern_base = ch.base;
                    a.cross = cross ? 1 : 0;
                    a.sink = sb.sink();
                    launch_generic(ch.P, a, s);
                    HIPCHK(hipGetLastError());
                }
                HIPCHK(hipEventRecord(ev.b, s));
                bool overflow = false;
                total = sink_total(db, sb, counts, overflow);
                if (!overflow) break;
                require(attempt == 0, "internal: hit bins overflowed twice");
                expected = (uint64_t)(*std::max_element(counts.begin(), counts.end())) * sb.nbins + sb.nbins;
            }
        }
        double kms = 0.0;
        if (done && jit)
            for (auto& e : jev) kms += e->ms();
        else
            kms = ev.ms();
        bool lens_done = hit_list != nullptr;
        pm_hits* h = hit_list ? hit_list
                              : sink_to_hits(db, sb, counts, total, reinterpret_cast<const int32_t*>(d_up + o_len),
                                             &lens_done);
        h->kernel_ms = kms;
        if (total && !lens_done) {
            hipLaunchKernelGGL(k_linear_lens, dim3(blocks_for(total, 256)), dim3(256), 0, s, h->keys, total,
                               reinterpret_cast<const int32_t*>(d_up + o_len), h->lens);
            HIPCHK(hipGetLastError());
        }
        if (report && async && batch && total) {
            // pipelined batch (the q-gram filter's path syncs once, for the
            // verify's counts): the report pass is enqueued and the reported
            // count lands in pinned memory with the pass's last dispatch; the
            // list resolves on first use (hits_finalize), so the caller can
            // collect the previous query and launch the next one while this
            // one's sort and report run (round 6: ~0.1 ms of GPU idle per
            // configs[4] step before)
            std::unique_ptr<pm_pending> pd(new pm_pending());
            pd->db = db;
            pd->count_only = true;
            pd->counts_h = static_cast<uint32_t*>(pinned_get(8, &pd->counts_cap));
            pd->counts_h[0] = 0u;
            const ReportWs ws = report_ws(db, h->keys_cap / 8);
            if (!h->ready) HIPCHK(hipEventCreate(&h->ready));
            report_enqueue_ws(db, h, flags, ws, false, total, pd->counts_h, s, h->ready, cross, es);
            lane_end(db, s);
            h->pending = pd.release();
            db->pending.insert(h);
            *out = h;
            return;
        }
        if (report) report_sync(db, h, flags, total, cross, es);
        // no host sync here: consumers wait on h->ready (pm_hits_copy*,
        // pm_hits_device, pm_hits_destroy)
        hits_ready(db, h);
        *out = h;
    }
}

}  // namespace

namespace pm {

std::vector<char> hiprtc_compile(const std::string& src) { return jit_compile(src); }

void hits_finalize(pm_hits* h) {
    if (!h || !h->pending) return;
    pm_db* db = h->pending->db;
    std::lock_guard<std::recursive_mutex> lk(db->mu);
    if (!h->pending) return;   // resolved meanwhile (by pm_db_destroy)
    std::unique_ptr<pm_pending> pd(h->pending);
    h->pending = nullptr;
    db->pending.erase(h);
    DeviceGuard g(h->device);
    HIPCHK(hipEventSynchronize(pd->counted ? pd->counted : h->ready));
    if (pd->count_only) {   // a pipelined batch: only the reported count was pending
        h->count = pd->counts_h[0];
        return;
    }
    uint64_t total = 0;
    uint32_t maxc = 0;
    bool overflow = false;
    for (uint32_t b = 0; b < pd->nbins; ++b) {
        const uint32_t c = pd->counts_h[b];
        total += c;
        maxc = std::max(maxc, c);
        overflow |= c > pd->slot_cap_h[b / pd->bins_per_pattern];
    }
    const bool rec_over = pd->counts_h[pd->nbins] != 0;
    if (!overflow && !rec_over && maxc <= LDS_SORT_CAP_MAX) {   // the speculative list is the answer
        h->count = pd->reported ? pd->counts_h[pd->nbins + 1] : total;
        double kms = 0.0;
        for (auto& e : pd->jev) kms += e->ms();
        h->kernel_ms = kms;
        if (pd->clk) clock_report(pd->clk, pd->clk_nwg, kms);
        std::lock_guard<std::mutex> lk(g_cap_mu);
        if (g_cap_hint.size() > 256) g_cap_hint.clear();
        g_cap_hint[{db, pd->hint_key}] = {pd->slot_caps, pd->rcap};
        return;
    }
    if (!overflow && !rec_over) {   // bins too large for the LDS sort: this batch stays synchronous
        std::lock_guard<std::mutex> lk(g_nospec_mu);
        if (g_nospec.size() > 256) g_nospec.clear();
        g_nospec.insert({db, pd->hint_key});
    }
    // re-run synchronously (grows the capacities, remembers them) and adopt
    // the result's buffers
    pm_hits* r = nullptr;
    scan_linear_impl(db, pd->n_patterns, pd->lengths.data(), pd->pos_class.data(), pd->n_classes,
                     pd->class_acgt.data(), pd->class_bytes.data(), pd->class_is_any.data(), pd->k, pd->flags, &r,
                     false);
    pool_put(h->device, h->keys, h->keys_cap);
    pool_put(h->device, h->lens, h->lens_cap);
    if (h->ready && (h->old_keys || h->old_lens)) HIPCHK(hipEventSynchronize(h->ready));
    pool_put(h->device, h->old_keys, h->old_keys_cap);
    pool_put(h->device, h->old_lens, h->old_lens_cap);
    h->old_keys = nullptr;
    h->old_lens = nullptr;
    h->keys = r->keys;
    h->lens = r->lens;
    h->keys_cap = r->keys_cap;
    h->lens_cap = r->lens_cap;
    h->count = r->count;
    h->kernel_ms = r->kernel_ms;
    if (h->ready) quiet(hipEventDestroy(h->ready));
    h->ready = r->ready;
    delete r;
}

}  // namespace pm

extern "C" {

int pm_scan_linear(pm_db* db, int n_patterns, const int32_t* lengths, const uint8_t* pos_class, int n_classes,
                   const uint8_t* class_acgt, const uint32_t* class_bytes, const uint8_t* class_is_any, int k,
                   int flags, pm_hits** out) {
    return guarded([&] {
        require(db != nullptr, "db is NULL");
        std::lock_guard<std::recursive_mutex> lk(db->mu);
        scan_linear_impl(db, n_patterns, lengths, pos_class, n_classes, class_acgt, class_bytes, class_is_any, k,
                         (uint32_t)flags, out, false);
    });
}

int pm_scan_linear_async(pm_db* db, int n_patterns, const int32_t* lengths, const uint8_t* pos_class, int n_classes,
                         const uint8_t* class_acgt, const uint32_t* class_bytes, const uint8_t* class_is_any, int k,
                         int flags, pm_hits** out) {
    return guarded([&] {
        require(db != nullptr, "db is NULL");
        std::lock_guard<std::recursive_mutex> lk(db->mu);
        scan_linear_impl(db, n_patterns, lengths, pos_class, n_classes, class_acgt, class_bytes, class_is_any, k,
                         (uint32_t)flags, out, true);
    });
}

int pm_linear_jit_compile(int n_patterns, const int32_t* lengths, const uint8_t* pos_class, int n_classes,
                          const uint8_t* class_acgt, const uint8_t* class_is_any, int k, uint64_t* code_bytes) {
    return guarded([&] {
        require(lengths && pos_class && class_acgt && class_is_any, "null argument");
        require(n_patterns >= 1 && n_patterns <= JIT_MAX_P, "n_patterns out of range for one specialized kernel");
        require(n_classes >= 1 && n_classes <= 256, "n_classes out of range");
        require(k >= 0 && k <= PM_MAX_LINEAR_K, "k out of range", PM_E_UNSUPPORTED);
        for (int p = 0; p < n_patterns; ++p)
            require(lengths[p] >= 1 && lengths[p] <= PM_MAX_LINEAR_POSITIONS, "pattern length out of range");
        const std::string src =
            gen_linear_source(n_patterns, k, lengths, pos_class, class_acgt, class_is_any, 4, jit_parts());
        const std::vector<char> code = jit_compile(src);
        if (code_bytes) *code_bytes = code.size();
    });
}

}  // extern "C"
