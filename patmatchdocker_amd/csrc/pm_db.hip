// pm_db.hip -- the device-resident sequence database (pm_db_* entry points).
//
// Replaces nrgrep_coords' per-call read of '<datafile>'
// (www/FlaskApp/FlaskApp/patmatch.py:733-742): the FASTA file is uploaded
// once and kept in HBM in the stream-tile layout described in pm_internal.h
// (nucleotides) or as folded bytes (peptides).  Header lines (/^>\S/, the
// record names of generate_sequence_index.pl:33) and '\n' are record breaks.
#include <hipcub/hipcub.hpp>

#include "pm_internal.h"

namespace pm {

thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

void note_cleared_capture_status() {
    static std::once_flag once;
    std::call_once(once, [] {
        fprintf(stderr, "patmatch_hip: cleared hipErrorStreamCaptureUnsupported left pending on the calling thread "
                        "by an earlier call (not this library's)\n");
    });
}

namespace {

// code of a folded byte: 0..3 = A C G T, 4 = delimiter, 5 = other
__constant__ uint8_t c_code[256];

void init_code_table() {
    static bool done = false;
    if (done) return;
    uint8_t t[256];
    for (int i = 0; i < 256; ++i) t[i] = 5;
    t[(int)'A'] = 0; t[(int)'C'] = 1; t[(int)'G'] = 2; t[(int)'T'] = 3;
    t[(int)'a'] = 0; t[(int)'c'] = 1; t[(int)'g'] = 2; t[(int)'t'] = 3;
    t[(int)'\n'] = 4;
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(c_code), t, sizeof(t)));
    done = true;
}

// ---------------------------------------------------------------------------
// packing kernels (one thread per logical word of the 2048 main words of a
// tile; halo words are derived afterwards by k_fill_halo)
// ---------------------------------------------------------------------------
__global__ void k_pack_nuc(const uint8_t* __restrict__ raw, uint64_t n, uint64_t ntiles,
                           uint2* __restrict__ hl, uint2* __restrict__ bo) {
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (g >= ntiles * STREAM) return;
    const uint64_t t = g / STREAM;
    const uint32_t w = (uint32_t)(g % STREAM);
    uint32_t h = 0, l = 0, br = 0, ot = 0;
    for (uint32_t b = 0; b < 32; ++b) {
        const uint64_t p = pos_of(t, w, b);
        const uint32_t c = p < n ? c_code[raw[p]] : 4u;
        if (c < 4) {
            h |= (c >> 1) << b;
            l |= (c & 1) << b;
        } else if (c == 4) {
            br |= 1u << b;
        } else {
            ot |= 1u << b;
            if ((raw[p] & 0xdf) == 'N') h |= 1u << b;   // an "other" byte's hi bit: it is N (NUC_N_MARK)
        }
    }
    const uint64_t pw = phys_word(t, w);
    hl[pw] = make_uint2(h, l);
    bo[pw] = make_uint2(br, ot);
}

__device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

constexpr uint64_t SYN_HDR = 10;  // ">r%08u" then '\n'

// Exceptions of the synthetic text, at genome-like density: every record has
// one run of N (length 50..499 at a hashed offset) and IUPAC ambiguity
// letters at ~1e-5 of the bases (hashed per position).  Returns the byte of
// sequence offset `b` (0-based inside the record) of record `r`, or 0 for
// an A/C/G/T base (drawn from the per-word hash by k_pack_synth).
__device__ inline uint8_t synth_other(uint64_t r, uint64_t b, uint64_t p, uint64_t rec_len, uint64_t seed) {
    const uint64_t h = mix64(seed ^ (r * 0xd6e8feb86659fd93ull + 0x5bd1e995ull));
    const uint64_t run_len = 50 + (h >> 40) % 450;
    const uint64_t run_beg = (h % rec_len);
    if (b >= run_beg && b < run_beg + run_len) return (uint8_t)'N';
    const uint64_t x = mix64(p * 0x9e3779b97f4a7c15ull ^ seed ^ 0x2545f4914f6cdd1dull);
    if (x < 184467440737096ull) return (uint8_t)"RYKMSWBDHV"[(x >> 8) % 10];   // ~1e-5
    return 0;
}

// Synthetic FASTA-shaped text: records of SYN_HDR header bytes + '\n' +
// rec_len bases + '\n'; bases from a counter-based hash of (seed, word),
// exceptions from synth_other.
__global__ void k_pack_synth(uint64_t n, uint64_t ntiles, uint64_t rec_len, uint64_t seed,
                             uint2* __restrict__ hl, uint2* __restrict__ bo) {
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (g >= ntiles * STREAM) return;
    const uint64_t t = g / STREAM;
    const uint32_t w = (uint32_t)(g % STREAM);
    const uint64_t stride = SYN_HDR + 1 + rec_len + 1;
    const uint64_t r = mix64(seed * 0x9e3779b97f4a7c15ull + g);
    uint32_t br = 0, ot = 0, nn = 0;
    const uint64_t p0 = pos_of(t, w, 0);
    uint64_t q = p0 % stride;
    const uint64_t d = STREAM % stride;
    for (uint32_t b = 0; b < 32; ++b) {
        const uint64_t p = p0 + (uint64_t)b * STREAM;
        const bool is_base = p < n && q >= SYN_HDR + 1 && q < SYN_HDR + 1 + rec_len;
        if (!is_base) br |= 1u << b;
        else if (const uint8_t x = synth_other(p / stride, q - (SYN_HDR + 1), p, rec_len, seed)) {
            ot |= 1u << b;
            if (x == 'N') nn |= 1u << b;
        }
        q += d;
        if (q >= stride) q -= stride;
    }
    const uint64_t pw = phys_word(t, w);
    hl[pw] = make_uint2(((uint32_t)(r >> 32) & ~(br | ot)) | nn, (uint32_t)r & ~(br | ot));
    bo[pw] = make_uint2(br, ot);
}

// Header lines become breaks: one thread per [beg, end) range.
__global__ void k_mark_ranges(const uint64_t* __restrict__ ranges, uint64_t nr, uint2* __restrict__ bo) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= nr) return;
    for (uint64_t p = ranges[2 * i]; p < ranges[2 * i + 1]; ++p) {
        const Loc l = loc_of(p);
        atomicOr(&bo[l.word].x, 1u << l.bit);
    }
}

// Halo word i of tile t: bit b = bit b+1 of main word i (b < 31), bit 31 =
// bit 0 of main word i of tile t+1 (a break past the last tile).
__global__ void k_fill_halo(uint64_t ntiles, uint2* __restrict__ hl, uint2* __restrict__ bo) {
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (g >= ntiles * HALO) return;
    const uint64_t t = g / HALO;
    const uint32_t i = (uint32_t)(g % HALO);
    const uint64_t src = phys_word(t, i);
    const uint64_t dst = phys_word(t, (uint32_t)STREAM + i);
    const bool last = t + 1 >= ntiles;
    const uint64_t nxt = last ? src : phys_word(t + 1, i);
    auto shift_in = [](uint32_t cur, uint32_t next_bit) { return (cur >> 1) | (next_bit << 31); };
    const uint2 a = hl[src], b = bo[src];
    const uint2 an = last ? make_uint2(0u, 0u) : hl[nxt];
    const uint2 bn = last ? make_uint2(1u, 0u) : bo[nxt];
    hl[dst] = make_uint2(shift_in(a.x, an.x & 1u), shift_in(a.y, an.y & 1u));
    bo[dst] = make_uint2(shift_in(b.x, bn.x & 1u), shift_in(b.y, bn.y & 1u));
}

// superblock flags (32 physical words each)
__global__ void k_sb_flags(const uint2* __restrict__ bo, uint64_t nsb, uint32_t* __restrict__ sbflag,
                           uint32_t* __restrict__ sbcnt) {
    const uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (s >= nsb) return;
    uint32_t f = 0;
    for (int i = 0; i < 32; ++i) {
        const uint64_t w = s * 32 + i;
        const uint2 e = bo[w];
        if (e.x | e.y) f |= 1u << i;
    }
    sbflag[s] = f;
    sbcnt[s] = __popc(f);
}

// byte p of the synthetic FASTA text (k_pack_synth): ">r%08u\n" header
// lines (record index, 0-based), rec_len bases, "\n"; folded like every
// stored byte.  Only exception positions (header bytes, '\n', N, IUPAC
// letters) are asked for.
__device__ inline uint8_t synth_byte(uint64_t p, uint64_t rec_len, uint64_t seed) {
    const uint64_t stride = SYN_HDR + 1 + rec_len + 1;
    const uint64_t r = p / stride, q = p % stride;
    if (q >= SYN_HDR + 1 && q < SYN_HDR + 1 + rec_len) return synth_other(r, q - (SYN_HDR + 1), p, rec_len, seed);
    if (q == 0) return (uint8_t)'>';
    if (q == 1) return (uint8_t)'R';
    if (q < SYN_HDR) {
        uint64_t v = r % 100000000ull;
        for (uint64_t d = q; d < SYN_HDR - 1; ++d) v /= 10;
        return (uint8_t)('0' + v % 10);
    }
    return (uint8_t)'\n';
}

// Side tables of every flagged word: the break / other masks, the physical
// word, and the raw (folded) byte of each of its exception positions --
// header-line bytes and '\n' included, so the simple engine's windows that
// span a line break (k_linear_others) and the '^'/'$' checks see the file's
// own bytes.  Positions past the end of the file store 0.
__global__ void k_fill_exceptions(const uint8_t* __restrict__ raw, uint64_t n, uint64_t nwords,
                                  const uint2* __restrict__ bo,
                                  const uint32_t* __restrict__ sbflag, const uint32_t* __restrict__ sbbase,
                                  uint32_t* __restrict__ xbrk, uint32_t* __restrict__ xoth,
                                  uint64_t* __restrict__ xword, uint8_t* __restrict__ xbytes,
                                  uint32_t* __restrict__ n_oth_words, uint64_t syn_rec_len, uint64_t syn_seed) {
    const uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (w >= nwords) return;
    const uint32_t f = sbflag[w >> 5];
    const uint32_t bit = (uint32_t)(w & 31);
    if (!((f >> bit) & 1)) return;
    const uint64_t idx = sbbase[w >> 5] + __popc(f & ((1u << bit) - 1));
    const uint2 e = bo[w];
    const uint32_t br = e.x, ot = e.y & ~br;
    xbrk[idx] = br;
    xoth[idx] = ot;
    if (ot) atomicAdd(n_oth_words, 1u);
    xword[idx] = w;
    const uint64_t t = w / TILE_WORDS;
    const uint32_t lw = logical_word((uint32_t)(w % TILE_WORDS));
    for (uint32_t i = 0; i < 32; ++i) {
        const uint64_t p = pos_of(t, lw, i);
        uint8_t c = 0;
        if ((((br | ot) >> i) & 1) && p < n) c = raw != nullptr ? fold(raw[p]) : synth_byte(p, syn_rec_len, syn_seed);
        xbytes[idx * 32 + i] = c;
    }
}

// Run interiors (one thread per flagged word): bit b of xint = position e
// (bit b of logical word lw) has an exception at e - 1 (bit b of word lw - 1)
// and "other" bytes at e .. e + RUN_SKIP (words lw .. lw + RUN_SKIP, halo
// included).  Flagged words with a break or "other" bit outside xint are
// appended to xedge: only they can own a live window for patterns whose
// first k+1 A/C/G/T-only classes lie within RUN_SKIP (k_linear_others).
__global__ void k_run_interior(uint64_t nflag, const uint64_t* __restrict__ xword, const uint32_t* __restrict__ xbrk,
                               const uint32_t* __restrict__ xoth, const uint2* __restrict__ bo,
                               uint32_t* __restrict__ xint, uint32_t* __restrict__ xedge,
                               uint32_t* __restrict__ xedge_oth, unsigned long long* __restrict__ nedge) {
    const uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (idx >= nflag) return;
    const uint64_t w = xword[idx];
    const uint64_t tile = w / TILE_WORDS;
    const uint32_t lw = logical_word((uint32_t)(w % TILE_WORDS));
    uint32_t m = 0;
    if (lw >= 1 && lw < STREAM) {
        const uint2 pv = bo[phys_word(tile, lw - 1)];
        m = (pv.x | pv.y) & xoth[idx];
        for (uint32_t j = 1; j <= (uint32_t)RUN_SKIP && m; ++j) m &= bo[phys_word(tile, lw + j)].y;
    }
    xint[idx] = m;
    if (lw >= STREAM) return;
    if ((xoth[idx] | xbrk[idx]) & ~m) xedge[atomicAdd(&nedge[0], 1ull)] = (uint32_t)idx;
    if (xoth[idx] & ~m) xedge_oth[atomicAdd(&nedge[1], 1ull)] = (uint32_t)idx;
}

// The "other"-position list (pm_db::xlist): one thread per edge word of
// xedge_oth; every "other" bit outside the run interiors becomes one entry
// e | ahead << 48 | prev << 56, read from the position-contiguous planes.
// fill = false: count only.
__global__ void k_build_xlist(uint64_t nedge, const uint32_t* __restrict__ xedge_oth,
                              const uint64_t* __restrict__ xword, const uint32_t* __restrict__ xoth,
                              const uint32_t* __restrict__ xint, const uint4* __restrict__ lin, uint64_t nlin,
                              uint64_t* __restrict__ out, unsigned long long* __restrict__ cnt, int fill) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (t >= nedge) return;
    const uint32_t idx = xedge_oth[t];
    const uint64_t w = xword[idx];
    const uint64_t tile = w / TILE_WORDS;
    const uint32_t lw = logical_word((uint32_t)(w % TILE_WORDS));
    if (lw >= STREAM) return;   // a halo copy of a main word
    uint32_t bits = xoth[idx] & ~xint[idx];
    if (!fill) {
        if (bits) atomicAdd(cnt, (unsigned long long)__popc(bits));
        return;
    }
    const auto exc = [&](uint64_t p) {   // brk | oth at position p (past the planes: a break)
        if ((p >> 5) >= nlin) return true;
        const uint4 v = lin[p >> 5];
        return (((v.z | v.w) >> (uint32_t)(p & 31)) & 1u) != 0;
    };
    for (; bits; bits &= bits - 1) {
        const uint64_t e = pos_of(tile, lw, (uint32_t)__builtin_ctz(bits));
        const uint64_t prev = e > 0 && exc(e - 1) ? 1 : 0;
        uint64_t ahead = 0;
        while (ahead < 255 && exc(e + ahead)) ++ahead;
        out[atomicAdd(cnt, 1ull)] = e | ahead << XL_AHEAD_SHIFT | prev << XL_PREV_SHIFT;
    }
}

// oth = oth & ~brk everywhere (a header byte is a break, not an "other")
__global__ void k_clean_oth(uint64_t nwords, uint2* __restrict__ bo) {
    const uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (w < nwords) bo[w].y &= ~bo[w].x;
}

// lflag[t] bit l: lane l of tile t sees brk|oth in logical words
// [32 l, 32 l + 32 + HALO - 1).  One wave per tile.
__global__ void k_lane_flags(uint64_t ntiles, const uint2* __restrict__ bo, uint64_t* __restrict__ lflag) {
    const uint64_t t = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    if (t >= ntiles) return;
    bool any = false;
    for (uint32_t i = 0; i < LANE_WORDS + HALO - 1; ++i) {
        const uint32_t w = lane * LANE_WORDS + i;
        if (w >= TILE_WORDS) break;
        const uint2 e = bo[phys_word(t, w)];
        any |= (e.x | e.y) != 0;
    }
    const uint64_t bal = __ballot(any);
    if (lane == 0) lflag[t] = bal;
}

// hflag[t] bit l: a position of lane l's own words of tile t (logical words
// [32 l, 32 l + 32), every stream) is a header byte -- a break whose raw byte
// is not '\n' (nuc_is_header).  The report pass's header check (rep_keep)
// settles a start whose lane and predecessor's lane have none from this
// word.  One wave per tile.
__global__ void k_header_flags(uint64_t ntiles, const uint2* __restrict__ bo, const uint32_t* __restrict__ sbflag,
                               const uint32_t* __restrict__ sbbase, const uint8_t* __restrict__ xbytes,
                               uint64_t* __restrict__ hflag) {
    const uint64_t t = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    if (t >= ntiles) return;
    bool any = false;
    for (uint32_t i = 0; i < LANE_WORDS && !any; ++i) {
        const uint64_t pw = phys_word(t, lane * LANE_WORDS + i);
        for (uint32_t brk = bo[pw].x; brk && !any; brk &= brk - 1) {
            const uint32_t idx = exception_index(sbflag, sbbase, pw);
            any = xbytes[(uint64_t)idx * 32 + __builtin_ctz(brk)] != (uint8_t)'\n';
        }
    }
    const uint64_t bal = __ballot(any);
    if (lane == 0) hflag[t] = bal;
}

// The position-contiguous copy (lin): lin[p / 32] holds bit p % 32 of the
// hi, lo, brk and oth planes of positions p..  One block per tile: the
// tile's 2048 physical words of hl and bo in LDS, then every lin word of the
// tile is a 32 x 1-bit gather over one lane's column (conflict-free: a wave
// reads 64 consecutive physical words).  Random access to a few consecutive
// positions (the report pass's text windows) then costs one line instead of
// one line per position.
__global__ __launch_bounds__(256) void k_build_lin(uint64_t ntiles, const uint2* __restrict__ hl,
                                                   const uint2* __restrict__ bo, uint4* __restrict__ lin) {
    __shared__ uint2 shl[STREAM], sbo[STREAM];
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        for (uint32_t i = threadIdx.x; i < STREAM; i += blockDim.x) {
            shl[i] = hl[t * TILE_WORDS + i];
            sbo[i] = bo[t * TILE_WORDS + i];
        }
        __syncthreads();
        for (uint32_t o = threadIdx.x; o < STREAM; o += blockDim.x) {
            // lin word o of the tile: stream b = o / 64, logical words
            // 32 j .. 32 j + 31 (j = o % 64), i.e. physical i * 64 + j
            const uint32_t b = o >> 6, j = o & 63;
            uint32_t h = 0, l = 0, k = 0, x = 0;
#pragma unroll 8
            for (uint32_t i = 0; i < 32; ++i) {
                const uint2 d = shl[i * 64 + j], e = sbo[i * 64 + j];
                h |= ((d.x >> b) & 1u) << i;
                l |= ((d.y >> b) & 1u) << i;
                k |= ((e.x >> b) & 1u) << i;
                x |= ((e.y >> b) & 1u) << i;
            }
            lin[t * STREAM + o] = make_uint4(h, l, k, x);
        }
        __syncthreads();
    }
}

__global__ void k_pack_bytes(const uint8_t* __restrict__ raw, uint64_t n, uint64_t nalloc,
                             uint8_t* __restrict__ out) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= nalloc) return;
    out[i] = i < n ? fold(raw[i]) : (uint8_t)'\n';
}

__global__ void k_mark_ranges_bytes(const uint64_t* __restrict__ ranges, uint64_t nr, uint8_t* __restrict__ bytes) {
    const uint64_t i = blockIdx.x;
    if (i >= nr) return;
    const uint64_t b = ranges[2 * i], e = ranges[2 * i + 1];
    for (uint64_t p = b + threadIdx.x; p < e; p += blockDim.x) bytes[p] = '\n';
}

// which byte values occur (BYTE databases): one flag per value
__global__ void k_byte_seen(const uint8_t* __restrict__ bytes, uint64_t n, uint32_t* __restrict__ seen) {
    __shared__ uint32_t s[8];
    if (threadIdx.x < 8) s[threadIdx.x] = 0u;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t b = bytes[i];
        atomicOr(&s[b >> 5], 1u << (b & 31));
    }
    __syncthreads();
    if (threadIdx.x < 8 && s[threadIdx.x]) atomicOr(&seen[threadIdx.x], s[threadIdx.x]);
}

// The 5-bit residue planes: thread per 32-position word; plane q bit i =
// bit q of the code of position 32 w + i (padding words stay 0: breaks).
__global__ void k_pack_p5(const uint8_t* __restrict__ bytes, const uint8_t* __restrict__ raw, uint64_t nbytes, uint64_t nw,
                          const uint8_t* __restrict__ code, uint32_t* __restrict__ p5) {
    const uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (w >= nw) return;
    uint32_t pl[5] = {0u, 0u, 0u, 0u, 0u};
    const uint64_t b0 = w * 32;
    for (int i = 0; i < 32; ++i) {
        const uint64_t p = b0 + i;
        // header bytes read '\n' in the byte copy, themselves in raw
        const uint32_t c = p >= nbytes ? 0u : bytes[p] != '\n' ? code[bytes[p]] : raw[p] == '\n' ? P5_NL : 0u;
#pragma unroll
        for (int q = 0; q < 5; ++q) pl[q] |= ((c >> q) & 1u) << i;
    }
#pragma unroll
    for (int q = 0; q < 5; ++q) p5[(uint64_t)q * nw + w] = pl[q];
}

__global__ void k_decode(NucView v, uint64_t beg, uint32_t len, uint8_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < len) out[i] = nuc_raw_at(v, beg + i);
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
template <class T>
T* dalloc(pm_db* db, uint64_t count) {
    void* p = nullptr;
    if (count == 0) count = 1;
    HIPCHK(hipMalloc(&p, count * sizeof(T)));
    db->device_bytes += count * sizeof(T);
    return static_cast<T*>(p);
}

template <class T>
T* tmp_alloc(std::vector<void*>& owned, uint64_t count) {
    void* p = nullptr;
    HIPCHK(hipMalloc(&p, std::max<uint64_t>(count, 1) * sizeof(T)));
    owned.push_back(p);
    return static_cast<T*>(p);
}

void free_all(pm_db* db, std::vector<void*>& owned) {
    HIPCHK(hipStreamSynchronize(db->stream));
    for (void* p : owned) HIPCHK(hipFree(p));
    owned.clear();
}

// header lines (/^>\S/) as [beg, end) ranges, end excluding the '\n'
std::vector<uint64_t> header_ranges(const uint8_t* t, uint64_t n) {
    std::vector<uint64_t> r;
    uint64_t p = 0;
    while (p < n) {
        const void* nl = memchr(t + p, '\n', n - p);
        const uint64_t e = nl ? (uint64_t)((const uint8_t*)nl - t) : n;
        if (t[p] == '>' && p + 1 < e) {
            const uint8_t c = t[p + 1];
            const bool space = c == ' ' || c == '\t' || c == '\r' || c == '\f' || c == '\v';
            if (!space) { r.push_back(p); r.push_back(e); }
        }
        p = e + 1;
    }
    return r;
}

// the header line starts, kept on the device for the eextended walk
void set_headers(pm_db* db, const std::vector<uint64_t>& starts) {
    db->nhdr = starts.size();
    if (!db->nhdr) return;
    db->hdr = dalloc<uint64_t>(db, db->nhdr);
    HIPCHK(hipMemcpy(db->hdr, starts.data(), db->nhdr * 8, hipMemcpyHostToDevice));
}

// Tiles cover the file plus room for the longest NFA halo after the last
// chunk; every position >= n is a break.
uint64_t tiles_for(uint64_t n) { return (n + MAX_NFA_CHUNK + 2048 + TILE_POS - 1) / TILE_POS; }

void alloc_planes(pm_db* db) {
    db->ntiles = tiles_for(db->n);
    db->nwords = db->ntiles * TILE_WORDS;
    db->nsb = db->nwords / 32;
    db->hl = dalloc<uint2>(db, db->nwords + 128);   // + LDS-DMA over-read of the last tile
    db->bo = dalloc<uint2>(db, db->nwords);
    db->lflag = dalloc<uint64_t>(db, db->ntiles);
    db->hflag = dalloc<uint64_t>(db, db->ntiles);
}

// halo words, flags, compacted exception side tables, lane flags
void finish_nuc(pm_db* db, std::vector<void*>& owned, const uint8_t* d_raw, uint64_t syn_rec_len = 0,
                uint64_t syn_seed = 0) {
    hipStream_t s = db->stream;
    hipLaunchKernelGGL(k_clean_oth, dim3(blocks_for(db->nwords, 256)), dim3(256), 0, s, db->nwords, db->bo);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_fill_halo, dim3(blocks_for(db->ntiles * HALO, 256)), dim3(256), 0, s, db->ntiles, db->hl,
                       db->bo);
    HIPCHK(hipGetLastError());
    db->sbflag = dalloc<uint32_t>(db, db->nsb);
    db->sbbase = dalloc<uint32_t>(db, db->nsb);
    uint32_t* sbcnt = tmp_alloc<uint32_t>(owned, db->nsb);
    hipLaunchKernelGGL(k_sb_flags, dim3(blocks_for(db->nsb, 256)), dim3(256), 0, s, db->bo, db->nsb, db->sbflag,
                       sbcnt);
    HIPCHK(hipGetLastError());
    size_t tmp_bytes = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, sbcnt, db->sbbase, (int)db->nsb, s));
    clear_stale_capture_status("rocPRIM call (pm_db)");   // (a check after the call, pm_internal.h)
    void* tmp = tmp_alloc<uint8_t>(owned, tmp_bytes);
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, sbcnt, db->sbbase, (int)db->nsb, s));
    clear_stale_capture_status("rocPRIM call (pm_db)");   // (fails on any status but a caller's capture code)
    uint32_t* h = static_cast<uint32_t*>(reserve_host(db, db->pin_down, 16));
    HIPCHK(hipMemcpyAsync(h, db->sbbase + db->nsb - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(h + 1, sbcnt + db->nsb - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    db->nflag = (uint64_t)h[0] + h[1];
    db->xbrk = dalloc<uint32_t>(db, db->nflag);
    db->xoth = dalloc<uint32_t>(db, db->nflag);
    db->xword = dalloc<uint64_t>(db, db->nflag);
    db->xbytes = dalloc<uint8_t>(db, db->nflag * 32);
    uint32_t* d_noth = static_cast<uint32_t*>(reserve(db, db->ws_post, sizeof(uint32_t)));
    HIPCHK(hipMemsetAsync(d_noth, 0, sizeof(uint32_t), s));
    hipLaunchKernelGGL(k_fill_exceptions, dim3(blocks_for(db->nwords, 256)), dim3(256), 0, s, d_raw, db->n,
                       db->nwords, db->bo, db->sbflag, db->sbbase, db->xbrk, db->xoth, db->xword,
                       db->xbytes, d_noth, syn_rec_len, syn_seed);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(h, d_noth, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    db->n_oth_words = h[0];   // 0: scans skip the "other byte" pass
    hipLaunchKernelGGL(k_lane_flags, dim3(blocks_for(db->ntiles * 64, 256)), dim3(256), 0, s, db->ntiles, db->bo,
                       db->lflag);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_header_flags, dim3(blocks_for(db->ntiles * 64, 256)), dim3(256), 0, s, db->ntiles, db->bo,
                       db->sbflag, db->sbbase, db->xbytes, db->hflag);
    HIPCHK(hipGetLastError());
    db->lin = dalloc<uint4>(db, db->ntiles * STREAM);   // 0.5 byte per position
    hipLaunchKernelGGL(k_build_lin, dim3((uint32_t)std::min<uint64_t>(db->ntiles, 8192)), dim3(256), 0, s, db->ntiles,
                       db->hl, db->bo, db->lin);
    HIPCHK(hipGetLastError());
    require(db->nflag < (1ull << 32), "too many exception words for the run index", PM_E_UNSUPPORTED);
    db->xint = dalloc<uint32_t>(db, db->nflag);
    db->xedge = dalloc<uint32_t>(db, db->nflag);
    db->xedge_oth = dalloc<uint32_t>(db, db->nflag);
    unsigned long long* d_nedge = static_cast<unsigned long long*>(reserve(db, db->ws_post, 2 * sizeof(uint64_t)));
    HIPCHK(hipMemsetAsync(d_nedge, 0, 2 * sizeof(uint64_t), s));
    if (db->nflag) {
        hipLaunchKernelGGL(k_run_interior, dim3(blocks_for(db->nflag, 256)), dim3(256), 0, s, db->nflag, db->xword,
                           db->xbrk, db->xoth, db->bo, db->xint, db->xedge, db->xedge_oth, d_nedge);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipMemcpyAsync(h, d_nedge, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    db->nedge = reinterpret_cast<uint64_t*>(h)[0];
    db->nedge_oth = reinterpret_cast<uint64_t*>(h)[1];
    // the "other"-position list: count, allocate, fill
    for (int fill = 0; fill < 2; ++fill) {
        HIPCHK(hipMemsetAsync(d_nedge, 0, sizeof(uint64_t), s));
        if (db->nedge_oth)
            hipLaunchKernelGGL(k_build_xlist, dim3(blocks_for(db->nedge_oth, 256)), dim3(256), 0, s, db->nedge_oth,
                               db->xedge_oth, db->xword, db->xoth, db->xint, db->lin, db->ntiles * STREAM, db->xlist,
                               d_nedge, fill);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(h, d_nedge, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (!fill) {
            db->nxlist = reinterpret_cast<uint64_t*>(h)[0];
            db->xlist = dalloc<uint64_t>(db, db->nxlist);
        }
    }
    if (env_flag("PM_DEBUG_DB", false))
        fprintf(stderr, "pm_db: n=%llu tiles=%llu flagged words=%llu other words=%llu edge words=%llu (other %llu)\n",
                (unsigned long long)db->n, (unsigned long long)db->ntiles, (unsigned long long)db->nflag,
                (unsigned long long)db->n_oth_words, (unsigned long long)db->nedge,
                (unsigned long long)db->nedge_oth);
}

void init_stream(pm_db* db, void* stream) {
    if (stream) {
        db->stream = (hipStream_t)stream;
    } else {
        // non-blocking: work a caller queues on the null stream (e.g. copying
        // out the previous query's hits) must not wait for -- or stall the
        // host behind -- the scan in flight; consumers order on events
        HIPCHK(hipStreamCreateWithFlags(&db->stream, hipStreamNonBlocking));
        db->own_stream = true;
    }
}

void free_db(pm_db* db) {
    if (!db) return;
    // pipelined scans still pending resolve now (a re-run needs the database)
    while (!db->pending.empty()) {
        pm_hits* h = *db->pending.begin();
        try {
            hits_finalize(h);
        } catch (...) {
            db->pending.erase(h);   // the list stays unresolved (count 0)
        }
    }
    if (db->stream) quiet(hipStreamSynchronize(db->stream));
    if (db->post) {
        quiet(hipStreamSynchronize(db->post));
        quiet(hipStreamDestroy(db->post));
    }
    if (db->exc) {
        quiet(hipStreamSynchronize(db->exc));
        quiet(hipStreamDestroy(db->exc));
    }
    for (hipEvent_t e : {db->exc_fork, db->exc_join, db->scan_ev, db->join_ev})
        if (e) quiet(hipEventDestroy(e));
    void* ptrs[] = {db->hdr, db->reg_t, db->reg_e, db->reg_lut, db->reg_near, db->hl, db->bo, db->lin, db->sbflag, db->sbbase, db->xbrk, db->xoth, db->xword, db->xbytes,
                    db->lflag, db->hflag, db->xint, db->xedge, db->xedge_oth, db->xlist, db->p5, db->hdr_end, db->bytes, db->bytes_raw, db->ws_post.p,
                    db->ws_batch.p};
    for (void* p : ptrs)
        if (p) quiet(hipFree(p));
    if (db->pin_down.p) quiet(hipHostFree(db->pin_down.p));
    if (db->pin_ord.p) quiet(hipHostFree(db->pin_ord.p));
    for (pm_lane* l : {static_cast<pm_lane*>(db), &db->alt}) {
        for (void* p : {l->ws_tab.p, l->ws_sink.p, l->ws_rec.p, l->ws_rep.p, l->ws_oth.p})
            if (p) quiet(hipFree(p));
        for (void* p : {l->pin_up.p, l->pin_slots.p})
            if (p) quiet(hipHostFree(p));
        for (hipEvent_t e : {l->up_fence, l->slots_fence, l->free_ev})
            if (e) quiet(hipEventDestroy(e));
    }
    if (db->own_stream && db->stream) quiet(hipStreamDestroy(db->stream));
    delete db;
}

void check_device(int device) {
    int ndev = 0;
    const hipError_t e = hipGetDeviceCount(&ndev);
    quiet(e);   // reported as PM_E_NODEV below, not left pending
    if (e != hipSuccess || ndev == 0) throw failure(PM_E_NODEV, "no HIP device");
    require(device >= 0 && device < ndev, "device out of range");
}

}  // namespace

// Grow a workspace.  Growing waits for the stream first, so no queued work
// can still reference the old allocation.
void lane_begin(pm_db* db) {
    if (db->free_ev) HIPCHK(hipStreamWaitEvent(db->stream, db->free_ev, 0));
}

void lane_end(pm_db* db, hipStream_t s) {
    // while every scan of this database ran on its own stream (no post
    // stream yet), stream order already serializes the lane's users: no
    // marker packet between one scan's sort and the next scan's kernel
    if (!db->post && s == db->stream) return;
    if (!db->free_ev) HIPCHK(hipEventCreateWithFlags(&db->free_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(db->free_ev, s));
}

void switch_lane(pm_db* db) { std::swap(static_cast<pm_lane&>(*db), db->alt); }

int post_mode() {
    static const int v = [] {
        const char* e = getenv("PM_POST_STREAM");
        return e && (e[0] == '1' || e[0] == '2') ? e[0] - '0' : 0;
    }();
    return v;
}

hipStream_t post_stream(pm_db* db) {
    if (!db->post) {
        if (post_mode() == 2) {
            int least = 0, greatest = 0;
            HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
            HIPCHK(hipStreamCreateWithPriority(&db->post, hipStreamNonBlocking, greatest));
        } else {
            HIPCHK(hipStreamCreateWithFlags(&db->post, hipStreamNonBlocking));
        }
        HIPCHK(hipEventCreateWithFlags(&db->scan_ev, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&db->join_ev, hipEventDisableTiming));
    }
    return db->post;
}

void post_join(pm_db* db) {
    if (!db->post) return;
    HIPCHK(hipEventRecord(db->join_ev, db->post));
    HIPCHK(hipStreamWaitEvent(db->stream, db->join_ev, 0));
}

hipStream_t exc_stream(pm_db* db) {
    if (!db->exc) {
        HIPCHK(hipStreamCreateWithFlags(&db->exc, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&db->exc_fork, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&db->exc_join, hipEventDisableTiming));
    }
    return db->exc;
}

void* reserve(pm_db* db, pm_devbuf& b, size_t bytes) {
    if (b.cap < bytes) {
        HIPCHK(hipStreamSynchronize(db->stream));
        if (db->post) HIPCHK(hipStreamSynchronize(db->post));
        if (db->exc) HIPCHK(hipStreamSynchronize(db->exc));
        if (b.p) HIPCHK(hipFree(b.p));
        b.p = nullptr;
        b.cap = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 20);
        HIPCHK(hipMalloc(&b.p, want));
        b.cap = want;
    }
    return b.p;
}

void* reserve_host(pm_db* db, pm_hostbuf& b, size_t bytes) {
    if (b.cap < bytes) {
        HIPCHK(hipStreamSynchronize(db->stream));
        if (b.p) HIPCHK(hipHostFree(b.p));
        b.p = nullptr;
        b.cap = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 16);
        HIPCHK(hipHostMalloc(&b.p, want, hipHostMallocDefault));
        b.cap = want;
    }
    return b.p;
}

uint8_t* Upload::commit(pm_db* db) {
    uint8_t* d = static_cast<uint8_t*>(reserve(db, db->ws_tab, std::max<size_t>(blob.size(), 256)));
    if (db->up_cache_p == (void*)d && db->up_cache == blob) return d;   // a repeated query: tables in place
    // the pinned staging buffer is rewritten only after its last copy ran
    // (a pipelined scan may still have it queued)
    if (db->up_fence) HIPCHK(hipEventSynchronize(db->up_fence));
    uint8_t* h = static_cast<uint8_t*>(reserve_host(db, db->pin_up, std::max<size_t>(blob.size(), 256)));
    memcpy(h, blob.data(), blob.size());
    HIPCHK(hipMemcpyAsync(d, h, blob.size(), hipMemcpyHostToDevice, db->stream));
    if (!db->up_fence) HIPCHK(hipEventCreateWithFlags(&db->up_fence, hipEventDisableTiming));
    HIPCHK(hipEventRecord(db->up_fence, db->stream));
    db->up_cache = blob;
    db->up_cache_p = d;
    return d;
}

// The 5-bit residue planes of a BYTE database (pm_db::p5), when its folded
// bytes take at most 30 values besides '\n'; `ranges`: the header lines.
void build_p5(pm_db* db, std::vector<void*>& owned, const std::vector<uint64_t>& ranges) {
    hipStream_t s = db->stream;
    uint32_t* d_seen = tmp_alloc<uint32_t>(owned, 8);
    HIPCHK(hipMemsetAsync(d_seen, 0, 32, s));
    hipLaunchKernelGGL(k_byte_seen, dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(1024, blocks_for(db->n, 256)))),
                       dim3(256), 0, s, db->bytes, db->n, d_seen);
    HIPCHK(hipGetLastError());
    uint32_t seen[8];
    HIPCHK(hipMemcpyAsync(seen, d_seen, 32, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    memset(db->code_of, 0, sizeof db->code_of);
    db->code_of['\n'] = (uint8_t)P5_NL;
    int nc = (int)P5_NL;
    for (int b = 0; b < 256; ++b)
        if (b != '\n' && ((seen[b >> 5] >> (b & 31)) & 1)) {
            if (++nc > 31) {
                memset(db->code_of, 0, sizeof db->code_of);
                db->n_codes = 0;
                return;   // the byte copy is scanned
            }
            db->code_of[b] = (uint8_t)nc;
        }
    db->n_codes = nc;
    if (db->nhdr) {
        std::vector<uint64_t> ends(db->nhdr);
        for (uint64_t r = 0; r < db->nhdr; ++r) ends[r] = ranges[2 * r + 1];
        db->hdr_end = dalloc<uint64_t>(db, db->nhdr);
        HIPCHK(hipMemcpy(db->hdr_end, ends.data(), db->nhdr * 8, hipMemcpyHostToDevice));
    }
    db->nw5 = (db->n + 31) / 32 + P5_PAD;
    db->p5 = dalloc<uint32_t>(db, 5 * db->nw5);
    HIPCHK(hipMemsetAsync(db->p5, 0, 5 * db->nw5 * 4, s));
    uint8_t* d_code = tmp_alloc<uint8_t>(owned, 256);
    HIPCHK(hipMemcpyAsync(d_code, db->code_of, 256, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_pack_p5, dim3(blocks_for(db->nw5, 256)), dim3(256), 0, s, db->bytes, db->bytes_raw, db->n, db->nw5,
                       d_code, db->p5);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));   // d_code is freed with the other temporaries
}

NucView nuc_view(const pm_db* db) {
    return NucView{db->hl, db->bo, db->sbflag, db->sbbase, db->xbytes, db->lin};
}

// the region table on the device: starts, ends, and the bucket lookup
void set_regions(pm_db* db, const std::vector<uint64_t>& t, const std::vector<uint64_t>& e) {
    require(t.size() == e.size() && !t.empty() && t.size() < (1ull << 31), "bad region table");
    for (size_t r = 0; r < t.size(); ++r) {
        require(t[r] <= e[r] && e[r] <= db->n, "region outside the database");
        require(r == 0 ? t[r] == 0 : t[r] > t[r - 1], "region starts must increase from 0");
    }
    const uint64_t nlut = (db->n >> REG_LUT_SHIFT) + 1;
    std::vector<uint32_t> lut(nlut);
    for (uint64_t b = 0, r = 0; b < nlut; ++b) {
        while (r + 1 < t.size() && t[r + 1] <= (b << REG_LUT_SHIFT)) ++r;
        lut[b] = (uint32_t)r;
    }
    // blocks with a region start (> 0) within REG_NEAR_SPAN on either side
    const uint64_t nblk = (db->n >> REG_NEAR_SHIFT) + 1;
    std::vector<uint32_t> near((nblk + 31) / 32, 0u);
    for (size_t r = 1; r < t.size(); ++r) {
        const uint64_t lo = t[r] > REG_NEAR_SPAN ? t[r] - REG_NEAR_SPAN : 0, hi = t[r] + REG_NEAR_SPAN;
        for (uint64_t b = lo >> REG_NEAR_SHIFT; b <= (hi >> REG_NEAR_SHIFT) && b < nblk; ++b) near[b >> 5] |= 1u << (b & 31);
    }
    // the new tables are built completely before the old ones go: a failed
    // allocation or copy leaves the database with its previous regions
    void* nt[4] = {nullptr, nullptr, nullptr, nullptr};
    try {
        HIPCHK(hipMalloc(&nt[0], t.size() * 8));
        HIPCHK(hipMalloc(&nt[1], e.size() * 8));
        HIPCHK(hipMalloc(&nt[2], nlut * 4));
        HIPCHK(hipMalloc(&nt[3], near.size() * 4));
        HIPCHK(hipMemcpy(nt[0], t.data(), t.size() * 8, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(nt[1], e.data(), e.size() * 8, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(nt[2], lut.data(), nlut * 4, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(nt[3], near.data(), near.size() * 4, hipMemcpyHostToDevice));
    } catch (...) {
        for (void* p : nt)
            if (p) quiet(hipFree(p));
        throw;
    }
    HIPCHK(hipStreamSynchronize(db->stream));   // queued scans may still read the old table
    if (db->post) HIPCHK(hipStreamSynchronize(db->post));   // (and their post-processing)
    for (void* p : {(void*)db->reg_t, (void*)db->reg_e, (void*)db->reg_lut, (void*)db->reg_near})
        if (p) HIPCHK(hipFree(p));
    db->reg_t = static_cast<uint64_t*>(nt[0]);
    db->reg_e = static_cast<uint64_t*>(nt[1]);
    db->reg_lut = static_cast<uint32_t*>(nt[2]);
    db->reg_near = static_cast<uint32_t*>(nt[3]);
    db->nreg = (uint32_t)t.size();
    db->reg_blind = false;
    for (size_t r = 0; r + 1 < t.size(); ++r) db->reg_blind |= e[r] != t[r + 1] + 1;
}

}  // namespace pm

using namespace pm;

extern "C" {

const char* pm_last_error(void) { return g_err.c_str(); }
const char* pm_version(void) { return "patmatch_hip 0.3 (gfx950, stream-tile layout)"; }

int pm_device_count(int* count) {
    return guarded([&] {
        require(count != nullptr, "count is NULL");
        int c = 0;
        const hipError_t e = hipGetDeviceCount(&c);
        quiet(e);   // no device is an answer (0), not a status for the next call
        if (e != hipSuccess) c = 0;
        *count = c;
    });
}

int pm_db_create(const uint8_t* fasta, uint64_t n, int alphabet, int device, void* stream, pm_db** out) {
    pm_db* db = nullptr;
    std::vector<void*> owned;
    int rc = guarded([&] {
        require(out != nullptr && (fasta != nullptr || n == 0), "null argument");
        require(alphabet == PM_ALPHA_NUC || alphabet == PM_ALPHA_BYTE, "unknown alphabet");
        check_device(device);
        DeviceGuard g(device);
        init_code_table();
        db = new pm_db();
        db->device = device;
        db->alphabet = alphabet;
        db->n = n;
        init_stream(db, stream);
        hipStream_t s = db->stream;
        const std::vector<uint64_t> ranges = header_ranges(fasta, n);
        const uint64_t nr = ranges.size() / 2;
        {
            std::vector<uint64_t> hs(nr);
            for (uint64_t i = 0; i < nr; ++i) hs[i] = ranges[2 * i];
            set_headers(db, hs);
        }
        uint64_t* d_ranges = tmp_alloc<uint64_t>(owned, ranges.size());
        if (nr) HIPCHK(hipMemcpy(d_ranges, ranges.data(), ranges.size() * 8, hipMemcpyHostToDevice));
        uint8_t* d_raw = tmp_alloc<uint8_t>(owned, n + 64);
        if (n) HIPCHK(hipMemcpy(d_raw, fasta, n, hipMemcpyHostToDevice));
        if (alphabet == PM_ALPHA_NUC) {
            alloc_planes(db);
            hipLaunchKernelGGL(k_pack_nuc, dim3(blocks_for(db->ntiles * STREAM, 256)), dim3(256), 0, s, d_raw, n,
                               db->ntiles, db->hl, db->bo);
            HIPCHK(hipGetLastError());
            if (nr) {
                hipLaunchKernelGGL(k_mark_ranges, dim3(blocks_for(nr, 64)), dim3(64), 0, s, d_ranges, nr, db->bo);
                HIPCHK(hipGetLastError());
            }
            finish_nuc(db, owned, d_raw);
        } else {
            db->nbytes_alloc = round_up(n + BYTE_PAD, 4096);
            db->bytes = dalloc<uint8_t>(db, db->nbytes_alloc);
            hipLaunchKernelGGL(k_pack_bytes, dim3(blocks_for(db->nbytes_alloc, 256)), dim3(256), 0, s, d_raw, n,
                               db->nbytes_alloc, db->bytes);
            HIPCHK(hipGetLastError());
            // the file's own bytes (headers kept): nrgrep's simple engine may
            // match across a line break, and '^'/'$' look at real bytes
            db->bytes_raw = dalloc<uint8_t>(db, db->nbytes_alloc);
            HIPCHK(hipMemcpyAsync(db->bytes_raw, db->bytes, db->nbytes_alloc, hipMemcpyDeviceToDevice, s));
            if (nr) {
                hipLaunchKernelGGL(k_mark_ranges_bytes, dim3((uint32_t)nr), dim3(256), 0, s, d_ranges, nr, db->bytes);
                HIPCHK(hipGetLastError());
            }
            build_p5(db, owned, ranges);
        }
        free_all(db, owned);
        std::vector<uint64_t> rt, re;
        nrgrep_regions(n, PM_NRGREP_BUFFER, [&](uint64_t lo, uint64_t hi) {
            const void* p = memrchr(fasta + lo, '\n', hi - lo);
            return p ? (uint64_t)(static_cast<const uint8_t*>(p) - fasta) : ~0ull;
        }, rt, re);
        set_regions(db, rt, re);
        *out = db;
    });
    if (rc != PM_OK) {
        if (db && db->stream) quiet(hipStreamSynchronize(db->stream));
        for (void* p : owned) quiet(hipFree(p));
        free_db(db);
    }
    return rc;
}

int pm_db_create_synthetic(uint64_t n_records, uint64_t rec_len, uint64_t seed, int device, void* stream,
                           pm_db** out) {
    pm_db* db = nullptr;
    std::vector<void*> owned;
    int rc = guarded([&] {
        require(out != nullptr && n_records > 0 && rec_len > 0, "bad synthetic shape");
        check_device(device);
        DeviceGuard g(device);
        init_code_table();
        db = new pm_db();
        db->device = device;
        db->alphabet = PM_ALPHA_NUC;
        db->n = n_records * (SYN_HDR + 1 + rec_len + 1);
        init_stream(db, stream);
        alloc_planes(db);
        hipLaunchKernelGGL(k_pack_synth, dim3(blocks_for(db->ntiles * STREAM, 256)), dim3(256), 0, db->stream,
                           db->n, db->ntiles, rec_len, seed, db->hl, db->bo);
        HIPCHK(hipGetLastError());
        finish_nuc(db, owned, nullptr, rec_len, seed);
        free_all(db, owned);
        // the layout's line breaks: after each header and each record
        const uint64_t rb = SYN_HDR + 1 + rec_len + 1;
        {
            std::vector<uint64_t> hs(n_records);
            for (uint64_t r = 0; r < n_records; ++r) hs[r] = r * rb;
            set_headers(db, hs);
        }
        std::vector<uint64_t> rt, re;
        nrgrep_regions(db->n, PM_NRGREP_BUFFER, [&](uint64_t lo, uint64_t hi) {
            if (hi == 0) return ~0ull;
            const uint64_t q = hi - 1, r = q / rb, o = q % rb;
            const uint64_t d = o >= rb - 1 ? r * rb + rb - 1 : o >= SYN_HDR ? r * rb + SYN_HDR
                             : r ? (r - 1) * rb + rb - 1 : ~0ull;
            return d != ~0ull && d >= lo ? d : ~0ull;
        }, rt, re);
        set_regions(db, rt, re);
        *out = db;
    });
    if (rc != PM_OK) {
        if (db && db->stream) quiet(hipStreamSynchronize(db->stream));
        for (void* p : owned) quiet(hipFree(p));
        free_db(db);
    }
    return rc;
}

int pm_db_set_regions(pm_db* db, uint64_t count, const uint64_t* starts, const uint64_t* ends) {
    return guarded([&] {
        require(db != nullptr && starts != nullptr && ends != nullptr && count >= 1, "null argument");
        std::lock_guard<std::recursive_mutex> lk(db->mu);
        DeviceGuard g(db->device);
        set_regions(db, std::vector<uint64_t>(starts, starts + count), std::vector<uint64_t>(ends, ends + count));
    });
}

int pm_db_regions(const pm_db* db, uint64_t cap, uint64_t* starts, uint64_t* ends, uint64_t* count) {
    return guarded([&] {
        require(db != nullptr && count != nullptr && (cap == 0 || (starts && ends)), "null argument");
        std::lock_guard<std::recursive_mutex> lk(const_cast<pm_db*>(db)->mu);
        *count = db->nreg;
        const uint64_t n = std::min<uint64_t>(cap, db->nreg);
        if (n) {
            DeviceGuard g(db->device);
            HIPCHK(hipMemcpy(starts, db->reg_t, n * 8, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(ends, db->reg_e, n * 8, hipMemcpyDeviceToHost));
        }
    });
}

int pm_db_destroy(pm_db* db) {
    return guarded([&] {
        if (!db) return;
        DeviceGuard g(db->device);
        {   // wait for a scan in flight on another thread; its pending lists resolve here
            std::lock_guard<std::recursive_mutex> lk(db->mu);
            while (!db->pending.empty()) {
                pm_hits* h = *db->pending.begin();
                try {
                    hits_finalize(h);
                } catch (...) {
                    db->pending.erase(h);   // the list stays unresolved (count 0)
                }
            }
        }
        free_db(db);
    });
}

int pm_db_info(const pm_db* db, uint64_t* n_positions, int* alphabet, uint64_t* n_exception_words,
               uint64_t* device_bytes) {
    return guarded([&] {
        require(db != nullptr, "db is NULL");
        if (n_positions) *n_positions = db->n;
        if (alphabet) *alphabet = db->alphabet;
        if (n_exception_words) *n_exception_words = db->nflag;
        if (device_bytes) *device_bytes = db->device_bytes;
    });
}

int pm_db_residue_codes(const pm_db* db, int* n_codes, uint8_t* code_of_byte) {
    return guarded([&] {
        require(db != nullptr, "db is NULL");
        if (n_codes) *n_codes = db->n_codes;
        if (code_of_byte) memcpy(code_of_byte, db->code_of, 256);
    });
}

int pm_db_decode(pm_db* db, uint64_t beg, uint32_t len, uint8_t* out) {
    return guarded([&] {
        require(db != nullptr && out != nullptr, "null argument");
        std::lock_guard<std::recursive_mutex> lk(db->mu);
        require(beg + len <= db->n, "decode range outside the database");
        if (len == 0) return;
        DeviceGuard g(db->device);
        uint8_t* d = static_cast<uint8_t*>(reserve(db, db->ws_post, len));
        if (db->alphabet == PM_ALPHA_NUC) {
            hipLaunchKernelGGL(k_decode, dim3(blocks_for(len, 256)), dim3(256), 0, db->stream, nuc_view(db), beg, len, d);
            HIPCHK(hipGetLastError());
        } else {
            HIPCHK(hipMemcpyAsync(d, db->bytes + beg, len, hipMemcpyDeviceToDevice, db->stream));
        }
        HIPCHK(hipStreamSynchronize(db->stream));
        HIPCHK(hipMemcpy(out, d, len, hipMemcpyDeviceToHost));
    });
}

}  // extern "C"
