// pm_scan.hip -- MI355X (gfx950) PatMatch scan engine behind include/patmatch_hip.h.
//
// Replaces the reference's `nrgrep_coords` process boundary
// (www/FlaskApp/FlaskApp/patmatch.py:733-742, :818-828).  Design notes live
// in DESIGN.md; the short version:
//
//  * Database in HBM, coordinate space = byte offsets of the FASTA file.
//    Nucleotide files: two bit-planes (hi, lo) of 2-bit A/C/G/T codes, one
//    u32 word per 32 positions (0.25 B/base).  Everything else ('\n', header
//    lines, N and other IUPAC bytes, the tail padding) is an "exception":
//    one flag bit per word in a per-superblock (1024 positions) u32 plus a
//    compacted side table {brk mask, oth mask, 32 raw bytes} per flagged
//    word.  Peptide files: one case-folded byte per residue.
//  * k_linear: fixed-length patterns (the common DNA case) with <= k
//    substitutions, bit-sliced over 32 text positions per VALU word: per
//    pattern position one v_alignbit of a class-mismatch word plus k+1
//    v_and_or/v_bitop3 thermometer-counter updates.  No MFMA: this is
//    integer bit-twiddling bound by HBM/VALU.
//  * k_nfa_rev + k_nfa_verify: general patterns (classes, ? * + |, m <= 64)
//    as a bit-parallel Glushkov automaton, one 64-bit state word per lane
//    and error row; the reverse scan finds every match start, the verify
//    pass finds the shortest end from each start (the reported semantics).
//  * Hits leave the kernels through wave-aggregated atomics into 1024
//    independent bins (no single hot counter), are compacted and radix
//    sorted by (pattern, beg) on the device.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <map>
#include <mutex>
#include <sstream>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "patmatch_hip.h"

namespace {

thread_local std::string g_err;

struct pm_failure : std::runtime_error {
    int code;
    pm_failure(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIPCHK(expr)                                                                   \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            throw pm_failure(PM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

template <class F>
int guarded(F&& f) {
    try {
        f();
        return PM_OK;
    } catch (const pm_failure& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::exception& e) {
        g_err = e.what();
        return PM_E_ARG;
    }
}

void require(bool ok, const char* msg, int code = PM_E_ARG) {
    if (!ok) throw pm_failure(code, msg);
}

constexpr int PAD_WORDS = 1024;        // tail padding (32768 positions, all breaks)
constexpr uint32_t NBINS = 1024;       // independent hit counters
constexpr int MAX_NFA_CHUNK = 4096;    // positions per lane in k_nfa_rev

__host__ __device__ inline uint8_t fold(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }

// code of a folded byte: 0..3 = A C G T, 4 = delimiter, 5 = other
__constant__ uint8_t c_code[256];

uint64_t round_up(uint64_t x, uint64_t m) { return (x + m - 1) / m * m; }

}  // namespace

// ---------------------------------------------------------------------------
// device database
// ---------------------------------------------------------------------------
struct DevBuf {          // device buffer grown on demand, reused across calls
    void* p = nullptr;
    size_t cap = 0;
};
struct HostBuf {         // pinned host staging buffer
    void* p = nullptr;
    size_t cap = 0;
};

struct pm_db {
    int device = 0;
    int alphabet = PM_ALPHA_NUC;
    uint64_t n = 0;          // positions (file bytes)
    uint64_t nwords = 0;     // NUC: plane words incl. padding
    uint64_t nsb = 0;        // NUC: superblocks (32 words)
    uint64_t nflag = 0;      // NUC: exception words
    uint64_t nbytes_alloc = 0;
    uint32_t *hi = nullptr, *lo = nullptr, *sbflag = nullptr, *sbbase = nullptr;
    uint32_t *xbrk = nullptr, *xoth = nullptr;
    uint8_t* xbytes = nullptr;
    uint8_t* bytes = nullptr; // BYTE alphabet
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // per-call workspaces (never stream-ordered allocations)
    DevBuf ws_tab, ws_sink, ws_post;
    HostBuf pin_up, pin_down;
    uint64_t device_bytes = 0;
};

struct pm_hits {
    int device = 0;
    uint64_t count = 0;
    uint64_t* keys = nullptr;   // sorted, pattern << 48 | beg
    uint32_t* lens = nullptr;
    double kernel_ms = 0.0;
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        HIPCHK(hipGetDevice(&prev));
        if (prev != dev) HIPCHK(hipSetDevice(dev));
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

template <class T>
T* dalloc(pm_db* db, uint64_t count) {
    void* p = nullptr;
    if (count == 0) count = 1;
    HIPCHK(hipMalloc(&p, count * sizeof(T)));
    db->device_bytes += count * sizeof(T);
    return static_cast<T*>(p);
}

// Grow a workspace.  Growing waits for the stream first, so no queued work
// can still reference the old allocation.
void* reserve(pm_db* db, DevBuf& b, size_t bytes) {
    if (b.cap < bytes) {
        HIPCHK(hipStreamSynchronize(db->stream));
        if (b.p) HIPCHK(hipFree(b.p));
        b.p = nullptr;
        b.cap = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 20);
        HIPCHK(hipMalloc(&b.p, want));
        b.cap = want;
    }
    return b.p;
}

void* reserve_host(pm_db* db, HostBuf& b, size_t bytes) {
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

// Carves 256-byte aligned pieces out of one buffer.
struct Carve {
    size_t off = 0;
    size_t take(size_t bytes) {
        size_t at = off;
        off += (bytes + 255) / 256 * 256;
        return at;
    }
};

// Host blob staged through pinned memory and uploaded in one copy.
struct Upload {
    std::vector<uint8_t> blob;
    size_t add(const void* src, size_t bytes) {
        size_t at = (blob.size() + 255) / 256 * 256;
        blob.resize(at + bytes);
        if (bytes) memcpy(blob.data() + at, src, bytes);
        return at;
    }
    // uploads into db->ws_tab; returns its device base
    uint8_t* commit(pm_db* db) {
        uint8_t* d = static_cast<uint8_t*>(reserve(db, db->ws_tab, std::max<size_t>(blob.size(), 256)));
        uint8_t* h = static_cast<uint8_t*>(reserve_host(db, db->pin_up, std::max<size_t>(blob.size(), 256)));
        memcpy(h, blob.data(), blob.size());
        HIPCHK(hipMemcpyAsync(d, h, blob.size(), hipMemcpyHostToDevice, db->stream));
        return d;
    }
};

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
// packing kernels
// ---------------------------------------------------------------------------

// One thread per 32-position word: 2-bit planes + delimiter / other masks.
__global__ void k_pack_nuc(const uint8_t* __restrict__ raw, uint64_t n, uint64_t nwords,
                           uint32_t* __restrict__ hi, uint32_t* __restrict__ lo,
                           uint32_t* __restrict__ brk, uint32_t* __restrict__ oth) {
    uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (w >= nwords) return;
    uint64_t p0 = w * 32;
    uint8_t b[32];
    if (p0 + 32 <= n) {
        const uint4* src = reinterpret_cast<const uint4*>(raw + p0);
        uint4 v0 = src[0], v1 = src[1];
        memcpy(b, &v0, 16);
        memcpy(b + 16, &v1, 16);
    } else {
        for (int i = 0; i < 32; ++i) b[i] = (p0 + i < n) ? raw[p0 + i] : (uint8_t)'\n';
    }
    uint32_t h = 0, l = 0, br = 0, ot = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        uint32_t c = c_code[b[i]];
        if (c < 4) {
            h |= (c >> 1) << i;
            l |= (c & 1) << i;
        } else if (c == 4) {
            br |= 1u << i;
        } else {
            ot |= 1u << i;
        }
    }
    hi[w] = h; lo[w] = l; brk[w] = br; oth[w] = ot;
}

// Synthetic FASTA-shaped nucleotide text generated per word (no raw bytes).
__device__ inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

constexpr uint64_t SYN_HDR = 10;  // ">r%08u" then '\n'

__global__ void k_pack_synth(uint64_t n, uint64_t nwords, uint64_t rec_len, uint64_t seed,
                             uint32_t* __restrict__ hi, uint32_t* __restrict__ lo,
                             uint32_t* __restrict__ brk, uint32_t* __restrict__ oth) {
    uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (w >= nwords) return;
    const uint64_t stride = SYN_HDR + 1 + rec_len + 1;
    uint64_t r = mix64(seed * 0x9e3779b97f4a7c15ull + w);
    uint32_t h = (uint32_t)(r >> 32), l = (uint32_t)r;
    uint32_t br = 0;
    uint64_t p0 = w * 32;
    uint64_t q = p0 % stride;
    for (int i = 0; i < 32; ++i) {
        bool is_base = (p0 + i < n) && q >= SYN_HDR + 1 && q < SYN_HDR + 1 + rec_len;
        if (!is_base) br |= 1u << i;
        if (++q == stride) q = 0;
    }
    hi[w] = h & ~br; lo[w] = l & ~br; brk[w] = br; oth[w] = 0;
}

// Header lines become breaks: one thread per [beg, end) range.
__global__ void k_mark_ranges(const uint64_t* __restrict__ ranges, uint64_t nr, uint32_t* __restrict__ brk) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= nr) return;
    uint64_t b = ranges[2 * i], e = ranges[2 * i + 1];
    while (b < e) {
        uint64_t w = b >> 5;
        uint32_t lo_bit = b & 31;
        uint64_t wend = std::min<uint64_t>(e, (w + 1) * 32);
        uint32_t hi_bit = (uint32_t)(wend - w * 32);
        uint32_t mask = (hi_bit == 32 ? 0xffffffffu : ((1u << hi_bit) - 1)) & ~((1u << lo_bit) - 1);
        atomicOr(&brk[w], mask);
        b = wend;
    }
}

__global__ void k_sb_flags(const uint32_t* __restrict__ brk, const uint32_t* __restrict__ oth,
                           uint64_t nsb, uint32_t* __restrict__ sbflag, uint32_t* __restrict__ sbcnt) {
    uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (s >= nsb) return;
    uint32_t f = 0;
    for (int i = 0; i < 32; ++i) {
        uint64_t w = s * 32 + i;
        if (brk[w] | oth[w]) f |= 1u << i;
    }
    sbflag[s] = f;
    sbcnt[s] = __popc(f);
}

__global__ void k_fill_exceptions(const uint8_t* __restrict__ raw, uint64_t n, uint64_t nwords,
                                  const uint32_t* __restrict__ brk, const uint32_t* __restrict__ oth,
                                  const uint32_t* __restrict__ sbflag, const uint32_t* __restrict__ sbbase,
                                  uint32_t* __restrict__ xbrk, uint32_t* __restrict__ xoth,
                                  uint8_t* __restrict__ xbytes) {
    uint64_t w = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (w >= nwords) return;
    uint32_t f = sbflag[w >> 5];
    uint32_t bit = (uint32_t)(w & 31);
    if (!((f >> bit) & 1)) return;
    uint64_t idx = sbbase[w >> 5] + __popc(f & ((1u << bit) - 1));
    uint32_t br = brk[w], ot = oth[w];
    xbrk[idx] = br;
    xoth[idx] = ot & ~br;
    for (int i = 0; i < 32; ++i) {
        uint64_t p = w * 32 + i;
        uint8_t c = '\n';
        if (!((br >> i) & 1) && raw != nullptr && p < n) c = fold(raw[p]);
        xbytes[idx * 32 + i] = c;
    }
}

__global__ void k_pack_bytes(const uint8_t* __restrict__ raw, uint64_t n, uint64_t nalloc,
                             uint8_t* __restrict__ out) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= nalloc) return;
    out[i] = i < n ? fold(raw[i]) : (uint8_t)'\n';
}

__global__ void k_mark_ranges_bytes(const uint64_t* __restrict__ ranges, uint64_t nr, uint8_t* __restrict__ bytes) {
    uint64_t i = blockIdx.x;
    if (i >= nr) return;
    uint64_t b = ranges[2 * i], e = ranges[2 * i + 1];
    for (uint64_t p = b + threadIdx.x; p < e; p += blockDim.x) bytes[p] = '\n';
}

// ---------------------------------------------------------------------------
// device helpers shared by the automaton kernels
// ---------------------------------------------------------------------------
struct NucView {
    const uint32_t *hi, *lo, *sbflag, *sbbase, *xbrk, *xoth;
    const uint8_t* xbytes;
};

__device__ inline uint8_t nuc_char_at(const NucView& v, uint64_t p) {
    const uint64_t w = p >> 5;
    const uint32_t b = (uint32_t)(p & 31);
    const uint32_t f = v.sbflag[w >> 5];
    const uint32_t wb = (uint32_t)(w & 31);
    if ((f >> wb) & 1) {
        uint64_t idx = v.sbbase[w >> 5] + __popc(f & ((1u << wb) - 1));
        if (((v.xbrk[idx] | v.xoth[idx]) >> b) & 1) return v.xbytes[idx * 32 + b];
    }
    uint32_t code = (((v.hi[w] >> b) & 1) << 1) | ((v.lo[w] >> b) & 1);
    return (uint8_t)((0x54474341u >> (8 * code)) & 0xff);   // "ACGT"
}

// ---------------------------------------------------------------------------
// hit sink: 1024 bins, wave-aggregated atomics
// ---------------------------------------------------------------------------
struct Sink {
    uint64_t* out;       // [NBINS * cap]
    uint32_t* bin_cnt;   // [NBINS]
    uint32_t cap;
};

__device__ inline uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

// ---------------------------------------------------------------------------
// k_linear: bit-sliced k-mismatch scan of fixed-length patterns
// ---------------------------------------------------------------------------
// Program (u32, device, read through the scalar cache): prog[0] = number of
// classes nc; class c has a record of linear_rec(P, MW) words at
// 1 + c * REC: [acgt-subset | byte-table index << 8], then for p in P, q in
// MW the mask of shifts (j - 32q) at which pattern p has class c in word
// offset q.  '.' positions never appear (they cannot mismatch); breaks are
// handled through the exception path.
typedef const __attribute__((address_space(4))) uint32_t* cu32p;
typedef const __attribute__((address_space(4))) int32_t* ci32p;

__host__ __device__ constexpr int linear_rec(int P, int MW) {
    return (1 + P * MW) <= 2 ? 2 : (1 + P * MW) <= 4 ? 4 : (1 + P * MW) <= 8 ? 8 : 16;
}

struct LinearArgs {
    const uint32_t *hi, *lo, *sbflag, *sbbase, *xbrk, *xoth;
    const uint8_t* xbytes;
    const uint32_t* prog;
    const uint32_t* class_bytes;   // [nclass][8]
    const int32_t* lengths;        // [P]
    uint64_t n_iter;               // wave iterations over the start words
    int pattern_base;
    Sink sink;
};

// index of flagged word w in the compacted exception side tables
__device__ inline uint32_t exception_index(const uint32_t* sbflag, const uint32_t* sbbase, uint64_t w) {
    const uint32_t f = sbflag[w >> 5];
    const uint32_t wb = (uint32_t)(w & 31);
    return sbbase[w >> 5] + __popc(f & ((1u << wb) - 1));
}

template <int WPL, int NW>
struct LaneWords {
    uint32_t H[NW], L[NW];
    uint32_t f0, f1;   // superblock flag words covering w0 .. w0+NW-1
    // bit i = word w0+i has exceptions (evaluated late, so a prefetch of the
    // next iteration's words is not waited for)
    __device__ uint64_t flags(uint64_t w0) const {
        return ((((uint64_t)f1 << 32) | f0) >> (w0 & 31)) & ((1ull << NW) - 1);
    }
};

template <int WPL, int NW>
__device__ inline void load_lane_words(const LinearArgs& a, uint64_t w0, LaneWords<WPL, NW>& d) {
    if constexpr (WPL == 2) {
        const uint2 vh = *reinterpret_cast<const uint2*>(a.hi + w0);
        const uint2 vl = *reinterpret_cast<const uint2*>(a.lo + w0);
        d.H[0] = vh.x; d.H[1] = vh.y;
        d.L[0] = vl.x; d.L[1] = vl.y;
    } else {
#pragma unroll
        for (int v = 0; v < WPL / 4; ++v) {
            const uint4 vh = *reinterpret_cast<const uint4*>(a.hi + w0 + 4 * v);
            const uint4 vl = *reinterpret_cast<const uint4*>(a.lo + w0 + 4 * v);
            d.H[4 * v] = vh.x; d.H[4 * v + 1] = vh.y; d.H[4 * v + 2] = vh.z; d.H[4 * v + 3] = vh.w;
            d.L[4 * v] = vl.x; d.L[4 * v + 1] = vl.y; d.L[4 * v + 2] = vl.z; d.L[4 * v + 3] = vl.w;
        }
    }
#pragma unroll
    for (int i = WPL; i < NW; ++i) { d.H[i] = a.hi[w0 + i]; d.L[i] = a.lo[w0 + i]; }
    // both flag words are loaded unconditionally (sbflag is padded) so no
    // branch depends on the prefetched data
    d.f0 = a.sbflag[w0 >> 5];
    d.f1 = a.sbflag[(w0 >> 5) + 1];
}

// Per-window mismatch counters, bit-sliced over the 32 window starts of a
// word.  Mismatch bits arrive one or two at a time; pairs go through a
// carry-save adder (xor3 + majority, one v_bitop3 each) so the count is
// o + 2*C with o in {0,1} and C tracked as a thermometer (c[0] = C>=1, ...).
template <int K>
struct Counter {
    static constexpr int NC = K / 2 + 1;       // carry levels needed
    uint32_t o, c[NC];
    __device__ void clear() {
        o = 0;
#pragma unroll
        for (int i = 0; i < NC; ++i) c[i] = 0;
    }
    __device__ void carry_in(uint32_t cy) {
#pragma unroll
        for (int i = NC - 1; i > 0; --i) c[i] |= c[i - 1] & cy;
        c[0] |= cy;
    }
    __device__ void add1(uint32_t x) {
        if constexpr (K == 0) {
            o |= x;
        } else {
            const uint32_t cy = o & x;
            o ^= x;
            carry_in(cy);
        }
    }
    __device__ void add2(uint32_t x, uint32_t y) {
        if constexpr (K == 0) {
            o |= x | y;
        } else {
            const uint32_t cy = __builtin_amdgcn_bitop3_b32(o, x, y, 0xE8);   // majority
            o = __builtin_amdgcn_bitop3_b32(o, x, y, 0x96);                  // xor3
            carry_in(cy);
        }
    }
    // windows with more than K mismatches
    __device__ uint32_t dead() const {
        if constexpr (K == 0) return o;
        else if constexpr (K % 2 == 1) return c[NC - 1];              // C > K/2
        else return c[NC - 1] | (c[NC - 2] & o);                     // C > K/2 or (C == K/2 and o)
    }
};

// Mismatch word of one ACGT subset (bit0=A, bit1=C, bit2=G, bit3=T; codes
// A=00 C=01 G=10 T=11 as (H,L)): one VALU op per word given H, L, ~H, ~L.
template <int NW>
__device__ inline void class_mismatch(uint32_t subset, const uint32_t (&H)[NW], const uint32_t (&L)[NW],
                                      const uint32_t (&nH)[NW], const uint32_t (&nL)[NW], uint32_t (&X)[NW]) {
#define PM_CASE(code, expr)                                   \
    case code:                                                \
        _Pragma("unroll") for (int i = 0; i < NW; ++i) X[i] = (expr); \
        break;
    switch (subset) {
        PM_CASE(0x0, ~0u)
        PM_CASE(0x1, H[i] | L[i])
        PM_CASE(0x2, H[i] | nL[i])
        PM_CASE(0x4, nH[i] | L[i])
        PM_CASE(0x8, nH[i] | nL[i])
        PM_CASE(0x3, H[i])
        PM_CASE(0x5, L[i])
        PM_CASE(0x9, H[i] ^ L[i])
        PM_CASE(0x6, H[i] ^ nL[i])
        PM_CASE(0xA, nL[i])
        PM_CASE(0xC, nH[i])
        PM_CASE(0x7, H[i] & L[i])
        PM_CASE(0xB, H[i] & nL[i])
        PM_CASE(0xD, nH[i] & L[i])
        PM_CASE(0xE, nH[i] & nL[i])
        default:
            _Pragma("unroll") for (int i = 0; i < NW; ++i) X[i] = 0u;
            break;
    }
#undef PM_CASE
}

// Mismatch counters of the WPL words of one lane.  EXC: some word of the
// lane is flagged, so non-ACGT bytes are looked up and breaks kill windows.
template <int P, int K, int MW, int WPL, bool EXC>
__device__ inline void count_mismatches(const LinearArgs& a, const LaneWords<WPL, WPL + MW>& cur, uint64_t w0,
                                        Counter<K> (&t)[P][WPL], uint32_t (&kill)[P][WPL],
                                        const int (&len)[P], uint64_t fl) {
    constexpr int NW = WPL + MW;
    constexpr int REC = linear_rec(P, MW);
    const cu32p prog = (cu32p)(uintptr_t)a.prog;
    const uint32_t nc = prog[0];
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
        for (int r = 0; r < WPL; ++r) {
            kill[p][r] = 0;
            t[p][r].clear();
        }
    uint32_t nH[NW], nL[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) { nH[i] = ~cur.H[i]; nL[i] = ~cur.L[i]; }
    uint32_t rec[REC], rec_next[REC];
#pragma unroll
    for (int i = 0; i < REC; ++i) rec[i] = prog[1 + i];
    for (uint32_t c = 0; c < nc; ++c) {
        const uint32_t cn = (c + 1 < nc) ? c + 1 : c;
#pragma unroll
        for (int i = 0; i < REC; ++i) rec_next[i] = prog[1 + cn * REC + i];
        const uint32_t desc = rec[0];
        uint32_t X[NW];
        class_mismatch<NW>(desc & 15, cur.H, cur.L, nH, nL, X);
        if constexpr (EXC) {
            // non-ACGT bytes (N, other IUPAC letters, ...) of flagged words:
            // membership from the class's 256-bit byte table (rare path,
            // side-table words re-read from cache instead of held live)
            const cu32p cb = (cu32p)(uintptr_t)a.class_bytes + 8 * (desc >> 8);
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                if (!((fl >> i) & 1)) continue;
                const uint32_t idx = exception_index(a.sbflag, a.sbbase, w0 + i);
                uint32_t o = a.xoth[idx];
                const uint32_t oth = o;
                uint32_t mem = 0;
                while (o) {
                    const int b = __builtin_ctz(o);
                    o &= o - 1;
                    const uint8_t ch = a.xbytes[(uint64_t)idx * 32 + b];
                    if ((cb[ch >> 5] >> (ch & 31)) & 1) mem |= 1u << b;
                }
                X[i] = (X[i] & ~oth) | (oth & ~mem);
            }
        }
#pragma unroll
        for (int p = 0; p < P; ++p) {
#pragma unroll
            for (int q = 0; q < MW; ++q) {
                uint32_t sh = rec[1 + p * MW + q];
                while (sh) {
                    const int j = __builtin_ctz(sh);
                    sh &= sh - 1;
                    if (sh) {
                        const int j2 = __builtin_ctz(sh);
                        sh &= sh - 1;
#pragma unroll
                        for (int r = 0; r < WPL; ++r)
                            t[p][r].add2(__builtin_amdgcn_alignbit(X[r + q + 1], X[r + q], j),
                                         __builtin_amdgcn_alignbit(X[r + q + 1], X[r + q], j2));
                    } else {
#pragma unroll
                        for (int r = 0; r < WPL; ++r)
                            t[p][r].add1(__builtin_amdgcn_alignbit(X[r + q + 1], X[r + q], j));
                    }
                }
            }
        }
#pragma unroll
        for (int i = 0; i < REC; ++i) rec[i] = rec_next[i];
    }
    if constexpr (EXC) {
        // windows overlapping a break (newline, header byte, tail padding)
        uint32_t BRK[NW];
#pragma unroll
        for (int i = 0; i < NW; ++i)
            BRK[i] = ((fl >> i) & 1) ? a.xbrk[exception_index(a.sbflag, a.sbbase, w0 + i)] : 0u;
#pragma unroll
        for (int p = 0; p < P; ++p)
#pragma unroll
            for (int r = 0; r < WPL; ++r) {
                uint32_t k = 0;
                for (int j = 0; j < len[p]; ++j) {
                    const int q = j >> 5;
                    uint32_t lo_w = 0, hi_w = 0;
#pragma unroll
                    for (int qq = 0; qq < MW; ++qq)
                        if (q == qq) { lo_w = BRK[r + qq]; hi_w = BRK[r + qq + 1]; }
                    k |= __builtin_amdgcn_alignbit(hi_w, lo_w, j & 31);
                }
                kill[p][r] = k;
            }
    }
}

// Counts one lane-iteration and emits its hits.
template <int P, int K, int MW, int WPL>
__device__ inline void linear_iteration(const LinearArgs& a, const LaneWords<WPL, WPL + MW>& cur, uint64_t w0,
                                        const int (&len)[P], int lane, uint64_t wave) {
    Counter<K> t[P][WPL];
    uint32_t kill[P][WPL];
    const uint64_t fl = cur.flags(w0);
    if (fl == 0) count_mismatches<P, K, MW, WPL, false>(a, cur, w0, t, kill, len, fl);
    else count_mismatches<P, K, MW, WPL, true>(a, cur, w0, t, kill, len, fl);
    uint32_t hits[P][WPL];
    uint32_t cnt = 0;
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
        for (int r = 0; r < WPL; ++r) {
            hits[p][r] = ~t[p][r].dead() & ~kill[p][r];
            cnt += __popc(hits[p][r]);
        }
    if (__ballot(cnt != 0)) {
        const uint32_t incl = wave_incl_scan(cnt, lane);
        const uint32_t total = __shfl(incl, 63, 64);
        const uint32_t bin = (uint32_t)(wave % NBINS);
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&a.sink.bin_cnt[bin], total);
        base = __shfl(base, 0, 64);
        uint32_t o = base + incl - cnt;
        uint64_t* dst = a.sink.out + (uint64_t)bin * a.sink.cap;
#pragma unroll
        for (int p = 0; p < P; ++p) {
#pragma unroll
            for (int r = 0; r < WPL; ++r) {
                uint32_t h = hits[p][r];
                while (h) {
                    const int b = __builtin_ctz(h);
                    h &= h - 1;
                    if (o < a.sink.cap) dst[o] = ((uint64_t)(a.pattern_base + p) << 48) | ((w0 + r) * 32 + b);
                    ++o;
                }
            }
        }
    }
}

// Grid-stride over wave iterations (64 lanes x WPL consecutive words each).
// DBUF: unrolled by two with alternating register buffers, so the planes of
// the next iteration are in flight while this one computes; the prefetch
// address is clamped instead of predicated so the compiler can count its
// loads (no vmcnt(0) drain).
template <int P, int K, int MW, int WPL, bool DBUF>
__global__ __launch_bounds__(256) void k_linear(LinearArgs a) {
    constexpr int NW = WPL + MW;
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = (gridDim.x * (uint64_t)blockDim.x) >> 6;
    if (wave >= a.n_iter) return;
    int len[P];
#pragma unroll
    for (int p = 0; p < P; ++p) len[p] = ((ci32p)(uintptr_t)a.lengths)[p];
    const uint64_t last = a.n_iter - 1;
    auto words_of = [&](uint64_t it) { return (std::min(it, last) * 64 + lane) * WPL; };
    LaneWords<WPL, NW> A, B;
    uint64_t it = wave;
    if constexpr (DBUF) {
        load_lane_words<WPL, NW>(a, words_of(it), A);
        while (true) {
            load_lane_words<WPL, NW>(a, words_of(it + nwaves), B);
            linear_iteration<P, K, MW, WPL>(a, A, words_of(it), len, lane, wave);
            it += nwaves;
            if (it >= a.n_iter) break;
            load_lane_words<WPL, NW>(a, words_of(it + nwaves), A);
            linear_iteration<P, K, MW, WPL>(a, B, words_of(it), len, lane, wave);
            it += nwaves;
            if (it >= a.n_iter) break;
        }
    } else {
        for (; it < a.n_iter; it += nwaves) {
            load_lane_words<WPL, NW>(a, words_of(it), A);
            linear_iteration<P, K, MW, WPL>(a, A, words_of(it), len, lane, wave);
        }
    }
}

// ---------------------------------------------------------------------------
// k_nfa_rev: reverse Glushkov scan -> every start with a match (<= K subs)
// ---------------------------------------------------------------------------
struct NfaArgs {
    NucView nuc;
    const uint8_t* bytes;
    const uint64_t* prec;     // [nt][256]   positions preceding the set
    const uint64_t* follow;   // [nt][256]   positions following the set
    const uint64_t* bmask;    // [256]
    uint64_t first, last;
    int nt;
    int halo;
    int chunk;                // positions per lane (multiple of 32)
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

template <int K, bool NUC>
__global__ __launch_bounds__(256) void k_nfa_rev(NfaArgs a) {
    __shared__ uint64_t s_prec[8 * 256];
    __shared__ uint64_t s_b[256];
    for (int i = threadIdx.x; i < a.nt * 256; i += blockDim.x) s_prec[i] = a.prec[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s_b[i] = a.bmask[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint64_t gid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t wave = gid >> 6;
    const bool live = gid < a.nchunks;
    const uint64_t chunk_id = live ? gid : a.nchunks - 1;
    const uint64_t c0 = chunk_id * a.chunk;
    const uint64_t c1 = c0 + a.chunk;           // emit for [c0, c1) ∩ [0, n)
    const uint64_t top = c1 + a.halo;           // process (top .. c0], padded storage
    const uint32_t bin = (uint32_t)(wave % NBINS);
    uint64_t* dst = a.sink.out + (uint64_t)bin * a.sink.cap;
    uint64_t R[K + 1];
#pragma unroll
    for (int j = 0; j <= K; ++j) R[j] = 0;

    if constexpr (NUC) {
        const uint64_t wtop = (top + 31) >> 5;
        for (uint64_t w = wtop; w-- > (c0 >> 5);) {
            const uint32_t H = a.nuc.hi[w], L = a.nuc.lo[w];
            const uint32_t f = a.nuc.sbflag[w >> 5];
            const uint32_t wb = (uint32_t)(w & 31);
            uint32_t EXC = 0, idx = 0;
            if ((f >> wb) & 1) {
                idx = a.nuc.sbbase[w >> 5] + __popc(f & ((1u << wb) - 1));
                EXC = a.nuc.xbrk[idx] | a.nuc.xoth[idx];
            }
            for (int b = 31; b >= 0; --b) {
                uint8_t ch;
                if ((EXC >> b) & 1) ch = a.nuc.xbytes[(uint64_t)idx * 32 + b];
                else ch = (uint8_t)((0x54474341u >> (8 * ((((H >> b) & 1) << 1) | ((L >> b) & 1)))) & 0xff);
                const uint64_t bc = s_b[ch];
                const uint64_t nb = ch == '\n' ? 0ull : ~0ull;
                nfa_rev_step<K>(R, bc, nb, s_prec, a.nt, a.last);
                const uint64_t p = w * 32 + b;
                uint64_t any = 0;
#pragma unroll
                for (int j = 0; j <= K; ++j) any |= R[j];
                const bool st = live && p < c1 && p < a.n && (any & a.first);
                const uint64_t bal = __ballot(st);
                if (bal) {
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(&a.sink.bin_cnt[bin], (uint32_t)__popcll(bal));
                    base = __shfl(base, 0, 64);
                    const uint32_t o = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
                    if (st && o < a.sink.cap) dst[o] = ((uint64_t)a.pattern_id << 48) | p;
                }
            }
        }
    } else {
        const uint32_t* b32 = reinterpret_cast<const uint32_t*>(a.bytes);
        const uint64_t wtop = (top + 3) >> 2;
        for (uint64_t w = wtop; w-- > (c0 >> 2);) {
            const uint32_t word = b32[w];
            for (int b = 3; b >= 0; --b) {
                const uint8_t ch = (uint8_t)(word >> (8 * b));
                const uint64_t bc = s_b[ch];
                const uint64_t nb = ch == '\n' ? 0ull : ~0ull;
                nfa_rev_step<K>(R, bc, nb, s_prec, a.nt, a.last);
                const uint64_t p = w * 4 + b;
                uint64_t any = 0;
#pragma unroll
                for (int j = 0; j <= K; ++j) any |= R[j];
                const bool st = live && p < c1 && p < a.n && (any & a.first);
                const uint64_t bal = __ballot(st);
                if (bal) {
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(&a.sink.bin_cnt[bin], (uint32_t)__popcll(bal));
                    base = __shfl(base, 0, 64);
                    const uint32_t o = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1));
                    if (st && o < a.sink.cap) dst[o] = ((uint64_t)a.pattern_id << 48) | p;
                }
            }
        }
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
        const uint64_t p = s + d;
        uint8_t ch;
        if constexpr (NUC) ch = nuc_char_at(a.nuc, p);
        else ch = a.bytes[p];
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

// ---------------------------------------------------------------------------
// compaction of bins + lengths
// ---------------------------------------------------------------------------
__global__ void k_gather_bins(const uint64_t* __restrict__ out, const uint32_t* __restrict__ cnt,
                              const uint64_t* __restrict__ off, uint32_t cap, uint64_t* __restrict__ dst) {
    const uint32_t bin = blockIdx.x;
    const uint32_t c = min(cnt[bin], cap);
    const uint64_t o = off[bin];
    for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) dst[o + i] = out[(uint64_t)bin * cap + i];
}

__global__ void k_linear_lens(const uint64_t* __restrict__ keys, uint64_t n, const int32_t* __restrict__ lengths,
                              int pattern_base, uint32_t* __restrict__ lens) {
    uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    lens[i] = (uint32_t)lengths[(int)(keys[i] >> 48) - pattern_base];
}

__global__ void k_decode(NucView v, uint64_t beg, uint32_t len, uint8_t* out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < len) out[i] = nuc_char_at(v, beg + i);
}

// bin counters -> exclusive offsets, one block of NBINS threads
__global__ void k_bin_offsets(const uint32_t* __restrict__ cnt, uint32_t cap, uint64_t* __restrict__ off) {
    __shared__ uint64_t buf[NBINS];
    const uint32_t t = threadIdx.x;
    buf[t] = min(cnt[t], cap);
    __syncthreads();
    for (uint32_t d = 1; d < NBINS; d <<= 1) {
        uint64_t v = t >= d ? buf[t - d] : 0;
        __syncthreads();
        buf[t] += v;
        __syncthreads();
    }
    off[t] = buf[t] - min(cnt[t], cap);
}

// ---------------------------------------------------------------------------
// host helpers
// ---------------------------------------------------------------------------
NucView nuc_view(const pm_db* db) {
    return NucView{db->hi, db->lo, db->sbflag, db->sbbase, db->xbrk, db->xoth, db->xbytes};
}

uint32_t blocks_for(uint64_t n, uint32_t threads) { return (uint32_t)std::max<uint64_t>(1, (n + threads - 1) / threads); }

// header lines (/^>\S/) as [beg, end) ranges, end excluding the '\n'
std::vector<uint64_t> header_ranges(const uint8_t* t, uint64_t n) {
    std::vector<uint64_t> r;
    uint64_t p = 0;
    while (p < n) {
        const void* nl = memchr(t + p, '\n', n - p);
        uint64_t e = nl ? (uint64_t)((const uint8_t*)nl - t) : n;
        if (t[p] == '>' && p + 1 < e) {
            uint8_t c = t[p + 1];
            bool space = c == ' ' || c == '\t' || c == '\r' || c == '\f' || c == '\v';
            if (!space) { r.push_back(p); r.push_back(e); }
        }
        p = e + 1;
    }
    return r;
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

// flags per superblock, compacted exception side tables
void finish_exceptions(pm_db* db, std::vector<void*>& owned, const uint8_t* d_raw, uint32_t* brk, uint32_t* oth) {
    hipStream_t s = db->stream;
    db->sbflag = dalloc<uint32_t>(db, db->nsb);
    db->sbbase = dalloc<uint32_t>(db, db->nsb);
    uint32_t* sbcnt = tmp_alloc<uint32_t>(owned, db->nsb);
    hipLaunchKernelGGL(k_sb_flags, dim3(blocks_for(db->nsb, 256)), dim3(256), 0, s, brk, oth, db->nsb,
                       db->sbflag, sbcnt);
    HIPCHK(hipGetLastError());
    size_t tmp_bytes = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, sbcnt, db->sbbase, (int)db->nsb, s));
    void* tmp = tmp_alloc<uint8_t>(owned, tmp_bytes);
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, sbcnt, db->sbbase, (int)db->nsb, s));
    uint32_t* h = static_cast<uint32_t*>(reserve_host(db, db->pin_down, 8));
    HIPCHK(hipMemcpyAsync(h, db->sbbase + db->nsb - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(h + 1, sbcnt + db->nsb - 1, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    db->nflag = (uint64_t)h[0] + h[1];
    db->xbrk = dalloc<uint32_t>(db, db->nflag);
    db->xoth = dalloc<uint32_t>(db, db->nflag);
    db->xbytes = dalloc<uint8_t>(db, db->nflag * 32);
    hipLaunchKernelGGL(k_fill_exceptions, dim3(blocks_for(db->nwords, 256)), dim3(256), 0, s, d_raw, db->n,
                       db->nwords, brk, oth, db->sbflag, db->sbbase, db->xbrk, db->xoth, db->xbytes);
    HIPCHK(hipGetLastError());
}

void init_stream(pm_db* db, void* stream) {
    if (stream) {
        db->stream = (hipStream_t)stream;
    } else {
        HIPCHK(hipStreamCreate(&db->stream));   // blocking: ordered with the null stream
        db->own_stream = true;
    }
}

void free_db(pm_db* db) {
    if (!db) return;
    if (db->stream) (void)hipStreamSynchronize(db->stream);
    void* ptrs[] = {db->hi, db->lo, db->sbflag, db->sbbase, db->xbrk, db->xoth, db->xbytes, db->bytes,
                    db->ws_tab.p, db->ws_sink.p, db->ws_post.p};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (db->pin_up.p) (void)hipHostFree(db->pin_up.p);
    if (db->pin_down.p) (void)hipHostFree(db->pin_down.p);
    if (db->own_stream && db->stream) (void)hipStreamDestroy(db->stream);
    delete db;
}

struct SinkBuffers {
    uint64_t* out = nullptr;
    uint32_t* cnt = nullptr;
    uint32_t cap = 0;
};

SinkBuffers make_sink(pm_db* db, uint64_t expected) {
    SinkBuffers sb;
    uint64_t cap = std::max<uint64_t>(1024, (expected + NBINS - 1) / NBINS * 2);
    cap = std::min<uint64_t>(cap, 1ull << 26);
    sb.cap = (uint32_t)cap;
    Carve c;
    const size_t o_out = c.take((uint64_t)NBINS * sb.cap * sizeof(uint64_t));
    const size_t o_cnt = c.take(NBINS * sizeof(uint32_t));
    uint8_t* base = static_cast<uint8_t*>(reserve(db, db->ws_sink, c.off));
    sb.out = reinterpret_cast<uint64_t*>(base + o_out);
    sb.cnt = reinterpret_cast<uint32_t*>(base + o_cnt);
    HIPCHK(hipMemsetAsync(sb.cnt, 0, NBINS * sizeof(uint32_t), db->stream));
    return sb;
}

// Reads bin counters; returns total, sets `overflow` if a bin exceeded cap.
uint64_t sink_total(pm_db* db, const SinkBuffers& sb, std::vector<uint32_t>& counts, bool& overflow) {
    uint32_t* h = static_cast<uint32_t*>(reserve_host(db, db->pin_down, NBINS * sizeof(uint32_t)));
    HIPCHK(hipMemcpyAsync(h, sb.cnt, NBINS * sizeof(uint32_t), hipMemcpyDeviceToHost, db->stream));
    HIPCHK(hipStreamSynchronize(db->stream));
    counts.assign(h, h + NBINS);
    uint64_t total = 0;
    overflow = false;
    for (uint32_t c : counts) {
        total += c;
        overflow |= c > sb.cap;
    }
    return total;
}

// bins -> contiguous -> radix sorted keys (owned by the returned hits)
pm_hits* sink_to_hits(pm_db* db, const SinkBuffers& sb, uint64_t total, int key_bits) {
    hipStream_t s = db->stream;
    pm_hits* h = new pm_hits();
    h->device = db->device;
    h->count = total;
    try {
        HIPCHK(hipMalloc((void**)&h->keys, std::max<uint64_t>(total, 1) * sizeof(uint64_t)));
        HIPCHK(hipMalloc((void**)&h->lens, std::max<uint64_t>(total, 1) * sizeof(uint32_t)));
        if (total == 0) return h;
        size_t sort_bytes = 0;
        HIPCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, sort_bytes, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                                 (int)total, 0, key_bits, s));
        Carve c;
        const size_t o_off = c.take(NBINS * sizeof(uint64_t));
        const size_t o_uns = c.take(total * sizeof(uint64_t));
        const size_t o_tmp = c.take(sort_bytes);
        uint8_t* base = static_cast<uint8_t*>(reserve(db, db->ws_post, c.off));
        uint64_t* d_off = reinterpret_cast<uint64_t*>(base + o_off);
        uint64_t* unsorted = reinterpret_cast<uint64_t*>(base + o_uns);
        hipLaunchKernelGGL(k_bin_offsets, dim3(1), dim3(NBINS), 0, s, sb.cnt, sb.cap, d_off);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(k_gather_bins, dim3(NBINS), dim3(256), 0, s, sb.out, sb.cnt, d_off, sb.cap, unsorted);
        HIPCHK(hipGetLastError());
        HIPCHK(hipcub::DeviceRadixSort::SortKeys(base + o_tmp, sort_bytes, unsorted, h->keys, (int)total, 0,
                                                 key_bits, s));
    } catch (...) {
        if (h->keys) (void)hipFree(h->keys);
        if (h->lens) (void)hipFree(h->lens);
        delete h;
        throw;
    }
    return h;
}

// --- runtime-specialized k_linear (hipRTC) -----------------------------------
// For large databases the batch's patterns are compiled into the kernel:
// every shift is an immediate of v_alignbit, every class word a single op
// on (H, L, ~H, ~L), all positions of a pattern are paired through the
// carry-save counter, and no scalar loop or program load is left in the
// hot loop.  Code objects are cached per generated source and device.
const char* kJitCommon = R"JIT(
typedef unsigned int u32;
typedef unsigned long long u64;
struct JArgs {
    const u32 *hi, *lo, *sbflag, *sbbase, *xbrk, *xoth;
    const unsigned char* xbytes;
    const u32* cb;
    u64 n_iter;
    u64* out;
    u32* bin_cnt;
    u32 cap;
    int pattern_base;
};
#define NBINS 1024u
#define AL(h, l, s) __builtin_amdgcn_alignbit((h), (l), (s))
template <int K>
struct Ctr {
    static constexpr int NC = K / 2 + 1;
    u32 o, c[NC];
    __device__ __forceinline__ void clear() { o = 0; for (int i = 0; i < NC; ++i) c[i] = 0; }
    __device__ __forceinline__ void carry(u32 cy) {
        for (int i = NC - 1; i > 0; --i) c[i] |= c[i - 1] & cy;
        c[0] |= cy;
    }
    __device__ __forceinline__ void add1(u32 x) {
        if constexpr (K == 0) { o |= x; } else { const u32 cy = o & x; o ^= x; carry(cy); }
    }
    __device__ __forceinline__ void add2(u32 x, u32 y) {
        if constexpr (K == 0) { o |= x | y; }
        else {
            const u32 cy = __builtin_amdgcn_bitop3_b32(o, x, y, 0xE8);
            o = __builtin_amdgcn_bitop3_b32(o, x, y, 0x96);
            carry(cy);
        }
    }
    __device__ __forceinline__ u32 dead() const {
        if constexpr (K == 0) return o;
        else if constexpr (K % 2 == 1) return c[NC - 1];
        else return c[NC - 1] | (c[NC - 2] & o);
    }
};
__device__ __forceinline__ u32 exc_index(const u32* sbflag, const u32* sbbase, u64 w) {
    const u32 f = sbflag[w >> 5];
    const u32 wb = (u32)(w & 31);
    return sbbase[w >> 5] + __popc(f & ((1u << wb) - 1));
}
// non-ACGT bytes of a flagged word: class membership from the byte table
__device__ __forceinline__ u32 fix_class(const JArgs& a, u32 x, u64 w, int cls) {
    const u32 idx = exc_index(a.sbflag, a.sbbase, w);
    u32 o = a.xoth[idx];
    const u32 oth = o;
    u32 mem = 0;
    while (o) {
        const int b = __builtin_ctz(o);
        o &= o - 1;
        const unsigned char ch = a.xbytes[(u64)idx * 32 + b];
        if ((a.cb[8 * cls + (ch >> 5)] >> (ch & 31)) & 1) mem |= 1u << b;
    }
    return (x & ~oth) | (oth & ~mem);
}
__device__ __forceinline__ u32 wave_incl_scan(u32 v, int lane) {
    for (int d = 1; d < 64; d <<= 1) {
        u32 o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}
)JIT";

struct JitKernel {
    hipModule_t module = nullptr;
    hipFunction_t fn = nullptr;
};

std::mutex g_jit_mu;
std::map<std::pair<int, std::string>, JitKernel> g_jit_cache;

struct JArgsHost {           // must match JArgs in kJitCommon
    const uint32_t *hi, *lo, *sbflag, *sbbase, *xbrk, *xoth;
    const uint8_t* xbytes;
    const uint32_t* cb;
    uint64_t n_iter;
    uint64_t* out;
    uint32_t* bin_cnt;
    uint32_t cap;
    int pattern_base;
};

const char* subset_expr(int subset) {
    switch (subset & 15) {
        case 0x0: return "~0u";
        case 0x1: return "H[i] | L[i]";
        case 0x2: return "H[i] | nL[i]";
        case 0x4: return "nH[i] | L[i]";
        case 0x8: return "nH[i] | nL[i]";
        case 0x3: return "H[i]";
        case 0x5: return "L[i]";
        case 0x9: return "H[i] ^ L[i]";
        case 0x6: return "H[i] ^ nL[i]";
        case 0xA: return "nL[i]";
        case 0xC: return "nH[i]";
        case 0x7: return "H[i] & L[i]";
        case 0xB: return "H[i] & nL[i]";
        case 0xD: return "nH[i] & L[i]";
        case 0xE: return "nH[i] & nL[i]";
        default: return "0u";
    }
}

// Source of the specialized kernel for patterns [base, base+P).
std::string gen_linear_source(int P, int K, int MW, const int32_t* lengths, const uint8_t* pos_class,
                              const uint8_t* class_acgt, const uint8_t* class_is_any) {
    constexpr int W = 4;                      // words per lane
    const int NW = W + MW;
    std::vector<int> used;
    std::map<int, int> slot;
    for (int p = 0; p < P; ++p)
        for (int j = 0; j < lengths[p]; ++j) {
            const int c = pos_class[64 * p + j];
            if (!class_is_any[c] && !slot.count(c)) { slot[c] = (int)used.size(); used.push_back(c); }
        }
    std::ostringstream o;
    o << kJitCommon;
    o << "#define P " << P << "\n#define K " << K << "\n#define W " << W << "\n#define NW " << NW << "\n";
    o << "__device__ __forceinline__ void body(const JArgs& a, const u32 (&H)[NW], const u32 (&L)[NW], u32 f0, "
         "u32 f1, u64 w0, int lane, u64 wave) {\n";
    o << "  const u64 fl = ((((u64)f1 << 32) | f0) >> (w0 & 31)) & ((1ull << NW) - 1);\n";
    o << "  u32 nH[NW], nL[NW];\n#pragma unroll\n  for (int i = 0; i < NW; ++i) { nH[i] = ~H[i]; nL[i] = ~L[i]; }\n";
    for (size_t u = 0; u < used.size(); ++u) {
        o << "  u32 X" << u << "[NW];\n#pragma unroll\n  for (int i = 0; i < NW; ++i) X" << u << "[i] = "
          << subset_expr(class_acgt[used[u]]) << ";\n";
    }
    o << "  if (fl) {\n#pragma unroll\n    for (int i = 0; i < NW; ++i) if ((fl >> i) & 1) {\n";
    for (size_t u = 0; u < used.size(); ++u)
        o << "      X" << u << "[i] = fix_class(a, X" << u << "[i], w0 + i, " << used[u] << ");\n";
    o << "    }\n  }\n";
    o << "  Ctr<K> t[P][W];\n#pragma unroll\n  for (int p = 0; p < P; ++p)\n#pragma unroll\n"
         "    for (int r = 0; r < W; ++r) t[p][r].clear();\n";
    o << "#pragma unroll\n  for (int r = 0; r < W; ++r) {\n";
    for (int p = 0; p < P; ++p) {
        std::vector<std::pair<int, int>> pos;   // (shift, slot)
        for (int j = 0; j < lengths[p]; ++j) {
            const int c = pos_class[64 * p + j];
            if (!class_is_any[c]) pos.push_back({j, slot[c]});
        }
        auto term = [&](const std::pair<int, int>& e) {
            std::ostringstream t;
            const int q = e.first >> 5, sh = e.first & 31;
            t << "AL(X" << e.second << "[r + " << q + 1 << "], X" << e.second << "[r + " << q << "], " << sh << ")";
            return t.str();
        };
        size_t i = 0;
        for (; i + 1 < pos.size(); i += 2)
            o << "    t[" << p << "][r].add2(" << term(pos[i]) << ", " << term(pos[i + 1]) << ");\n";
        if (i < pos.size()) o << "    t[" << p << "][r].add1(" << term(pos[i]) << ");\n";
    }
    o << "  }\n";
    // windows overlapping breaks (newline, header bytes, tail padding)
    o << "  u32 kill[P][W];\n#pragma unroll\n  for (int p = 0; p < P; ++p)\n#pragma unroll\n"
         "    for (int r = 0; r < W; ++r) kill[p][r] = 0;\n";
    o << "  if (fl) {\n    u32 B[NW + 1];\n#pragma unroll\n    for (int i = 0; i < NW; ++i) B[i] = ((fl >> i) & 1) ? "
         "a.xbrk[exc_index(a.sbflag, a.sbbase, w0 + i)] : 0u;\n    B[NW] = 0;\n";
    for (int p = 0; p < P; ++p)
        o << "#pragma unroll\n    for (int r = 0; r < W; ++r) {\n      u32 k = 0;\n#pragma unroll\n"
             "      for (int j = 0; j < " << lengths[p] << "; ++j) k |= AL(B[r + (j >> 5) + 1], B[r + (j >> 5)], j & 31);\n"
             "      kill[" << p << "][r] = k;\n    }\n";
    o << "  }\n";
    o << R"JIT(  u32 hits[P][W];
  u32 cnt = 0;
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int r = 0; r < W; ++r) { hits[p][r] = ~t[p][r].dead() & ~kill[p][r]; cnt += __popc(hits[p][r]); }
  if (__ballot(cnt != 0)) {
    const u32 incl = wave_incl_scan(cnt, lane);
    const u32 total = __shfl(incl, 63, 64);
    const u32 bin = (u32)(wave % NBINS);
    u32 base = 0;
    if (lane == 0) base = atomicAdd(&a.bin_cnt[bin], total);
    base = __shfl(base, 0, 64);
    u32 o = base + incl - cnt;
    u64* dst = a.out + (u64)bin * a.cap;
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
      for (int r = 0; r < W; ++r) {
        u32 h = hits[p][r];
        while (h) {
          const int b = __builtin_ctz(h);
          h &= h - 1;
          if (o < a.cap) dst[o] = ((u64)(a.pattern_base + p) << 48) | ((w0 + r) * 32 + b);
          ++o;
        }
      }
  }
}
__device__ __forceinline__ void load(const JArgs& a, u64 w0, u32 (&H)[NW], u32 (&L)[NW], u32& f0, u32& f1) {
  const uint4 vh = *reinterpret_cast<const uint4*>(a.hi + w0);
  const uint4 vl = *reinterpret_cast<const uint4*>(a.lo + w0);
  H[0] = vh.x; H[1] = vh.y; H[2] = vh.z; H[3] = vh.w;
  L[0] = vl.x; L[1] = vl.y; L[2] = vl.z; L[3] = vl.w;
#pragma unroll
  for (int i = W; i < NW; ++i) { H[i] = a.hi[w0 + i]; L[i] = a.lo[w0 + i]; }
  f0 = a.sbflag[w0 >> 5];
  f1 = a.sbflag[(w0 >> 5) + 1];
}
extern "C" __global__ __launch_bounds__(256) void pm_linear_jit(JArgs a) {
  const int lane = threadIdx.x & 63;
  const u64 wave = (blockIdx.x * (u64)blockDim.x + threadIdx.x) >> 6;
  const u64 nwaves = (gridDim.x * (u64)blockDim.x) >> 6;
  if (wave >= a.n_iter) return;
  const u64 last = a.n_iter - 1;
  u32 HA[NW], LA[NW], HB[NW], LB[NW], fa0, fa1, fb0, fb1;
  u64 it = wave;
  load(a, (it * 64 + lane) * W, HA, LA, fa0, fa1);
  while (true) {
    u64 nx = it + nwaves < last ? it + nwaves : last;
    load(a, (nx * 64 + lane) * W, HB, LB, fb0, fb1);
    body(a, HA, LA, fa0, fa1, (it * 64 + lane) * W, lane, wave);
    it += nwaves;
    if (it >= a.n_iter) break;
    nx = it + nwaves < last ? it + nwaves : last;
    load(a, (nx * 64 + lane) * W, HA, LA, fa0, fa1);
    body(a, HB, LB, fb0, fb1, (it * 64 + lane) * W, lane, wave);
    it += nwaves;
    if (it >= a.n_iter) break;
  }
}
)JIT";
    return o.str();
}

#define RTCCHK(expr)                                                                     \
    do {                                                                                 \
        hiprtcResult r_ = (expr);                                                        \
        if (r_ != HIPRTC_SUCCESS)                                                        \
            throw pm_failure(PM_E_HIP, std::string(#expr) + ": " + hiprtcGetErrorString(r_)); \
    } while (0)

// Compiles (cached) and returns the code object of `src`.
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
        throw pm_failure(PM_E_HIP, "hipRTC compile failed: " + log.substr(0, 2000));
    }
    size_t n = 0;
    RTCCHK(hiprtcGetCodeSize(prog, &n));
    std::vector<char> code(n);
    RTCCHK(hiprtcGetCode(prog, code.data()));
    hiprtcDestroyProgram(&prog);
    return code;
}

hipFunction_t jit_function(int device, const std::string& src) {
    std::lock_guard<std::mutex> lk(g_jit_mu);
    auto key = std::make_pair(device, src);
    auto it = g_jit_cache.find(key);
    if (it != g_jit_cache.end()) return it->second.fn;
    std::vector<char> code = jit_compile(src);
    JitKernel jk;
    HIPCHK(hipModuleLoadData(&jk.module, code.data()));
    HIPCHK(hipModuleGetFunction(&jk.fn, jk.module, "pm_linear_jit"));
    g_jit_cache[key] = jk;
    return jk.fn;
}

// PM_JIT: "0" never, "1" always, default: databases of >= 64 Mi positions
bool use_jit(const pm_db* db) {
    const char* e = getenv("PM_JIT");
    if (e && e[0] == '0') return false;
    if (e && e[0] == '1') return true;
    return db->n >= (64ull << 20);
}

// --- linear-scan dispatch ----------------------------------------------------
// Lane shape (words per lane, double buffering).  The default is the
// measured best; PM_LINEAR_SHAPE=<wpl><d|s> selects the experimental shapes
// (instantiated for the two-pattern batch only).
struct LinearShape {
    int wpl = 4;
    bool dbuf = true;
};

LinearShape linear_shape() {
    LinearShape sh;
    if (const char* e = getenv("PM_LINEAR_SHAPE")) {
        if (e[0] == '2' || e[0] == '4' || e[0] == '8') sh.wpl = e[0] - '0';
        if (e[0] && e[1] == 's') sh.dbuf = false;
    }
    return sh;
}

template <int P, int K, int MW, int WPL, bool DBUF>
void launch_linear(const LinearArgs& a, hipStream_t s) {
    const uint64_t blocks = std::min<uint64_t>((a.n_iter + 3) / 4, 256 * 16);
    hipLaunchKernelGGL((k_linear<P, K, MW, WPL, DBUF>), dim3((uint32_t)std::max<uint64_t>(blocks, 1)), dim3(256),
                       0, s, a);
}

template <int P, int K, int MW>
void launch_linear_shape(const LinearShape& sh, const LinearArgs& a, hipStream_t s) {
    if constexpr (P == 2 && K == 2 && MW == 1) {
        if (sh.wpl == 2) { sh.dbuf ? launch_linear<P, K, MW, 2, true>(a, s) : launch_linear<P, K, MW, 2, false>(a, s); return; }
        if (sh.wpl == 8) { sh.dbuf ? launch_linear<P, K, MW, 8, true>(a, s) : launch_linear<P, K, MW, 8, false>(a, s); return; }
        if (!sh.dbuf) { launch_linear<P, K, MW, 4, false>(a, s); return; }
    }
    launch_linear<P, K, MW, 4, true>(a, s);
}

template <int P, int K>
void launch_linear_mw(int mw, const LinearShape& sh, const LinearArgs& a, hipStream_t s) {
    if (mw == 1) launch_linear_shape<P, K, 1>(sh, a, s);
    else launch_linear_shape<P, K, 2>(sh, a, s);
}

template <int P>
void launch_linear_k(int k, int mw, const LinearShape& sh, const LinearArgs& a, hipStream_t s) {
    switch (k) {
        case 0: launch_linear_mw<P, 0>(mw, sh, a, s); break;
        case 1: launch_linear_mw<P, 1>(mw, sh, a, s); break;
        case 2: launch_linear_mw<P, 2>(mw, sh, a, s); break;
        default: launch_linear_mw<P, 3>(mw, sh, a, s); break;
    }
}

void launch_linear_any(int P, int k, int mw, const LinearShape& sh, const LinearArgs& a, hipStream_t s) {
    switch (P) {
        case 1: launch_linear_k<1>(k, mw, sh, a, s); break;
        case 2: launch_linear_k<2>(k, mw, sh, a, s); break;
        default: launch_linear_k<4>(k, mw, sh, a, s); break;
    }
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

struct EventPair {
    hipEvent_t a = nullptr, b = nullptr;
    EventPair() {
        HIPCHK(hipEventCreate(&a));
        HIPCHK(hipEventCreate(&b));
    }
    ~EventPair() {
        if (a) (void)hipEventDestroy(a);
        if (b) (void)hipEventDestroy(b);
    }
    double ms() {
        float v = 0.f;
        HIPCHK(hipEventElapsedTime(&v, a, b));
        return v;
    }
};

void check_device(int device) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) throw pm_failure(PM_E_NODEV, "no HIP device");
    require(device >= 0 && device < ndev, "device out of range");
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

const char* pm_last_error(void) { return g_err.c_str(); }
const char* pm_version(void) { return "patmatch_hip 0.2 (gfx950)"; }

int pm_device_count(int* count) {
    return guarded([&] {
        require(count != nullptr, "count is NULL");
        int c = 0;
        if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
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
        uint64_t* d_ranges = tmp_alloc<uint64_t>(owned, ranges.size());
        if (nr) HIPCHK(hipMemcpy(d_ranges, ranges.data(), ranges.size() * 8, hipMemcpyHostToDevice));
        uint8_t* d_raw = tmp_alloc<uint8_t>(owned, n + 64);
        if (n) HIPCHK(hipMemcpy(d_raw, fasta, n, hipMemcpyHostToDevice));
        if (alphabet == PM_ALPHA_NUC) {
            db->nwords = round_up((n + 31) / 32 + PAD_WORDS, 1024);
            db->nsb = db->nwords / 32;
            db->hi = dalloc<uint32_t>(db, db->nwords);
            db->lo = dalloc<uint32_t>(db, db->nwords);
            uint32_t* brk = tmp_alloc<uint32_t>(owned, db->nwords);
            uint32_t* oth = tmp_alloc<uint32_t>(owned, db->nwords);
            hipLaunchKernelGGL(k_pack_nuc, dim3(blocks_for(db->nwords, 256)), dim3(256), 0, s, d_raw, n, db->nwords,
                               db->hi, db->lo, brk, oth);
            HIPCHK(hipGetLastError());
            if (nr) {
                hipLaunchKernelGGL(k_mark_ranges, dim3(blocks_for(nr, 256)), dim3(256), 0, s, d_ranges, nr, brk);
                HIPCHK(hipGetLastError());
            }
            finish_exceptions(db, owned, d_raw, brk, oth);
        } else {
            db->nbytes_alloc = round_up(n + 2 * MAX_NFA_CHUNK + 4096, 4096);
            db->bytes = dalloc<uint8_t>(db, db->nbytes_alloc);
            hipLaunchKernelGGL(k_pack_bytes, dim3(blocks_for(db->nbytes_alloc, 256)), dim3(256), 0, s, d_raw, n,
                               db->nbytes_alloc, db->bytes);
            HIPCHK(hipGetLastError());
            if (nr) {
                hipLaunchKernelGGL(k_mark_ranges_bytes, dim3((uint32_t)nr), dim3(256), 0, s, d_ranges, nr, db->bytes);
                HIPCHK(hipGetLastError());
            }
        }
        free_all(db, owned);
        *out = db;
    });
    if (rc != PM_OK) {
        if (db && db->stream) (void)hipStreamSynchronize(db->stream);
        for (void* p : owned) (void)hipFree(p);
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
        hipStream_t s = db->stream;
        db->nwords = round_up((db->n + 31) / 32 + PAD_WORDS, 1024);
        db->nsb = db->nwords / 32;
        db->hi = dalloc<uint32_t>(db, db->nwords);
        db->lo = dalloc<uint32_t>(db, db->nwords);
        uint32_t* brk = tmp_alloc<uint32_t>(owned, db->nwords);
        uint32_t* oth = tmp_alloc<uint32_t>(owned, db->nwords);
        hipLaunchKernelGGL(k_pack_synth, dim3(blocks_for(db->nwords, 256)), dim3(256), 0, s, db->n, db->nwords,
                           rec_len, seed, db->hi, db->lo, brk, oth);
        HIPCHK(hipGetLastError());
        finish_exceptions(db, owned, nullptr, brk, oth);
        free_all(db, owned);
        *out = db;
    });
    if (rc != PM_OK) {
        if (db && db->stream) (void)hipStreamSynchronize(db->stream);
        for (void* p : owned) (void)hipFree(p);
        free_db(db);
    }
    return rc;
}

int pm_db_destroy(pm_db* db) {
    return guarded([&] {
        if (!db) return;
        DeviceGuard g(db->device);
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

int pm_db_decode(pm_db* db, uint64_t beg, uint32_t len, uint8_t* out) {
    return guarded([&] {
        require(db != nullptr && out != nullptr, "null argument");
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

int pm_scan_linear(pm_db* db, int n_patterns, const int32_t* lengths, const uint8_t* pos_class, int n_classes,
                   const uint8_t* class_acgt, const uint32_t* class_bytes, const uint8_t* class_is_any, int k,
                   pm_hits** out) {
    return guarded([&] {
        require(db != nullptr && out != nullptr && lengths && pos_class && class_acgt && class_bytes && class_is_any,
                "null argument");
        require(db->alphabet == PM_ALPHA_NUC, "pm_scan_linear needs a nucleotide database", PM_E_UNSUPPORTED);
        require(n_patterns >= 1 && n_patterns <= 4096, "n_patterns out of range");
        require(n_classes >= 1 && n_classes <= 256, "n_classes out of range");
        require(k >= 0 && k <= PM_MAX_K, "k out of range for the GPU kernels", PM_E_UNSUPPORTED);
        for (int p = 0; p < n_patterns; ++p) {
            require(lengths[p] >= 1 && lengths[p] <= PM_MAX_POSITIONS, "pattern length out of range");
            for (int j = 0; j < lengths[p]; ++j) require(pos_class[64 * p + j] < n_classes, "class id out of range");
        }
        DeviceGuard g(db->device);
        hipStream_t s = db->stream;
        const LinearShape shape = linear_shape();
        const uint64_t wave_words = 64ull * shape.wpl;
        const uint64_t start_words = (db->n + 31) / 32;
        const uint64_t n_iter = (start_words + wave_words - 1) / wave_words;
        require(n_iter * wave_words + 64 <= db->nwords, "internal: padding too small");

        // one upload: class byte tables, lengths, then one program per chunk
        struct Chunk { int base, P, MW; size_t off; hipFunction_t jit; };
        std::vector<Chunk> chunks;
        const bool jit = use_jit(db);
        Upload up;
        const size_t o_cb = up.add(class_bytes, (size_t)n_classes * 32);
        const size_t o_len = up.add(lengths, (size_t)n_patterns * 4);
        for (int base = 0; base < n_patterns;) {
            const int rem = n_patterns - base;
            const int P = rem >= 4 ? 4 : (rem >= 2 ? 2 : 1);   // instantiated widths
            int maxlen = 0;
            for (int p = 0; p < P; ++p) maxlen = std::max(maxlen, (int)lengths[base + p]);
            const int MW = maxlen > 32 ? 2 : 1;
            std::vector<int> used, slot(n_classes, -1);
            for (int p = 0; p < P; ++p)
                for (int j = 0; j < lengths[base + p]; ++j) {
                    const int c = pos_class[64 * (base + p) + j];
                    if (class_is_any[c] || slot[c] >= 0) continue;
                    slot[c] = (int)used.size();
                    used.push_back(c);
                }
            const int REC = linear_rec(P, MW);
            std::vector<uint32_t> prog(1 + (used.size() + 1) * REC, 0);   // +1: prefetch slack
            prog[0] = (uint32_t)used.size();
            for (size_t u = 0; u < used.size(); ++u)
                prog[1 + u * REC] = (uint32_t)(class_acgt[used[u]] & 15) | ((uint32_t)used[u] << 8);
            for (int p = 0; p < P; ++p)
                for (int j = 0; j < lengths[base + p]; ++j) {
                    const int c = pos_class[64 * (base + p) + j];
                    if (!class_is_any[c]) prog[1 + slot[c] * REC + 1 + p * MW + (j >> 5)] |= 1u << (j & 31);
                }
            hipFunction_t fn = nullptr;
            if (jit)
                fn = jit_function(db->device, gen_linear_source(P, k, MW, lengths + base, pos_class + 64 * base,
                                                                class_acgt, class_is_any));
            chunks.push_back({base, P, MW, up.add(prog.data(), prog.size() * 4), fn});
            base += P;
        }
        uint8_t* d_up = up.commit(db);
        const uint64_t jit_iter = (start_words + 255) / 256;        // W = 4 words per lane

        uint64_t expected = std::max<uint64_t>(db->n / 64, 1 << 16);
        SinkBuffers sb;
        std::vector<uint32_t> counts;
        uint64_t total = 0;
        EventPair ev;
        for (int attempt = 0; attempt < 2; ++attempt) {
            sb = make_sink(db, expected);
            HIPCHK(hipEventRecord(ev.a, s));
            for (const Chunk& ch : chunks) {
                if (ch.jit) {
                    JArgsHost ja{db->hi, db->lo, db->sbflag, db->sbbase, db->xbrk, db->xoth, db->xbytes,
                                 reinterpret_cast<const uint32_t*>(d_up + o_cb), jit_iter, sb.out, sb.cnt, sb.cap,
                                 ch.base};
                    void* params[] = {&ja};
                    const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((jit_iter + 3) / 4, 256 * 16));
                    HIPCHK(hipModuleLaunchKernel(ch.jit, blocks, 1, 1, 256, 1, 1, 0, s, params, nullptr));
                    continue;
                }
                LinearArgs a{};
                a.hi = db->hi; a.lo = db->lo; a.sbflag = db->sbflag; a.sbbase = db->sbbase;
                a.xbrk = db->xbrk; a.xoth = db->xoth; a.xbytes = db->xbytes;
                a.prog = reinterpret_cast<const uint32_t*>(d_up + ch.off);
                a.class_bytes = reinterpret_cast<const uint32_t*>(d_up + o_cb);
                a.lengths = reinterpret_cast<const int32_t*>(d_up + o_len) + ch.base;
                a.n_iter = n_iter;
                a.pattern_base = ch.base;
                a.sink = Sink{sb.out, sb.cnt, sb.cap};
                launch_linear_any(ch.P, k, ch.MW, shape, a, s);
                HIPCHK(hipGetLastError());
            }
            HIPCHK(hipEventRecord(ev.b, s));
            bool overflow = false;
            total = sink_total(db, sb, counts, overflow);
            if (!overflow) break;
            require(attempt == 0, "internal: hit bins overflowed twice");
            expected = (uint64_t)(*std::max_element(counts.begin(), counts.end())) * NBINS + NBINS;
        }
        const double kms = ev.ms();
        int key_bits = 48;
        while ((1 << (key_bits - 48)) < n_patterns) ++key_bits;
        pm_hits* h = sink_to_hits(db, sb, total, key_bits);
        h->kernel_ms = kms;
        if (total) {
            hipLaunchKernelGGL(k_linear_lens, dim3(blocks_for(total, 256)), dim3(256), 0, s, h->keys, total,
                               reinterpret_cast<const int32_t*>(d_up + o_len), 0, h->lens);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipStreamSynchronize(s));
        *out = h;
    });
}

int pm_linear_jit_compile(int n_patterns, const int32_t* lengths, const uint8_t* pos_class, int n_classes,
                          const uint8_t* class_acgt, const uint8_t* class_is_any, int k, uint64_t* code_bytes) {
    return guarded([&] {
        require(lengths && pos_class && class_acgt && class_is_any, "null argument");
        require(n_patterns >= 1 && n_patterns <= 4, "n_patterns out of range for one specialized kernel");
        require(n_classes >= 1 && n_classes <= 256, "n_classes out of range");
        require(k >= 0 && k <= PM_MAX_K, "k out of range", PM_E_UNSUPPORTED);
        int maxlen = 0;
        for (int p = 0; p < n_patterns; ++p) {
            require(lengths[p] >= 1 && lengths[p] <= PM_MAX_POSITIONS, "pattern length out of range");
            maxlen = std::max(maxlen, (int)lengths[p]);
        }
        const std::string src = gen_linear_source(n_patterns, k, maxlen > 32 ? 2 : 1, lengths, pos_class,
                                                  class_acgt, class_is_any);
        const std::vector<char> code = jit_compile(src);
        if (code_bytes) *code_bytes = code.size();
    });
}

int pm_scan_nfa(pm_db* db, int m, const uint64_t* byte_mask, const uint64_t* follow, uint64_t first, uint64_t last,
                int max_len, int k, int pattern_id, pm_hits** out) {
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
        // chunk per lane: enough lanes to fill the chip, bounded for latency
        uint64_t chunk = db->n / (256ull * 4 * 64 * 2);
        chunk = std::max<uint64_t>(64, std::min<uint64_t>(MAX_NFA_CHUNK, round_up(std::max<uint64_t>(chunk, 1), 32)));
        a.chunk = (int)chunk;
        a.nchunks = std::max<uint64_t>(1, (db->n + chunk - 1) / chunk);
        const bool nuc = db->alphabet == PM_ALPHA_NUC;
        const uint64_t need = a.nchunks * chunk + a.halo + 64;   // storage must cover the last halo
        if (nuc) require(need <= db->nwords * 32, "internal: NUC padding too small");
        else require(need <= db->nbytes_alloc, "internal: byte padding too small");

        uint64_t expected = std::max<uint64_t>(db->n / 64, 1 << 16);
        SinkBuffers sb;
        std::vector<uint32_t> counts;
        uint64_t total = 0;
        EventPair ev;
        const uint32_t blocks = blocks_for(a.nchunks, 256);
        for (int attempt = 0; attempt < 2; ++attempt) {
            sb = make_sink(db, expected);
            a.sink = Sink{sb.out, sb.cnt, sb.cap};
            HIPCHK(hipEventRecord(ev.a, s));
            if (nuc) launch_nfa_rev<true>(k, a, blocks, s);
            else launch_nfa_rev<false>(k, a, blocks, s);
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventRecord(ev.b, s));
            bool overflow = false;
            total = sink_total(db, sb, counts, overflow);
            if (!overflow) break;
            require(attempt == 0, "internal: hit bins overflowed twice");
            expected = (uint64_t)(*std::max_element(counts.begin(), counts.end())) * NBINS + NBINS;
        }
        double kms = ev.ms();
        int key_bits = 48;
        while ((1 << (key_bits - 48)) <= pattern_id) ++key_bits;
        pm_hits* h = sink_to_hits(db, sb, total, key_bits);
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
        *out = h;
    });
}

int pm_hits_count(const pm_hits* h, uint64_t* count) {
    return guarded([&] {
        require(h != nullptr && count != nullptr, "null argument");
        *count = h->count;
    });
}

int pm_hits_copy(const pm_hits* h, int32_t* pattern, int64_t* beg, int64_t* end, uint64_t max_count) {
    return guarded([&] {
        require(h != nullptr, "hits is NULL");
        const uint64_t n = std::min<uint64_t>(h->count, max_count);
        if (n == 0) return;
        DeviceGuard g(h->device);
        std::vector<uint64_t> keys(n);
        std::vector<uint32_t> lens(n);
        HIPCHK(hipDeviceSynchronize());
        HIPCHK(hipMemcpy(keys.data(), h->keys, n * 8, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(lens.data(), h->lens, n * 4, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < n; ++i) {
            const int64_t b = (int64_t)(keys[i] & ((1ull << 48) - 1));
            if (pattern) pattern[i] = (int32_t)(keys[i] >> 48);
            if (beg) beg[i] = b;
            if (end) end[i] = b + (int64_t)lens[i];
        }
    });
}

int pm_hits_copy_device(const pm_hits* h, uint64_t* keys_dst, uint32_t* lens_dst, uint64_t max_count,
                        void* stream) {
    return guarded([&] {
        require(h != nullptr, "hits is NULL");
        const uint64_t n = std::min<uint64_t>(h->count, max_count);
        if (n == 0) return;
        DeviceGuard g(h->device);
        hipStream_t s = (hipStream_t)stream;
        if (keys_dst) HIPCHK(hipMemcpyAsync(keys_dst, h->keys, n * 8, hipMemcpyDeviceToDevice, s));
        if (lens_dst) HIPCHK(hipMemcpyAsync(lens_dst, h->lens, n * 4, hipMemcpyDeviceToDevice, s));
        if (!stream) HIPCHK(hipStreamSynchronize(s));
    });
}

int pm_hits_kernel_ms(const pm_hits* h, double* ms) {
    return guarded([&] {
        require(h != nullptr && ms != nullptr, "null argument");
        *ms = h->kernel_ms;
    });
}

int pm_hits_device(const pm_hits* h, void** keys, void** lens, uint64_t* count) {
    return guarded([&] {
        require(h != nullptr, "hits is NULL");
        if (keys) *keys = h->keys;
        if (lens) *lens = h->lens;
        if (count) *count = h->count;
    });
}

int pm_hits_destroy(pm_hits* h) {
    return guarded([&] {
        if (!h) return;
        DeviceGuard g(h->device);
        HIPCHK(hipDeviceSynchronize());
        if (h->keys) HIPCHK(hipFree(h->keys));
        if (h->lens) HIPCHK(hipFree(h->lens));
        delete h;
    });
}

}  // extern "C"
