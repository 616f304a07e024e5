// pm_internal.h -- shared internals of libpatmatch_hip.so (not part of the ABI).
//
// The public boundary is include/patmatch_hip.h; everything here is private
// to the library's translation units (pm_db.hip, pm_hits.hip, pm_linear.hip,
// pm_nfa.hip).
//
// Nucleotide database layout ("stream tiles")
// ---------------------------------------------------------
// The file is cut into tiles of TILE_POS = 65536 positions.  Inside a tile,
// bit b (0..31) of logical word w (0..2047) holds position
//        T * 65536 + b * 2048 + w,
// i.e. each of the 32 bits of a word walks its own 2048-position "stream".
// Consequence: the window starting at (w, b) reads its j-th position from
// bit b of word w + j -- no bit shifts at all in the scan kernels, a pattern
// position is just a register index.  The logical words of a tile are stored
// lane-interleaved (physical (w % 32) * 64 + w / 32), so a wave whose lane l
// owns logical words [32 l, 32 l + 32) loads them with perfectly coalesced
// dword loads.  A tile stores HALO more logical words 2048..2111 (the
// continuation of every stream into the next one: bit b of word 2048 + i is
// position T * 65536 + (b + 1) * 2048 + i), so windows near a stream end need
// no neighbour-tile access.  The formula pos = T * 65536 + b * 2048 + w holds
// for halo words too.
//
// Planes per physical word, stored as two uint2 arrays: hl = {hi, lo} (2-bit
// code A=00 C=01 G=10 T=11, folded case) and bo = {brk, oth}: brk = the
// position is a record break ('\n', a header-line byte, or past the end of
// the file), oth = any other non-ACGT byte (N, IUPAC letters, '\r', ...).
// One dwordx2 load per word gives both bits of every base.  Sparse side tables give the exact byte of every
// exception position: sbflag (1 bit per physical word with brk|oth, 32 words
// per u32), sbbase (exclusive prefix), xbrk/xoth masks, the physical word
// index (xword) and 32 folded bytes per flagged word.  lflag has one u64 per
// tile: bit l = lane l of the tile sees an exception among its 32 words and
// the HALO-1 words after them.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "patmatch_hip.h"

namespace pm {

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
struct failure : std::runtime_error {
    int code;
    failure(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIPCHK(expr)                                                                    \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            throw ::pm::failure(PM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

void set_error(const std::string& msg);

// A HIP error stays on the thread until it is read: a successful call does
// not reset it (tools/micro/status_probe.hip, round 6).  So a launch check
// (HIPCHK(hipGetLastError())) also reports any earlier unchecked call's
// failure on the same thread.  hipErrorStreamCaptureUnsupported is what a
// capture-unsafe call (hipMalloc, a synchronize) returns while any thread
// captures a stream in global mode; this library never captures, but a
// caller's thread may carry that code from such a call of its own.  It is
// the one code cleared without failing; every other pending status is an
// error.  (Round 5 cleared after every rocPRIM call, on the theory that
// rocPRIM leaves that code behind; the probe shows none of the rocPRIM /
// hipCUB calls made here leaves any status, on a non-blocking stream or the
// null stream.  The checks stay after those calls, now failing on any other
// code.)
inline void clear_stale_capture_status(const char* after) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess && e != hipErrorStreamCaptureUnsupported)
        throw failure(PM_E_HIP, std::string(after) + ": " + hipGetErrorString(e));
}

// A call whose failure is deliberately ignored (teardown: frees, destroys,
// a final synchronize; a query whose "no" is an answer) must not leave its
// code pending for the next launch check on the thread: read it back.
inline void quiet(hipError_t e) {
    if (e != hipSuccess) (void)hipGetLastError();
}

void note_cleared_capture_status();   // one stderr line per process (pm_db.hip)

template <class F>
int guarded(F&& f) {
    // a C-ABI entry starts from a clean thread status: a pending capture
    // code (above) is cleared and noted once on stderr; any other status
    // pending from an earlier call (another library's, or a launch nobody
    // checked) is reported as this entry's failure rather than thrown away,
    // and is cleared by reading it, so the next call starts clean
    // (hipErrorNoDevice is left by the runtime's own start-up on a host
    // without a GPU; the host-only entries -- the hipRTC compile checks --
    // run there, and every entry that needs a device reports PM_E_NODEV)
    const hipError_t prior = hipGetLastError();
    if (prior == hipErrorStreamCaptureUnsupported) {
        note_cleared_capture_status();
    } else if (prior != hipSuccess && prior != hipErrorNoDevice) {
        set_error(std::string("a HIP error was pending on this thread before the call: ") +
                  hipGetErrorString(prior));
        return PM_E_HIP;
    }
    try {
        f();
        return PM_OK;
    } catch (const failure& e) {
        set_error(e.what());
        return e.code;
    } catch (const std::exception& e) {
        set_error(e.what());
        return PM_E_ARG;
    }
}

inline void require(bool ok, const char* msg, int code = PM_E_ARG) {
    if (!ok) throw failure(code, msg);
}

// ---------------------------------------------------------------------------
// layout constants
// ---------------------------------------------------------------------------
constexpr int LANE_WORDS = 32;                       // logical words per lane
constexpr int TILE_LANES = 64;                       // one wave per tile
constexpr uint64_t STREAM = LANE_WORDS * TILE_LANES; // 2048 positions per stream
constexpr uint64_t TILE_POS = 32 * STREAM;           // 65536 positions per tile
constexpr int HALO = 64;                             // halo words per tile (63 used)
constexpr uint64_t TILE_WORDS = STREAM + HALO;       // 2112 physical words per tile
constexpr int MAX_WINDOW = HALO;                     // longest linear pattern (64)
constexpr uint32_t NBINS = 1024;                     // hit bins (at least)
constexpr uint32_t MAX_BINS = 8192;
constexpr int MAX_NFA_CHUNK = 4096;                  // positions per lane in k_nfa_rev
constexpr uint32_t LDS_SORT_CAP = 2048;              // keys per bin sorted in LDS (16 KB: 8 sort blocks per CU)
constexpr uint32_t LDS_SORT_CAP_MAX = 4096;          // the larger sort variant (32 KB), for bins above LDS_SORT_CAP
constexpr uint32_t LDS_SORT_CAP_HUGE = 16384;        // large bins, sorted in a second pass (128 KB of LDS)
constexpr uint32_t LDS_SORT_SMALL = 256;             // many-bin lists: the small-bin pass (rank sort, 2 KB of LDS)
constexpr uint64_t BYTE_PAD = 2 * MAX_NFA_CHUNK + 4096;
constexpr int RUN_SKIP = 8;                          // run-interior lookahead (xint)

__host__ __device__ inline uint8_t fold(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }

// exact 64-bit min / max: device max()/min() on uint64_t can resolve to the
// floating-point overloads (53-bit mantissa), which corrupts (pattern, pos)
// keys above 2^53
__host__ __device__ inline uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }
__host__ __device__ inline uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// physical word index of logical word w (0 <= w < TILE_WORDS) of tile t
__host__ __device__ inline uint64_t phys_word(uint64_t tile, uint32_t w) {
    return tile * TILE_WORDS + (w < STREAM ? (uint64_t)((w & 31u) * 64u + (w >> 5)) : (uint64_t)w);
}
// logical word of physical offset r (0 <= r < TILE_WORDS) inside its tile
__host__ __device__ inline uint32_t logical_word(uint32_t r) {
    return r < STREAM ? (r & 63u) * 32u + (r >> 6) : r;
}
// file position of bit b of logical word w of tile t (valid for halo words)
__host__ __device__ inline uint64_t pos_of(uint64_t tile, uint32_t w, uint32_t b) {
    return tile * TILE_POS + (uint64_t)b * STREAM + w;
}
struct Loc {
    uint64_t word;   // physical word
    uint32_t bit;
};
__host__ __device__ inline Loc loc_of(uint64_t p) {
    const uint64_t t = p / TILE_POS;
    const uint32_t q = (uint32_t)(p % TILE_POS);
    return Loc{phys_word(t, q % (uint32_t)STREAM), q / (uint32_t)STREAM};
}

// an on/off knob from the environment ("0" off, anything else on)
inline bool env_flag(const char* name, bool dflt) {
    const char* e = getenv(name);
    return e ? e[0] != '0' : dflt;
}
inline uint64_t round_up(uint64_t x, uint64_t m) { return (x + m - 1) / m * m; }
inline uint32_t blocks_for(uint64_t n, uint32_t threads) {
    return (uint32_t)std::max<uint64_t>(1, (n + threads - 1) / threads);
}

// ---------------------------------------------------------------------------
// device views
// ---------------------------------------------------------------------------
// NUC_N_MARK: at an "other" position (bo.y bit set, no break) the hi plane
// bit is 1 iff the byte is N -- the common exception byte, whose class
// membership then needs no side-table lookup (k_others_lane); every other
// reader takes exception bytes from xbytes and ignores the planes there.
struct NucView {
    const uint2 *hl, *bo;
    const uint32_t *sbflag, *sbbase;
    const uint8_t* xbytes;
    const uint4* lin;   // the position-contiguous planes (pm_db::lin)
};

// the "other"-position list (pm_db::xlist)
constexpr uint32_t P5_NL = 1;      // the residue code of '\n' (0: header bytes and padding)
constexpr uint64_t P5_PAD = 4;   // zero words past a 5-bit plane (a window reads up to 3 words ahead)
constexpr uint64_t XL_POS_MASK = (1ull << 48) - 1;
constexpr int XL_AHEAD_SHIFT = 48;
constexpr int XL_PREV_SHIFT = 56;

// index of flagged physical word w in the compacted side tables
__device__ inline uint32_t exception_index(const uint32_t* sbflag, const uint32_t* sbbase, uint64_t w) {
    const uint32_t f = sbflag[w >> 5];
    const uint32_t wb = (uint32_t)(w & 31);
    return sbbase[w >> 5] + __popc(f & ((1u << wb) - 1));
}

// orders one wave's LDS stores before its later LDS loads (and loads before
// later stores) across lanes, without a block barrier: a wave's DS
// operations execute in issue order, so only the compiler must not move them
__device__ inline void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// the exact (folded) file byte at position p < n: breaks and "other" bytes
// come from the side table (xbytes holds the raw byte of every flagged
// position: header-line bytes, '\n', N, IUPAC letters, ...)
__device__ inline uint8_t nuc_raw_at(const NucView& v, uint64_t p) {
    const Loc l = loc_of(p);
    const uint2 e = v.bo[l.word];
    if (((e.x | e.y) >> l.bit) & 1) {
        const uint32_t idx = exception_index(v.sbflag, v.sbbase, l.word);
        return v.xbytes[(uint64_t)idx * 32 + l.bit];
    }
    const uint2 d = v.hl[l.word];
    const uint32_t code = (((d.x >> l.bit) & 1) << 1) | ((d.y >> l.bit) & 1);
    return (uint8_t)((0x54474341u >> (8 * code)) & 0xff);   // "ACGT"
}

// a header-line byte (/^>\S/ lines, generate_sequence_index.pl:33) -- a break
// whose raw byte is not the delimiter
__device__ inline bool nuc_is_header(const NucView& v, uint64_t p) {
    const Loc l = loc_of(p);
    if (!((v.bo[l.word].x >> l.bit) & 1)) return false;
    const uint32_t idx = exception_index(v.sbflag, v.sbbase, l.word);
    return v.xbytes[(uint64_t)idx * 32 + l.bit] != (uint8_t)'\n';
}

// folded byte at file position p as the line-bounded scans see it: '\n' for
// every break (header bytes included) and the tail padding
__device__ inline uint8_t nuc_char_at(const NucView& v, uint64_t p) {
    const Loc l = loc_of(p);
    const uint2 e = v.bo[l.word];
    if ((e.x >> l.bit) & 1) return (uint8_t)'\n';
    if ((e.y >> l.bit) & 1) {
        const uint32_t idx = exception_index(v.sbflag, v.sbbase, l.word);
        return v.xbytes[(uint64_t)idx * 32 + l.bit];
    }
    const uint2 d = v.hl[l.word];
    const uint32_t code = (((d.x >> l.bit) & 1) << 1) | ((d.y >> l.bit) & 1);
    return (uint8_t)((0x54474341u >> (8 * code)) & 0xff);   // "ACGT"
}

// Hit sink: NBINS bins of `cap` keys.  Bins are ranges of (pattern, position)
// in increasing order, so sorting every bin sorts the whole list.
struct Sink {
    uint64_t* out;       // [NBINS * cap]
    uint32_t* bin_cnt;   // [NBINS]
    uint32_t cap;
    uint32_t bins_per_pattern;
    uint32_t pos_shift;  // bin within a pattern = position >> pos_shift
    __device__ uint32_t bin_of(uint32_t pattern_slot, uint64_t pos) const {
        return pattern_slot * bins_per_pattern + (uint32_t)(pos >> pos_shift);
    }
    __device__ void push(uint32_t bin, uint64_t key) const {
        const uint32_t o = atomicAdd(&bin_cnt[bin], 1u);
        if (o < cap) out[(uint64_t)bin * cap + o] = key;
    }
};

__device__ inline uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

struct EventPair {
    hipEvent_t a = nullptr, b = nullptr;
    EventPair() {
        HIPCHK(hipEventCreate(&a));
        HIPCHK(hipEventCreate(&b));
    }
    ~EventPair() {
        if (a) quiet(hipEventDestroy(a));
        if (b) quiet(hipEventDestroy(b));
    }
    double ms() {
        float v = 0.f;
        HIPCHK(hipEventElapsedTime(&v, a, b));
        return v;
    }
};

}  // namespace pm

// ---------------------------------------------------------------------------
// opaque ABI types
// ---------------------------------------------------------------------------
struct pm_devbuf {       // device buffer grown on demand, reused across calls
    void* p = nullptr;
    size_t cap = 0;
};
struct pm_hostbuf {      // pinned host staging buffer
    void* p = nullptr;
    size_t cap = 0;
};

// Per-scan workspaces ("lane"): device buffers the kernels of one scan
// write, the pinned staging they are uploaded from, and `free_ev`, recorded
// after the last work that reads them (a scan waits for it on the GPU before
// reusing the lane).  Never stream-ordered allocations.
struct pm_lane {
    pm_devbuf ws_tab, ws_sink, ws_rec, ws_rep, ws_oth;
    pm_hostbuf pin_up, pin_slots;
    // slot tables last uploaded into ws_sink (skip the copy when unchanged)
    void* slot_cache_p = nullptr;
    uint32_t slot_cache_per = 0;
    std::vector<uint32_t> slot_cache_caps;
    // pinned staging buffers are rewritten by the host only after the copy
    // that last read them has run (pipelined scans keep work in flight)
    hipEvent_t up_fence = nullptr, slots_fence = nullptr;
    std::vector<uint8_t> up_cache;    // tables last uploaded into ws_tab
    void* up_cache_p = nullptr;
    hipEvent_t free_ev = nullptr;
};

struct pm_db : pm_lane {
    // every entry point that uses the database (scans, decode, destroy, the
    // resolution of a pending list) holds this lock: ctypes releases the GIL
    // around a call, so a multi-threaded server (mod_wsgi's 15 threads) may
    // enter from several threads at once; the workspaces, slot caches and
    // the pending set are per database.  Recursive: resolving a pending list
    // can re-run its scan.
    std::recursive_mutex mu;
    int device = 0;
    int alphabet = PM_ALPHA_NUC;
    uint64_t n = 0;          // positions (file bytes)
    uint64_t ntiles = 0;     // NUC: tiles (incl. break-only padding tiles)
    uint64_t nwords = 0;     // NUC: physical words (ntiles * TILE_WORDS)
    uint64_t nsb = 0;        // NUC: superblocks (32 physical words)
    uint64_t nflag = 0;      // NUC: exception words
    uint64_t n_oth_words = ~0ull;   // NUC: words holding an "other" byte (~0: not counted)
    uint64_t nbytes_alloc = 0;
    uint2 *hl = nullptr, *bo = nullptr;   // NUC planes {hi, lo}, {brk, oth}
    uint32_t *sbflag = nullptr, *sbbase = nullptr;
    uint32_t *xbrk = nullptr, *xoth = nullptr;
    uint8_t* xbytes = nullptr;
    uint64_t* xword = nullptr;   // NUC: physical word of each flagged word
    uint64_t* lflag = nullptr;   // NUC: per tile, lanes with exceptions
    uint64_t* hflag = nullptr;   // NUC: per tile, lanes whose own words hold a header byte (k_header_flags)
    uint4* lin = nullptr;        // NUC: {hi, lo, brk, oth} bits of positions 32 q .. 32 q + 31 (k_build_lin)
    // NUC, runs of N: per flagged word, the bits whose position is preceded
    // by an exception and followed by RUN_SKIP more "other" bytes (xint);
    // the flagged words with a bit outside that mask (xedge, nedge of them;
    // xedge_oth / nedge_oth: those with an "other" bit outside it)
    uint32_t* xint = nullptr;
    uint32_t* xedge = nullptr;
    uint64_t nedge = 0;
    uint32_t* xedge_oth = nullptr;
    uint64_t nedge_oth = 0;
    // NUC: every "other" position outside the run interiors, as
    // e | ahead << 48 | prev << 56 (XL_*): ahead = consecutive exception
    // positions from e on (at most 255), prev = e - 1 is an exception
    // (k_others_lane's work list, built once per database)
    uint64_t* xlist = nullptr;
    uint64_t nxlist = 0;
    // BYTE databases: the folded bytes as 5-bit residue codes (0 = a header
    // byte or the padding, 1 = '\n', 2..31 = the database's other distinct
    // bytes, in increasing byte order), bit-sliced: plane q of word w holds
    // bit q of the codes of positions 32 w .. 32 w + 31 (p5[q * nw5 + w]).
    // None when the file holds more than 30 distinct bytes besides '\n'
    // (the byte copy is scanned then).  hdr_end[r]: the end of header line r
    // (its '\n'; hdr[r] its start) for windows that read header bytes.
    uint64_t* hdr_end = nullptr;
    uint32_t* p5 = nullptr;
    uint64_t nw5 = 0;      // words per plane (+ P5_PAD zero words read past the end)
    int n_codes = 0;       // residue codes in use (0: no planes)
    uint8_t code_of[256] = {};
    uint8_t* bytes = nullptr;    // BYTE alphabet: folded bytes, header lines stored as '\n'
    uint8_t* bytes_raw = nullptr;   // BYTE alphabet: folded bytes as in the file (headers kept)
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // synchronous-path workspaces
    pm_devbuf ws_post;
    // the q-gram batch filter's device tables (pm_batch.hip) and the batch
    // signature they were built for: a repeated batch uploads nothing
    pm_devbuf ws_batch;
    std::string batch_sig;
    pm_hostbuf pin_down;
    pm_hostbuf pin_ord;   // the ordered batch verify's list counts
    // pipelined scans: record expansion + sort of scan i run on `post` while
    // scan i+1's kernel runs on `stream`, each on its own workspace lane (the
    // inherited pm_lane is the active one, `alt` the other; switch_lane swaps)
    hipStream_t post = nullptr;
    pm_lane alt;
    bool lane_flip = false;          // PM_POST_STREAM: the next pipelined scan takes `alt`
    hipEvent_t scan_ev = nullptr;    // PM_POST_STREAM: a scan's end, waited for by `post`
    hipEvent_t join_ev = nullptr;    // post_join: `post`'s queued work, waited for by `stream`
    // the exception pass (k_linear_others) runs on `exc`, concurrently with
    // the specialized scan: forked from the scan stream after the counters
    // are zeroed, joined before the sort
    hipStream_t exc = nullptr;
    hipEvent_t exc_fork = nullptr, exc_join = nullptr;
    std::set<pm_hits*> pending;       // pipelined scans not yet resolved
    uint64_t device_bytes = 0;
    // nrgrep's search regions (Regions; set by pm_db_create* for the file
    // itself, or by pm_db_set_regions)
    uint64_t *reg_t = nullptr, *reg_e = nullptr;
    uint32_t *reg_lut = nullptr, *reg_near = nullptr;
    uint32_t nreg = 0;
    bool reg_blind = false;   // some region ends without a '\n' (a buffer holding none)
    // the first position of every header line (/^>\S/, sorted): the
    // eextended walk starts a cluster at each (pm_eextended.hip)
    uint64_t* hdr = nullptr;
    uint64_t nhdr = 0;
};

// A pipelined scan (pm_scan_linear_async) between launch and resolution: the
// hit list was sorted speculatively into segment-sized capacity; its bin
// counts travel to pinned memory behind `counted`.  Resolution validates
// them (no overflow, no record overflow, every bin LDS-sortable) or re-runs
// the query synchronously.
struct pm_pending {
    pm_db* db = nullptr;
    hipEvent_t counted = nullptr;
    uint32_t* counts_h = nullptr;     // nbins counts + the record-overflow counter
    size_t counts_cap = 0;
    uint32_t nbins = 0, bins_per_pattern = 0;
    std::vector<uint32_t> slot_cap_h;
    std::vector<std::unique_ptr<pm::EventPair>> jev;   // per specialized launch
    std::string hint_key;
    std::vector<uint32_t> slot_caps;
    uint32_t rcap = 0;
    // the query itself, for the synchronous re-run
    int n_patterns = 0, n_classes = 0, k = 0;
    uint32_t flags = 0;               // PM_REPORT_* / PM_ANCHOR_*
    bool reported = false;            // counts_h[nbins + 1] holds the reported count
    bool count_only = false;          // a pipelined batch: counts_h[0] is the reported count, nothing else pends
    std::vector<int32_t> lengths;
    std::vector<uint8_t> pos_class, class_acgt, class_is_any;
    std::vector<uint32_t> class_bytes;
    uint64_t* clk = nullptr;          // PM_JIT_CLOCK: the launch's per-workgroup clock samples
    uint64_t clk_nwg = 0;
    ~pm_pending();
};

struct pm_hits {
    int device = 0;
    uint64_t count = 0;
    uint64_t* keys = nullptr;   // sorted, pattern << 48 | beg
    uint32_t* lens = nullptr;
    size_t keys_cap = 0, lens_cap = 0;
    // set: lens[] is unwritten and a key's length is plen[pattern] (a batch
    // of exact patterns; the report pass reads it and writes its own lens)
    const int32_t* plen = nullptr;
    double kernel_ms = 0.0;
    hipEvent_t ready = nullptr;     // recorded after the last kernel writing keys/lens
    hipEvent_t last_use = nullptr;  // recorded by pm_hits_copy_device on the caller's stream
    pm_pending* pending = nullptr;  // pipelined scan not yet resolved (count unknown)
    // the list's buffers before its report pass compacted it: free once
    // `ready` (bound to the pass's last dispatch) has completed
    uint64_t* old_keys = nullptr;
    uint32_t* old_lens = nullptr;
    size_t old_keys_cap = 0, old_lens_cap = 0;
};

namespace pm {

// ---------------------------------------------------------------------------
// host helpers (pm_db.hip)
// ---------------------------------------------------------------------------
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        HIPCHK(hipGetDevice(&prev));
        if (prev != dev) HIPCHK(hipSetDevice(dev));
    }
    ~DeviceGuard() {
        if (prev >= 0) quiet(hipSetDevice(prev));
    }
};

// workspace lanes (pm_lane): a scan waits on the GPU for its lane's last
// reader (lane_begin) and marks its own last reader (lane_end, also done by
// hits_ready on db->stream); switch_lane alternates lanes (pipelined scans)
void lane_begin(pm_db* db);
void lane_end(pm_db* db, hipStream_t s);
void switch_lane(pm_db* db);
hipStream_t post_stream(pm_db* db);
// PM_POST_STREAM (A/B, round 6): 0 (default) the expansion, exception pass,
// sort and report of a pipelined scan run on the scan's own stream; 1 on
// `post` with the workspaces double-buffered (lane_flip), so scan i+1 runs
// while scan i is post-processed; 2 the same with `post` at high priority
int post_mode();
// every other user of a database's workspaces waits for `post` first
void post_join(pm_db* db);
hipStream_t exc_stream(pm_db* db);   // creates exc, exc_fork and exc_join on first use
void* reserve(pm_db* db, pm_devbuf& b, size_t bytes);
// Per-device pool of hit-list buffers (sizes rounded to powers of two):
// scans allocate their result from it and pm_hits_destroy returns it, so a
// query costs no hipMalloc/hipFree (hipFree synchronizes the device).
void* pool_get(int device, size_t bytes, size_t* cap);
void pool_put(int device, void* p, size_t cap);
void* reserve_host(pm_db* db, pm_hostbuf& b, size_t bytes);
NucView nuc_view(const pm_db* db);
// nrgrep's regions of a text read in buffers of `bufsize` bytes
// (recSearchFile 0x402250): last_nl(lo, hi) = the last '\n' in [lo, hi), or
// ~0.  Region r = [t[r], e[r]).  bufsize 0: one region.
template <class LastNl>
void nrgrep_regions(uint64_t n, uint64_t bufsize, LastNl last_nl, std::vector<uint64_t>& t, std::vector<uint64_t>& e) {
    t.clear();
    e.clear();
    for (uint64_t at = 0;;) {
        if (bufsize == 0 || at + bufsize > n) {   // bufEof (0x41bfc0): the buffer is not full
            t.push_back(at);
            e.push_back(n);
            return;
        }
        t.push_back(at);
        // simpleRevSearch (0x402475) for the record delimiter; the region ends
        // after it and the next buffer starts AT it (bufLoad 0x4023e6 from its
        // start); none, or only at the buffer start: the whole buffer, and the
        // next one starts after it (0x4024a0 -> 0x4022ba)
        const uint64_t d = last_nl(at, at + bufsize);
        if (d != ~0ull && d != at) {
            e.push_back(d + 1);
            at = d;
        } else {
            e.push_back(at + bufsize);
            at += bufsize;
        }
        if (at >= n) return;   // bufEmpty after the load
    }
}
void set_regions(pm_db* db, const std::vector<uint64_t>& t, const std::vector<uint64_t>& e);

// hipRTC: compiles generated kernel source for gfx950 (pm_linear.hip)
std::vector<char> hiprtc_compile(const std::string& src);

// The reverse (start-finding) pass of a class-sequence automaton with
// insertions / deletions / substitutions, bit-sliced over the 32 streams of
// the nucleotide planes (pm_ids.hip).  Emits every start into `sink` as
// k_nfa_rev would.  Returns false (nothing launched) when the shape is not
// covered (positions x rows too many for registers).
struct IdsSpec {
    int m, k, errs;
    const uint64_t* byte_mask;   // [256] positions accepting each folded byte (host)
    const uint64_t* d_bmask;     // the same table on the device ('\n' accepted by none)
    uint64_t rev_pre[PM_MAX_K + 1], rev_ins[PM_MAX_K + 1];   // the injected start config (scan_nfa)
    int pattern_id;
    bool keep = false;           // (set by ids_rev_scan) the warm-up words' planes kept in LDS
};
bool ids_rev_scan(pm_db* db, const IdsSpec& spec, const Sink& sink, hipStream_t s, hipEvent_t ev_a, hipEvent_t ev_b);

// Large k = 0 batches of fixed-length patterns: a q-gram filter in one pass
// over the planes (pm_batch.hip).
constexpr int BQ = 10;                                     // q-gram length
constexpr uint32_t BQ_TABLE_WORDS = 1u << (2 * BQ - 5);    // 2^20 bits: 128 KB of LDS
constexpr int BATCH_WAVES = 16;                            // waves per workgroup (one workgroup per CU)
constexpr int BATCH_THREADS = 64 * BATCH_WAVES;
constexpr int BATCH_MAX_P = 1024;
constexpr int BATCH_MAX_LEN = 16;                          // a window's bases fit one 32-bit code word
constexpr uint32_t BATCH_MAX_WPO = 64;                     // scan waves per output segment
constexpr uint32_t BATCH_VERIFY_WAVES = 16;                // waves per verify block (one per segment)
constexpr uint32_t ORD_HIST_MAX_P = 256;                   // patterns counted per list by the ordered verify
constexpr uint64_t BATCH_MAX_EXPANSIONS = 1ull << 18;      // indexed codes (a quarter of the table)

struct BatchIndex {
    uint32_t omax = 0;     // the largest piece offset: probes start there
    uint64_t expansions = 0;
    std::vector<uint32_t> table;      // [BQ_TABLE_WORDS]: the codes present (bit code & 31 of word code >> 5)
    // [2^(2 BQ)]: first entry << 8 | entries, per code (4 MB, read once per
    // candidate; an L2-resident hash table measured slower: 2.22 vs 2.08 ms)
    std::vector<uint32_t> code_off;
    std::vector<uint32_t> ents;       // BATCH_ENT_WORDS per (code, pattern) entry, in increasing code order
    std::vector<uint32_t> pmask;      // [P][4]: bit 2j + 1 = position j accepts A / C / G / T
    std::vector<uint32_t> popt;       // [P]: o_p, the indexed piece's offset
    // [BQ_HASH_SLOTS] open-addressing table of the codes present, for the
    // verify's LDS (empty when there are too many codes): code | x << 20 |
    // entries << 52, ~0 = empty slot; x = the entry's first word (p | o_p <<
    // 16 | len << 24) for a code with one entry, else its first entry's index
    // (bq_slot_entry)
    std::vector<uint64_t> hash;
    // device image (ws_batch): table | code_off | ents | pmask | popt | hash
    size_t o_table = 0, o_code = 0, o_ents = 0, o_pmask = 0, o_popt = 0, o_hash = 0, bytes = 0;
};
constexpr uint32_t BQ_HASH_BITS = 14;                      // 16 Ki slots: 128 KB of LDS
constexpr uint32_t BQ_HASH_SLOTS = 1u << BQ_HASH_BITS;
constexpr uint32_t BQ_HASH_MAX_CODES = BQ_HASH_SLOTS * 7 / 10;
__host__ __device__ inline uint32_t bq_hash(uint32_t code) { return (code * 0x9E3779B1u) >> (32 - BQ_HASH_BITS); }
// one verification entry (two uint4): {p | o_p << 16 | len << 24, length mask
// (bits 2j + 1), 0, 0}, {mA, mC, mG, mT}
constexpr int BATCH_ENT_WORDS = 8;
// a hash slot -> co: first entry << 8 | entries (entries >= 2; 0: absent),
// or, for a one-entry code, that entry's first word | BQ_CO_ONE (the slot
// holds it: p | o_p << 16 | len << 24, len < 32 leaves bit 31 free; entry
// indices stay below 2^23, build_batch_index)
constexpr uint32_t BQ_CO_ONE = 1u << 31;
__host__ __device__ inline uint32_t bq_slot_entry(uint64_t sl) {
    const uint32_t cnt = (uint32_t)(sl >> 52) & 255u;
    if (cnt == 1) return (uint32_t)(sl >> 20) | BQ_CO_ONE;
    return (uint32_t)((sl >> 20) & 0xFFFFFFu) << 8 | cnt;
}
// the length mask of a pattern of `len` positions (bits 2j + 1, j < len)
__host__ __device__ inline uint32_t bq_len_mask(uint32_t len) {
    return 0xAAAAAAAAu & (len >= 16 ? ~0u : (1u << (2 * len)) - 1u);
}
// false: the batch is not for the filter (lengths outside [BQ, BATCH_MAX_LEN],
// too many patterns or expansions, a code shared by more than 255 patterns)
bool build_batch_index(int P, const int32_t* lengths, const uint8_t* pos_class, const uint8_t* class_acgt,
                       const uint8_t* class_is_any, BatchIndex& bi);

struct BatchScanArgs {
    const uint2* hl;
    uint64_t ntiles;
    const uint32_t* table;
    uint32_t omax, tiles_per_wave, nwaves, ccap;
    uint4* cand;            // [nwaves][ccap] candidate entries
    uint32_t* cand_cnt;     // [nwaves]
    uint32_t *zero_a, *zero_b;   // counters zeroed by the first workgroup (the sink's aux counter, xcnt)
};
struct BatchVerifyArgs {
    const uint4* cand;
    const uint32_t* cand_cnt;
    uint32_t ccap;
    uint32_t* aux;          // the largest candidate count above ccap (0: none)
    const uint32_t* code_off;
    const uint64_t* hash;   // BatchIndex::hash (null: code_off)
    const uint4* ents;      // two uint4 per entry
    const uint4* pmask;
    const uint32_t* popt;
    const int32_t* lengths;
    uint32_t omax, tiles_per_wave, wpo, nwaves, nout;
    int P;
    const uint2 *hl, *bo;
    const uint64_t* lflag;
    uint64_t ntiles, n;
    uint64_t* out;
    uint32_t* seg_cnt;
    const uint64_t* slot_base;
    const uint32_t* slot_cap;
    uint64_t* xkeys;        // keys of the next segment
    uint32_t* xcnt;
    uint32_t xcap;
    // the ordered form (null: the unordered one): per (segment, verify wave)
    // list of ord_cap keys in position order, their counts, and a flag set
    // when a lane's round held more matches than it keeps
    uint64_t* ord_out = nullptr;
    uint32_t* ord_cnt = nullptr;
    uint32_t* ord_bad = nullptr;
    uint32_t ord_cap = 0;
    uint32_t sink_segs = 0;   // segments per pattern of the bins k_batch_fixup fills (0: nout)
    uint32_t* ord_hist = nullptr;   // [P][nout * BATCH_VERIFY_WAVES] keys per (pattern, list); null: none
    const uint4* lin = nullptr;     // the position-contiguous planes: a window's exception bits in 1-2 loads
};
// k_batch_scan (timed by ev_a / ev_b), k_batch_verify, k_batch_fixup on s
void batch_launch(const BatchScanArgs& sa, const BatchVerifyArgs& va, uint32_t nblocks, hipStream_t s,
                  hipEvent_t ev_a, hipEvent_t ev_b);

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
    uint8_t* commit(pm_db* db);   // uploads into db->ws_tab; returns its device base
};


// ---------------------------------------------------------------------------
// hit collection (pm_hits.hip)
// ---------------------------------------------------------------------------
struct SinkBuffers {
    uint64_t* out = nullptr;
    uint32_t* cnt = nullptr;
    uint32_t cap = 0;              // uniform capacity (make_sink) / the largest slot capacity
    // per pattern slot: bin b of slot p = b / bins_per_pattern holds up to
    // slot_cap[p] keys at out + slot_base[p] + (b % bins_per_pattern) * slot_cap[p]
    uint64_t* slot_base = nullptr;
    uint32_t* slot_cap = nullptr;
    std::vector<uint32_t> slot_cap_h;
    // cnt[nbins]: one auxiliary device counter zeroed and read back with the
    // bin counters (pm_linear: the record-overflow maximum); sink_total sets aux
    uint32_t aux = 0;
    uint32_t bins_per_pattern = NBINS;
    uint32_t pos_shift = 0;
    uint32_t nbins = NBINS;
    Sink sink() const { return Sink{out, cnt, cap, bins_per_pattern, pos_shift}; }
};

// Bins for `n_slots` pattern slots over positions [0, n_positions);
// `expected` sizes the per-bin capacity.
SinkBuffers make_sink(pm_db* db, int n_slots, uint64_t n_positions, uint64_t expected);
// Bins filled by the producer itself: n_slots x per_slot segments of `cap`
// keys, each a position range in increasing order (pm_linear_jit).
SinkBuffers make_sink_segments(pm_db* db, int n_slots, uint32_t per_slot, const std::vector<uint32_t>& slot_caps,
                               bool zero_counts = true);
// Reads bin counters; returns total, sets `overflow` if a bin exceeded cap.
uint64_t sink_total(pm_db* db, const SinkBuffers& sb, std::vector<uint32_t>& counts, bool& overflow);
// bins -> one sorted key list (pattern << 48 | pos) owned by the returned
// hits; lens are left for the caller to fill.
// Sorts every bin (<= 4096 bins, lists <= LDS_SORT_CAP_MAX keys) into a list
// sized for all capacities BEFORE the counts reach the host, so a scan needs
// one host sync; count unset -- the caller validates the counts it reads
// afterwards and keeps the result (count = total) or discards it.
// counts_host (mapped pinned, optional): the sort also stores the raw bin
// counts and the aux counter there (the pipelined scan's readback).
// total_out (device, optional): the list length (sum of the clamped counts).
pm_hits* sink_sort_speculative(pm_db* db, const SinkBuffers& sb, const int32_t* slot_len, uint32_t* counts_host,
                               hipStream_t stream, uint64_t* total_out = nullptr, bool bind_ready = true);
void discard_hits(pm_hits* h);   // buffers back to the pool (no event waits)
// slot_len (device, per slot, optional): fixed match length of every key of
// a slot -- the LDS sort writes h->lens with the keys.
// The ordered batch verify's result: nlists lists of position-ordered keys
// (list l at ord + l * ord_cap, cnt[l] <= ord_cap keys; d_cnt on the device)
// and the sink's bins (counts, sink_total keys: the exception pass, keys of
// the next segment, the first starts) into one (pattern, position)-sorted
// list: one stable radix pass over the pattern bits, the sink sorted by
// sink_to_hits, a merge of the two.  Lens are the caller's.
// d_hist (may be null): keys per (pattern, list), [P][nlists] -- then a
// stable scatter by pattern replaces the radix sort.
pm_hits* ordered_to_hits(pm_db* db, const SinkBuffers& sb, const std::vector<uint32_t>& counts, uint64_t sink_total,
                         const uint64_t* ord, uint32_t ord_cap, const uint32_t* d_cnt, const uint32_t* cnt,
                         uint32_t nlists, int n_patterns, const uint32_t* d_hist = nullptr);
pm_hits* sink_to_hits(pm_db* db, const SinkBuffers& sb, const std::vector<uint32_t>& counts, uint64_t total,
                      const int32_t* slot_len = nullptr, bool* lens_done = nullptr);
// records h->ready on the db stream: call after the last kernel filling h
void hits_ready(pm_db* db, pm_hits* h);
// Resolves a pipelined scan's hit list (no-op for a resolved one): waits for
// its counts, keeps the speculative list or replaces it by a synchronous
// re-run of the query (pm_linear.hip).
void hits_finalize(pm_hits* h);
// mapped pinned host buffers for count readbacks (pooled, no hipHostMalloc
// per scan; kernels write them directly)
void* pinned_get(size_t bytes, size_t* cap);
void pinned_put(void* p, size_t cap);

// ---------------------------------------------------------------------------
// nrgrep report selection (pm_hits.hip)
// ---------------------------------------------------------------------------
// The scan kernels produce candidates: every start with a match (and its
// end).  nrgrep_coords prints a subset: recSearchFile (0x402250) calls the
// scanner on [R, buffer end), prints the match it returns and resumes at its
// end (R = end, 0x4022de-0x4022f4), so reported matches never overlap and the
// first one found wins; '^' / '$' (main 0x40164d / 0x40162a) are checked by
// recCheckLeftContext / recCheckRightContext (0x402170 / 0x4021e0) against
// the region start R and the line ends.  Hits whose start lies on a header
// line (incl. its '\n') are dropped afterwards (process_output discards them,
// patmatch.py:548).
// nrgrep's search regions (pm_db::reg_*, DESIGN.md §1 "Regions"): region r
// is [reg_t[r], reg_e[r]); a match is found in the region whose start is the
// last one at or before its start, must lie inside it, and the report rule
// restarts at every region start.
struct Regions {
    const uint64_t* t = nullptr;    // starts (increasing)
    const uint64_t* e = nullptr;    // ends
    const uint32_t* lut = nullptr;  // [p >> REG_LUT_SHIFT]: the last region starting at or before that bucket
    const uint32_t* near = nullptr; // bit per REG_NEAR_SHIFT block: a region start within REG_NEAR_SPAN
    uint32_t n = 0;                 // <= 1: one region, the whole text (nothing to check)
};
constexpr int REG_LUT_SHIFT = 20;
constexpr int REG_NEAR_SHIFT = 12;
// >= the widest gap inside one esimple cluster (es_gap: 2 (m + k) + 2), so a
// cluster never straddles a region start unseen
constexpr uint64_t REG_NEAR_SPAN = 1024;
static_assert(REG_NEAR_SPAN >= 2 * (PM_MAX_POSITIONS + PM_MAX_K) + 2, "REG_NEAR_SPAN below the esimple gap");
__device__ inline uint32_t region_of(const Regions& g, uint64_t s) {
    uint32_t r = g.lut[s >> REG_LUT_SHIFT];
    while (r + 1 < g.n && g.t[r + 1] <= s) ++r;
    return r;
}
// a region start (other than 0) lies within REG_NEAR_SPAN of s: only then
// can the regions change anything about a window starting at s (one cached
// load; regions are ~1.6 MB apart)
__device__ inline bool region_near(const Regions& g, uint64_t s) {
    if (g.n <= 1) return false;
    const uint64_t b = s >> REG_NEAR_SHIFT;
    return (g.near[b >> 5] >> (b & 31)) & 1u;
}

struct TextView {
    NucView nuc;
    const uint8_t* bytes;   // BYTE layout (header bytes stored as '\n')
    const uint8_t* raw;     // BYTE layout, the file's own bytes
    uint64_t n;
    int nuc_layout;
    const uint64_t* hflag;  // NUC: per tile, the lanes whose own words hold a header byte (pm_db::hflag)
    Regions reg;
};
TextView text_view(const pm_db* db);

// the file's own text as nrgrep's extended walks read it (pm_extended.hip,
// pm_eextended.hip)
__device__ inline uint8_t xt_fold(uint8_t c) { return (c >= 'a' && c <= 'z') ? (uint8_t)(c - 32) : c; }

// the file's own byte at p (headers and '\n' included), folded
__device__ inline uint8_t xt_byte(const TextView& tv, uint64_t p) {
    if (tv.nuc_layout) {
        const uint4 v = tv.nuc.lin[p >> 5];
        const uint32_t i = (uint32_t)(p & 31);
        if (((v.z | v.w) >> i) & 1) return xt_fold(nuc_raw_at(tv.nuc, p));
        return (uint8_t)((0x54474341u >> (8 * ((((v.x >> i) & 1) << 1) | ((v.y >> i) & 1)))) & 0xff);
    }
    return xt_fold(tv.raw[p]);
}

// a line break or header byte at p (the breaks of the line-bounded scans)
__device__ inline bool xt_brk(const TextView& tv, uint64_t p) {
    if (tv.nuc_layout) return (tv.nuc.lin[p >> 5].z >> (uint32_t)(p & 31)) & 1;
    return tv.bytes[p] == (uint8_t)'\n';
}

// the start of a header line (process_output drops such matches)
__device__ inline bool xt_header(const TextView& tv, uint64_t p) {
    if (tv.nuc_layout) return nuc_is_header(tv.nuc, p);
    return tv.bytes[p] == (uint8_t)'\n' && tv.raw[p] != (uint8_t)'\n';
}

// a break in (a, b): a and b are starts of matches (sequence positions), so
// a header byte in between implies the '\n' before its line.  Looks back
// from b at most `cap` positions; false when none was found there.
__device__ inline bool xt_brk_between(const TextView& tv, uint64_t a, uint64_t b, uint64_t cap) {
    const uint64_t lo = b - a > cap ? b - cap : a + 1;
    if (lo + 1 > b) return false;   // nothing between
    if (tv.nuc_layout) {
        for (uint64_t w = (b - 1) >> 5;; --w) {
            uint32_t z = tv.nuc.lin[w].z;
            const uint64_t w0 = w << 5;
            if (w0 + 31 > b - 1) z &= (2u << (uint32_t)((b - 1) - w0)) - 1u;   // positions <= b - 1
            if (w0 < lo) z &= ~((1u << (uint32_t)(lo - w0)) - 1u);            // positions >= lo
            if (z) return true;
            if (w0 <= lo) return false;
        }
    }
    for (uint64_t p = b - 1; p >= lo; --p) {
        if (tv.bytes[p] == (uint8_t)'\n') return true;
        if (p == lo) break;
    }
    return false;
}

__device__ inline uint32_t xt_region(const TextView& tv, uint64_t p) { return tv.reg.n > 1 ? region_of(tv.reg, p) : 0u; }

// A walk thread's window of the file's own folded bytes (xt_byte) in LDS:
// the per-cluster walks of nrgrep's report (pm_extended / pm_eextended /
// pm_regular.hip) read the text one character per dependent step, so each
// read from memory was a full round trip.  A miss refills TC_WIN bytes from
// TC_BACK before the position with independent 16-byte loads (one round trip
// per refill); the scanners move forward and every verify phase reads at most
// a pattern's span back.
constexpr uint32_t TC_WIN = 256, TC_BACK = 96;
constexpr uint32_t WALK_T = 128;   // walk threads per block: WALK_T * TC_WIN bytes of LDS
__device__ inline uint32_t fold4(uint32_t v) {   // xt_fold on four bytes
    const uint32_t ge_a = (v | 0x80808080u) - 0x61616161u, gt_z = (v | 0x80808080u) - 0x7b7b7b7bu;
    const uint32_t lower = ge_a & ~gt_z & ~v & 0x80808080u;   // 0x61 <= b <= 0x7a
    return v - (lower >> 2);                                   // 0x80 >> 2 = 0x20
}
// A refill is out of line (one copy for every read site of a walk; a walk
// inlines dozens) and takes plain pointers, not the TextView aggregate.
// NUC: [l, h) from the position planes four bytes at a time, then the
// flagged positions (exceptions, breaks) from the side tables.
static __device__ __attribute__((noinline)) void tc_fill_nuc(uint8_t* buf, const uint4* lin, const uint2* hl,
                                                             const uint2* bo, const uint32_t* sbflag,
                                                             const uint32_t* sbbase, const uint8_t* xbytes,
                                                             uint64_t l, uint64_t h) {
    const NucView nv{hl, bo, sbflag, sbbase, xbytes, lin};
    uint4 w[TC_WIN / 32];
#pragma unroll
    for (uint32_t q = 0; q < TC_WIN / 32; ++q) w[q] = l + 32ull * q < h ? lin[(l >> 5) + q] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t q = 0; q < TC_WIN / 32; ++q) {
        uint32_t o[8];
#pragma unroll
        for (uint32_t g = 0; g < 8; ++g) {
            uint32_t v = 0;
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i) {
                const uint32_t b = 4 * g + i;
                const uint32_t code = (((w[q].x >> b) & 1) << 1) | ((w[q].y >> b) & 1);
                v |= ((0x54474341u >> (8 * code)) & 0xffu) << (8 * i);   // "ACGT"
            }
            o[g] = v;
        }
        uint4* d = reinterpret_cast<uint4*>(buf + 32 * q);
        d[0] = make_uint4(o[0], o[1], o[2], o[3]);
        d[1] = make_uint4(o[4], o[5], o[6], o[7]);
    }
    for (uint32_t q = 0; q < TC_WIN / 32; ++q) {
        uint32_t ex = w[q].z | w[q].w;
        while (ex) {
            const uint32_t i = (uint32_t)__builtin_ctz(ex);
            ex &= ex - 1;
            const uint64_t pos = l + 32ull * q + i;
            if (pos < h) buf[32 * q + i] = xt_fold(nuc_raw_at(nv, pos));
        }
    }
}
// BYTE: [l, h) with 16-byte loads, folded four bytes at a time
static __device__ __attribute__((noinline)) void tc_fill_raw(uint8_t* buf, const uint8_t* raw, uint64_t n, uint64_t l) {
    uint4 v[TC_WIN / 16];
#pragma unroll
    for (uint32_t q = 0; q < TC_WIN / 16; ++q)
        v[q] = l + 16ull * q + 16 <= n ? *reinterpret_cast<const uint4*>(raw + l + 16ull * q) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t q = 0; q < TC_WIN / 16; ++q)
        *reinterpret_cast<uint4*>(buf + 16 * q) = make_uint4(fold4(v[q].x), fold4(v[q].y), fold4(v[q].z), fold4(v[q].w));
    for (uint64_t p = l + 16ull * ((n > l ? n - l : 0) / 16); p < n && p < l + TC_WIN; ++p)   // the last partial chunk
        buf[p - l] = xt_fold(raw[p]);
}
struct TxtCache {
    uint8_t* buf;       // TC_WIN bytes of LDS (16-byte aligned)
    uint64_t lo, hi;    // positions cached: [lo, hi)
    __device__ void fill(const TextView& tv, uint64_t p) {
        if (tv.nuc_layout) {
            const uint64_t l = p > TC_BACK ? (p - TC_BACK) & ~31ull : 0ull;
            hi = umin64(l + TC_WIN, tv.n);
            tc_fill_nuc(buf, tv.nuc.lin, tv.nuc.hl, tv.nuc.bo, tv.nuc.sbflag, tv.nuc.sbbase, tv.nuc.xbytes, l, hi);
            lo = l;
            return;
        }
        const uint64_t l = p > TC_BACK ? (p - TC_BACK) & ~15ull : 0ull;
        tc_fill_raw(buf, tv.raw, tv.n, l);
        lo = l;
        hi = umin64(l + TC_WIN, tv.n);
    }
    __device__ uint8_t get(const TextView& tv, uint64_t p) {
        if (p >= tv.n) return (uint8_t)'\n';
        if (p - lo >= hi - lo) fill(tv, p);
        return buf[p - lo];
    }
};
// the first '\n' at or after p (n: none), p < n <= tv.n: a word of break
// flags (NUC) or 16 bytes (BYTE) per dependent load
__device__ inline uint64_t xt_next_nl(const TextView& tv, uint64_t p, uint64_t n) {
    if (tv.nuc_layout) {
        while (p < n) {
            uint32_t z = tv.nuc.lin[p >> 5].z >> (uint32_t)(p & 31);
            if (!z) {
                p = ((p >> 5) + 1) << 5;
                continue;
            }
            p += (uint64_t)__builtin_ctz(z);
            if (p >= n) break;
            if (xt_byte(tv, p) == (uint8_t)'\n') return p;
            ++p;
        }
        return n;
    }
    for (; p < n && (p & 15); ++p)
        if (tv.raw[p] == (uint8_t)'\n') return p;
    for (; p + 16 <= n; p += 16) {
        const uint4 v = *reinterpret_cast<const uint4*>(tv.raw + p);
        const uint32_t w[4] = {v.x ^ 0x0a0a0a0au, v.y ^ 0x0a0a0a0au, v.z ^ 0x0a0a0a0au, v.w ^ 0x0a0a0a0au};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t z = (w[q] - 0x01010101u) & ~w[q] & 0x80808080u;   // a zero byte = a '\n'
            if (z) return p + 4ull * q + (uint64_t)(__builtin_ctz(z) >> 3);
        }
    }
    for (; p < n; ++p)
        if (tv.raw[p] == (uint8_t)'\n') return p;
    return n;
}

// the walks' dynamic LDS: the plan's tables (when they fit, TAB_LDS_MAX) then
// TC_WIN bytes per thread
constexpr size_t TAB_LDS_MAX = 24 << 10;
__host__ __device__ inline size_t walk_tab_bytes(uint32_t tab_words) {
    return tab_words * 8ull <= TAB_LDS_MAX ? ((tab_words * 8ull + 15) & ~15ull) : 0;
}

// true when the pass changes anything for `flags` (cross: candidates may
// start on header lines)
bool report_needed(const pm_db* db, uint32_t flags, bool cross);
// report_enqueue_ws (below) enqueues the pass on s: h's keys/lens are
// replaced by the reported subset (the old buffers are recycled once the pass
// has read them).  The input count is *ws.total (device; the speculative
// sort's sum) or total_h.  The selected count is stored in ws.count and at
// host_count (mapped pinned, optional).  `done` (optional) is bound to the
// last kernel's dispatch.
// Synchronous form: enqueue on db->stream, read the count back, set h->count.
// hdr: candidates may start on a header line (the simple engine's cross
// windows) -- only then is every start checked against the header bytes.
struct EsPrep;
struct XtPrep;
void report_sync(pm_db* db, pm_hits* h, uint32_t flags, uint64_t total, bool hdr, const EsPrep* es = nullptr,
                 const XtPrep* xt = nullptr);
// Workspace of one pass (db's current lane), sized for `cap_items` keys;
// reserve it BEFORE enqueueing the producer of *total (reserve() may move it).
struct ReportWs {
    uint64_t* total = nullptr;   // input count written by the producer (speculative sort)
    uint32_t* count = nullptr;   // selected count
    uint64_t* bmax = nullptr;
    uint32_t* bcnt = nullptr;
    uint8_t* acc = nullptr;
    uint32_t* wlist = nullptr;   // esimple: the clusters to walk
    uint32_t* wcount = nullptr;
    uint64_t cap = 0;
};
ReportWs report_ws(pm_db* db, uint64_t cap_items);

// ---------------------------------------------------------------------------
// nrgrep's esimple engine (pm_esimple.hip): the report of a class sequence
// at k > 0 (PM_ESIMPLE) -- nrgrep's own candidate order and two-phase verify
// replayed per cluster of candidate starts
// ---------------------------------------------------------------------------
struct EsPlan {               // esimplePreproc 0x415540
    int type = 0;             // 1 pieces (BNDM), 2 backward window (ABNDM), 3 forward prefix (shift-or)
    int piece_len = 0;        // type 1
    int wbeg = 0, wend = 0;   // simpleFindBest's window (types 2, 3)
    int npieces = 0;          // k + 1 (type 1) or 1
    int L[PM_MAX_K + 1] = {}; // pattern positions left of each piece / window
};
// B: [256][W] position sets of the folded bytes (bit i = position i)
EsPlan es_plan(const uint64_t* B, int W, int m, int k);

struct EsSlot {               // one pattern of a report (device, uploaded as is)
    int32_t m, k, errs, type, mpc, wbeg, wend, W, np, anchors, pid, lone;
    int32_t L[PM_MAX_K + 1];
    uint64_t test[PM_MAX_K + 1];   // type 1: the piece test mask (0x41384b)
    uint64_t o_B, o_TL, o_TR;      // word offsets of B / TL[np] / TR[np] ([256][W] each) in the table blob
    uint64_t o_P;                  // type 1: word offset of the packed piece table [256]
    uint64_t pstart, pend;         // type 1: the pieces' first / last bits in the packed table
};
struct EsBuild {
    std::vector<EsSlot> slots;
    std::vector<uint64_t> tab;
};
struct EsUpload {
    size_t o_slots = 0, o_tab = 0, o_map = 0;
    uint32_t tab_words = 0;   // the compact tables ([codes][W] rows per table)
    int ncodes = 0;
    int nslots = 0;
    int32_t pid_base = 0;
    int wmax = 1;   // position words of the widest pattern
    int kmax = 1;   // the largest k
};
struct EsPrep {
    const EsSlot* slots = nullptr;
    const uint64_t* tab = nullptr;   // compact tables: [ncodes][W] rows (es_upload)
    const uint8_t* cmap = nullptr;   // byte -> code (code 0: '\n', a break)
    uint32_t tab_words = 0;
    int ncodes = 0;
    int nslots = 0;
    int32_t pid_base = 0;   // slot = pattern id - pid_base
    int32_t gap_max = 0;    // candidate starts further apart never interact
    int wmax = 1;           // position words of the widest pattern (1, 2 or 4)
    int kmax = 1;           // the largest k (rows of the verify automaton)
    uint32_t dl_off = 0;    // k_es_walk's piece words in its LDS
    int lines = 0;          // every position is a key (es_all_positions): clusters are lines
    uint32_t win = 0;       // k_es_walk's per-thread text ring (bytes, a power of two; 0: none)
    uint32_t tab_off = 0, map_off = 0;   // k_es_walk's LDS: the compact tables, the code map
    int tab_lds = 0;        // the tables are read from LDS
    uint32_t slots_off = 0; // k_es_walk's LDS copy of the slots (slots_lds)
    int slots_lds = 0;      // the slots are read from LDS
};
// Deletions with k >= m (the whole pattern may be deleted): every position
// can be reported, so the walk takes every position as a key and each line
// as a cluster (EsPrep::lines).  At most ES_ALL_MAX positions.
constexpr uint64_t ES_ALL_MAX = 1ull << 28;
pm_hits* es_all_positions(pm_db* db, int32_t pattern_id);
// slots get pattern ids pid, in increasing order
void es_add_slot(EsBuild& b, const uint64_t* B, int W, int m, int k, int errs, uint32_t flags, int32_t pid);
void es_upload(const EsBuild& b, Upload& up, EsUpload& u);
int32_t es_gap(const EsBuild& b);
EsPrep es_bind(const EsUpload& u, const uint8_t* d_up, int32_t gap_max);
// k_es_heads + k_es_walk + k_es_count on s: rewrites keys/lens in place and
// sets acc (bit 0 = reported) and the per-chunk counts bcnt (G chunks) for
// k_rep_scatter; wlist / wcount: the walk list (one entry per list item)
void es_launch(const EsPrep& P, uint64_t* keys, uint32_t* lens, const uint64_t* total_d, uint64_t total_h,
               uint8_t* acc, uint32_t* wlist, uint32_t* wcount, uint32_t* bcnt, uint32_t G, const TextView& tv,
               hipStream_t s);

// letterProb (.data 0x621120), 256 entries (pm_esimple.hip)
void letter_probs(double out[256]);

// ---------------------------------------------------------------------------
// nrgrep's extended engine at k = 0 (pm_extended.hip): the report of a class
// sequence with '?', '*', '+' (detClass() == 2, PM_EXTENDED) -- extendedFindBest's
// plan, the window / prefix scanners and checkMatch replayed per cluster of
// candidate starts
// ---------------------------------------------------------------------------
struct XtPlan {                // extendedPreproc 0x413260
    int type = 0;              // 2: a window scanned backward, 3: the prefix scanned forward
    int fwd = 0;               // extendedFindBest's count: the window's non-optional positions
    int beg = 0, end = 0;      // the window / prefix [beg, end)
    int L = 0;                 // pattern positions left of the candidate (beg, or end for type 3)
    int simple = 0;            // no '?*+' in [beg, end): simpleScan instead of extendedScan
};
// B: [256][W] position sets of the folded bytes; opt / rep: [W] masks
XtPlan xt_plan(const uint64_t* B, int W, int m, const uint64_t* opt, const uint64_t* rep);

struct XtSlot {                // one pattern (device, uploaded as is)
    int32_t m, type, fwd, len, simple, L, anchors, pid;
    int32_t plen[2], pw[2];    // verify parts: [0] left (reversed), [1] right; positions, words
    int64_t max_len;           // the longest match, -1: unbounded
    uint64_t fI, fF, fS;       // scanner: optional-block masks (extendedLoadFast)
    uint64_t vI[2][4], vF[2][4], vS[2][4], vX[2][4];
    uint64_t o_T, o_TA, o_vB[2], o_vA[2];   // word offsets of [256] / [256][pw] tables in the blob
};
// nrgrep's extended engine with errors (eextended, k > 0): the plan of
// eextendedPreproc 0x40fe30 and one verify part of checkMatch1 0x40e340
struct EePlan {
    int type = 0;              // 1: k + 1 pieces, 2: a window backward, 3: the prefix forward
    int simple = 0;            // no '?*+' in the scanned positions: esimpleScan's loops
    int np = 1;                // pieces (k + 1 for type 1)
    int plen = 0;              // the pieces' length in characters (type 1)
    int fwd = 0, wbeg = 0, wend = 0;   // extendedFindBest's window (K = k)
    int off[PM_MAX_K + 1] = {}, pend[PM_MAX_K + 1] = {};   // pieces [off, pend) / the window
    int L[PM_MAX_K + 1] = {};  // pattern positions left of each piece's candidate
};
double find_best_ext(const std::vector<double>& prob, const std::vector<double>& aprob, const uint64_t* opt, int m,
                     int K, int* fwd, int* beg, int* end);
EePlan ee_plan(const uint64_t* B, int W, int m, const uint64_t* opt, const uint64_t* rep, int k);

struct EePart {                // extendedLoadVerif 0x412c60: len positions, [256][pw] tables
    int32_t len, pw;
    uint64_t I[4], F[4], S[4], X[4];
    uint64_t o_B, o_A;
};
struct EeSlot {                // one pattern (device, uploaded as is)
    int32_t m, k, errs, type, simple, np, plen, flen, fspan, wbeg, wend, anchors, pid;
    int32_t lines;             // every position is a key, every line a cluster (es_all_positions): deletions
                               // reaching the shortest match, or a part over 64 positions with substitutions
    int64_t max_len;           // the longest alignment (insertions included), -1: unbounded or `lines`
    uint64_t fI, fF, fS;       // scanner: optional-block masks
    uint64_t top[PM_MAX_K + 1];   // type 1 (extended): each piece's top bit
    uint64_t o_T, o_TA, o_T2;  // [256] scanner tables in the blob
    EePart lv[PM_MAX_K + 1], rv[PM_MAX_K + 1];
};
// returns EeSlot::lines
bool ee_build(const uint64_t* B, int W, int m, const uint64_t* opt, const uint64_t* rep, int k, int errs,
              int64_t max_len, uint32_t flags, int32_t pid, bool all_lines, Upload& up, size_t& o_slot,
              size_t& o_tab);


// nrgrep's regular engine at k = 0 (pm_regular.hip): a pattern with '|' or a
// repeated group (detClass() == 3, PM_REGULAR) -- regularFindBest's plan
// over nrgrep's tree, regularScan and checkMatch replayed per cluster
constexpr int RG_NW = 5;       // words of a state set: positions + 1 <= 320
struct RgTree {                // Program.tree (regex.py): node i = type, left, right, position
    int nodes = 0;
    const int32_t* tree = nullptr;
    const int32_t* nullable = nullptr;
};
struct RgSlot {                // one pattern (device, uploaded as is)
    int32_t ms, nw, mp, type, ell, anchors, pid;   // states, words (1 / RG_NW), window states
    int64_t max_len;           // the longest text a match covers, -1: walk whole lines
    int64_t gap;               // consecutive starts further apart start a new cluster (-1: lines)
    uint64_t finit, ffinal;    // the window scanner's initial / final states
    uint64_t final_[RG_NW], vis[RG_NW];   // the automaton's final states; the states SLICE sees
    int32_t unmap[64];         // window state -> automaton state (P->0x860 / P->0x858), -1 none
    uint64_t o_arr, o_rev, o_B, o_Bw, o_A, o_fw, o_rw;   // word offsets in the table blob
    // eregular (k > 0, one word; pm_regular.hip): type 1 pieces, 2 backward
    // window, 3 forward; cls 1 (esimple's scanners) or 3 (eregularScan)
    int32_t k, errs, cls, nstates, lines;   // nstates: P->0x24; lines: clusters break at '\n' too
    uint64_t match0;           // class 1: checkMatch's state word P->0x28
    int32_t first[PM_MAX_K + 1];   // class 1: each window's first state
    uint64_t o_T0, o_T2;       // class 1: esimpleLoadFast's tables
};
// builds the plan and tables into `up`; false when nothing can be printed
// (k = 0: the window is a class / extended sequence, P->match is never set;
// k > 0: detClass 2, the binary dies)
bool rg_build(const RgTree& t, const uint64_t* B, int W, int npos, int64_t max_len, int k, int errs, uint32_t flags,
              int32_t pid, Upload& up, size_t& o_slot, size_t& o_tab);

struct XtPrep {
    const XtSlot* slot = nullptr;
    const RgSlot* rg = nullptr;   // the regular walk instead
    const EeSlot* ee = nullptr;   // k > 0: the eextended walk instead
    const uint64_t* tab = nullptr;
    int32_t pid = 0;
    int32_t words = 1;            // eextended: the verify parts' widest word count
    int32_t eregular = 0;         // rg: k > 0 (pm_regular.hip k_erg_walk)
    int32_t k = 0;                // errors (the walks' row count template argument)
    int32_t scanner = 0;          // xt / ee / eregular: xt_scanner / ee_scanner / erg_scanner of the slot (a template argument of the walk)
    uint32_t tab_words = 0;       // words of the table blob at tab (copied to LDS when small)
};
// eextended heads + walk on s (keys/lens rewritten in place, acc bit 0 =
// reported); xt_launch calls it when X.ee is set
// appends pid << 48 | each header line start to the sorted start list of h
// (total entries) and sorts it again; returns the new length
uint64_t ee_add_headers(pm_db* db, pm_hits* h, uint64_t total, int32_t pid);

// the eextended walk's scanner kind: 0..2 esimpleScan pieces / window /
// prefix, 3..5 eextendedScan pieces / window / prefix
int ee_scanner(const Upload& up, size_t o_slot);
// the extended walk's scanner kind (k = 0): 0 extendedScan window, 1
// simpleScan window, 2 simpleScan prefix, 3 extendedScan prefix
int xt_scanner(const Upload& up, size_t o_slot);
// the eregular walk's scanner kind: 0..1 esimpleScan pieces / window,
// 2 the pieces exactly, 3 bwdScanrk, 4 fwdScanrk
int erg_scanner(const Upload& up, size_t o_slot);
void ee_launch(const XtPrep& X, uint64_t* keys, uint32_t* lens, const uint64_t* total_d, uint64_t total_h,
               uint8_t* acc, const TextView& tv, int words, hipStream_t s);
// regular heads + walk on s (keys/lens rewritten in place, acc bit 0 =
// reported); xt_launch calls it when X.rg is set
void rg_launch(const XtPrep& X, uint64_t* keys, uint32_t* lens, const uint64_t* total_d, uint64_t total_h,
               uint8_t* acc, const TextView& tv, hipStream_t s);
// builds the plan and tables of one pattern into `up`; returns the slot's
// and the table blob's offsets
void xt_build(const uint64_t* B, int W, int m, const uint64_t* opt, const uint64_t* rep, int64_t max_len,
              uint32_t flags, int32_t pid, Upload& up, size_t& o_slot, size_t& o_tab);
// heads + walk + per-chunk counts on s (keys/lens rewritten in place, acc
// bit 0 = reported), like es_launch
void xt_launch(const XtPrep& X, uint64_t* keys, uint32_t* lens, const uint64_t* total_d, uint64_t total_h,
               uint8_t* acc, uint32_t* bcnt, uint32_t G, const TextView& tv, hipStream_t s);

// es (optional): the list holds a class sequence's candidate starts at
// k > 0 and the selection is nrgrep's esimple engine (pm_esimple.hip); xt
// (optional): an extended pattern's starts at k = 0 (pm_extended.hip)
void report_enqueue_ws(pm_db* db, pm_hits* h, uint32_t flags, const ReportWs& ws, bool total_on_device,
                       uint64_t total_h, uint32_t* host_count, hipStream_t s, hipEvent_t done, bool hdr,
                       const EsPrep* es = nullptr, const XtPrep* xt = nullptr);

}  // namespace pm
