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
#include <map>
#include <mutex>
#include <sstream>

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
                        kill |= e.x;
                    }
                    if (a.class_any[cls]) continue;
                    const uint2 v = a.nuc.hl[pw];
                    uint32_t x = subset_mismatch(a.class_acgt[cls], v.x, v.y);
                    if (e.y) {
                        const uint32_t idx = exception_index(a.nuc.sbflag, a.nuc.sbbase, pw);
                        uint32_t o = e.y;
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
                    if (pos < a.n) {
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
        default: hipLaunchKernelGGL(k_linear_generic<4>, dim3(blocks), dim3(256), 0, s, a); break;
    }
}

// Windows of a specialized scan that overlap an "other" byte (N, IUPAC
// letter, ...) and no break, evaluated exactly.  One thread per flagged word;
// a window is owned by the first "other" position it contains, so each is
// evaluated once.  (The fast path drops every window that overlaps any
// exception; windows with a break are dead.)
struct OthersArgs {
    NucView nuc;
    const uint32_t* xoth;
    const uint64_t* xword;
    uint64_t nflag, n;
    const uint8_t* pos_class;
    const int32_t* lengths;
    const uint8_t* class_any;
    const uint32_t* class_bytes;
    int P, k, pattern_base;
    uint64_t* out;       // the specialized kernel's (pattern, workgroup) segments
    uint32_t* seg_cnt;
    uint32_t cap, nwg, tiles_per_wg;
};

__global__ __launch_bounds__(256) void k_linear_others(OthersArgs a) {
    const uint64_t idx = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (idx >= a.nflag) return;
    uint32_t ot = a.xoth[idx];
    if (!ot) return;
    const uint64_t w = a.xword[idx];
    const uint64_t tile = w / TILE_WORDS;
    const uint32_t lw = logical_word((uint32_t)(w % TILE_WORDS));
    if (lw >= STREAM) return;   // halo copy of a main word
    while (ot) {
        const uint32_t b = __builtin_ctz(ot);
        ot &= ot - 1;
        const uint64_t e = pos_of(tile, lw, b);
        if (e >= a.n) continue;
        for (int p = 0; p < a.P; ++p) {
            const int len = a.lengths[p];
            for (int d = 0; d < len && (uint64_t)d <= e; ++d) {
                const uint64_t s = e - d;
                int mm = 0;
                bool ok = true;
                for (int j = 0; j < len && ok; ++j) {
                    const uint8_t ch = nuc_char_at(a.nuc, s + j);
                    if (ch == '\n') { ok = false; break; }
                    const bool other = !(ch == 'A' || ch == 'C' || ch == 'G' || ch == 'T');
                    if (other && s + j < e) { ok = false; break; }   // owned by an earlier other
                    const int c = a.pos_class[p * 64 + j];
                    if (a.class_any[c]) continue;
                    if (!((a.class_bytes[c * 8 + (ch >> 5)] >> (ch & 31)) & 1) && ++mm > a.k) ok = false;
                }
                if (ok) {
                    const uint32_t slot = (uint32_t)(a.pattern_base + p);
                    const uint64_t seg = (uint64_t)slot * a.nwg + (s / TILE_POS) / a.tiles_per_wg;
                    const uint32_t o = atomicAdd(&a.seg_cnt[seg], 1u);
                    if (o < a.cap) a.out[seg * a.cap + o] = ((uint64_t)slot << 48) | s;
                }
            }
        }
    }
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
struct JArgs {
    const uint2 *hl, *bo;
    const u64* lflag;
    const u8* pos_class;    // [P][64]
    const u8* class_any;    // [nc]
    const u8* class_acgt;   // [nc]
    u64 ntiles, n;
    u64* out;               // [slot][nwg][cap] hit keys, one segment per (pattern, workgroup)
    u32* seg_cnt;           // [slot][nwg]
    u64* dummy;             // [nwg] sink of the always-issued flush stores
    u32 cap, nwg, tiles_per_wg;
    int pattern_base;
};
#define STREAM 2048u
#define TILE_POS 65536ull
#define TILE_WORDS 2112ull
#define B3(a, b, c, t) ((u32)__builtin_amdgcn_bitop3_b32((a), (b), (c), (t)))
__device__ __forceinline__ u64 phys_word(u64 tile, u32 w) {
    return tile * TILE_WORDS + (w < STREAM ? (u64)((w & 31u) * 64u + (w >> 5)) : (u64)w);
}
// Hit output (rare path, out of line: inlined, even never-executed emission
// code perturbs the allocation and schedule of the 16-step fast path).  A
// slot of the (pattern, workgroup) segment is reserved with an LDS atomic
// (lgkmcnt; a returning global atomic would be waited for on vmcnt, which
// retires in order and would drain the tile prefetch in flight).  Workgroups
// own contiguous tile ranges, so each segment is a position range.
typedef __attribute__((address_space(3))) u32 lds_u32;
typedef __attribute__((address_space(3))) const uint2 lds_uint2;
struct HitStage {
    u32 cnt[4];      // per pattern: next slot of this workgroup's segment
};
// the kernel arguments the rare path needs, passed by value (no struct copy
// to scratch)
typedef __attribute__((address_space(1))) const uint2 glb_uint2;
typedef __attribute__((address_space(1))) u64 glb_u64;
struct RareArgs {
    glb_uint2* bo;   // global address space: flat accesses would also count in lgkmcnt
    glb_u64* out;
    u32 cap, nwg;
    int pattern_base;
};
__device__ __forceinline__ void emit(const RareArgs& a, lds_u32* cnt, int p, u64 pos) {
    const u32 slot = (u32)(a.pattern_base + p);
    const u32 o = __atomic_fetch_add(cnt + p, 1u, __ATOMIC_RELAXED);
    if (o < a.cap) a.out[((u64)slot * a.nwg + blockIdx.x) * a.cap + o] = ((u64)slot << 48) | pos;
}
)JIT";

struct JitKernel {
    hipModule_t module = nullptr;
    hipFunction_t fn = nullptr;
};

std::mutex g_jit_mu;
std::map<std::pair<int, std::string>, JitKernel> g_jit_cache;

struct JArgsHost {           // must match JArgs in kJitCommon
    const uint2 *hl, *bo;
    const uint64_t* lflag;
    const uint8_t* pos_class;
    const uint8_t* class_any;
    const uint8_t* class_acgt;
    uint64_t ntiles, n;
    uint64_t* out;
    uint32_t* seg_cnt;
    uint64_t* dummy;
    uint32_t cap, nwg, tiles_per_wg;
    int pattern_base;
};

// mismatch of an ACGT subset as an expression of the plane words h, l
std::string subset_expr(int subset, const std::string& h, const std::string& l) {
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

// Emits a bit-sliced "count > K" network over `in` (mismatch words) and
// returns the name of the result.  Columns of equal weight are compressed
// with full adders (xor3 + majority, one v_bitop3 each); carries whose
// weight exceeds K go straight into the dead mask, the few bits left are
// compared with K at the end.  ~1.6 ops per input for K = 2.
std::string emit_dead_network(std::ostringstream& o, const std::vector<std::string>& in, int K, int& uid,
                              const std::string& ind) {
    auto fresh = [&](const char* pfx) { return std::string(pfx) + std::to_string(uid++); };
    if (in.empty()) return "0u";
    if (K == 0) {
        std::string acc = in[0];
        size_t i = 1;
        for (; i + 1 < in.size(); i += 2) {
            const std::string v = fresh("d");
            o << ind << "const u32 " << v << " = " << acc << " | " << in[i] << " | " << in[i + 1] << ";\n";
            acc = v;
        }
        if (i < in.size()) {
            const std::string v = fresh("d");
            o << ind << "const u32 " << v << " = " << acc << " | " << in[i] << ";\n";
            acc = v;
        }
        return acc;
    }
    const int lmax = K >= 2 ? 1 : 0;   // highest column whose weight is <= K
    std::deque<std::string> col[3];
    col[0].assign(in.begin(), in.end());
    // compress every column to at most 2 bits with full adders; carries of
    // weight > K go straight into the dead mask
    for (int L = 0; L <= lmax; ++L) {
        auto& c = col[L];
        while (c.size() > 2) {
            const std::string a = c.front(); c.pop_front();
            const std::string b = c.front(); c.pop_front();
            const std::string d = c.front(); c.pop_front();
            const std::string s = fresh("s"), cy = fresh("c");
            o << ind << "const u32 " << s << " = B3(" << a << ", " << b << ", " << d << ", 0x96);\n";
            o << ind << "const u32 " << cy << " = B3(" << a << ", " << b << ", " << d << ", 0xE8);\n";
            c.push_back(s);
            col[L + 1].push_back(cy);
        }
    }
    std::vector<std::string> terms(col[lmax + 1].begin(), col[lmax + 1].end());
    // what is left: a, b (weight 1) and, for K >= 2, c, d (weight 2)
    auto at = [&](int L, size_t i) { return i < col[L].size() ? col[L][i] : std::string("0u"); };
    if (K == 1) {
        if (col[0].size() == 2) terms.push_back("(" + at(0, 0) + " & " + at(0, 1) + ")");
    } else if (!col[1].empty()) {
        // count = a + b + 2 (c + d) (+ 4 per dead carry):
        //   K = 2: dead iff c & d, or (c | d) & (a | b)  = maj(c, d, a | b)
        //   K = 3: dead iff c & d, or (c | d) & a & b    = maj(c, d, a & b)
        const std::string ab = col[0].size() < 2 ? at(0, 0)
                               : "(" + at(0, 0) + (K == 2 ? " | " : " & ") + at(0, 1) + ")";
        if (K == 3 && col[0].size() < 2) terms.push_back("(" + at(1, 0) + " & " + at(1, 1) + ")");
        else terms.push_back("B3(" + at(1, 0) + ", " + at(1, 1) + ", " + ab + ", 0xE8)");
    }
    if (terms.empty()) return "0u";
    std::string acc = terms[0];
    size_t i = 1;
    for (; i + 1 < terms.size(); i += 2) {
        const std::string v = fresh("d");
        o << ind << "const u32 " << v << " = " << acc << " | " << terms[i] << " | " << terms[i + 1] << ";\n";
        acc = v;
    }
    if (i < terms.size()) {
        const std::string v = fresh("d");
        o << ind << "const u32 " << v << " = " << acc << " | " << terms[i] << ";\n";
        acc = v;
    }
    return acc;
}

#define PROF_TAIL                                                                              \
    "#ifdef PM_PROF\n  if (lane == 0) { u64* pr = a.dummy + (u64)gridDim.x + (blockIdx.x * 4 + wid) * 3;\n" \
    "    pr[0] = c_wait; pr[1] = c_bar; pr[2] = c_rest; }\n#endif\n"

// Source of the specialized kernel for a batch of P <= 4 patterns.
//
// Workgroup = 4 waves = one tile at a time: wave w scans pattern w % P over
// the step range part w / P (4 / P parts of the tile's 32 steps).  Tiles
// arrive in a 3-deep LDS ring by global_load_lds_dwordx4 (LDS-DMA, no
// VGPRs, 1 KiB per wave-instruction): while the workgroup computes tile i
// the DMAs of tiles i+1 and i+2 are in flight (~104 KB per CU at 3
// workgroups/CU), so HBM latency is off the critical path and every tile is
// read from HBM once however many waves scan it.  Per wave, lane l walks its
// window words t; the class words X_c(w) of the wave's pattern live in a
// register ring from first to last use and each step is a straight-line
// Wallace tree.  The steps are one basic block (no branch): hits are rare,
// so the fast path only records which steps had a live window (hs) and the
// XOR of the live masks (acc); the rare path emits them.
std::string gen_linear_source(int P, int K, const int32_t* lengths, const uint8_t* pos_class,
                              const uint8_t* class_acgt, const uint8_t* class_is_any) {
    const int PARTS = 4 / P;                   // step ranges per pattern
    const int STEPS = LANE_WORDS / PARTS;      // steps per wave
    int RING = 3;                              // LDS tile buffers
    if (const char* e = getenv("PM_JIT_RING")) RING = atoi(e);   // experiment: 2 or 3
    const int TILE_BYTES = (int)(TILE_WORDS * 8);         // 16896: 16.5 KiB
    const int DMA_PIECES = (TILE_BYTES + 1023) / 1024;   // 1 KiB per glds wave-instruction (last one half)
    const int LDS_TILE = TILE_BYTES;
    std::ostringstream o;
    o << kJitCommon;
    o << "#define P " << P << "\n#define K " << K << "\n";
    auto word_off = [&](int i) {   // physical word of logical word 32 lane + i, relative to the tile
        std::ostringstream s;
        if (i < LANE_WORDS) s << (i * 64) << " + lane";
        else if (i < 2 * LANE_WORDS) s << "hb1 + " << (i - 32) << " * hs1";
        else s << "hb2 + " << (i - 64) << " * hs2";
        return s.str();
    };
    int max_est = 0;
    for (int p = 0; p < P; ++p) {
        const int L = lengths[p];
        const uint8_t* pc = pos_class + 64 * p;
        std::vector<int> used;
        std::map<int, int> slot;
        std::map<int, std::pair<int, int>> span;
        for (int j = 0; j < L; ++j) {
            if (class_is_any[pc[j]]) continue;
            if (!slot.count(pc[j])) { slot[pc[j]] = (int)used.size(); used.push_back(pc[j]); span[pc[j]] = {j, j}; }
            span[pc[j]].second = j;
        }
        int ring = 0;
        for (auto& kv : span) ring += kv.second.second - kv.second.first + 1;
        max_est = std::max(max_est, ring + 2 * L + 32);
        // --- rare path: emit the live windows of step t (exception-free ones
        // for a lane that sees exceptions; k_linear_others owns the rest)
        o << "__device__ __forceinline__ void emit_hits" << p
          << "(const RareArgs& a, lds_u32* cnt, u64 tile, u32 lane, u32 t, u64 lf, u32 lv) {\n"
             "  const u32 w0 = 32u * lane + t;\n"
             "  if ((lf >> lane) & 1) {\n    glb_uint2* bo = a.bo + tile * TILE_WORDS;\n    u32 ex = 0;\n"
             "#pragma unroll\n    for (int j = 0; j < " << L << "; ++j) {\n"
             "      const u32 w = w0 + j;\n      const uint2 v = bo[w < STREAM ? (w & 31u) * 64u + (w >> 5) : w];\n"
             "      ex |= v.x | v.y;\n    }\n    lv &= ~ex;\n  }\n"
             "  for (u32 h = lv; h; h &= h - 1) emit(a, cnt, " << p
          << ", tile * TILE_POS + (u64)__builtin_ctz(h) * STREAM + w0);\n}\n";
        // --- rare path: re-evaluate step t (several live steps in a lane)
        o << "__device__ __forceinline__ void recompute_step" << p
          << "(const RareArgs& a, lds_u32* cnt, lds_uint2* hl, u64 tile, u32 lane, u32 t, u64 lf) {\n"
             "  const u32 w0 = 32u * lane + t;\n"
             "  uint2 v[" << L << "];\n#pragma unroll\n  for (int j = 0; j < " << L << "; ++j) {\n"
             "    const u32 w = w0 + j;\n    v[j] = hl[w < STREAM ? (w & 31u) * 64u + (w >> 5) : w];\n  }\n";
        {
            int ruid = 0;
            std::vector<std::string> in;
            for (int j = 0; j < L; ++j) {
                if (class_is_any[pc[j]]) continue;
                const std::string nm = "r" + std::to_string(ruid++);
                o << "  const u32 " << nm << " = "
                  << subset_expr(class_acgt[pc[j]], "v[" + std::to_string(j) + "].x", "v[" + std::to_string(j) + "].y")
                  << ";\n";
                in.push_back(nm);
            }
            const std::string d = emit_dead_network(o, in, K, ruid, "  ");
            o << "  emit_hits" << p << "(a, cnt, tile, lane, t, lf, ~" << d << ");\n}\n";
        }
        o << "__device__ __noinline__ void rare" << p << "(u32 hs, u32 acc, u64 tile, u32 lane, u64 lf, u32 sw_addr, "
             "u32 cnt_addr, const uint2* bo, u64* out, u32 cap, u32 nwg, int pattern_base) {\n"
             "  const RareArgs a{(glb_uint2*)bo, (glb_u64*)out, cap, nwg, pattern_base};\n"
             "  lds_u32* cnt = (lds_u32*)(size_t)cnt_addr;\n  lds_uint2* sw = (lds_uint2*)(size_t)sw_addr;\n"
             "  if ((hs & (hs - 1)) == 0) emit_hits" << p << "(a, cnt, tile, lane, __builtin_ctz(hs), lf, acc);\n"
             "  else for (u32 h = hs; h; h &= h - 1) recompute_step" << p << "(a, cnt, sw, tile, lane, __builtin_ctz(h), lf);\n}\n";
        // --- fast path over steps [t0, t1) of one tile, words from LDS
        for (int part = 0; part < PARTS; ++part) {
            const int t0 = part * STEPS, t1 = t0 + STEPS;
            const int wend = t1 + L - 1;   // words [t0, wend)
            o << "__device__ __forceinline__ void tile_body" << p << "_" << part
              << "(const JArgs& a, u32 sw_addr, u32 cnt_addr, const uint2* __restrict__ sw, u64 tile, int lane, u32 hb1, "
                 "u32 hs1, u32 hb2, u32 hs2, u64 lf) {\n  u32 hs = 0, acc = 0;\n";
            std::vector<bool> loaded(wend, false);
            std::vector<std::vector<bool>> done(wend, std::vector<bool>(used.size(), false));
            auto ensure_class = [&](int i, int u) {
                if (!loaded[i]) {
                    loaded[i] = true;
                    o << "  const uint2 v" << i << " = sw[" << word_off(i) << "];\n";
                }
                if (done[i][u]) return;
                done[i][u] = true;
                o << "  const u32 x" << u << "_" << i << " = "
                  << subset_expr(class_acgt[used[u]], "v" + std::to_string(i) + ".x", "v" + std::to_string(i) + ".y")
                  << ";\n";
            };
            int uid = 0;
            for (int t = t0; t < t1; ++t) {
                std::vector<std::string> in;
                for (int j = 0; j < L; ++j) {
                    if (class_is_any[pc[j]]) continue;
                    ensure_class(t + j, slot[pc[j]]);
                    in.push_back("x" + std::to_string(slot[pc[j]]) + "_" + std::to_string(t + j));
                }
                o << "  {  // step " << t << "\n";
                const std::string d = emit_dead_network(o, in, K, uid, "    ");
                o << "    hs |= min(~" << d << ", 1u) << " << t << ";\n    acc ^= ~" << d << ";\n  }\n";
            }
            if (getenv("PM_JIT_EMIT") && getenv("PM_JIT_EMIT")[0] == '0')   // experiment: no emission
                o << "  if (hs == 0x12345678u && acc == 0x9abcdef0u) a.seg_cnt[0] = 1;\n  hs = 0;\n";
            if (getenv("PM_JIT_EMIT") && getenv("PM_JIT_EMIT")[0] == '2')   // experiment: code present, never taken
                o << "  if (hs == 0x12345678u && acc == 0x9abcdef0u) a.seg_cnt[1] = 1;\n  if (lf != 0x1234567812345678ull) hs = 0;\n";
            o << "  if (hs) rare" << p << "(hs, acc, tile, lane, lf, sw_addr, cnt_addr, a.bo, a.out, a.cap, a.nwg, "
                 "a.pattern_base);\n}\n";
        }
    }
    // Occupancy target from the widest body's register ring; LDS allows 3
    // workgroups (12 waves) per CU.
    int waves = 1;
    while (waves < 3 && 512 / (waves + 1) >= max_est * 5 / 4) ++waves;
    if (const char* e = getenv("PM_JIT_WAVES")) waves = atoi(e);   // experiment override
    o << "#define RING " << RING << "\n#define LDS_TILE " << LDS_TILE << "\n#define DMA_PIECES " << DMA_PIECES << "\n";
    // experiment knobs: PM_JIT_NODMA=1 computes on whatever is in LDS (no
    // staging), PM_JIT_NOCOMPUTE=1 only streams the tiles
    const bool nodma = getenv("PM_JIT_NODMA") && getenv("PM_JIT_NODMA")[0] == '1';
    const bool nocompute = getenv("PM_JIT_NOCOMPUTE") && getenv("PM_JIT_NOCOMPUTE")[0] == '1';
    if (nodma) o << "#define PM_NODMA 1\n";
    o << R"JIT(// Raw barrier: __syncthreads()'s release fence would wait vmcnt(0) for the
// hit stores and with them drain the tile prefetch in flight.  LDS writes
// (hit counters, register-staged tiles) are complete at lgkmcnt(0); the
// empty asm statements keep the compiler from moving memory accesses across.
#define BARRIER()                                                   \
  do {                                                              \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");              \
    __builtin_amdgcn_s_barrier();                                   \
    asm volatile("" ::: "memory");                                  \
  } while (0)
// DMA tile t into the ring slot at LDS byte address `dst0`: DMA_PIECES 1-KiB
// pieces, piece q issued by wave q % 4 (lane-linear LDS image of the tile).
// Inline asm so that the compiler's wait bookkeeping does not drain it
// before the ds_reads of the slot being computed; waited for explicitly.
__device__ __forceinline__ void stage(const JArgs& a, u32 dst0, u64 tile, u64 tend, u32 wid, int lane) {
#ifdef PM_NODMA
  return;
#endif
  if (tile >= tend) return;
  const unsigned char* src = reinterpret_cast<const unsigned char*>(a.hl + tile * TILE_WORDS) + lane * 16;
#pragma unroll
  for (int q = 0; q < DMA_PIECES; q += 4) {
    if (q + (int)wid >= DMA_PIECES) break;
    if ((q + (int)wid + 1) * 1024 > LDS_TILE && lane * 16 >= LDS_TILE % 1024) continue;   // half last piece
    const u32 dst = __builtin_amdgcn_readfirstlane(dst0 + (q + wid) * 1024);
    u32 keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src + (q + wid) * 1024), "s"(dst) : "memory");
  }
}
)JIT";
    // PM_JIT_PROF=1: per-wave s_memtime totals (wait / barrier / rest of the
    // iteration) into the dummy buffer, for tools/jit_sweep.py
    const bool prof = getenv("PM_JIT_PROF") && getenv("PM_JIT_PROF")[0] == '1';
    if (prof) o << "#define PM_PROF 1\n";
    o << R"JIT(#ifdef PM_PROF
#define PT(v) const u64 v = __builtin_amdgcn_s_memtime()
#else
#define PT(v)
#endif
)JIT";
    o << "extern \"C\" __global__ __launch_bounds__(256, " << waves << ") void pm_linear_jit(JArgs a) {\n"
         "  __shared__ __attribute__((aligned(1024))) unsigned char lds[RING * LDS_TILE];\n"
         "  __shared__ HitStage hsg;\n"
         "  const int lane = threadIdx.x & 63;\n"
         "  const u32 wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n"
         "  const u32 pat = wid % " << P << ", part = wid / " << P << ";\n"
         "  if (threadIdx.x < 4) hsg.cnt[threadIdx.x] = 0;\n"
         "  // pieces this wave DMAs per tile (its share of DMA_PIECES)\n"
         "  const u32 mine = (DMA_PIECES - wid + 3) / 4;\n"
         "  // halo word offsets (logical words 32 lane + 32 g + r, r < 32)\n"
         "  const u32 hb1 = lane + 1 < 64 ? lane + 1 : 32u * lane + 32u, hs1 = lane + 1 < 64 ? 64u : 1u;\n"
         "  const u32 hb2 = lane + 2 < 64 ? lane + 2 : 32u * lane + 64u, hs2 = lane + 2 < 64 ? 64u : 1u;\n"
         "  const u32 lds_base = (u32)reinterpret_cast<u64>(lds);   // LDS byte address (low bits of the flat address)\n"
         "  // this workgroup's contiguous tile range\n"
         "  const u64 t0 = (u64)blockIdx.x * a.tiles_per_wg;\n"
         "  const u64 tend = t0 + a.tiles_per_wg < a.ntiles ? t0 + a.tiles_per_wg : a.ntiles;\n"
         "  stage(a, lds_base, t0, tend, wid, lane);\n"
         "  stage(a, lds_base + LDS_TILE, t0 + 1, tend, wid, lane);\n"
         "  u32 slot = 0;\n"
         "  const u32 cnt_addr = (u32)reinterpret_cast<u64>(&hsg.cnt[0]);\n"
         "#ifdef PM_PROF\n  u64 c_wait = 0, c_bar = 0, c_rest = 0;\n#endif\n"
         "  for (u64 tile = t0; tile < tend; ++tile) {\n"
         "    PT(ta);\n"
         "    // wait for this tile's pieces (own DMAs; the next tile's stay in\n"
         "    // flight: vmcnt retires in order), then the barrier makes everyone's\n"
         "    // pieces visible and frees the previous tile's slot\n"
         "    if (tile + 1 < tend) {\n"
         "      if (mine == 5) asm volatile(\"s_waitcnt vmcnt(5)\" ::: \"memory\");\n"
         "      else asm volatile(\"s_waitcnt vmcnt(4)\" ::: \"memory\");\n"
         "    } else {\n"
         "      asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n"
         "    }\n"
         "    PT(tb);\n"
         "    BARRIER();\n"
         "    PT(tc);\n"
         "    stage(a, lds_base + (slot == 0 ? RING - 1 : slot - 1) * LDS_TILE, tile + RING - 1, tend, wid, lane);\n"
         "    u64 lf;   // scalar load (lgkmcnt): a vector load's vmcnt wait would drain the DMAs\n"
         "    asm volatile(\"s_load_dwordx2 %0, %1, 0x0\\n\\ts_waitcnt lgkmcnt(0)\" : \"=s\"(lf) : \"s\"(a.lflag + tile) : \"memory\");\n"
         "    const uint2* sw = reinterpret_cast<const uint2*>(lds + slot * LDS_TILE);\n";
    bool first = true;
    if (nocompute) o << "    if (lf == 0x123456789ull) a.seg_cnt[0] = sw[lane].x;\n";
    for (int p = 0; p < P && !nocompute; ++p)
        for (int part = 0; part < PARTS; ++part) {
            o << "    " << (first ? "" : "else ") << "if (pat == " << p << " && part == " << part << ") tile_body" << p
              << "_" << part << "(a, (u32)reinterpret_cast<u64>(sw), cnt_addr, sw, tile, lane, hb1, hs1, hb2, hs2, lf);\n";
            first = false;
        }
    o << "#ifdef PM_PROF\n    { PT(td); c_wait += tb - ta; c_bar += tc - tb; c_rest += td - tc; }\n#endif\n";
    o << "    slot = slot == RING - 1 ? 0 : slot + 1;\n  }\n"
         "  BARRIER();\n"
         "  if (threadIdx.x < " << P << ") a.seg_cnt[(u64)(a.pattern_base + threadIdx.x) * a.nwg + blockIdx.x] = "
         "hsg.cnt[threadIdx.x];\n"
         PROF_TAIL "}\n";
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
    for (const char* knob : {"PM_JIT_WAVES", "PM_JIT_RING", "PM_JIT_EMIT", "PM_JIT_NODMA", "PM_JIT_NOCOMPUTE",
                             "PM_JIT_PROF"})
        if (const char* e = getenv(knob)) sig += std::string(";") + knob + "=" + e;
    return sig;
}

hipFunction_t jit_function(int device, int P, int K, const int32_t* lengths, const uint8_t* pos_class,
                           const uint8_t* class_acgt, const uint8_t* class_is_any) {
    const auto key = std::make_pair(device, jit_signature(P, K, lengths, pos_class, class_acgt, class_is_any));
    std::lock_guard<std::mutex> lk(g_jit_mu);
    auto it = g_jit_cache.find(key);
    if (it != g_jit_cache.end()) return it->second.fn;
    std::vector<char> code = jit_compile(gen_linear_source(P, K, lengths, pos_class, class_acgt, class_is_any));
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

}  // namespace
}  // namespace pm

using namespace pm;

extern "C" {

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
        const bool jit = use_jit(db);

        Upload up;
        const size_t o_cb = up.add(class_bytes, (size_t)n_classes * 32);
        const size_t o_len = up.add(lengths, (size_t)n_patterns * 4);
        const size_t o_pc = up.add(pos_class, (size_t)n_patterns * 64);
        const size_t o_acgt = up.add(class_acgt, (size_t)n_classes);
        const size_t o_any = up.add(class_is_any, (size_t)n_classes);
        struct Chunk { int base, P; hipFunction_t jit; };
        std::vector<Chunk> chunks;
        for (int base = 0; base < n_patterns;) {
            const int rem = n_patterns - base;
            const int P = rem >= 4 ? 4 : (rem >= 2 ? 2 : 1);   // instantiated widths
            hipFunction_t fn = nullptr;
            if (jit)
                fn = jit_function(db->device, P, k, lengths + base, pos_class + 64 * base, class_acgt, class_is_any);
            chunks.push_back({base, P, fn});
            base += P;
        }
        uint8_t* d_up = up.commit(db);

        SinkBuffers sb;
        std::vector<uint32_t> counts;
        uint64_t total = 0;
        EventPair ev;
        bool done = false;
        if (jit) {
            // one output segment per (pattern, workgroup); workgroups own
            // contiguous tile ranges (3 per CU resident)
            uint64_t nwg = std::min<uint64_t>(db->ntiles, 256 * 3);
            const uint64_t tpw = (db->ntiles + nwg - 1) / nwg;
            nwg = (db->ntiles + tpw - 1) / tpw;
            uint32_t cap = 1024;
            while (cap > 256 && (uint64_t)n_patterns * nwg * cap * 8 > (1ull << 30)) cap /= 2;
            const uint64_t dummy_words = nwg + nwg * 4 * 3;   // flush sink + PM_JIT_PROF counters
            uint64_t* dummy = static_cast<uint64_t*>(reserve(db, db->ws_post, dummy_words * sizeof(uint64_t)));
            if (getenv("PM_JIT_PROF")) HIPCHK(hipMemsetAsync(dummy, 0, dummy_words * sizeof(uint64_t), s));
            for (int attempt = 0; attempt < 2 && !done; ++attempt) {
                sb = make_sink_segments(db, n_patterns, (uint32_t)nwg, cap);
                HIPCHK(hipEventRecord(ev.a, s));
                for (const Chunk& ch : chunks) {
                    JArgsHost ja{db->hl, db->bo, db->lflag, d_up + o_pc + 64 * ch.base, d_up + o_any, d_up + o_acgt,
                                 db->ntiles, db->n, sb.out, sb.cnt, dummy, sb.cap, (uint32_t)nwg, (uint32_t)tpw, ch.base};
                    void* params[] = {&ja};
                    HIPCHK(hipModuleLaunchKernel(ch.jit, (uint32_t)nwg, 1, 1, 256, 1, 1, 0, s, params, nullptr));
                    if (db->nflag) {
                        OthersArgs oa{nuc_view(db), db->xoth, db->xword, db->nflag, db->n,
                                      d_up + o_pc + 64 * ch.base, reinterpret_cast<const int32_t*>(d_up + o_len) + ch.base,
                                      d_up + o_any, reinterpret_cast<const uint32_t*>(d_up + o_cb), ch.P, k, ch.base,
                                      sb.out, sb.cnt, sb.cap, (uint32_t)nwg, (uint32_t)tpw};
                        hipLaunchKernelGGL(k_linear_others, dim3(blocks_for(db->nflag, 256)), dim3(256), 0, s, oa);
                        HIPCHK(hipGetLastError());
                    }
                }
                HIPCHK(hipEventRecord(ev.b, s));
                bool overflow = false;
                total = sink_total(db, sb, counts, overflow);
                if (getenv("PM_JIT_PROF") && getenv("PM_JIT_PROF")[0] == '1') {
                    std::vector<uint64_t> pr(nwg * 4 * 3);
                    HIPCHK(hipMemcpy(pr.data(), dummy + nwg, pr.size() * 8, hipMemcpyDeviceToHost));
                    double w[4][3] = {};
                    for (uint64_t b = 0; b < nwg; ++b)
                        for (int wv = 0; wv < 4; ++wv)
                            for (int c = 0; c < 3; ++c) w[wv][c] += (double)pr[(b * 4 + wv) * 3 + c] / nwg;
                    for (int wv = 0; wv < 4; ++wv)
                        fprintf(stderr, "PM_JIT_PROF wave %d: wait %.0f  barrier %.0f  rest %.0f cycles/workgroup\n", wv,
                                w[wv][0], w[wv][1], w[wv][2]);
                }
                if (!overflow) { done = true; break; }
                const uint32_t maxc = *std::max_element(counts.begin(), counts.end());
                if (maxc > LDS_SORT_CAP) break;   // pathological hit density: generic kernels below
                while (cap < maxc) cap *= 2;
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
        const double kms = ev.ms();
        pm_hits* h = sink_to_hits(db, sb, counts, total);
        h->kernel_ms = kms;
        if (total) {
            hipLaunchKernelGGL(k_linear_lens, dim3(blocks_for(total, 256)), dim3(256), 0, s, h->keys, total,
                               reinterpret_cast<const int32_t*>(d_up + o_len), h->lens);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipStreamSynchronize(s));
        hits_ready(db, h);
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
        for (int p = 0; p < n_patterns; ++p)
            require(lengths[p] >= 1 && lengths[p] <= PM_MAX_POSITIONS, "pattern length out of range");
        const std::string src = gen_linear_source(n_patterns, k, lengths, pos_class, class_acgt, class_is_any);
        const std::vector<char> code = jit_compile(src);
        if (code_bytes) *code_bytes = code.size();
    });
}

}  // extern "C"
