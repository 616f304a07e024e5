// pm_ids.hip -- the web default `-k <k>ids` (insertions, deletions,
// substitutions; patmatch.py:299-314) for a class sequence on the nucleotide
// planes: the start-finding pass of the Glushkov kernels (k_nfa_rev, one
// text stream per lane, one character per step) restated bit-sliced over
// the 32 streams of a stream tile.
//
// The reverse automaton of a class sequence has shift transitions (position
// i + 1 -> i), so with one 32-bit register per (error row j, position i) --
// bit b = stream b -- a transition is a register renaming and a step over
// 32 characters (one logical word of every stream) is, per (j, i),
//     N[j][i] = (R[j][i+1] & M[c_i]) | R[j-1][i+1] | R[j-1][i] | N[j-1][i+1]
// (match, substitution, insertion, deletion), where M[c] = the class-match
// word of the word's 32 bases (one v_bitop3 of the hi/lo planes).  A start
// of a match is emitted where any row holds position 0 -- exactly the
// candidates k_nfa_rev emits; k_nfa_verify then finds each one's shortest
// end.  The kernel is generated per pattern (hipRTC): positions and rows are
// register names, the injected start configuration is folded into
// constants.  Line breaks (bo.x) zero every state, "other" bytes (N, IUPAC
// letters: bo.y) take their class membership from the byte's mask; both are
// handled in a second copy of the step taken only when a lane of the wave
// sees one.
//
// Lanes: one wave per tile, lane c owns the tile's stream column c (32
// logical words) and scans it right to left after a warm-up of L - 1 words
// (L = the longest match, m + k) read from the next column or the halo.
#include <map>
#include <sstream>
#include <tuple>

#include <hip/hip_ext.h>

#include "pm_internal.h"

namespace pm {
namespace {

constexpr int IDS_MAX_REGS = 64;   // m * (k + 1) state registers at most
// Words in flight per wave: a step's plane word is DMA'd into a per-wave LDS
// ring IDS_DEPTH steps before it is used (the step itself is ~100 dependent
// VALU ops, too short to cover an HBM miss, and the compiler's waits drained
// register prefetches right after issuing them)
constexpr int IDS_DEPTH = 4;

const char* kIdsCommon = R"IDS(
typedef unsigned int u32;
typedef unsigned long long u64;
typedef unsigned char u8;
#define STREAM 2048u
#define TILE_POS 65536ull
#define TILE_WORDS 2112ull
#define B3(a, b, c, t) ((u32)__builtin_amdgcn_bitop3_b32((a), (b), (c), (t)))
struct IArgs {
    const uint2* hl;
    const uint2* bo;
    const u32* sbflag;
    const u32* sbbase;
    const u8* xbytes;
    const u64* lflag;
    const u64* bmask;      // [256] positions accepting each folded byte
    u64 ntiles, n;
    u64* sink_out;
    u32* sink_cnt;
    u32 sink_cap, bins_per_pattern, pos_shift, pattern_id;
};
__device__ inline u64 phys(u64 tile, u32 w) {
    return tile * TILE_WORDS + (w < STREAM ? (u64)((w & 31u) * 64u + (w >> 5)) : (u64)w);
}
// LDS-DMA of one plane word per lane: the hi plane's dword lands at
// lds + 4 lane, the lo plane's at lds + 256 + 4 lane (no VGPR destination;
// waited for with vmcnt).  Inline asm, so that the compiler's own wait
// bookkeeping does not drain the loads in flight.
#if IDS_M0_CLOBBER
// m0 declared clobbered: the compiler keeps nothing in it across the DMA
// (no save / restore around each of a step's four DMAs)
__device__ __forceinline__ void dma_dword(u64 ga, u32 lds) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" : : "v"(ga), "s"(lds) : "memory", "m0");
}
#else
__device__ __forceinline__ void dma_dword(u64 ga, u32 lds) {
    u32 keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(ga), "s"(lds) : "memory");
}
#endif
// a step's word of both planes: {hi, lo} at lds, lds + 256 and the
// exception plane's {brk, oth} at lds + 512, lds + 768 (4 lane-linear dwords).
// A row with no break or "other" byte in any lane (`ex` false, wave-uniform)
// never reads its exception slots: they get the plane word again, a hit on
// the line just fetched, so the exception plane costs HBM bytes only for
// flagged rows while every step still issues 4 DMAs (the vmcnt waits count
// them).
// The planes' {hi, lo} may come from another address (ph, the lane-0 word
// every lane loads when only lane 0 needs it) and land elsewhere (lhl, a
// keep slot: same {hi, lo} offsets) than the exception dwords (lex).
__device__ __forceinline__ void dma_word(const uint2* ph, const uint2* p, long dbo, u32 lhl, u32 lex, bool ex) {
    const u64 ga = (u64)ph, ge = ex ? (u64)(p + dbo) : ga;
    dma_dword(ga, lhl);
    dma_dword(ga + 4ull, lhl + 256u);
    dma_dword(ge, lex);
    dma_dword(ge + 4ull, lex + 256u);
}
__device__ inline void push(const IArgs& a, u64 pos) {
    const u32 bin = (u32)(pos >> a.pos_shift);
    const u32 o = atomicAdd(&a.sink_cnt[bin], 1u);
    if (o < a.sink_cap) a.sink_out[(u64)bin * a.sink_cap + o] = ((u64)a.pattern_id << 48) | pos;
}
)IDS";

struct IArgsHost {   // must match IArgs in kIdsCommon
    const uint2* hl;
    const uint2* bo;
    const uint32_t* sbflag;
    const uint32_t* sbbase;
    const uint8_t* xbytes;
    const uint64_t* lflag;
    const uint64_t* bmask;
    uint64_t ntiles, n;
    uint64_t* sink_out;
    uint32_t* sink_cnt;
    uint32_t sink_cap, bins_per_pattern, pos_shift, pattern_id;
};

// ACGT subset of the class of position i (bit 0 = A .. bit 3 = T) and
// whether it takes every byte but '\n' ('.')
struct PosClass {
    int acgt;
    bool any;
};

PosClass pos_class_of(const uint64_t* bm, int i) {
    PosClass c{0, true};
    const char* acgt = "ACGT";
    for (int x = 0; x < 4; ++x)
        if ((bm[(uint8_t)acgt[x]] >> i) & 1) c.acgt |= 1 << x;
    for (int b = 0; b < 256; ++b)
        if (b != '\n' && !((bm[b] >> i) & 1)) c.any = false;
    return c;
}

// v_bitop3 truth table of "the base coded (hi, lo) is in subset s"
// (A=00 C=01 G=10 T=11), inputs (hi, lo, lo)
int subset_table(int s) {
    int t = 0;
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b)
            for (int c = 0; c < 2; ++c)
                if ((s >> (2 * a + b)) & 1) t |= 1 << (4 * a + 2 * b + c);
    return t;
}

// Logical words per lane column (WPL; the generator takes 32, 64 or 128:
// 2048 / WPL lanes per tile, WPL / 32 tiles per wave).  Longer columns pay
// the WU warm-up words once per WPL words instead of once per 32 (17 / 28 %
// fewer steps at the bench's WU = 16), but a step's 64 lanes then read words
// WPL / 32 apart, over 2 or 4 tiles: 2 or 4 times the cache lines per DMA,
// each fetched again WPL / 32 times.  Measured per strand on `-k 2ids`:
// 1.62 / 2.04 ms at 32 / 64 (kernel trace), the step 4.44 / 5.36 / 7.15 ms
// at 32 / 64 / 128 (round 4, tools/gpu_idsab.sh).
int ids_wpl(int) { return 32; }

// PM_IDS_KEEP=1: the warm-up words stay in LDS for the lane that owns them
// (WPL = 32: lane c's warm-up column is lane c + 1's own, read 32 steps
// later) instead of being read again from memory.  Measured slower and off
// by default: its 8 KB of LDS per wave leave 3 workgroups per CU instead of
// 4, and the kernel took 1.84 vs 1.58 ms per strand (-k 2ids 2,056 vs 2,262
// Gbases/s, profiles/r05k_ids_keep.txt).
bool ids_keep() {
    const char* e = getenv("PM_IDS_KEEP");
    return e && e[0] == '1';
}

// PM_IDS_BRKSPLIT=0 (A/B): a step whose words hold an exception masks every
// new state register with the break mask (45 more VALU ops at the bench's
// m = 15, k = 2) whether or not a line break is among them.  Default: that
// step tests the wave's break bits first and takes the masked update only
// when some lane's word holds a break (rare: N runs and IUPAC letters are
// the common exceptions; breaks come once per line)
// PM_IDS_M0=0 (A/B): each LDS-DMA saves and restores m0 around itself (the
// round-5 form); default: m0 is a declared clobber of the DMA's asm
bool ids_m0_clobber() {
    static const bool on = !(getenv("PM_IDS_M0") && getenv("PM_IDS_M0")[0] == '0');
    return on;
}

bool ids_brk_split() {
    static const bool on = !(getenv("PM_IDS_BRKSPLIT") && getenv("PM_IDS_BRKSPLIT")[0] == '0');
    return on;
}

// The kernel's source and its cache signature (everything the source
// depends on); with want_source false only the signature (a query's cache
// lookup: generating the source cost ~0.1 ms per query).
std::string gen_ids_source(const IdsSpec& sp, std::string* sig, bool want_source = true) {
    const int m = sp.m, k = sp.k;
    const bool SUB = sp.errs & PM_ERR_SUB, INS = sp.errs & PM_ERR_INS, DEL = sp.errs & PM_ERR_DEL;
    const int L = m + (INS ? k : 0);   // the longest match
    const int WU = L - 1;              // warm-up words
    std::vector<PosClass> pc(m);
    std::map<std::tuple<int, bool, bool>, int> cls;   // distinct classes (ACGT subset, any, takes N) -> register
    std::vector<int> rep;                       // a position of each class
    std::vector<int> ci(m);
    for (int i = 0; i < m; ++i) {
        pc[i] = pos_class_of(sp.byte_mask, i);
        auto key = std::make_tuple(pc[i].any ? 15 : pc[i].acgt, pc[i].any,
                                   !pc[i].any && ((sp.byte_mask[(uint8_t)'N'] >> i) & 1));
        auto it = cls.find(key);
        if (it == cls.end()) {
            it = cls.emplace(key, (int)rep.size()).first;
            rep.push_back(i);
        }
        ci[i] = it->second;
    }
    std::ostringstream sg;
    const int WPL = ids_wpl(WU);
    const bool keep = sp.keep && WPL == 32 && WU >= 1;   // lane c's warm-up column is lane c + 1's
    const bool brk_split = ids_brk_split();
    const bool m0c = ids_m0_clobber();
    sg << "ids13:" << WPL << ":" << (keep ? 1 : 0) << ":" << (brk_split ? 1 : 0) << (m0c ? "c" : "s") << ":" << m << ":" << k << ":" << sp.errs << ":";
    for (int i = 0; i < m; ++i) {
        sg << (pc[i].any ? '.' : (char)('a' + pc[i].acgt));
        if (!pc[i].any && ((sp.byte_mask[(uint8_t)'N'] >> i) & 1)) sg << 'N';   // the class takes N
    }
    for (int j = 0; j <= k; ++j) sg << ":" << sp.rev_pre[j] << "," << sp.rev_ins[j];
    *sig = sg.str();
    if (!want_source) return std::string();

    // two register banks, r and s: a step reads one and writes the other,
    // and the loop body is two steps (r -> s, s -> r), so no state moves
    auto V = [](char bank, int j, int i) { return std::string(1, bank) + std::to_string(j) + "_" + std::to_string(i); };
    auto bit = [](uint64_t set, int i) { return (set >> i) & 1; };
    // one step over word t (`tv`): new state (bank dst) from the old (bank
    // src) and the class words; `kill` masks every register with nb (a
    // line break zeroes all states)
    auto update = [&](std::ostringstream& o, char src, char dst, bool kill, const std::string& ind) {
        for (int j = 0; j <= k; ++j)
            for (int i = 0; i < m; ++i) {
                // A(j, i) = R(j, i+1) | injected constant
                auto A = [&](int jj) -> std::string {
                    if (bit(sp.rev_pre[jj], i)) return "0xffffffffu";
                    return i + 1 < m ? V(src, jj, i + 1) : "0u";
                };
                // match term: A & M (or A, or M alone), then the error terms
                // ORed in; emitted as explicit v_bitop3 ((a & m) | x: 0xEA,
                // a | b | c: 0xFE) -- written as C the compiler picks
                // v_or3_b32 / v_and_or_b32, which issue ~1.5x slower on
                // gfx950 (profiles/r01c_valu_rates.txt)
                const std::string a = A(j);
                std::string ta, tm;   // the match term as (ta & tm), or ta alone (tm empty)
                if (a == "0xffffffffu") ta = pc[i].any ? "0xffffffffu" : "M" + std::to_string(ci[i]);
                else if (a == "0u") ta = "0u";
                else {
                    ta = a;
                    if (!pc[i].any) tm = "M" + std::to_string(ci[i]);
                }
                std::vector<std::string> rest;
                if (j > 0 && SUB) rest.push_back(A(j - 1));
                if (j > 0 && INS) rest.push_back(bit(sp.rev_ins[j - 1], i) ? "0xffffffffu" : V(src, j - 1, i));
                if (j > 0 && DEL) {
                    if (i + 1 < m) rest.push_back(V(dst, j - 1, i + 1));
                    if (j >= 2 && INS && i == m - 1) rest.push_back("0xffffffffu");
                }
                std::vector<std::string> terms;
                bool ones = ta == "0xffffffffu" && tm.empty();
                for (const std::string& x : rest) {
                    if (x == "0xffffffffu") ones = true;
                    else if (x != "0u") terms.push_back(x);
                }
                std::string e;
                if (ones) {
                    e = "0xffffffffu";
                } else {
                    size_t q = 0;
                    if (ta == "0u") e = "";
                    else if (tm.empty()) e = ta;
                    else if (!terms.empty()) e = "B3(" + ta + ", " + tm + ", " + terms[q++] + ", 0xEA)";
                    else e = "(" + ta + " & " + tm + ")";
                    for (; q < terms.size();) {
                        if (e.empty()) e = terms[q++];
                        else if (q + 1 < terms.size()) {
                            e = "B3(" + e + ", " + terms[q] + ", " + terms[q + 1] + ", 0xFE)";
                            q += 2;
                        } else e = "(" + e + " | " + terms[q++] + ")";
                    }
                    if (e.empty()) e = "0u";
                }
                o << ind << V(dst, j, i) << " = " << (kill ? "(" + e + ") & nb" : e) << ";\n";
            }
    };
    // one step over word t = `tv` of the lane's stream column, whose plane /
    // exception words are `vv` / `ev` and whose plane word is at pointer `pv`;
    // `emit`: t < 32 (the lane's own column) -- report starts
    // kept_phase: own words t < WU, which the lane to the left kept (keep)
    bool kept_phase = false;
    auto step = [&](std::ostringstream& o, char src, char dst, const std::string& tv, const std::string& vv,
                    const std::string& pv, bool emit) {
        const std::string in = "            ";
        (void)vv;
        o << in << "{\n";
        // this step's word landed (the DEPTH - 1 later steps' DMAs may
        // still be in flight), then the DMA DEPTH steps ahead goes into the
        // slot the previous step read
        o << in << "    asm volatile(\"s_waitcnt vmcnt(" << 4 * (IDS_DEPTH - 1) << ")\" ::: \"memory\");\n";
        // the word's planes: the ring slot, or (keep) the warm-up word's keep
        // slot / the kept own word of the lane to the left
        if (!keep)
            o << in << "    const u32* vs_ = ring + sl * 256u + col;\n";
        else if (!emit)
            o << in << "    const u32* vs_ = keep + ((u32)(" << tv << ") - WPL) * 128u + col;\n";
        else if (kept_phase)
            o << in << "    const u32* vs_ = col ? keep + (u32)(" << tv << ") * 128u + col - 1u : ring + sl * 256u;\n";
        else
            o << in << "    const u32* vs_ = ring + sl * 256u + col;\n";
        o << in << "    const uint2 v = make_uint2(vs_[0], vs_[64]);\n";
        o << in << "    issue(qs + IDS_DEPTH, snx);\n";
        if (emit)
            o << in << "    const uint2* " << pv << " = pm + (long)(((" << tv << ") & 31) * 64 + ((" << tv << ") >> 5));\n";
        else
            o << in << "    const u32 u_ = (u32)(" << tv << ") - WPL;\n"
              << in << "    const uint2* " << pv << " = pn + (long)((u_ & 31u) * s1 + (u_ >> 5) * s2);\n";
        o << in << "    const u32 sl_ = sl;\n";
        o << in << "    ++qs; sl = sl + 1u == IDS_SLOTS ? 0u : sl + 1u; snx = snx + 1u == IDS_SLOTS ? 0u : snx + 1u;\n";
        if (brk_split) o << in << "    bool killed_ = false;\n";
        for (size_t c = 0; c < rep.size(); ++c) {
            const PosClass& p = pc[rep[c]];
            if (p.any) o << in << "    u32 M" << c << " = 0xffffffffu;\n";
            else o << in << "    u32 M" << c << " = B3(v.x, v.y, v.y, " << subset_table(p.acgt) << ");\n";
        }
        // the step's exception flag (wave-uniform, from the group's masks):
        // only a step with a break or an "other" byte in some lane's word
        // reads the exception plane
        o << in << "    if (" << (emit ? "exo((u32)(" + tv + "))" : "exw(u_)") << ") {   // wave-uniform, rare\n";
        o << in << "        const uint2 e = make_uint2(ring[sl_ * 256u + 128u + col], ring[sl_ * 256u + 192u + col]);\n";
        o << in << "        const u32 nb = ~e.x;\n";
        // "other" bytes: an N (NUC_N_MARK: its hi bit) matches '.' only;
        // any other byte takes its own class membership from the side tables
        o << in << "        const u32 en = e.y & v.x, eo = e.y & ~v.x;\n";
        for (size_t c = 0; c < rep.size(); ++c) {
            const bool n_in = (sp.byte_mask[(uint8_t)'N'] >> rep[c]) & 1;   // the class takes N ('.', [ACGTN] ...)
            o << in << "        M" << c << (n_in ? " |= en;\n" : " &= ~en;\n");
        }
        o << in << "        if (eo) {\n";
        o << in << "            const u64 pw = (u64)(" << pv << " - a.hl);\n";
        o << in << "            const u32 f = a.sbflag[pw >> 5];\n";
        o << in << "            const u32 xi = a.sbbase[pw >> 5] + __popc(f & ((1u << (u32)(pw & 31)) - 1u));\n";
        o << in << "            for (u32 ob = eo; ob; ob &= ob - 1) {\n";
        o << in << "                const u32 b = __builtin_ctz(ob);\n";
        o << in << "                const u64 mk = a.bmask[a.xbytes[(u64)xi * 32 + b]];\n";
        for (size_t c = 0; c < rep.size(); ++c)
            o << in << "                M" << c << " = ((mk >> " << rep[c] << ") & 1ull) ? (M" << c << " | (1u << b)) : (M"
              << c << " & ~(1u << b));\n";
        o << in << "            }\n";
        o << in << "        }\n";
        if (brk_split) {
            // only a break kills: without one in any lane's word the
            // exception step takes the plain update below with the adjusted
            // classes (one copy of each update, as without the split)
            o << in << "        if (__builtin_amdgcn_ballot_w64(e.x != 0u)) {   // wave-uniform: a line break\n";
            update(o, src, dst, true, in + "            ");
            o << in << "            killed_ = true;\n";
            o << in << "        }\n";
            o << in << "    }\n";
            o << in << "    if (!killed_) {\n";
            update(o, src, dst, false, in + "        ");
            o << in << "    }\n";
        } else {   // (the round-5 form)
            update(o, src, dst, true, in + "        ");
            o << in << "    } else {\n";
            update(o, src, dst, false, in + "        ");
            o << in << "    }\n";
        }
        if (emit) {
            o << in << "    u32 em = 0u";
            for (int j = 0; j <= k; ++j) o << " | " << V(dst, j, 0);
            o << ";\n";
            o << in << "    for (; em; em &= em - 1) {\n";
            o << in << "        const u64 pos = posb + (u64)__builtin_ctz(em) * STREAM + (u32)(" << tv << ");\n";
            o << in << "        if (pos < a.n) push(a, pos);\n";
            o << in << "    }\n";
        }
        o << in << "}\n";
    };

    std::ostringstream o;
    o << "#define IDS_M0_CLOBBER " << (m0c ? 1 : 0) << "\n";
    o << kIdsCommon;
    o << "#define WU " << WU << "\n";
    // keep: the warm-up words' planes stay in LDS for the lane that owns
    // them (ids_keep_ok); 4 workgroups per CU without it (<= 128 VGPRs, 4
    // waves per SIMD; staging each tile in LDS by LDS-DMA first measured no
    // faster, round 2), as many as the keep slots leave LDS for with it
    const int per_wg = 4 * ((IDS_DEPTH + 1) * 1024 + (keep ? WU * 512 : 0));
    const int wg = keep ? std::max(1, std::min(4, (160 << 10) / per_wg)) : 4;
    o << "#define IDS_KEEP " << (keep ? 1 : 0) << "\n#define IDS_KEEP_WORDS " << (keep ? WU : 1) << "\n";
    o << "#define IDS_WG " << wg << "\n#define IDS_DEPTH " << IDS_DEPTH << "\n#define IDS_SLOTS " << IDS_DEPTH + 1 << "\n";
    o << "#define WPL " << WPL << "u\n#define TPW " << WPL / 32 << "u\n#define LPT " << 2048 / WPL << "u\n";
    o << "#define STRIDE_MASK " << (WPL == 32 ? "0xffffffffffffffffull" : WPL == 64 ? "0x5555555555555555ull"
                                                                                      : "0x1111111111111111ull") << "\n";
    o << R"IDS(
// One wave per TPW tiles; lane c scans column cc = c % LPT of tile c / LPT:
// logical words WPL cc .. WPL cc + WPL - 1 of its 32 streams (word t of the
// column: physical row t & 31, column TPW cc + (t >> 5)).  It first scans
// the next column's first WU words (the tile's halo for the last column)
// right to left as warm-up, then its own WPL words, reporting starts: WU +
// WPL steps per WPL words (at WPL = 32 the warm-up was a third of the
// steps).  The exception plane is read only at steps where some lane's word
// has a break or an "other" byte: the group's sbflag rows are folded into a
// wave-uniform mask over t once per group (bit t: own word t; warm-up word u
// adds the halo's bit u).
extern "C" __global__ __launch_bounds__(256, IDS_WG) void pm_ids_rev(IArgs a) {   // IDS_WG workgroups per CU
    __shared__ __attribute__((aligned(16))) u32 ids_ring[4][IDS_SLOTS * 256];   // per wave: {hi, lo, brk, oth} x 64 lanes per slot
    // per wave (IDS_KEEP): the warm-up words' {hi, lo} x 64 lanes, slot u =
    // warm-up word u -- lane c's warm-up word u is lane c + 1's own word u,
    // which lane c + 1 reads here 32 steps later instead of from memory
    __shared__ __attribute__((aligned(16))) u32 ids_keep[4][IDS_KEEP_WORDS * 128];
    const u32 col = threadIdx.x & 63;
    const u32 wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    u32* const ring = ids_ring[wid];
    const u32 rbase = __builtin_amdgcn_readfirstlane((u32)reinterpret_cast<u64>(ring));   // its LDS byte address
    u32* const keep = ids_keep[wid];
    const u32 kbase = __builtin_amdgcn_readfirstlane((u32)reinterpret_cast<u64>(keep));
    const u64 wave = (u64)blockIdx.x * 4u + wid, nwaves = gridDim.x * 4ull;
    const long dbo = a.bo - a.hl;   // the exception plane has the planes' layout
    const u64 ngroups = (a.ntiles + TPW - 1) / TPW;
    const u32 cc = col % LPT;
    const bool last_col = cc == LPT - 1u;
    const u32 s1 = last_col ? 1u : 64u, s2 = last_col ? 32u : 1u;   // warm-up word u: (u & 31) s1 + (u >> 5) s2
    for (u64 tg = wave; tg < ngroups; tg += nwaves) {
        // (WPL > 32) lanes of a tile past the end scan the last tile again
        // and report nothing (their positions are >= n)
        const u64 tile = tg * TPW + col / LPT;
        const uint2* tb = a.hl + (tile < a.ntiles ? tile : a.ntiles - 1) * TILE_WORDS;
        const uint2* pm = tb + TPW * cc;                                  // own words
        const uint2* pn = last_col ? tb + STREAM : tb + TPW * (cc + 1);   // warm-up words
        const u64 posb = tile * TILE_POS + (u64)WPL * cc;
        // the group's exception masks: lane r < 32 folds row r of every
        // tile into TPW bits (bit g: a flagged word in column group g)
        u32 fold = 0;
        u64 hm = 0;
        for (u32 tau = 0; tau < TPW; ++tau) {
            const u64 tt = tg * TPW + tau < a.ntiles ? tg * TPW + tau : a.ntiles - 1;
            const u64 base = tt * TILE_WORDS;   // a multiple of 32: rows are sbflag word pairs
            if (col < 32u) {
                const u32* sf = a.sbflag + (base >> 5) + 2u * col;
                const u64 rf = (u64)sf[0] | ((u64)sf[1] << 32);
                for (u32 g = 0; g < TPW; ++g) fold |= (u32)((rf & (STRIDE_MASK << g)) != 0ull) << g;
            }
            const u32* hf = a.sbflag + ((base + STREAM) >> 5);
            hm |= (u64)hf[0] | ((u64)hf[1] << 32);   // halo words 2048 .. 2111
        }
        u64 mlo = 0, mhi = 0;
        for (u32 g = 0; g < TPW; ++g) {
            const u64 bl = __ballot((fold >> g) & 1u) & 0xffffffffull;
            if (g < 2u) mlo |= bl << (32u * g);
            else mhi |= bl << (32u * (g - 2u));
        }
        auto exo = [&](u32 t) { return (((t < 64u ? mlo : mhi) >> (t & 63u)) & 1ull) != 0ull; };
        auto exw = [&](u32 u) { return ((((mlo | hm) >> u) & 1ull)) != 0ull; };
        // step q (0 .. WU + WPL - 1) reads word t = WPL - 1 + WU - q (warm-up
        // word u = t - WPL while q < WU); its DMA goes IDS_DEPTH steps ahead
        auto issue = [&](int q, u32 slot) {
            const int t2 = (int)WPL - 1 + WU - q;
            const bool w2 = q < WU, o2 = !w2 && q < WU + (int)WPL;
            const u32 u2 = (u32)(t2 - (int)WPL);
            const bool ex2 = w2 ? exw(u2) : (o2 && exo((u32)t2));
            const uint2* g2 = w2 ? pn + (long)((u2 & 31u) * s1 + (u2 >> 5) * s2)
                                 : o2 ? pm + (long)((t2 & 31) * 64 + (t2 >> 5)) : tb;
            const u32 lr = rbase + slot * 1024u;
            if (IDS_KEEP && w2) {            // a warm-up word: its planes into keep slot u2
                dma_word(g2, g2, dbo, kbase + u2 * 512u, lr + 512u, ex2);
            } else if (IDS_KEEP && o2 && t2 < WU) {
                // an own word the lane to the left kept: only lane 0 (whose
                // word nobody kept) needs the planes, the others load lane
                // 0's word (one line)
                const uint2* g0 = tb + (long)((t2 & 31) * 64 + (t2 >> 5));
                dma_word(col ? g0 : g2, g2, dbo, lr, lr + 512u, ex2);
            } else {
                dma_word(g2, g2, dbo, lr, lr + 512u, ex2);
            }
        };
        // the first IDS_DEPTH words go in flight now (the previous group's
        // DMAs have all landed: the slots are free)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int qs = 0;
        u32 sl = 0, snx = IDS_DEPTH;
        for (int q = 0; q < IDS_DEPTH; ++q) issue(q, (u32)q);
)IDS";
    for (int j = 0; j <= k; ++j)
        for (int i = 0; i < m; ++i) o << "        u32 " << V('r', j, i) << " = 0, " << V('s', j, i) << " = 0;\n";
    // a phase: `n` steps from t = `t0` down, pointer form `own`; pairs of
    // steps alternate the register banks (each step's word comes from the
    // LDS ring)
    char b0 = 'r', b1 = 's';
    auto phase = [&](int t0, int n, bool own) {
        int t = t0;
        if (n % 2) {   // a single step first
            o << "        {\n";
            step(o, b0, b1, std::to_string(t), "", "p0", own);
            o << "        }\n";
            std::swap(b0, b1);
            --t;
            --n;
        }
        if (!n) return;
        const std::string ind = "            ";
        const int last = t - n + 1;
        o << "        for (int t = " << t << "; t >= " << last + 1 << "; t -= 2) {\n";
        step(o, b0, b1, "t", "", "p0", own);
        step(o, b1, b0, "t - 1", "", "p1", own);
        o << "        }\n";
    };
    phase(WPL - 1 + WU, WU, false);   // warm-up: t = WPL + WU - 1 .. WPL
    if (keep) {                       // own column: t = WPL - 1 .. WU, then the kept words WU - 1 .. 0
        phase(WPL - 1, WPL - WU, true);
        kept_phase = true;
        phase(WU - 1, WU, true);
    } else {
        phase(WPL - 1, WPL, true);    // own column: t = WPL - 1 .. 0
    }
    // the last tile's look-ahead DMAs land before the wave ends (its LDS is
    // released with the workgroup)
    o << "    }\n    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n}\n";
    return o.str();
}

struct IdsKernel {
    hipModule_t module = nullptr;
    hipFunction_t fn = nullptr;
};
std::mutex g_ids_mu;
std::map<std::pair<int, std::string>, IdsKernel> g_ids_cache;

}  // namespace

bool ids_rev_scan(pm_db* db, const IdsSpec& sp, const Sink& sink, hipStream_t s, hipEvent_t ev_a, hipEvent_t ev_b) {
    if (db->alphabet != PM_ALPHA_NUC || sp.m * (sp.k + 1) > IDS_MAX_REGS || sp.m > 64) return false;
    const int WU = sp.m + ((sp.errs & PM_ERR_INS) ? sp.k : 0) - 1;
    if (WU > std::min(HALO - 1, ids_wpl(WU))) return false;   // the warm-up must fit the next lane column or the halo
    IdsSpec spk = sp;
    spk.keep = ids_keep();
    std::string sig;
    gen_ids_source(spk, &sig, false);
    hipFunction_t fn;
    {
        std::lock_guard<std::mutex> lk(g_ids_mu);
        auto key = std::make_pair(db->device, sig);
        auto it = g_ids_cache.find(key);
        if (it == g_ids_cache.end()) {
            std::vector<char> code = hiprtc_compile(gen_ids_source(spk, &sig));
            IdsKernel kk;
            HIPCHK(hipModuleLoadData(&kk.module, code.data()));
            HIPCHK(hipModuleGetFunction(&kk.fn, kk.module, "pm_ids_rev"));
            it = g_ids_cache.emplace(key, kk).first;
        }
        fn = it->second.fn;
    }
    const NucView nv = nuc_view(db);
    IArgsHost a{nv.hl, nv.bo, nv.sbflag, nv.sbbase, nv.xbytes, db->lflag, sp.d_bmask, db->ntiles, db->n,
                sink.out, sink.bin_cnt, sink.cap, sink.bins_per_pattern, sink.pos_shift, (uint32_t)sp.pattern_id};
    void* params[] = {&a};
    // one wave per group of TPW tiles, waves loop over groups (every wave
    // reaches the end);
    // four rounds of the resident waves (the kernel needs 120 VGPRs: 4 per
    // SIMD): later rounds' workgroups start wherever earlier ones finish,
    // which evens out CUs that run slower (per strand: one round 1.80 ms,
    // two 1.71, four 1.68; r03z, r03i2, r03i4)
    int ncu = 0, per_cu = 0;
    HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, db->device));
    HIPCHK(hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, 0));
    const uint64_t resident = (uint64_t)std::max(ncu, 1) * (uint64_t)std::max(per_cu, 1) * 4;
    const uint64_t tpw = (uint64_t)ids_wpl(WU) / 32, ngroups = (db->ntiles + tpw - 1) / tpw;
    const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((ngroups + 3) / 4, resident));
    HIPCHK(hipExtModuleLaunchKernel(fn, blocks * 256u, 1, 1, 256, 1, 1, 0, s, params, nullptr, ev_a, ev_b, 0));
    return true;
}

}  // namespace pm

using namespace pm;

extern "C" int pm_ids_jit_compile(int m, const uint64_t* byte_mask, int k, int errs, uint64_t* code_bytes) {
    return guarded([&] {
        require(byte_mask != nullptr && code_bytes != nullptr, "null argument");
        require(m >= 1 && m <= 64 && k >= 0 && k <= PM_MAX_K && m * (k + 1) <= IDS_MAX_REGS,
                "shape not covered by the bit-sliced kernel", PM_E_UNSUPPORTED);
        require((errs & ~(PM_ERR_INS | PM_ERR_DEL | PM_ERR_SUB)) == 0, "bad error-type mask");
        // the start configuration of a plain class sequence, as scan_nfa builds it
        IdsSpec sp{m, k, errs, byte_mask, nullptr, {}, {}, 0};
        sp.keep = ids_keep();
        const uint64_t last = 1ull << (m - 1);
        uint64_t S = 0;
        for (int j = 0; j <= k; ++j) {
            sp.rev_ins[j] = S;
            sp.rev_pre[j] = (S >> 1) | ((j == 0 || (errs & PM_ERR_INS)) ? last : 0);
            if (errs & PM_ERR_DEL) S = (S >> 1) | ((j == 0 || (errs & PM_ERR_INS)) ? last : 0);
            else S = 0;
        }
        std::string sig;
        *code_bytes = hiprtc_compile(gen_ids_source(sp, &sig)).size();
    });
}
