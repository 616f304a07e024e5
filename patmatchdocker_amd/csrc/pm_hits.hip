// pm_hits.hip -- hit collection: bins -> one sorted (pattern, beg) list, and
// the pm_hits_* entry points.
//
// The reference reads hits as nrgrep_coords' "[beg, end]: match" lines, one
// run per pattern/strand, each in increasing beg order (parsed at
// www/FlaskApp/FlaskApp/patmatch.py:505-531).  Here every scan kernel pushes
// 64-bit keys (pattern << 48 | beg) into bins that partition (pattern,
// position) space in increasing order; each bin is sorted in LDS by one
// workgroup and written at its exclusive offset, which yields the same
// order as the reference's concatenated runs without a global sort.  Bins
// too large for LDS (a dense pattern of a big batch) are gathered and radix
// sorted by themselves, then copied to their offsets.
#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_merge.hpp>

#include <map>
#include <mutex>

#include "pm_internal.h"

namespace pm {
namespace {

struct BinShape {
    const uint64_t* slot_base;
    const uint32_t* slot_cap;
    uint32_t bins_per_slot;
    __device__ uint32_t cap(uint32_t bin) const { return slot_cap[bin / bins_per_slot]; }
    __device__ const uint64_t* src(const uint64_t* out, uint32_t bin) const {
        const uint32_t sl = bin / bins_per_slot;
        return out + slot_base[sl] + (uint64_t)(bin % bins_per_slot) * slot_cap[sl];
    }
};

// One workgroup per bin: bitonic sort in LDS, write at the bin's offset.
// CAP keys per bin at most (2048: 16 KB of LDS; 4096 when a bin may hold
// more, 32 KB); larger bins are left to the caller.
// One bin, sorted by the whole block (uniform control flow: c is the same
// for every thread).
template <uint32_t CAP>
__device__ __forceinline__ void sort_one_bin(uint64_t* s, uint32_t bin, const uint64_t* __restrict__ out,
                                             const uint32_t* __restrict__ cnt, const uint64_t* __restrict__ off,
                                             const BinShape& sh, uint64_t* __restrict__ dst,
                                             const int32_t* __restrict__ slot_len, uint32_t* __restrict__ lens) {
    const uint32_t c = min(cnt[bin], sh.cap(bin));
    if (c == 0 || c > CAP) return;   // (a speculative sort's caller redoes such lists)
    uint64_t base;
    if (off) {
        base = off[bin];
    } else {   // few bins: the block sums the counts before it (no offsets pass)
        uint64_t acc = 0;
        for (uint32_t b = threadIdx.x; b < bin; b += blockDim.x) acc += min(cnt[b], sh.cap(b));
        for (int d2 = 32; d2 > 0; d2 >>= 1) acc += __shfl_xor(acc, d2, 64);   // wave sum
        if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
        __syncthreads();
        base = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; ++w) base += s[w];
        __syncthreads();
    }
    const uint64_t* src = sh.src(out, bin);
    uint64_t* d = dst + base;
    if (slot_len) {   // every key of a bin has its slot's fixed length
        const uint32_t len = (uint32_t)slot_len[bin / sh.bins_per_slot];
        for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) lens[base + i] = len;
    }
    if (c == 1) {
        if (threadIdx.x == 0) d[0] = src[0];
        return;
    }
    if (c <= blockDim.x) {
        // small bin (the common case: ~100 keys): rank sort -- every thread
        // counts the keys before its own (LDS broadcast reads, ties broken by
        // index) and stores its key at that rank; one barrier instead of the
        // bitonic network's log^2 rounds
        const uint32_t i = threadIdx.x;
        uint64_t mine = 0;
        if (i < c) s[i] = mine = src[i];
        __syncthreads();
        if (i < c) {
            uint32_t r = 0;
            for (uint32_t j = 0; j < c; ++j) {
                const uint64_t v = s[j];
                r += (v < mine) | ((v == mine) & (j < i));
            }
            d[r] = mine;
        }
        return;
    }
    uint32_t n2 = 2;
    while (n2 < c) n2 <<= 1;
    for (uint32_t i = threadIdx.x; i < n2; i += blockDim.x) s[i] = i < c ? src[i] : ~0ull;
    __syncthreads();
    for (uint32_t k = 2; k <= n2; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < n2; i += blockDim.x) {
                const uint32_t ix = i ^ j;
                if (ix > i) {
                    const uint64_t a = s[i], b = s[ix];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) { s[i] = b; s[ix] = a; }
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) d[i] = s[i];
}

// One workgroup per bin at a time (item it -> bin it, or bin_list[it]; the
// grid strides over nitems): bitonic sort in LDS, write at the bin's offset.
// CAP keys per bin at most (2048: 16 KB of LDS; 4096 when a bin may hold
// more, 32 KB; 16384 for the large-bin pass, 128 KB); larger bins are left
// to the caller.
template <uint32_t CAP, int THREADS = 256>
__global__ __launch_bounds__(THREADS) void k_sort_bins(const uint64_t* __restrict__ out, const uint32_t* __restrict__ cnt,
                                                       const uint64_t* __restrict__ off, BinShape sh,
                                                       uint64_t* __restrict__ dst, const int32_t* __restrict__ slot_len,
                                                       uint32_t* __restrict__ lens, uint32_t* counts_host,
                                                       uint32_t nbins, uint64_t* total_out,
                                                       const uint32_t* __restrict__ bin_list, uint32_t nitems) {
    __shared__ uint64_t s[CAP];
    if (counts_host && blockIdx.x == 0) {   // the pipelined scan's count readback (mapped host memory)
        for (uint32_t i = threadIdx.x; i <= nbins; i += blockDim.x) counts_host[i] = cnt[i];
        __threadfence_system();
    }
    if (total_out && blockIdx.x == 0) {     // list length for the report pass (device-side count)
        uint64_t acc = 0;
        for (uint32_t b = threadIdx.x; b < nbins; b += blockDim.x) acc += min(cnt[b], sh.cap(b));
        for (int d2 = 32; d2 > 0; d2 >>= 1) acc += __shfl_xor(acc, d2, 64);
        __shared__ uint64_t wsum[THREADS / 64];
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = acc;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t t = 0;
            for (int w = 0; w < THREADS / 64; ++w) t += wsum[w];
            *total_out = t;
            // the report workspace's walk-list counter follows the total
            // (report_ws): zeroed here, no memset before the report pass
            *reinterpret_cast<uint32_t*>(total_out + 1) = 0u;
        }
    }
    for (uint32_t it = blockIdx.x; it < nitems; it += gridDim.x) {
        sort_one_bin<CAP>(s, bin_list ? bin_list[it] : it, out, cnt, off, sh, dst, slot_len, lens);
        __syncthreads();   // s is reused by the next bin
    }
}

// Bins of up to T * IPT keys from a list (one bin per block at a time): a
// bin holds one pattern slot and a position range, so its keys sort as the
// 32-bit offsets from its smallest position -- a block radix sort over the
// range's significant bits (4096 keys: ~4 passes of an LDS rank, where the
// bitonic network took 78 barrier rounds).  A range of 2^32 positions or
// more (no sink makes one) takes a rank sort over the bin in memory.
template <int T, int IPT>
__global__ __launch_bounds__(T) void k_radix_bins(const uint64_t* __restrict__ out, const uint32_t* __restrict__ cnt,
                                                  const uint64_t* __restrict__ off, BinShape sh,
                                                  uint64_t* __restrict__ dst, const int32_t* __restrict__ slot_len,
                                                  uint32_t* __restrict__ lens, const uint32_t* __restrict__ bin_list,
                                                  uint32_t nitems) {
    using Sort = hipcub::BlockRadixSort<uint32_t, T, IPT>;
    __shared__ typename Sort::TempStorage ts;
    __shared__ uint64_t red_lo[T / 64], red_hi[T / 64];
    constexpr uint64_t PM = (1ull << 48) - 1;
    for (uint32_t it = blockIdx.x; it < nitems; it += gridDim.x) {
        const uint32_t bin = bin_list[it];
        const uint32_t c = min(cnt[bin], sh.cap(bin));
        const uint64_t* src = sh.src(out, bin);
        const uint64_t base = off[bin];
        uint64_t k[IPT];
        uint64_t lo = ~0ull, hi = 0;
#pragma unroll
        for (int j = 0; j < IPT; ++j) {   // striped: a wave's loads are contiguous
            const uint32_t q = (uint32_t)j * T + threadIdx.x;
            k[j] = q < c ? src[q] : 0ull;
            if (q < c) {
                lo = umin64(lo, k[j] & PM);
                hi = umax64(hi, k[j] & PM);
            }
        }
        for (int d = 32; d > 0; d >>= 1) {
            const uint64_t ol = ((uint64_t)__shfl_xor((uint32_t)(lo >> 32), d, 64) << 32) | __shfl_xor((uint32_t)lo, d, 64);
            const uint64_t oh = ((uint64_t)__shfl_xor((uint32_t)(hi >> 32), d, 64) << 32) | __shfl_xor((uint32_t)hi, d, 64);
            lo = umin64(lo, ol);
            hi = umax64(hi, oh);
        }
        if ((threadIdx.x & 63) == 0) {
            red_lo[threadIdx.x >> 6] = lo;
            red_hi[threadIdx.x >> 6] = hi;
        }
        __syncthreads();
        lo = ~0ull;
        hi = 0;
        for (int w = 0; w < T / 64; ++w) {
            lo = umin64(lo, red_lo[w]);
            hi = umax64(hi, red_hi[w]);
        }
        const uint64_t tag = src[0] & ~PM;   // the bin's pattern slot
        const uint32_t len = slot_len ? (uint32_t)slot_len[bin / sh.bins_per_slot] : 0u;
        if (hi - lo < 0xFFFFFFFFull) {
            // offsets from lo; the padding (hi - lo + 1) sorts after every key
            const uint32_t pad = (uint32_t)(hi - lo + 1);
            const int bits = 32 - __builtin_clz(pad);
            uint32_t v[IPT];
            // blocked input (thread t: items t * IPT + j); any order will do
#pragma unroll
            for (int j = 0; j < IPT; ++j) v[j] = (uint32_t)j * T + threadIdx.x < c ? (uint32_t)((k[j] & PM) - lo) : pad;
            Sort(ts).SortBlockedToStriped(v, 0, bits);
#pragma unroll
            for (int j = 0; j < IPT; ++j) {   // striped: rank j * T + t
                const uint32_t r = (uint32_t)j * T + threadIdx.x;
                if (r < c) {
                    dst[base + r] = tag | (lo + v[j]);
                    if (slot_len) lens[base + r] = len;
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                const uint32_t q = (uint32_t)j * T + threadIdx.x;
                if (q >= c) continue;
                const uint64_t kq = src[q];   // (reloaded: k[] is dead past the offsets)
                uint32_t r = 0;
                for (uint32_t x = 0; x < c; ++x) {
                    const uint64_t y = src[x];
                    r += (y < kq) | ((y == kq) & (x < q));
                }
                dst[base + r] = kq;
                if (slot_len) lens[base + r] = len;
            }
        }
        __syncthreads();   // ts and red_* are reused by the next bin
    }
}

// clamped bin count (the keys a bin contributes to the list)
struct BinCount {
    const uint32_t* cnt;
    BinShape sh;
    __device__ uint64_t operator()(uint32_t b) const { return min(cnt[b], sh.cap(b)); }
};

// The whole list radix sorted (many large bins): gathered at the bins'
// offsets, packed as pattern << pos_bits | position when pos_bits > 0
__global__ void k_gather_bins(const uint64_t* __restrict__ out, const uint32_t* __restrict__ cnt,
                              const uint64_t* __restrict__ off, BinShape sh, uint64_t* __restrict__ dst,
                              uint32_t pos_bits) {
    const uint32_t bin = blockIdx.x;
    const uint32_t c = min(cnt[bin], sh.cap(bin));
    const uint64_t o = off[bin];
    const uint64_t* src = sh.src(out, bin);
    for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) {
        const uint64_t k = src[i];
        dst[o + i] = pos_bits ? ((k >> 48) << pos_bits) | (k & ((1ull << 48) - 1)) : k;
    }
}
// the ordered batch verify's lists gathered at their offsets (list order =
// position order)
__global__ void k_gather_lists(const uint64_t* __restrict__ ord, uint32_t cap, const uint32_t* __restrict__ cnt,
                               const uint64_t* __restrict__ off, uint64_t* __restrict__ dst) {
    const uint32_t l = blockIdx.x;
    const uint32_t c = min(cnt[l], cap);
    const uint64_t o = off[l];
    const uint64_t* src = ord + (uint64_t)l * cap;
    for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) dst[o + i] = src[i];
}
// The lists' keys to their (pattern, position) places: one wave per list,
// its keys in list order (= position order), 8 x 64 per round (4: 270 vs 262 us).  Per
// sub-round the lanes holding the same pattern find each other (a ballot
// per pattern bit), take base[p] + their rank among them, and the group's
// last lane advances base[p] (LDS, this wave's alone): a stable scatter, no
// sort.  base[p] starts at the exclusive scan of keys per (pattern, list)
// in pattern-major order.
constexpr uint32_t SCAT_U = 8;
__global__ __launch_bounds__(64) void k_list_scatter(const uint64_t* __restrict__ ord, uint32_t cap,
                                                     const uint32_t* __restrict__ cnt, const uint32_t* __restrict__ off,
                                                     uint32_t nlists, uint32_t P, uint32_t pbits,
                                                     uint64_t* __restrict__ dst) {
    __shared__ uint32_t base[ORD_HIST_MAX_P];
    const uint32_t l = blockIdx.x, lane = threadIdx.x;
    for (uint32_t p = lane; p < P; p += 64) base[p] = off[(uint64_t)p * nlists + l];
    __syncthreads();
    const uint32_t c = min(cnt[l], cap);
    const uint64_t* src = ord + (uint64_t)l * cap;
    const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;   // lanes under this one
    uint64_t nk[SCAT_U];
#pragma unroll
    for (uint32_t u = 0; u < SCAT_U; ++u) nk[u] = u * 64 + lane < c ? src[u * 64 + lane] : 0ull;
    for (uint32_t i0 = 0; i0 < c; i0 += 64 * SCAT_U) {
        uint64_t k[SCAT_U];
#pragma unroll
        for (uint32_t u = 0; u < SCAT_U; ++u) {   // this round's keys; the next round's in flight
            k[u] = nk[u];
            const uint32_t i = i0 + 64 * SCAT_U + u * 64 + lane;
            nk[u] = i < c ? src[i] : 0ull;
        }
#pragma unroll
        for (uint32_t u = 0; u < SCAT_U; ++u) {
            const bool valid = i0 + u * 64 + lane < c;
            const uint32_t p = (uint32_t)(k[u] >> 48);
            uint64_t peers = __builtin_amdgcn_ballot_w64(valid);
            for (uint32_t b = 0; b < pbits; ++b) {
                const uint64_t bb = __builtin_amdgcn_ballot_w64((p >> b) & 1u);
                peers &= ((p >> b) & 1u) ? bb : ~bb;
            }
            if (valid) {
                dst[base[p] + (uint32_t)__builtin_popcountll(peers & below)] = k[u];
                if (!(peers >> lane >> 1)) base[p] += (uint32_t)__builtin_popcountll(peers);   // the group's last lane
            }
        }
    }
}
struct ListCount {
    const uint32_t* cnt;
    uint32_t cap;
    __device__ uint64_t operator()(uint32_t l) const { return min(cnt[l], cap); }
};
__global__ void k_unpack_keys(uint64_t* __restrict__ keys, uint64_t n, uint32_t pos_bits) {
    const uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = keys[i];
    keys[i] = ((k >> pos_bits) << 48) | (k & ((1ull << pos_bits) - 1));
}

// the bins too large for an LDS sort: gathered into one list (bin order),
// radix sorted, copied back to each bin's offset.  pos_bits > 0: keys
// packed as pattern << pos_bits | position while sorted, so the radix sort
// runs over the significant bits only
struct HugeBin {
    uint32_t bin, c;
    uint64_t src_off, dst_off;
};
__global__ void k_gather_huge(const uint64_t* __restrict__ out, BinShape sh, const HugeBin* __restrict__ hb,
                              uint64_t* __restrict__ dst, uint32_t pos_bits) {
    const HugeBin b = hb[blockIdx.x];
    const uint64_t* src = sh.src(out, b.bin);
    for (uint32_t i = threadIdx.x; i < b.c; i += blockDim.x) {
        const uint64_t k = src[i];
        dst[b.src_off + i] = pos_bits ? ((k >> 48) << pos_bits) | (k & ((1ull << 48) - 1)) : k;
    }
}
__global__ void k_scatter_huge(const uint64_t* __restrict__ sorted, BinShape sh, const HugeBin* __restrict__ hb,
                               uint64_t* __restrict__ dst, const int32_t* __restrict__ slot_len,
                               uint32_t* __restrict__ lens, uint32_t pos_bits) {
    const HugeBin b = hb[blockIdx.x];
    const uint32_t len = slot_len ? (uint32_t)slot_len[b.bin / sh.bins_per_slot] : 0u;
    for (uint32_t i = threadIdx.x; i < b.c; i += blockDim.x) {
        const uint64_t k = sorted[b.src_off + i];
        dst[b.dst_off + i] = pos_bits ? ((k >> pos_bits) << 48) | (k & ((1ull << pos_bits) - 1)) : k;
        if (slot_len) lens[b.dst_off + i] = len;
    }
}


std::mutex g_pool_mu;
std::map<std::pair<int, size_t>, std::vector<void*>> g_pool;   // (device, capacity) -> free buffers
std::map<size_t, std::vector<void*>> g_pinned;                 // capacity -> free pinned host buffers
// destroyed hit lists whose buffers some queued work may still touch (a
// copy out on the caller's stream, a pipelined scan): recycled once their
// events have completed, so pm_hits_destroy never blocks the host
std::vector<pm_hits*> g_deferred;

bool event_done(hipEvent_t e) {
    if (!e) return true;
    const hipError_t q = hipEventQuery(e);
    quiet(q);   // hipErrorNotReady is an answer, not a failure to leave pending
    return q == hipSuccess;
}

bool hits_idle(const pm_hits* h) {
    return event_done(h->ready) && event_done(h->last_use) && (!h->pending || event_done(h->pending->counted));
}

void release_hits(pm_hits* h) {   // every event of h has completed
    if (h->ready) quiet(hipEventDestroy(h->ready));
    if (h->last_use) quiet(hipEventDestroy(h->last_use));
    delete h->pending;
    pool_put(h->device, h->keys, h->keys_cap);
    pool_put(h->device, h->lens, h->lens_cap);
    pool_put(h->device, h->old_keys, h->old_keys_cap);
    pool_put(h->device, h->old_lens, h->old_lens_cap);
    delete h;
}

// caller holds g_pool_mu; recycles every deferred list that is idle
void sweep_deferred_locked(std::vector<pm_hits*>& idle) {
    for (size_t i = 0; i < g_deferred.size();) {
        if (hits_idle(g_deferred[i])) {
            idle.push_back(g_deferred[i]);
            g_deferred[i] = g_deferred.back();
            g_deferred.pop_back();
        } else {
            ++i;
        }
    }
}

void sweep_deferred() {
    std::vector<pm_hits*> idle;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        sweep_deferred_locked(idle);
    }
    for (pm_hits* h : idle) release_hits(h);   // pool_put takes the lock itself
}

}  // namespace

void* pinned_get(size_t bytes, size_t* cap) {
    size_t c = 4096;
    while (c < bytes) c <<= 1;
    *cap = c;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        auto& v = g_pinned[c];
        if (!v.empty()) {
            void* p = v.back();
            v.pop_back();
            return p;
        }
    }
    void* p = nullptr;
    // mapped + coherent: kernels store into it, the host reads after an event
    HIPCHK(hipHostMalloc(&p, c, hipHostMallocMapped | hipHostMallocCoherent));
    return p;
}

void pinned_put(void* p, size_t cap) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    auto& v = g_pinned[cap];
    if (v.size() < 8) v.push_back(p);
    else quiet(hipHostFree(p));
}

void* pool_get(int device, size_t bytes, size_t* cap) {
    size_t c = 256;
    while (c < bytes) c <<= 1;
    *cap = c;
    sweep_deferred();
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        auto it = g_pool.find({device, c});
        if (it != g_pool.end() && !it->second.empty()) {
            void* p = it->second.back();
            it->second.pop_back();
            return p;
        }
    }
    void* p = nullptr;
    HIPCHK(hipMalloc(&p, c));
    return p;
}

void hits_ready(pm_db* db, pm_hits* h) {
    if (!h->ready) HIPCHK(hipEventCreateWithFlags(&h->ready, hipEventDisableTiming));
    HIPCHK(hipEventRecord(h->ready, db->stream));
    lane_end(db, db->stream);
}

void pool_put(int device, void* p, size_t cap) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    auto& v = g_pool[{device, cap}];
    if (v.size() < 8) v.push_back(p);
    else quiet(hipFree(p));
}

// Allocates out/cnt/slot arrays for n_slots slots of `per_slot` bins with
// per-slot capacities; counters zeroed, slot tables uploaded.
static SinkBuffers alloc_sink(pm_db* db, int n_slots, uint32_t per_slot, const std::vector<uint32_t>& caps,
                              bool zero_counts = true) {
    SinkBuffers sb;
    require(n_slots >= 1 && per_slot >= 1 && caps.size() == (size_t)n_slots, "internal: bad sink shape");
    sb.bins_per_pattern = per_slot;
    sb.nbins = (uint32_t)n_slots * per_slot;
    sb.slot_cap_h = caps;
    std::vector<uint64_t> base(n_slots);
    uint64_t total = 0;
    sb.cap = 0;
    for (int i = 0; i < n_slots; ++i) {
        base[i] = total;
        total += (uint64_t)per_slot * caps[i];
        sb.cap = std::max(sb.cap, caps[i]);
    }
    Carve c;
    const size_t o_out = c.take(total * sizeof(uint64_t));
    const size_t o_cnt = c.take((sb.nbins + 1) * sizeof(uint32_t));   // + the aux counter
    const size_t o_base = c.take(n_slots * sizeof(uint64_t));
    const size_t o_cap = c.take(n_slots * sizeof(uint32_t));
    uint8_t* d = static_cast<uint8_t*>(reserve(db, db->ws_sink, c.off));
    sb.out = reinterpret_cast<uint64_t*>(d + o_out);
    sb.cnt = reinterpret_cast<uint32_t*>(d + o_cnt);
    sb.slot_base = reinterpret_cast<uint64_t*>(d + o_base);
    sb.slot_cap = reinterpret_cast<uint32_t*>(d + o_cap);
    // slot tables staged through pinned memory (ordered on the db stream);
    // the layout is a function of (buffer, per_slot, caps), so an identical
    // repeat finds them in place
    if (db->slot_cache_p != (void*)d || db->slot_cache_per != per_slot || db->slot_cache_caps != caps) {
        static_assert(sizeof(uint64_t) == 8, "");
        if (db->slots_fence) HIPCHK(hipEventSynchronize(db->slots_fence));   // last copy out of pin_slots ran
        uint8_t* h = static_cast<uint8_t*>(reserve_host(db, db->pin_slots, (size_t)n_slots * 12 + 16));
        memcpy(h, base.data(), n_slots * 8);
        memcpy(h + (size_t)n_slots * 8, caps.data(), n_slots * 4);
        // o_base and o_cap are adjacent (8-byte entries then 4-byte ones, 256-aligned carve)
        HIPCHK(hipMemcpyAsync(sb.slot_base, h, n_slots * 8, hipMemcpyHostToDevice, db->stream));
        HIPCHK(hipMemcpyAsync(sb.slot_cap, h + (size_t)n_slots * 8, n_slots * 4, hipMemcpyHostToDevice, db->stream));
        if (!db->slots_fence) HIPCHK(hipEventCreateWithFlags(&db->slots_fence, hipEventDisableTiming));
        HIPCHK(hipEventRecord(db->slots_fence, db->stream));
        db->slot_cache_p = d;
        db->slot_cache_per = per_slot;
        db->slot_cache_caps = caps;
    }
    if (zero_counts) HIPCHK(hipMemsetAsync(sb.cnt, 0, (sb.nbins + 1) * sizeof(uint32_t), db->stream));
    return sb;
}

SinkBuffers make_sink(pm_db* db, int n_slots, uint64_t n_positions, uint64_t expected) {
    require(n_slots >= 1 && (uint32_t)n_slots <= MAX_BINS, "internal: too many pattern slots");
    const uint32_t bpp = std::max<uint32_t>(1, NBINS / (uint32_t)n_slots);
    uint32_t shift = 0;
    const uint64_t last = std::max<uint64_t>(n_positions, 1) - 1;
    while ((last >> shift) >= bpp) ++shift;
    const uint32_t nbins = (uint32_t)n_slots * bpp;
    uint64_t cap = std::max<uint64_t>(1024, (expected + nbins - 1) / nbins * 2);
    cap = std::min<uint64_t>(cap, 1ull << 26);
    SinkBuffers sb = alloc_sink(db, n_slots, bpp, std::vector<uint32_t>(n_slots, (uint32_t)cap));
    sb.pos_shift = shift;   // uniform capacity: bin b lives at out + b * cap (Sink::push)
    return sb;
}

SinkBuffers make_sink_segments(pm_db* db, int n_slots, uint32_t per_slot, const std::vector<uint32_t>& slot_caps,
                               bool zero_counts) {
    SinkBuffers sb = alloc_sink(db, n_slots, per_slot, slot_caps, zero_counts);
    sb.pos_shift = 0;
    return sb;
}

uint64_t sink_total(pm_db* db, const SinkBuffers& sb, std::vector<uint32_t>& counts, bool& overflow) {
    uint32_t* h = static_cast<uint32_t*>(reserve_host(db, db->pin_down, (sb.nbins + 1) * sizeof(uint32_t)));
    HIPCHK(hipMemcpyAsync(h, sb.cnt, (sb.nbins + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost, db->stream));
    HIPCHK(hipStreamSynchronize(db->stream));
    counts.assign(h, h + sb.nbins);
    const_cast<SinkBuffers&>(sb).aux = h[sb.nbins];
    uint64_t total = 0;
    overflow = false;
    for (uint32_t b = 0; b < sb.nbins; ++b) {
        total += counts[b];
        overflow |= counts[b] > sb.slot_cap_h[b / sb.bins_per_pattern];
    }
    return total;
}

pm_hits* sink_sort_speculative(pm_db* db, const SinkBuffers& sb, const int32_t* slot_len, uint32_t* counts_host,
                               hipStream_t stream, uint64_t* total_out, bool bind_ready) {
    require(sb.nbins <= 4096, "internal: speculative sort needs <= 4096 bins");
    uint64_t cap_total = 0;
    for (uint32_t c : sb.slot_cap_h) cap_total += (uint64_t)c * sb.bins_per_pattern;
    pm_hits* h = new pm_hits();
    h->device = db->device;
    try {
        h->keys = static_cast<uint64_t*>(pool_get(db->device, std::max<uint64_t>(cap_total, 1) * 8, &h->keys_cap));
        h->lens = static_cast<uint32_t*>(pool_get(db->device, std::max<uint64_t>(cap_total, 1) * 4, &h->lens_cap));
        const BinShape sh{sb.slot_base, sb.slot_cap, sb.bins_per_pattern};
        // a bin holds at most its slot's capacity: the 4096-key sort when a
        // capacity exceeds 2048
        const bool big = *std::max_element(sb.slot_cap_h.begin(), sb.slot_cap_h.end()) > LDS_SORT_CAP;
        auto kern = big ? k_sort_bins<LDS_SORT_CAP_MAX> : k_sort_bins<LDS_SORT_CAP>;
        if (counts_host && bind_ready) {
            // pipelined scan: the list's ready event is bound to the sort's
            // own dispatch (no marker packet before the next scan's kernel)
            HIPCHK(hipEventCreate(&h->ready));
            hipExtLaunchKernelGGL(kern, dim3(sb.nbins), dim3(256), 0, stream, nullptr, h->ready, 0u, sb.out,
                                  sb.cnt, (const uint64_t*)nullptr, sh, h->keys, slot_len, h->lens, counts_host,
                                  sb.nbins, total_out, (const uint32_t*)nullptr, sb.nbins);
        } else {
            hipLaunchKernelGGL(kern, dim3(sb.nbins), dim3(256), 0, stream, sb.out,
                               sb.cnt, (const uint64_t*)nullptr, sh, h->keys, slot_len, h->lens, counts_host,
                               (counts_host || total_out) ? sb.nbins : 0u, total_out, (const uint32_t*)nullptr, sb.nbins);
        }
        HIPCHK(hipGetLastError());
    } catch (...) {
        discard_hits(h);
        throw;
    }
    return h;
}

void discard_hits(pm_hits* h) {
    if (!h) return;
    pool_put(h->device, h->keys, h->keys_cap);
    pool_put(h->device, h->lens, h->lens_cap);
    pool_put(h->device, h->old_keys, h->old_keys_cap);
    pool_put(h->device, h->old_lens, h->old_lens_cap);
    delete h;
}

pm_hits* sink_to_hits(pm_db* db, const SinkBuffers& sb, const std::vector<uint32_t>& counts, uint64_t total,
                      const int32_t* slot_len, bool* lens_done) {
    if (lens_done) *lens_done = false;
    hipStream_t s = db->stream;
    pm_hits* h = new pm_hits();
    h->device = db->device;
    h->count = total;
    try {
        h->keys = static_cast<uint64_t*>(pool_get(db->device, std::max<uint64_t>(total, 1) * sizeof(uint64_t),
                                                  &h->keys_cap));
        h->lens = static_cast<uint32_t*>(pool_get(db->device, std::max<uint64_t>(total, 1) * sizeof(uint32_t),
                                                  &h->lens_cap));
        if (total == 0) return h;
        const uint32_t maxc = *std::max_element(counts.begin(), counts.end());
        // bins of up to LDS_SORT_CAP_MAX keys: one LDS sort block each; a few
        // larger ones (dense patterns of a big batch) up to LDS_SORT_CAP_HUGE:
        // a second pass over their list, 128 KB of LDS per block; beyond
        // that (configs[4]: one pattern's ~24 Ki keys per segment) the bins
        // are radix sorted by themselves -- 6 M keys instead of the whole
        // 31 M-key list
        std::vector<uint32_t> big;
        std::vector<HugeBin> huge;
        uint64_t nhuge = 0, nlarge = 0;   // keys in bins over LDS_SORT_CAP_HUGE / over LDS_SORT_SMALL
        if (maxc > LDS_SORT_SMALL) {
            uint64_t at = 0;
            for (uint32_t b = 0; b < sb.nbins; ++b) {
                const uint32_t c = std::min(counts[b], sb.slot_cap_h[b / sb.bins_per_pattern]);
                if (c > LDS_SORT_CAP_HUGE) {
                    huge.push_back({b, c, nhuge, at});
                    nhuge += c;
                } else if (c > LDS_SORT_CAP_MAX) {
                    big.push_back(b);
                }
                if (c > LDS_SORT_SMALL) nlarge += c;
                at += c;
            }
        }
        // with a huge bin and most keys in large bins (configs[4]: 29 of 31 M)
        // one radix sort of the whole list: every per-bin form sorts at about
        // the same keys/s (block radix 27-32, huge-bin radix ~26 Gkeys/s,
        // r05k) and the whole list is one pass of kernels
        const bool whole = !huge.empty() && 2 * nlarge > total;
        if (whole) {
            big.clear();
            huge.clear();
            nhuge = 0;
        }
        const BinShape sh{sb.slot_base, sb.slot_cap, sb.bins_per_pattern};
        // up to 4096 bins each sort block sums the counts before it itself
        const bool inline_off = !whole && sb.nbins <= 4096 && big.empty() && huge.empty();
        auto counted = hipcub::TransformInputIterator<uint64_t, BinCount, hipcub::CountingInputIterator<uint32_t>>(
            hipcub::CountingInputIterator<uint32_t>(0u), BinCount{sb.cnt, sh});
        size_t scan_bytes = 0, sort_bytes = 0;
        // sort only the significant bits: positions < 2^pos_bits, pattern
        // slots < 2^slot_bits
        uint32_t pos_bits = 1, slot_bits = 1;
        while (pos_bits < 48 && (db->n >> pos_bits)) ++pos_bits;
        while (slot_bits < 16 && ((uint64_t)(sb.nbins / sb.bins_per_pattern - 1) >> slot_bits)) ++slot_bits;
        const bool pack = pos_bits + slot_bits < 56;
        size_t hsort_bytes = 0;
        if (!huge.empty())
            HIPCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, hsort_bytes, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                                     (int)nhuge, 0, pack ? (int)(pos_bits + slot_bits) : 64, s));
        if (whole)
            HIPCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, sort_bytes, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                                     (int)total, 0, pack ? (int)(pos_bits + slot_bits) : 64, s));
        if (!inline_off)
            HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, counted, (uint64_t*)nullptr, (int)sb.nbins, s));
        clear_stale_capture_status("rocPRIM call (pm_hits)");   // (status check after the size queries too, see the scan below)
        Carve c;
        const size_t o_off = c.take(sb.nbins * sizeof(uint64_t));
        const size_t o_scan = c.take(scan_bytes);
        const size_t o_big = c.take(inline_off ? 0 : (size_t)sb.nbins * sizeof(uint32_t));   // bin lists
        const size_t o_hb = c.take(huge.size() * sizeof(HugeBin));
        const size_t o_hin = c.take(nhuge * sizeof(uint64_t));
        const size_t o_hout = c.take(nhuge * sizeof(uint64_t));
        const size_t o_hsort = c.take(hsort_bytes);
        const size_t o_uns = c.take(whole ? total * sizeof(uint64_t) : 0);
        const size_t o_tmp = c.take(sort_bytes);
        uint8_t* base = static_cast<uint8_t*>(reserve(db, db->ws_post, c.off));
        uint64_t* d_off = reinterpret_cast<uint64_t*>(base + o_off);
        if (!inline_off) {
            HIPCHK(hipcub::DeviceScan::ExclusiveSum(base + o_scan, scan_bytes, counted, d_off, (int)sb.nbins, s));
            // (a status check after the library call: any status but a
            // caller's capture code fails here, pm_internal.h -- round 6's
            // probe found none of these rocPRIM calls leaves one)
            clear_stale_capture_status("rocPRIM call (pm_hits)");
        }
        if (whole) {
            uint64_t* unsorted = reinterpret_cast<uint64_t*>(base + o_uns);
            hipLaunchKernelGGL(k_gather_bins, dim3(sb.nbins), dim3(256), 0, s, sb.out, sb.cnt, d_off, sh, unsorted,
                               pack ? pos_bits : 0u);
            HIPCHK(hipGetLastError());
            HIPCHK(hipcub::DeviceRadixSort::SortKeys(base + o_tmp, sort_bytes, unsorted, h->keys, (int)total, 0,
                                                     pack ? (int)(pos_bits + slot_bits) : 64, s));
            clear_stale_capture_status("rocPRIM call (pm_hits)");   // (status check, see the scan above)
            if (pack) {
                hipLaunchKernelGGL(k_unpack_keys, dim3(blocks_for(total, 256)), dim3(256), 0, s, h->keys, total,
                                   pos_bits);
                HIPCHK(hipGetLastError());
            }
        } else if (inline_off) {
            auto kern = maxc > LDS_SORT_CAP ? k_sort_bins<LDS_SORT_CAP_MAX> : k_sort_bins<LDS_SORT_CAP>;
            hipLaunchKernelGGL(kern, dim3(sb.nbins), dim3(256), 0, s, sb.out, sb.cnt, (const uint64_t*)nullptr, sh,
                               h->keys, slot_len, h->lens, (uint32_t*)nullptr, 0u, (uint64_t*)nullptr,
                               (const uint32_t*)nullptr, sb.nbins);
            HIPCHK(hipGetLastError());
        } else {
            // many bins (a large batch: patterns x segments), each pass a
            // size class: a bin's sort is a short chain of dependent loads, so
            // the small-bin pass (most bins, 2 KB of LDS) keeps many blocks
            // in flight per CU; the larger classes go by bin lists
            std::vector<uint32_t> mid;
            for (uint32_t b = 0; b < sb.nbins; ++b) {
                const uint32_t c = std::min(counts[b], sb.slot_cap_h[b / sb.bins_per_pattern]);
                if (c > LDS_SORT_SMALL && c <= LDS_SORT_CAP_MAX) mid.push_back(b);
            }
            hipLaunchKernelGGL((k_sort_bins<LDS_SORT_SMALL, LDS_SORT_SMALL>), dim3(std::min<uint32_t>(sb.nbins, 65536)),
                               dim3(LDS_SORT_SMALL), 0, s, sb.out, sb.cnt, (const uint64_t*)d_off, sh, h->keys,
                               slot_len, h->lens, (uint32_t*)nullptr, 0u, (uint64_t*)nullptr,
                               (const uint32_t*)nullptr, sb.nbins);
            HIPCHK(hipGetLastError());
            std::vector<uint32_t> lists(mid);
            lists.insert(lists.end(), big.begin(), big.end());
            if (!huge.empty()) {
                HugeBin* d_hb = reinterpret_cast<HugeBin*>(base + o_hb);
                uint64_t* hin = reinterpret_cast<uint64_t*>(base + o_hin);
                uint64_t* hout = reinterpret_cast<uint64_t*>(base + o_hout);
                const uint32_t pb = pack ? pos_bits : 0u;
                HIPCHK(hipMemcpyAsync(d_hb, huge.data(), huge.size() * sizeof(HugeBin), hipMemcpyHostToDevice, s));
                hipLaunchKernelGGL(k_gather_huge, dim3((uint32_t)huge.size()), dim3(1024), 0, s, sb.out, sh, d_hb, hin, pb);
                HIPCHK(hipGetLastError());
                HIPCHK(hipcub::DeviceRadixSort::SortKeys(base + o_hsort, hsort_bytes, hin, hout, (int)nhuge, 0,
                                                         pack ? (int)(pos_bits + slot_bits) : 64, s));
                clear_stale_capture_status("rocPRIM call (pm_hits)");   // (status check, see the scan above)
                hipLaunchKernelGGL(k_scatter_huge, dim3((uint32_t)huge.size()), dim3(1024), 0, s, hout, sh, d_hb,
                                   h->keys, slot_len, h->lens, pb);
                HIPCHK(hipGetLastError());
                if (lists.empty()) HIPCHK(hipStreamSynchronize(s));   // `huge` (pageable) was read by the copy
            }
            if (!lists.empty()) {
                uint32_t* d_lists = reinterpret_cast<uint32_t*>(base + o_big);
                HIPCHK(hipMemcpyAsync(d_lists, lists.data(), lists.size() * 4, hipMemcpyHostToDevice, s));
                static_assert(256 * 16 == LDS_SORT_CAP_MAX && 512 * 32 == LDS_SORT_CAP_HUGE, "radix bin shapes");
                if (!mid.empty())
                    hipLaunchKernelGGL((k_radix_bins<256, 16>), dim3((uint32_t)mid.size()), dim3(256), 0, s, sb.out,
                                       sb.cnt, (const uint64_t*)d_off, sh, h->keys, slot_len, h->lens,
                                       (const uint32_t*)d_lists, (uint32_t)mid.size());
                if (!big.empty())
                    hipLaunchKernelGGL((k_radix_bins<512, 32>), dim3((uint32_t)big.size()), dim3(512), 0, s, sb.out,
                                       sb.cnt, (const uint64_t*)d_off, sh, h->keys, slot_len, h->lens,
                                       (const uint32_t*)d_lists + mid.size(), (uint32_t)big.size());
                HIPCHK(hipGetLastError());
                HIPCHK(hipStreamSynchronize(s));   // `lists` (pageable) was read by the copy
            }
            if (lens_done) *lens_done = slot_len != nullptr;
        }
    } catch (...) {
        pool_put(h->device, h->keys, h->keys_cap);
        pool_put(h->device, h->lens, h->lens_cap);
        delete h;
        throw;
    }
    return h;
}

namespace {
void retire_buffers(pm_hits* h, hipStream_t s);   // below (report pass)
}

pm_hits* ordered_to_hits(pm_db* db, const SinkBuffers& sb, const std::vector<uint32_t>& counts, uint64_t sink_total,
                         const uint64_t* ord, uint32_t ord_cap, const uint32_t* d_cnt, const uint32_t* cnt,
                         uint32_t nlists, int n_patterns, const uint32_t* d_hist) {
    uint64_t t1 = 0;
    for (uint32_t l = 0; l < nlists; ++l) t1 += std::min(cnt[l], ord_cap);
    // the sink first (its sort reserves ws_post itself)
    pm_hits* hs = sink_total ? sink_to_hits(db, sb, counts, sink_total, nullptr, nullptr) : nullptr;
    if (t1 == 0 && hs) return hs;
    hipStream_t s = db->stream;
    const uint64_t total = t1 + sink_total;
    pm_hits* h = new pm_hits();
    h->device = db->device;
    h->count = total;
    try {
        h->keys = static_cast<uint64_t*>(pool_get(db->device, std::max<uint64_t>(total, 1) * 8, &h->keys_cap));
        h->lens = static_cast<uint32_t*>(pool_get(db->device, std::max<uint64_t>(total, 1) * 4, &h->lens_cap));
        if (total) {
            // the lists hold every pattern's keys in increasing position: one
            // stable radix sort over the pattern bits (48 + slot_bits) orders
            // them by (pattern, position)
            uint32_t slot_bits = 1;
            while (slot_bits < 16 && ((uint64_t)(n_patterns - 1) >> slot_bits)) ++slot_bits;
            auto counted = hipcub::TransformInputIterator<uint64_t, ListCount, hipcub::CountingInputIterator<uint32_t>>(
                hipcub::CountingInputIterator<uint32_t>(0u), ListCount{d_cnt, ord_cap});
            size_t scan_bytes = 0, sort_bytes = 0, merge_bytes = 0;
            const uint64_t nh = d_hist ? (uint64_t)n_patterns * nlists : 0;
            if (d_hist) {   // keys per (pattern, list) -> their first places
                HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, d_hist, (uint32_t*)nullptr, (int)nh, s));
            } else {
                HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, counted, (uint64_t*)nullptr, (int)nlists, s));
                HIPCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, sort_bytes, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                                         (int)t1, 48, 48 + (int)slot_bits, s));
            }
            if (hs)
                HIPCHK(rocprim::merge(nullptr, merge_bytes, (const uint64_t*)nullptr, (const uint64_t*)nullptr,
                                      (uint64_t*)nullptr, (size_t)t1, (size_t)sink_total, rocprim::less<uint64_t>(), s));
            clear_stale_capture_status("rocPRIM call (pm_hits)");   // (status check, see sink_to_hits)
            Carve c;
            const size_t o_off = c.take(d_hist ? nh * sizeof(uint32_t) : nlists * sizeof(uint64_t));
            const size_t o_scan = c.take(scan_bytes);
            const size_t o_in = c.take(d_hist ? 0 : t1 * sizeof(uint64_t));
            const size_t o_mid = c.take(hs ? t1 * sizeof(uint64_t) : 0);
            const size_t o_tmp = c.take(std::max(sort_bytes, merge_bytes));
            uint8_t* base = static_cast<uint8_t*>(reserve(db, db->ws_post, c.off));
            uint64_t* d_off = reinterpret_cast<uint64_t*>(base + o_off);
            uint64_t* in = reinterpret_cast<uint64_t*>(base + o_in);
            uint64_t* sorted = hs ? reinterpret_cast<uint64_t*>(base + o_mid) : h->keys;
            if (d_hist) {
                uint32_t* d_poff = reinterpret_cast<uint32_t*>(base + o_off);
                HIPCHK(hipcub::DeviceScan::ExclusiveSum(base + o_scan, scan_bytes, d_hist, d_poff, (int)nh, s));
                clear_stale_capture_status("rocPRIM call (pm_hits)");
                hipLaunchKernelGGL(k_list_scatter, dim3(nlists), dim3(64), 0, s, ord, ord_cap, d_cnt, d_poff, nlists,
                                   (uint32_t)n_patterns, slot_bits, sorted);
                HIPCHK(hipGetLastError());
            } else {
                HIPCHK(hipcub::DeviceScan::ExclusiveSum(base + o_scan, scan_bytes, counted, d_off, (int)nlists, s));
                clear_stale_capture_status("rocPRIM call (pm_hits)");
                hipLaunchKernelGGL(k_gather_lists, dim3(nlists), dim3(256), 0, s, ord, ord_cap, d_cnt, d_off, in);
                HIPCHK(hipGetLastError());
                HIPCHK(hipcub::DeviceRadixSort::SortKeys(base + o_tmp, sort_bytes, in, sorted, (int)t1, 48,
                                                         48 + (int)slot_bits, s));
                clear_stale_capture_status("rocPRIM call (pm_hits)");
            }
            if (hs) {
                HIPCHK(rocprim::merge(base + o_tmp, merge_bytes, (const uint64_t*)sorted, (const uint64_t*)hs->keys,
                                      h->keys, (size_t)t1, (size_t)sink_total, rocprim::less<uint64_t>(), s));
                clear_stale_capture_status("rocPRIM call (pm_hits)");
            }
        }
    } catch (...) {
        discard_hits(h);
        if (hs) discard_hits(hs);
        throw;
    }
    if (hs) {
        // its buffers go back to the pool once the merge has read them (an
        // event-tracked shell, no host sync)
        retire_buffers(hs, s);
        hs->keys = nullptr;
        hs->lens = nullptr;
        discard_hits(hs);
    }
    return h;
}

// ---------------------------------------------------------------------------
// nrgrep report selection (see pm_internal.h and DESIGN.md §1)
// ---------------------------------------------------------------------------
// Input: a (pattern, beg)-sorted candidate list with match lengths.  Output:
// what nrgrep_coords prints, per pattern: scanning from R = 0, the first
// candidate with beg >= R is reported and R becomes its end.  Parallel form:
// candidate i is a "head" when its key is >= the running maximum of
// (pattern, end) over every earlier candidate -- whatever was reported
// before it ended at or before its start, so it is reported; the head's
// thread then walks its cluster (the candidates up to the next head)
// sequentially.  Clusters are short (overlapping matches), so the walk is
// cheap; the running maximum comes from per-chunk maxima (k_rep_max) and an
// in-block scan.  With '^' a start passes the check at a line start or
// exactly at R (recCheckLeftContext 0x402182): a head must then lie strictly
// after every earlier end (a candidate touching the running end joins its
// cluster), and the head itself is reported only at a line start.  A class
// sequence at k > 0 takes nrgrep's esimple order instead (pm_esimple.hip).
namespace {

constexpr uint32_t REP_G = 512;           // chunks (blocks) of the list (at least)
constexpr uint32_t REP_G_MAX = 8192;      // long lists: ~16 Ki candidates per chunk
constexpr uint32_t REP_T = 256;           // threads per block
constexpr uint64_t POS_MASK = (1ull << 48) - 1;

__device__ inline uint8_t tv_raw(const TextView& tv, uint64_t p) {
    return tv.nuc_layout ? nuc_raw_at(tv.nuc, p) : tv.raw[p];
}
__device__ inline bool tv_header(const TextView& tv, uint64_t p) {
    return tv.nuc_layout ? nuc_is_header(tv.nuc, p) : (tv.bytes[p] == (uint8_t)'\n' && tv.raw[p] != (uint8_t)'\n');
}

struct RepArgs {
    const uint64_t* keys;
    const uint32_t* lens;
    const int32_t* plen;    // non-null: lens by pattern (lens unread)
    uint64_t* okeys;
    uint32_t* olens;
    uint8_t* acc;           // per candidate: 1 = reported and kept (written exactly once, or twice with 0)
    uint64_t* bmax;
    uint32_t* bcnt;         // kept candidates per chunk
    const uint64_t* total_d;
    uint64_t total_h;
    uint32_t* count;
    uint32_t* host_count;
    TextView tv;
    uint32_t flags;
    int hdr;                // candidates may start on a header line (simple engine, cross windows)
};

__device__ inline uint64_t rep_total(const RepArgs& a) { return a.total_d ? *a.total_d : a.total_h; }
// candidate i's length (key: its key)
__device__ inline uint32_t rep_len(const RepArgs& a, uint64_t i, uint64_t key) {
    return a.plen ? (uint32_t)a.plen[key >> 48] : a.lens[i];
}
__device__ inline uint64_t rep_chunk(uint64_t total, uint32_t G) { return (total + G - 1) / G; }

// '$': the match must end at a line end or at the end of the text (the
// region end, recCheckRightContext 0x4021e0)
// near: region_near(key's start), computed once per candidate by the caller
__device__ inline bool rep_valid(const RepArgs& a, uint64_t key, uint32_t len, bool near) {
    if (len == 0) return false;   // a start whose verify found no (anchored) end
    // a speculative list that will be discarded (a bin the LDS sort skipped)
    // holds stale keys: never read the text at a position outside it
    const uint64_t s = key & POS_MASK;
    if (s >= a.tv.n || len > a.tv.n - s) return false;
    const uint64_t e = s + len;
    // inside the region it is found in (only a simple-engine window over a
    // region's last '\n', or a cut without one, can stick out)
    if (near && e > a.tv.reg.e[region_of(a.tv.reg, s)]) return false;
    if (!(a.flags & PM_ANCHOR_END)) return true;
    // '$': a line end or the region end (recCheckRightContext 0x4021e0)
    return e >= a.tv.n || tv_raw(a.tv, e) == (uint8_t)'\n' || (near && e == a.tv.reg.e[region_of(a.tv.reg, s)]);
}
// (pattern, end), the running maximum the heads are found with; the report
// rule restarts at every region start, so an end past the next region's
// start (the '\n' both regions hold) counts as that start
__device__ inline uint64_t rep_val(const RepArgs& a, uint64_t key, uint32_t len, bool near) {
    uint64_t v = key + len;
    if (near) {
        const uint32_t r = region_of(a.tv.reg, key & POS_MASK);
        if (r + 1 < a.tv.reg.n) v = umin64(v, (key & ~POS_MASK) | a.tv.reg.t[r + 1]);
    }
    return v;
}
// s starts a region (the search restarts there: R = s)
__device__ inline bool rep_region_start(const RepArgs& a, uint64_t s) {
    return region_near(a.tv.reg, s) && a.tv.reg.t[region_of(a.tv.reg, s)] == s;
}

// a start on a header line or on the '\n' that ends it maps to the '>name'
// record in process_output (get_name_offset) and is discarded
__device__ inline bool rep_keep(const RepArgs& a, uint64_t key) {
    if (!a.hdr) return true;
    const uint64_t s = key & POS_MASK;
    if (a.tv.nuc_layout) {
        // positions whose lane holds no header byte (hflag: 1.5 MB per 12.5
        // Gbp, cache-resident) settle with one cached load.  (Until round 6
        // this was lflag, the lanes with ANY exception -- N runs, IUPAC
        // letters, every line break of a wrapped file: ~5 % of a synthetic
        // database's lanes and nearly all of a real genome's, each such start
        // then paying the exception-table chain of nuc_is_header)
        auto clean = [&](uint64_t p) {
            return !((a.tv.hflag[p / TILE_POS] >> ((uint32_t)(p % STREAM) >> 5)) & 1ull);
        };
        if (clean(s) && (s == 0 || clean(s - 1))) return true;
    }
    if (tv_header(a.tv, s)) return false;
    return !(s > 0 && tv_header(a.tv, s - 1) && tv_raw(a.tv, s) == (uint8_t)'\n');
}

// region_near for a candidate's start, false past the text: a speculative
// list that will be discarded holds stale keys, whose positions may lie
// beyond the region tables
__device__ inline bool rep_near(const RepArgs& a, uint64_t key) {
    const uint64_t s = key & POS_MASK;
    return s < a.tv.n && region_near(a.tv.reg, s);
}

// '^' passes at a line start or at R (recCheckLeftContext 0x402170): the
// region start is R when a region's search begins
__device__ inline bool rep_line_start(const RepArgs& a, uint64_t s) {
    return s == 0 || tv_raw(a.tv, s - 1) == (uint8_t)'\n' || rep_region_start(a, s);
}

// 64-bit wave shuffle as two 32-bit halves (a (pattern, end) key does not
// fit the 32-bit shuffle)
__device__ inline uint64_t shfl_xor64(uint64_t v, int d) {
    const uint32_t lo = __shfl_xor((uint32_t)v, d, 64), hi = __shfl_xor((uint32_t)(v >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ inline uint64_t shfl_up64(uint64_t v, int d) {
    const uint32_t lo = __shfl_up((uint32_t)v, d, 64), hi = __shfl_up((uint32_t)(v >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}
__device__ inline uint64_t block_max(uint64_t v, uint64_t* red) {
    for (int d = 32; d > 0; d >>= 1) v = umax64(v, shfl_xor64(v, d));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    uint64_t r = 0;
    for (uint32_t w = 0; w < REP_T / 64; ++w) r = umax64(r, red[w]);
    __syncthreads();
    return r;
}
__device__ inline uint64_t block_sum(uint64_t v, uint64_t* red) {
    for (int d = 32; d > 0; d >>= 1) v += shfl_xor64(v, d);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    uint64_t r = 0;
    for (uint32_t w = 0; w < REP_T / 64; ++w) r += red[w];
    __syncthreads();
    return r;
}

// fixed lengths by pattern, no anchors: a valid candidate's rep_val is
// monotone along the (pattern, start)-sorted list (the end grows with the
// start; a region's cap of it too)
__device__ inline bool rep_monotone(const RepArgs& a) {
    return a.plen && !(a.flags & (PM_ANCHOR_START | PM_ANCHOR_END));
}

// per chunk: the largest (pattern, end) of a valid candidate; the kept
// counters start at 0
__global__ __launch_bounds__(REP_T) void k_rep_max(RepArgs a) {
    __shared__ uint64_t red[REP_T / 64];
    const uint64_t total = rep_total(a), C = rep_chunk(total, gridDim.x);
    const uint64_t b0 = blockIdx.x * C, b1 = umin64(total, b0 + C);
    uint64_t m = 0;
    if (a.flags & PM_REPORT_NRGREP) {
        // 4 candidates per round: their loads (and the region lookups that
        // depend on them) are in flight together, the next round's loads
        // while this one's lookups run
        constexpr int U = 4;
        uint64_t nkey[U];
        uint32_t nlen[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = b0 + threadIdx.x + (uint64_t)u * REP_T;
            nkey[u] = i < b1 ? a.keys[i] : 0ull;
            nlen[u] = i < b1 && !a.plen ? a.lens[i] : 0u;
        }
        for (uint64_t i0 = b0 + threadIdx.x; i0 < b1; i0 += U * REP_T) {
            uint64_t key[U];
            uint32_t len[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                key[u] = nkey[u];
                len[u] = !a.plen ? nlen[u] : i0 + (uint64_t)u * REP_T < b1 ? (uint32_t)a.plen[key[u] >> 48] : 0u;
                const uint64_t i = i0 + (uint64_t)(U + u) * REP_T;
                nkey[u] = i < b1 ? a.keys[i] : 0ull;
                nlen[u] = i < b1 && !a.plen ? a.lens[i] : 0u;
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (len[u]) {
                    const bool nr = rep_near(a, key[u]);
                    if (rep_valid(a, key[u], len[u], nr)) m = umax64(m, rep_val(a, key[u], len[u], nr));
                }
        }
        m = block_max(m, red);
    }
    if (threadIdx.x == 0) {
        a.bmax[blockIdx.x] = m;
        a.bcnt[blockIdx.x] = 0u;
    }
}

// acc[] and the kept count of every chunk
__global__ __launch_bounds__(REP_T) void k_rep_walk(RepArgs a) {
    __shared__ uint64_t red[REP_T / 64];
    __shared__ uint64_t wmax[REP_T / 64];
    const uint64_t total = rep_total(a), C = rep_chunk(total, gridDim.x);
    const uint64_t b0 = blockIdx.x * C, b1 = umin64(total, b0 + C);
    if (!(a.flags & PM_REPORT_NRGREP)) {   // every candidate: only the anchors filter
        uint64_t own = 0;
        for (uint64_t i = b0 + threadIdx.x; i < b1; i += REP_T) {
            const uint64_t key = a.keys[i];
            const uint64_t s = key & POS_MASK;
            bool ok = rep_valid(a, key, rep_len(a, i, key), rep_near(a, key));
            if (ok && (a.flags & PM_ANCHOR_START)) ok = rep_line_start(a, s);
            ok = ok && rep_keep(a, key);
            a.acc[i] = ok ? 1 : 0;
            own += ok;
        }
        own = block_sum(own, red);
        if (threadIdx.x == 0) a.bcnt[blockIdx.x] = (uint32_t)own;
        return;
    }
    const bool anch = (a.flags & PM_ANCHOR_START) != 0;
    // running maximum of every chunk before this one
    uint64_t carry = 0;
    if (rep_monotone(a)) {
        // lengths by pattern and no anchors: a valid candidate's (pattern,
        // end) never decreases along the list, so the running maximum is the
        // last valid candidate's (no k_rep_max pass).  The block looks back
        // REP_T keys per round, nearest first: a long run of invalid keys
        // (dropped at region ends) costs rounds of REP_T parallel loads, not
        // one dependent load per key on one thread.  Values are monotone
        // along the valid keys, so a round's maximum is its last valid one's
        // (and a value is never 0: end > 0).
        for (uint64_t top = b0; top > 0;) {
            const uint64_t lo = top > REP_T ? top - REP_T : 0;
            uint64_t v = 0;
            if (threadIdx.x < top - lo) {
                const uint64_t j = top - 1 - threadIdx.x;
                const uint64_t kj = a.keys[j];
                const uint32_t lj = rep_len(a, j, kj);
                const bool nj = rep_near(a, kj);
                if (rep_valid(a, kj, lj, nj)) v = rep_val(a, kj, lj, nj);
            }
            v = block_max(v, red);   // uniform across the block
            if (v) {
                carry = v;
                break;
            }
            top = lo;
        }
    } else {
        for (uint32_t b = threadIdx.x; b < blockIdx.x; b += REP_T) carry = umax64(carry, a.bmax[b]);
        carry = block_max(carry, red);
    }
    uint64_t own = 0;   // kept candidates of this chunk found by this thread's walks
    // A tile is REP_T * RW candidates, RW consecutive ones per thread: the
    // block's serial chain of tiles (a load, the scan's exchange, two
    // barriers each) is RW times shorter.  The next tile's loads are in
    // flight while a tile is scanned.
    constexpr int RW = 4;
    constexpr uint64_t TT = (uint64_t)REP_T * RW;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t nkey[RW];
    uint32_t nlen[RW];
#pragma unroll
    for (int u = 0; u < RW; ++u) {
        const uint64_t i = b0 + (uint64_t)threadIdx.x * RW + u;
        nkey[u] = i < b1 ? a.keys[i] : 0ull;
        nlen[u] = i < b1 && !a.plen ? a.lens[i] : 0u;
    }
    for (uint64_t base = b0; base < b1; base += TT) {
        const uint64_t i0 = base + (uint64_t)threadIdx.x * RW;
        uint64_t key[RW], val[RW];
        uint32_t len[RW];
        bool valid[RW];
#pragma unroll
        for (int u = 0; u < RW; ++u) {
            key[u] = nkey[u];
            len[u] = !a.plen ? nlen[u] : i0 + u < b1 ? (uint32_t)a.plen[key[u] >> 48] : 0u;
            const uint64_t ni = i0 + TT + u;
            nkey[u] = ni < b1 ? a.keys[ni] : 0ull;
            nlen[u] = ni < b1 && !a.plen ? a.lens[ni] : 0u;
        }
        uint64_t tmax = 0;   // the thread's candidates' running maximum
#pragma unroll
        for (int u = 0; u < RW; ++u) {
            val[u] = 0;
            valid[u] = false;
            if (i0 + u < b1) {
                const bool nr = rep_near(a, key[u]);
                valid[u] = rep_valid(a, key[u], len[u], nr);
                if (valid[u]) val[u] = rep_val(a, key[u], len[u], nr);
                else a.acc[i0 + u] = 0;
            }
        }
#pragma unroll
        for (int u = 0; u < RW; ++u) tmax = umax64(tmax, val[u]);
        // exclusive max-scan over the tile: the threads' maxima within each
        // wave by shuffles, then the maxima of the waves before it (one LDS
        // exchange)
        uint64_t incl = tmax;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t o = shfl_up64(incl, d);
            if (lane >= (uint32_t)d) incl = umax64(incl, o);
        }
        if (lane == 63) wmax[w] = incl;
        __syncthreads();
        uint64_t pre = 0, tile_max = 0;
#pragma unroll
        for (uint32_t q = 0; q < REP_T / 64; ++q) {
            if (q < w) pre = umax64(pre, wmax[q]);
            tile_max = umax64(tile_max, wmax[q]);
        }
        __syncthreads();   // wmax is rewritten by the next tile
        const uint64_t below = shfl_up64(incl, 1);
        uint64_t excl = umax64(carry, lane ? umax64(below, pre) : pre);
        carry = umax64(carry, tile_max);
        // '^': a start is reported only at a line start or exactly at the
        // resume point R (recCheckLeftContext 0x402170), so a candidate that
        // touches the previous cluster's end belongs to that cluster
        // (with '^' a candidate at a region start is a head: R restarts
        // there -- the file's first position included, R = 0 before any
        // report, key == excl == 0 for pattern 0)
        bool head[RW];
#pragma unroll
        for (int u = 0; u < RW; ++u) {
            head[u] = valid[u] && !(anch ? key[u] < excl || (key[u] == excl && (key[u] & POS_MASK) != 0 &&
                                                              !rep_region_start(a, key[u] & POS_MASK))
                                         : key[u] < excl);
            excl = umax64(excl, val[u]);
        }
        // the next candidate a head: the walk below would stop at it (its
        // running maximum is this head's end), so it is skipped -- the
        // common case, the walk's dependent loads are not paid.  The next
        // thread's first candidate comes by a shuffle (lane 63: the walk).
        const bool nh0 = __shfl_down(head[0] ? 1 : 0, 1, 64) != 0 && lane < 63;
#pragma unroll
        for (int u = 0; u < RW; ++u) {
            if (!head[u]) continue;   // not a head: its head's walk writes it
            const uint64_t i = i0 + u;
            // head: every earlier report ends before it (R < its start)
            const uint64_t s0 = key[u] & POS_MASK;
            const bool first = !anch || rep_line_start(a, s0);
            uint8_t kept = first && rep_keep(a, key[u]) ? 1 : 0;
            a.acc[i] = kept;
            own += kept;
            const bool next_head = u + 1 < RW ? head[u + 1 < RW ? u + 1 : u] : nh0;
            if (!anch && next_head) continue;
            uint64_t R = first ? s0 + len[u] : s0 - 1, run = val[u];   // s0 - 1: below every start of the cluster
            for (uint64_t j = i + 1; j < total; ++j) {
                const uint64_t kj = a.keys[j];
                if (anch ? kj > run || (kj == run && rep_region_start(a, kj & POS_MASK)) : kj >= run) break;  // the next head
                const uint32_t lj = rep_len(a, j, kj);
                kept = 0;
                const bool nj = rep_near(a, kj);
                if (rep_valid(a, kj, lj, nj)) {
                    const uint64_t sj = kj & POS_MASK;
                    if (sj >= R && (!anch || sj == R || rep_line_start(a, sj))) {
                        R = sj + lj;
                        kept = rep_keep(a, kj) ? 1 : 0;
                    }
                    run = umax64(run, rep_val(a, kj, lj, nj));
                }
                a.acc[j] = kept;
                if (kept) {
                    if (j < b1) ++own;
                    else atomicAdd(&a.bcnt[j / C], 1u);   // a cluster running into a later chunk (rare)
                }
            }
        }
    }
    own = block_sum(own, red);
    if (threadIdx.x == 0 && own) atomicAdd(&a.bcnt[blockIdx.x], (uint32_t)own);
}

__global__ __launch_bounds__(REP_T) void k_rep_scatter(RepArgs a) {
    __shared__ uint64_t red[REP_T / 64];
    __shared__ uint32_t scan[REP_T / 64];
    const uint64_t total = rep_total(a), C = rep_chunk(total, gridDim.x);
    uint64_t base_out = 0;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += REP_T) base_out += a.bcnt[b];
    base_out = block_sum(base_out, red);
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
        const uint32_t cnt = (uint32_t)(base_out + a.bcnt[blockIdx.x]);
        *a.count = cnt;
        if (a.host_count) {
            *a.host_count = cnt;
            __threadfence_system();
        }
    }
    const uint64_t b0 = blockIdx.x * C, b1 = umin64(total, b0 + C);
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint8_t nacc = b0 + threadIdx.x < b1 ? a.acc[b0 + threadIdx.x] : 0;   // the next tile's flags in flight
    for (uint64_t base = b0; base < b1; base += REP_T) {
        const uint64_t i = base + threadIdx.x;
        const bool keep = i < b1 && (nacc & 1);   // bit 1: a cluster head (k_es_walk)
        nacc = i + REP_T < b1 ? a.acc[i + REP_T] : 0;
        // the kept entries before this one: a wave ballot, then the counts
        // of the waves before it (one LDS exchange).  (Four consecutive
        // entries per thread measured slower: 251 vs 141 us on configs[4].)
        const uint64_t m = __builtin_amdgcn_ballot_w64(keep);
        if (lane == 0) scan[w] = (uint32_t)__builtin_popcountll(m);
        __syncthreads();
        uint32_t pre = 0, tile = 0;
#pragma unroll
        for (uint32_t q = 0; q < REP_T / 64; ++q) {
            if (q < w) pre += scan[q];
            tile += scan[q];
        }
        __syncthreads();
        if (keep) {
            const uint64_t o = base_out + pre + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            const uint64_t k = a.keys[i];
            a.okeys[o] = k;
            a.olens[o] = rep_len(a, i, k);
        }
        base_out += tile;
    }
}

// old key/len buffers of a hit list: recycled once the pass that reads them
// has run (an event-tracked shell on the deferred list)
void retire_buffers(pm_hits* h, hipStream_t s) {
    pm_hits* old = new pm_hits();
    old->device = h->device;
    old->keys = h->keys;
    old->lens = h->lens;
    old->keys_cap = h->keys_cap;
    old->lens_cap = h->lens_cap;
    HIPCHK(hipEventCreateWithFlags(&old->ready, hipEventDisableTiming));
    HIPCHK(hipEventRecord(old->ready, s));
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_deferred.push_back(old);
}

}  // namespace

TextView text_view(const pm_db* db) {
    return TextView{nuc_view(db), db->bytes, db->bytes_raw, db->n, db->alphabet == PM_ALPHA_NUC ? 1 : 0, db->hflag,
                    Regions{db->reg_t, db->reg_e, db->reg_lut, db->reg_near, db->nreg}};
}

bool report_needed(const pm_db* db, uint32_t flags, bool cross) {
    // several search regions: windows over a region end are dropped
    return (flags & (PM_REPORT_NRGREP | PM_ANCHOR_START | PM_ANCHOR_END)) || cross || db->nreg > 1;
}

ReportWs report_ws(pm_db* db, uint64_t cap_items) {
    Carve c;
    // the walk-list counter right after the total: the sort that writes the
    // device-side total zeroes it too (k_sort_bins)
    const size_t o_t = c.take(16), o_wc = o_t + 8, o_c = c.take(8), o_m = c.take(REP_G_MAX * 8),
                 o_b = c.take(REP_G_MAX * 4), o_w = c.take(std::max<uint64_t>(cap_items, 1) * 4),
                 o_a = c.take(std::max<uint64_t>(cap_items, 1));
    uint8_t* d = static_cast<uint8_t*>(reserve(db, db->ws_rep, c.off));
    ReportWs ws;
    ws.total = reinterpret_cast<uint64_t*>(d + o_t);
    ws.count = reinterpret_cast<uint32_t*>(d + o_c);
    ws.bmax = reinterpret_cast<uint64_t*>(d + o_m);
    ws.bcnt = reinterpret_cast<uint32_t*>(d + o_b);
    ws.acc = d + o_a;
    ws.wlist = reinterpret_cast<uint32_t*>(d + o_w);
    ws.wcount = reinterpret_cast<uint32_t*>(d + o_wc);
    ws.cap = std::max<uint64_t>(cap_items, 1);
    return ws;
}

void report_enqueue_ws(pm_db* db, pm_hits* h, uint32_t flags, const ReportWs& ws, bool total_on_device,
                       uint64_t total_h, uint32_t* host_count, hipStream_t s, hipEvent_t done, bool hdr,
                       const EsPrep* es, const XtPrep* xt) {
    // acc is indexed below the list length, which never exceeds the
    // capacity the workspace was sized for (the sort's slot capacities)
    const uint64_t cap_items = std::min<uint64_t>(h->keys_cap / 8, ws.cap);
    RepArgs a{};
    a.keys = h->keys;
    a.lens = h->lens;
    a.plen = h->plen;
    require(!h->plen || (!es && !xt), "internal: lens by pattern only for the generic report");
    size_t kc = 0, lc = 0;
    a.okeys = static_cast<uint64_t*>(pool_get(h->device, h->keys_cap, &kc));
    a.olens = static_cast<uint32_t*>(pool_get(h->device, h->lens_cap, &lc));
    a.acc = ws.acc;
    a.bmax = ws.bmax;
    a.bcnt = ws.bcnt;
    a.total_d = total_on_device ? ws.total : nullptr;
    a.total_h = total_h;
    a.count = ws.count;
    a.host_count = host_count;
    a.tv = text_view(db);
    // Regions cut after a '\n': a line-bounded match never reaches one, and
    // '^' never starts on the '\n' a region starts at -- only the simple
    // engine's windows (hdr) and blind cuts need the region checks
    if (!hdr && !db->reg_blind) a.tv.reg.n = 0;
    a.flags = flags;
    a.hdr = hdr && !(flags & PM_KEEP_HEADERS) ? 1 : 0;
    (void)cap_items;   // every acc entry below the list length is written by k_rep_walk (no memset)
    // chunks: REP_G, more for long lists (a big batch's tens of millions of
    // candidates: every block's serial tile scans then stay short)
    const uint32_t G = (uint32_t)std::min<uint64_t>(REP_G_MAX, std::max<uint64_t>(REP_G, ws.cap / 16384));
    if (es && (flags & PM_REPORT_NRGREP)) {
        // nrgrep's esimple engine: its own candidate order and verify
        es_launch(*es, h->keys, h->lens, a.total_d, a.total_h, a.acc, ws.wlist, ws.wcount, a.bcnt, G, a.tv, s);
    } else if (xt && (flags & PM_REPORT_NRGREP)) {
        // nrgrep's extended engine (k = 0): its scanners and checkMatch; it
        // reads the file's own bytes, regions included
        xt_launch(*xt, h->keys, h->lens, a.total_d, a.total_h, a.acc, a.bcnt, G, text_view(db), s);
    } else {
        if (h->plen && !(flags & (PM_ANCHOR_START | PM_ANCHOR_END)) && (flags & PM_REPORT_NRGREP))
            HIPCHK(hipMemsetAsync(a.bcnt, 0, G * sizeof(uint32_t), s));   // rep_monotone: no k_rep_max
        else
            hipLaunchKernelGGL(k_rep_max, dim3(G), dim3(REP_T), 0, s, a);
        hipLaunchKernelGGL(k_rep_walk, dim3(G), dim3(REP_T), 0, s, a);
    }
    if (done)
        hipExtLaunchKernelGGL(k_rep_scatter, dim3(G), dim3(REP_T), 0, s, nullptr, done, 0u, a);
    else
        hipLaunchKernelGGL(k_rep_scatter, dim3(G), dim3(REP_T), 0, s, a);
    HIPCHK(hipGetLastError());
    if (done && !h->old_keys && !h->old_lens) {
        // the pass's own completion event covers the old buffers: no event
        // record (a marker packet, ~10 us before the next scan starts)
        h->old_keys = h->keys;
        h->old_lens = h->lens;
        h->old_keys_cap = h->keys_cap;
        h->old_lens_cap = h->lens_cap;
    } else {
        retire_buffers(h, s);
    }
    h->keys = a.okeys;
    h->lens = a.olens;
    h->plen = nullptr;   // the pass wrote every kept length
    h->keys_cap = kc;
    h->lens_cap = lc;
}

void report_sync(pm_db* db, pm_hits* h, uint32_t flags, uint64_t total, bool hdr, const EsPrep* es,
                 const XtPrep* xt) {
    if (total == 0) {
        h->count = 0;
        h->plen = nullptr;
        return;
    }
    const ReportWs ws = report_ws(db, h->keys_cap / 8);
    report_enqueue_ws(db, h, flags, ws, false, total, nullptr, db->stream, nullptr, hdr, es, xt);
    uint32_t* hc = static_cast<uint32_t*>(reserve_host(db, db->pin_down, 8));
    HIPCHK(hipMemcpyAsync(hc, ws.count, 4, hipMemcpyDeviceToHost, db->stream));
    HIPCHK(hipStreamSynchronize(db->stream));
    h->count = *hc;
}

}  // namespace pm

pm_pending::~pm_pending() {
    if (counted) pm::quiet(hipEventDestroy(counted));
    pm::pinned_put(counts_h, counts_cap);
}

using namespace pm;

extern "C" {

int pm_hits_count(const pm_hits* h, uint64_t* count) {
    return guarded([&] {
        require(h != nullptr && count != nullptr, "null argument");
        hits_finalize(const_cast<pm_hits*>(h));
        *count = h->count;
    });
}

int pm_hits_copy(const pm_hits* h, int32_t* pattern, int64_t* beg, int64_t* end, uint64_t max_count) {
    return guarded([&] {
        require(h != nullptr, "hits is NULL");
        hits_finalize(const_cast<pm_hits*>(h));
        const uint64_t n = std::min<uint64_t>(h->count, max_count);
        if (n == 0) return;
        DeviceGuard g(h->device);
        std::vector<uint64_t> keys(n);
        std::vector<uint32_t> lens(n);
        if (h->ready) HIPCHK(hipEventSynchronize(h->ready));
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
        hits_finalize(const_cast<pm_hits*>(h));
        const uint64_t n = std::min<uint64_t>(h->count, max_count);
        if (n == 0) return;
        DeviceGuard g(h->device);
        hipStream_t s = (hipStream_t)stream;
        if (h->ready && s) HIPCHK(hipStreamWaitEvent(s, h->ready, 0));
        if (h->ready && !s) HIPCHK(hipEventSynchronize(h->ready));
        if (keys_dst) HIPCHK(hipMemcpyAsync(keys_dst, h->keys, n * 8, hipMemcpyDeviceToDevice, s));
        if (lens_dst) HIPCHK(hipMemcpyAsync(lens_dst, h->lens, n * 4, hipMemcpyDeviceToDevice, s));
        if (!stream) {
            HIPCHK(hipStreamSynchronize(s));
        } else {   // pm_hits_destroy waits for this copy before recycling the buffers
            pm_hits* hm = const_cast<pm_hits*>(h);
            if (!hm->last_use) HIPCHK(hipEventCreateWithFlags(&hm->last_use, hipEventDisableTiming));
            HIPCHK(hipEventRecord(hm->last_use, s));
        }
    });
}

int pm_hits_record_use(const pm_hits* h, void* stream) {
    return guarded([&] {
        require(h != nullptr, "hits is NULL");
        DeviceGuard g(h->device);
        pm_hits* hm = const_cast<pm_hits*>(h);
        if (!hm->last_use) HIPCHK(hipEventCreateWithFlags(&hm->last_use, hipEventDisableTiming));
        HIPCHK(hipEventRecord(hm->last_use, (hipStream_t)stream));
    });
}

int pm_hits_kernel_ms(const pm_hits* h, double* ms) {
    return guarded([&] {
        require(h != nullptr && ms != nullptr, "null argument");
        hits_finalize(const_cast<pm_hits*>(h));
        *ms = h->kernel_ms;
    });
}

int pm_hits_device(const pm_hits* h, void** keys, void** lens, uint64_t* count) {
    return guarded([&] {
        require(h != nullptr, "hits is NULL");
        hits_finalize(const_cast<pm_hits*>(h));
        DeviceGuard g(h->device);
        if (h->ready) HIPCHK(hipEventSynchronize(h->ready));   // the pointers are read by foreign streams
        if (keys) *keys = h->keys;
        if (lens) *lens = h->lens;
        if (count) *count = h->count;
    });
}

int pm_hits_destroy(pm_hits* h) {
    return guarded([&] {
        if (!h) return;
        DeviceGuard g(h->device);
        // the producing stream's work and any async copy out must be done
        // before the buffers go back to the pool: recycled now if they are,
        // else by a later pool_get / pm_hits_destroy (the host never waits)
        if (h->pending) {   // never resolved: no re-run
            std::lock_guard<std::recursive_mutex> lk(h->pending->db->mu);
            h->pending->db->pending.erase(h);
        }
        if (hits_idle(h)) {
            release_hits(h);
        } else {
            std::lock_guard<std::mutex> lk(g_pool_mu);
            g_deferred.push_back(h);
        }
        sweep_deferred();
    });
}

}  // extern "C"
