// pm_merge.hip -- the serving rank's merge of the ranks' hit lists
// (pm_merge_parts), on the device.
//
// The reference prints one process's hits per strand in file order
// (www/FlaskApp/FlaskApp/patmatch.py:733-743); sharded by record over the
// GPUs of a node (shards.py), every rank's list is sorted by key (pattern
// << 48 | node-wide position) and covers its own increasing position range,
// so the node-wide order is, pattern by pattern, the ranks' slices in rank
// order: no sort.  Three launches: the (part, pattern) slice starts by
// binary search, their destinations by one block's scan over the patterns,
// and one pass that moves every key (and its length, or the pattern's fixed
// length) to its place.  Round 6: this replaced a torch formulation
// (searchsorted, repeat_interleave, two scatters: 35 ms for 8 x 30.7 M keys,
// tools/merge_cost.py) with ~one read and one write of the list.
#include "pm_internal.h"

namespace pm {
namespace {

constexpr int MERGE_MAX_PARTS = 64;
constexpr uint32_t MERGE_T = 1024;

struct Parts {
    uint64_t beg[MERGE_MAX_PARTS];   // part r = keys[beg[r], beg[r] + len[r])
    uint64_t len[MERGE_MAX_PARTS];
    uint32_t blk0[MERGE_MAX_PARTS + 1];   // prefix of the move's blocks per part
    int n;
};

// start[r * (P + 1) + p] = absolute index of part r's first key of pattern >= p
__global__ void k_merge_starts(const uint64_t* __restrict__ keys, Parts parts, uint32_t P, uint64_t* __restrict__ start) {
    const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (g >= (uint64_t)parts.n * (P + 1)) return;
    const int r = (int)(g / (P + 1));
    const uint32_t p = (uint32_t)(g % (P + 1));
    const uint64_t want = (uint64_t)p << 48;
    uint64_t lo = 0, hi = parts.len[r];
    const uint64_t* k = keys + parts.beg[r];
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (k[mid] < want) lo = mid + 1; else hi = mid;
    }
    start[g] = parts.beg[r] + lo;
}

// base[r * P + p] = destination of part r's pattern-p slice minus its start:
// every earlier pattern's keys (all parts), then pattern p's keys of the
// parts before r.  One block; patterns in contiguous runs per thread.
__global__ __launch_bounds__(MERGE_T) void k_merge_bases(const uint64_t* __restrict__ start, Parts parts, uint32_t P,
                                                        int64_t* __restrict__ base) {
    __shared__ uint64_t s_sum[MERGE_T];
    const uint32_t per = (P + MERGE_T - 1) / MERGE_T;
    const uint32_t p0 = min(P, threadIdx.x * per), p1 = min(P, p0 + per);
    uint64_t own = 0;
    for (uint32_t p = p0; p < p1; ++p)
        for (int r = 0; r < parts.n; ++r) own += start[r * (P + 1) + p + 1] - start[r * (P + 1) + p];
    s_sum[threadIdx.x] = own;
    __syncthreads();
    for (uint32_t d = 1; d < MERGE_T; d <<= 1) {   // inclusive scan (Hillis-Steele)
        const uint64_t v = threadIdx.x >= d ? s_sum[threadIdx.x - d] : 0;
        __syncthreads();
        s_sum[threadIdx.x] += v;
        __syncthreads();
    }
    uint64_t run = s_sum[threadIdx.x] - own;   // keys of every pattern before p0
    for (uint32_t p = p0; p < p1; ++p) {
        for (int r = 0; r < parts.n; ++r) {
            const uint64_t s = start[r * (P + 1) + p];
            base[r * P + p] = (int64_t)run - (int64_t)s;
            run += start[r * (P + 1) + p + 1] - s;
        }
    }
}

// The move: a block takes MOVE_KEYS consecutive keys of ONE part (its part
// from the blocks' prefix, blk0, wave-uniform), stages that part's base row
// and the pattern lengths in LDS when the batch has <= MOVE_STAGE_P
// patterns, and each thread moves MOVE_PER keys at stride MOVE_T: the loads
// and (within a pattern's slice) the stores coalesce, and each thread has
// MOVE_PER independent loads in flight.  (Round 6's first form, one thread
// per key with a per-key search over the parts' prefix: 1.71 ms for 8 x
// 30.7 M keys, ~2.9 TB/s of its 4.9 GB.)
constexpr uint32_t MOVE_T = 256, MOVE_PER = 8, MOVE_KEYS = MOVE_T * MOVE_PER;
constexpr uint32_t MOVE_STAGE_P = 512;    // (a block re-reads the staged row: 4 KB at most)

template <bool STAGE>
__global__ __launch_bounds__(MOVE_T) void k_merge_move(const uint64_t* __restrict__ keys, const int32_t* __restrict__ lens,
                                                       Parts parts, uint32_t P, const int64_t* __restrict__ base,
                                                       const int32_t* __restrict__ len_of, uint64_t* __restrict__ out_keys,
                                                       int32_t* __restrict__ out_lens) {
    __shared__ int64_t s_base[STAGE ? MOVE_STAGE_P : 1];
    __shared__ int32_t s_len[STAGE ? MOVE_STAGE_P : 1];
    int r = 0;
    while (r + 1 < parts.n && blockIdx.x >= parts.blk0[r + 1]) ++r;   // block-uniform
    const uint64_t c0 = (uint64_t)(blockIdx.x - parts.blk0[r]) * MOVE_KEYS;
    const uint64_t n = parts.len[r] > c0 ? umin64(parts.len[r] - c0, MOVE_KEYS) : 0;
    const int64_t* brow = base + (uint64_t)r * P;
    if constexpr (STAGE) {
        for (uint32_t p = threadIdx.x; p < P; p += MOVE_T) {
            s_base[p] = brow[p];
            if (out_lens && !lens) s_len[p] = len_of[p];
        }
        __syncthreads();
    }
    const uint64_t i0 = parts.beg[r] + c0;
    uint64_t k[MOVE_PER];
#pragma unroll
    for (uint32_t u = 0; u < MOVE_PER; ++u) {
        const uint64_t q = threadIdx.x + (uint64_t)u * MOVE_T;
        k[u] = q < n ? keys[i0 + q] : ~0ull;
    }
#pragma unroll
    for (uint32_t u = 0; u < MOVE_PER; ++u) {
        const uint64_t q = threadIdx.x + (uint64_t)u * MOVE_T;
        const uint32_t p = (uint32_t)(k[u] >> 48);
        if (q >= n || p >= P) continue;   // (p >= P: the caller's pattern count is too small, checked on the host)
        const uint64_t i = i0 + q;
        const uint64_t dst = (uint64_t)((STAGE ? s_base[p] : brow[p]) + (int64_t)i);
        out_keys[dst] = k[u];
        if (out_lens) out_lens[dst] = lens ? lens[i] : (STAGE ? s_len[p] : len_of[p]);
    }
}

}  // namespace
}  // namespace pm

using namespace pm;

extern "C" {

int pm_merge_parts(const uint64_t* keys, const int32_t* lens, const uint64_t* part_beg, const uint64_t* part_len,
                   int nparts, int n_patterns, const int32_t* len_of_pattern, uint64_t* out_keys, int32_t* out_lens,
                   void* work, uint64_t* work_bytes, int device, void* stream) {
    return guarded([&] {
        require(nparts >= 1 && nparts <= MERGE_MAX_PARTS, "pm_merge_parts: 1..64 parts");
        require(n_patterns >= 1 && n_patterns <= 65536, "pm_merge_parts: 1..65536 patterns");
        require(work_bytes != nullptr, "work_bytes is NULL");
        const uint32_t P = (uint32_t)n_patterns;
        const size_t o_start = 0;
        const size_t o_base = o_start + (size_t)nparts * (P + 1) * 8;
        const size_t need = o_base + (size_t)nparts * P * 8;
        if (work == nullptr) {   // size query
            *work_bytes = need;
            return;
        }
        require(*work_bytes >= need, "pm_merge_parts: workspace too small");
        require(part_beg && part_len, "part_beg / part_len is NULL");
        require(out_keys != nullptr, "out_keys is NULL");
        require(!out_lens || lens || len_of_pattern, "out_lens needs lens or len_of_pattern");
        Parts parts{};
        parts.n = nparts;
        uint64_t total = 0, blocks = 0;
        for (int r = 0; r < nparts; ++r) {
            parts.beg[r] = part_beg[r];
            parts.len[r] = part_len[r];
            parts.blk0[r] = (uint32_t)blocks;
            total += part_len[r];
            blocks += (part_len[r] + MOVE_KEYS - 1) / MOVE_KEYS;
        }
        parts.blk0[nparts] = (uint32_t)blocks;
        require(blocks < (1ull << 31), "pm_merge_parts: too many keys");
        if (total == 0) return;
        require(keys != nullptr, "keys is NULL");
        DeviceGuard g(device);
        hipStream_t s = (hipStream_t)stream;
        uint8_t* w = static_cast<uint8_t*>(work);
        uint64_t* start = reinterpret_cast<uint64_t*>(w + o_start);
        int64_t* base = reinterpret_cast<int64_t*>(w + o_base);
        const uint64_t ns = (uint64_t)nparts * (P + 1);
        hipLaunchKernelGGL(k_merge_starts, dim3(blocks_for(ns, 256)), dim3(256), 0, s, keys, parts, P, start);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(k_merge_bases, dim3(1), dim3(MERGE_T), 0, s, start, parts, P, base);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(P <= MOVE_STAGE_P ? k_merge_move<true> : k_merge_move<false>, dim3((uint32_t)blocks),
                           dim3(MOVE_T), 0, s, keys, lens, parts, P, base, len_of_pattern, out_keys, out_lens);
        HIPCHK(hipGetLastError());
        if (!stream) HIPCHK(hipStreamSynchronize(s));
    });
}

}  // extern "C"
