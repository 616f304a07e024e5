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
    uint64_t out0[MERGE_MAX_PARTS + 1];   // prefix of len: part r's first compacted index
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

// one thread per key: part by the compacted prefix, destination = base of
// its (part, pattern) slice + its absolute index
__global__ void k_merge_move(const uint64_t* __restrict__ keys, const int32_t* __restrict__ lens, Parts parts,
                             uint32_t P, const int64_t* __restrict__ base, const int32_t* __restrict__ len_of,
                             uint64_t total, uint64_t* __restrict__ out_keys, int32_t* __restrict__ out_lens) {
    const uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (j >= total) return;
    int r = 0;
    while (r + 1 < parts.n && j >= parts.out0[r + 1]) ++r;
    const uint64_t i = parts.beg[r] + (j - parts.out0[r]);
    const uint64_t key = keys[i];
    const uint32_t p = (uint32_t)(key >> 48);
    if (p >= P) return;   // the caller's pattern count is too small: checked on the host
    const uint64_t dst = (uint64_t)(base[r * P + p] + (int64_t)i);
    out_keys[dst] = key;
    if (out_lens) out_lens[dst] = lens ? lens[i] : len_of[p];
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
        uint64_t total = 0;
        for (int r = 0; r < nparts; ++r) {
            parts.beg[r] = part_beg[r];
            parts.len[r] = part_len[r];
            parts.out0[r] = total;
            total += part_len[r];
        }
        parts.out0[nparts] = total;
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
        hipLaunchKernelGGL(k_merge_move, dim3(blocks_for(total, 256)), dim3(256), 0, s, keys, lens, parts, P, base,
                           len_of_pattern, total, out_keys, out_lens);
        HIPCHK(hipGetLastError());
        if (!stream) HIPCHK(hipStreamSynchronize(s));
    });
}

}  // extern "C"
