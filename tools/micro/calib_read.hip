// FETCH_SIZE calibration: known-byte streaming reads in the two access forms
// the scan kernels use, for `rocprofv3 --pmc FETCH_SIZE` (MI355X_MICROARCH.md
// "HBM": FETCH_SIZE = TCC_EA0_RDREQ x 64 B; calibrate on your own pattern).
//   k_read_dwordx4 : global_load_dwordx4, 16 B per lane, grid-stride
//   k_read_lds_dma : global_load_lds_dwordx4, 1 KiB per wave-instruction into
//                    LDS (pm_linear_jit's tile staging)
// Each kernel reads exactly BYTES bytes once per launch (3 launches each).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/calib_read tools/micro/calib_read.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ __launch_bounds__(256) void k_read_dwordx4(const uint4* __restrict__ src, uint64_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;   // never true for the fill used: keeps the loads
}

// one wave per 1 KiB piece, pieces grid-strided; 256 threads = 4 waves
__global__ __launch_bounds__(256) void k_read_lds_dma(const unsigned char* __restrict__ src, uint64_t npieces,
                                                      uint32_t* sink) {
    __shared__ __attribute__((aligned(1024))) unsigned char lds[4 * 1024];
    const int lane = threadIdx.x & 63;
    const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t lds_base = (uint32_t)reinterpret_cast<uint64_t>(lds) + wid * 1024u;
    const uint32_t voff = (uint32_t)lane * 16u;
    uint32_t acc = 0;
    const uint64_t waves = (uint64_t)gridDim.x * 4;
    for (uint64_t q = blockIdx.x * 4ull + wid; q < npieces; q += waves) {
        const unsigned char* pb = src + q * 1024;
        const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_base);
        uint32_t keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(voff), "s"(pb), "s"(dst) : "memory");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc ^= reinterpret_cast<const uint32_t*>(lds + wid * 1024)[lane];
    }
    if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;
}

int main(int argc, char** argv) {
    const uint64_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 4096ull) << 20;   // MiB
    unsigned char* src = nullptr;
    uint32_t* sink = nullptr;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMalloc(&sink, 1 << 20));
    CHECK(hipMemset(src, 0x11, bytes));
    CHECK(hipDeviceSynchronize());
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(k_read_dwordx4, dim3(256 * 32), dim3(256), 0, 0, reinterpret_cast<const uint4*>(src), bytes / 16, sink);
        CHECK(hipGetLastError());
    }
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(k_read_lds_dma, dim3(256 * 32), dim3(256), 0, 0, src, bytes / 1024, sink);
        CHECK(hipGetLastError());
    }
    CHECK(hipDeviceSynchronize());
    printf("{\"bytes_per_launch\": %llu, \"launches_per_kernel\": 3}\n", (unsigned long long)bytes);
    CHECK(hipFree(src));
    CHECK(hipFree(sink));
    return 0;
}
