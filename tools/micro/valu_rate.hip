// Microbenchmark: VALU issue rate of candidate bit ops for the scan kernels
// (inline asm so the exact instruction runs), 8 independent chains per lane
// whose operands are all live chain registers, 8 waves/SIMD.  Prints
// lane-ops/s and cycles per wave-instruction per SIMD at the nominal 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define A3(ins) asm volatile(ins " %0, %1, %2, %3" : "=v"(a[i]) : "v"(a[i]), "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]))
#define A2(ins) asm volatile(ins " %0, %1, %2" : "=v"(a[i]) : "v"(a[i]), "v"(a[(i + 1) & 7]))
#define OPS(X)                                                                                      \
    X(0, "v_bitop3_b32 0x96", asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(a[i]) : "v"(a[i]), "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]))) \
    X(1, "v_bitop3_b32 0xe8", asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe8" : "=v"(a[i]) : "v"(a[i]), "v"(a[(i + 1) & 7]), "v"(a[(i + 2) & 7]))) \
    X(2, "v_or3_b32", A3("v_or3_b32"))                                                              \
    X(3, "v_bfi_b32", A3("v_bfi_b32"))                                                              \
    X(4, "v_and_or_b32", A3("v_and_or_b32"))                                                        \
    X(5, "v_xad_u32", A3("v_xad_u32"))                                                              \
    X(6, "v_add3_u32", A3("v_add3_u32"))                                                            \
    X(7, "v_lshl_or_b32", A3("v_lshl_or_b32"))                                                      \
    X(8, "v_alignbit_b32", A3("v_alignbit_b32"))                                                    \
    X(9, "v_xor_b32", A2("v_xor_b32"))                                                              \
    X(10, "v_or_b32", A2("v_or_b32"))                                                               \
    X(11, "v_and_b32", A2("v_and_b32"))                                                             \
    X(12, "v_bitop3_b32 0x96 (2 distinct)", asm volatile("v_bitop3_b32 %0, %1, %2, %2 bitop3:0x96" : "=v"(a[i]) : "v"(a[i]), "v"(a[(i + 1) & 7])))

template <int OP>
__global__ __launch_bounds__(256) void k(unsigned* out, unsigned seed, int iters) {
    unsigned a[8];
    for (int i = 0; i < 8; ++i) a[i] = seed * (threadIdx.x + 1) + i * 0x9e3779b9u;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#define CASE(n, name, stmt) if constexpr (OP == n) { stmt; }
            OPS(CASE)
#undef CASE
        }
    }
    unsigned r = 0;
    for (int i = 0; i < 8; ++i) r ^= a[i];
    if (r == 0x12345678u) out[0] = r;
}

static int g_wps = 8;   // blocks per CU = waves per SIMD (256-thread blocks)

template <int OP>
void run(const char* name, unsigned* out, hipEvent_t e0, hipEvent_t e1) {
    const int blocks = 256 * g_wps, iters = 4096;
    float ms = 0;
    for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        k<OP><<<blocks, 256>>>(out, 3, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
    }
    const double wave_instr = (double)blocks * 4 * iters * 8;
    printf("%-32s %.3f ms  %.1f Tlane-ops/s  %.2f cycles/wave-instr/SIMD @2.4GHz\n", name, ms,
           wave_instr * 64 / (ms * 1e-3) / 1e12, ms * 1e-3 * 2.4e9 / (wave_instr / 1024));
}

int main(int argc, char** argv) {
    if (argc > 1) g_wps = atoi(argv[1]);
    printf("waves per SIMD: %d\n", g_wps);
    unsigned* out;
    (void)hipMalloc(&out, 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
#define RUN(n, name, stmt) run<n>(name, out, e0, e1);
    OPS(RUN)
    return 0;
}
