// Which call leaves a status on the thread that a later hipGetLastError()
// picks up?  Round 5's GPU suite failed once with "operation not permitted
// when stream is capturing" (hipErrorStreamCaptureUnsupported) in a launch
// check, with no stream capture anywhere in the library or the tests.  This
// probe runs the HIP and rocPRIM/hipCUB calls the library makes, on a
// non-blocking stream and on the null stream, and prints the thread's status
// (hipPeekAtLastError, then cleared) after each; then it checks whether a
// successful HIP call resets an earlier error (HIP_RETURN semantics).
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/micro/status_probe tools/micro/status_probe.hip
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>

#include <cstdint>
#include <cstdio>

static int report(const char* what, hipError_t rc) {
    const hipError_t st = hipPeekAtLastError();
    printf("%-58s rc=%-4d status=%-4d %s\n", what, (int)rc, (int)st, st == hipSuccess ? "" : hipGetErrorString(st));
    (void)hipGetLastError();
    return st != hipSuccess;
}

int main() {
    int bad = 0;
    hipStream_t ns = nullptr;
    hipStreamCreateWithFlags(&ns, hipStreamNonBlocking);
    report("hipStreamCreateWithFlags(nonblocking)", hipSuccess);
    const int n = 1 << 20;
    uint64_t *a = nullptr, *b = nullptr;
    hipMalloc(&a, n * 8);
    hipMalloc(&b, n * 8);
    hipMemset(a, 0x5a, n * 8);
    report("hipMalloc + hipMemset", hipSuccess);
    for (int pass = 0; pass < 2; ++pass) {
        hipStream_t s = pass ? nullptr : ns;
        printf("--- %s stream\n", pass ? "null" : "non-blocking");
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        bad += report("hipStreamIsCapturing", hipStreamIsCapturing(s, &cs));
        bad += report("hipGetStreamDeviceId", hipGetStreamDeviceId(s) >= 0 ? hipSuccess : hipErrorInvalidHandle);
        hipDeviceProp_t p;
        bad += report("hipGetDeviceProperties", hipGetDeviceProperties(&p, 0));
        int v = 0;
        bad += report("hipDeviceGetAttribute(warpSize)", hipDeviceGetAttribute(&v, hipDeviceAttributeWarpSize, 0));
        size_t sb = 0;
        bad += report("hipcub::DeviceRadixSort::SortKeys (size query)",
                      hipcub::DeviceRadixSort::SortKeys(nullptr, sb, a, b, n, 0, 64, s));
        void* ws = nullptr;
        hipMalloc(&ws, sb);
        bad += report("hipcub::DeviceRadixSort::SortKeys", hipcub::DeviceRadixSort::SortKeys(ws, sb, a, b, n, 0, 64, s));
        bad += report("hipStreamSynchronize", hipStreamSynchronize(s));
        size_t mb = 0;
        bad += report("rocprim::merge (size query)", rocprim::merge(nullptr, mb, a, a, b, n / 2, n / 2,
                                                                     rocprim::less<uint64_t>(), s));
        void* mw = nullptr;
        hipMalloc(&mw, mb + 8);
        bad += report("rocprim::merge", rocprim::merge(mw, mb, a, a, b, n / 2, n / 2, rocprim::less<uint64_t>(), s));
        size_t xb = 0;
        bad += report("hipcub::DeviceScan::ExclusiveSum (size query)",
                      hipcub::DeviceScan::ExclusiveSum(nullptr, xb, a, b, n, s));
        void* xw = nullptr;
        hipMalloc(&xw, xb + 8);
        bad += report("hipcub::DeviceScan::ExclusiveSum", hipcub::DeviceScan::ExclusiveSum(xw, xb, a, b, n, s));
        bad += report("hipStreamSynchronize", hipStreamSynchronize(s));
        hipFree(ws);
        hipFree(mw);
        hipFree(xw);
    }
    // does a successful call reset an earlier, unread error?
    printf("--- HIP_RETURN semantics\n");
    const hipError_t e = hipSetDevice(4096);
    printf("hipSetDevice(4096) rc=%d\n", (int)e);
    hipStreamSynchronize(ns);
    const hipError_t after = hipGetLastError();
    printf("after a successful hipStreamSynchronize: hipGetLastError()=%d (%s): %s\n", (int)after,
           hipGetErrorString(after), after == hipSuccess ? "a successful call resets the status"
                                                         : "the error stays until read");
    // how a caller can leave hipErrorStreamCaptureUnsupported pending on
    // purpose (for the C-ABI test of guarded()): a capture-unsafe call while
    // a stream captures in global mode, the status read only at the end
    printf("--- capture sequences (status not cleared between steps)\n");
    (void)hipGetLastError();
    for (int form = 0; form < 3; ++form) {
        hipStream_t cs = nullptr;
        hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);
        (void)hipGetLastError();
        hipError_t r1 = hipStreamBeginCapture(cs, hipStreamCaptureModeGlobal);
        hipError_t st1 = hipPeekAtLastError();
        void* p = nullptr;
        hipError_t r2 = form == 0 ? hipMalloc(&p, 64) : form == 1 ? hipStreamSynchronize(cs) : hipDeviceSynchronize();
        hipError_t st2 = hipPeekAtLastError();
        hipGraph_t g = nullptr;
        hipError_t r3 = hipStreamEndCapture(cs, &g);
        hipError_t st3 = hipPeekAtLastError();
        hipError_t r4 = hipStreamSynchronize(ns);
        hipError_t st4 = hipPeekAtLastError();
        printf("form %d (%s): begin rc=%d st=%d | call rc=%d st=%d | end rc=%d st=%d | sync rc=%d st=%d\n", form,
               form == 0 ? "hipMalloc" : form == 1 ? "hipStreamSynchronize(capturing)" : "hipDeviceSynchronize",
               (int)r1, (int)st1, (int)r2, (int)st2, (int)r3, (int)st3, (int)r4, (int)st4);
        (void)hipGetLastError();
        if (g) hipGraphDestroy(g);
        if (p) hipFree(p);
        hipStreamDestroy(cs);
        (void)hipGetLastError();
    }
    hipFree(a);
    hipFree(b);
    hipStreamDestroy(ns);
    printf("probe: %d calls left a status\n", bad);
    return 0;
}
