// Copy-in of a small synchronous call's inputs (product code).
//
// l7g_classify_host with a handful of requests (the Envoy adapter's
// Allowed(), one proxylib OnData) is latency: the classifiers reading the
// inputs from pinned host memory in place would pay a PCIe round trip for
// every dependent read their framers make (the one-request HTTP kernel took
// 14-28 us that way).  This kernel moves the call's input pieces -- offsets,
// lengths, connections, request bytes -- into device memory with one
// coalesced read over PCIe per 16 KiB, all loads in flight before the first
// store; the classifiers that follow on the stream then read HBM.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "copy_in_types.h"
#include "gmem.h"

namespace l7 {

namespace {
constexpr int kBlock = 1024;
constexpr int kPer = 4;  // 16-byte units per thread per round: 64 KiB in flight per round
}  // namespace

__global__ __launch_bounds__(kBlock) void copy_in_kernel(CopyIn c) {
    for (int k = 0; k < c.n; k++) {
        const uint64_t units = (c.p[k].bytes + 15) / 16;
        const uint4 *s = reinterpret_cast<const uint4 *>(c.p[k].src);
        uint4 *d = reinterpret_cast<uint4 *>(c.p[k].dst);
        for (uint64_t u0 = (uint64_t)blockIdx.x * kBlock * kPer; u0 < units; u0 += (uint64_t)gridDim.x * kBlock * kPer) {
            uint4 v[kPer];
#pragma unroll
            for (int j = 0; j < kPer; j++) {
                const uint64_t u = u0 + (uint64_t)j * kBlock + threadIdx.x;
                if (u < units) v[j] = gload16((uint64_t)(uintptr_t)(s + u));
            }
#pragma unroll
            for (int j = 0; j < kPer; j++) {
                const uint64_t u = u0 + (uint64_t)j * kBlock + threadIdx.x;
                if (u < units) d[u] = v[j];
            }
        }
    }
}

hipError_t LaunchCopyIn(const CopyIn &c, hipStream_t stream) {
    uint64_t units = 0;
    for (int k = 0; k < c.n; k++) units = units > (c.p[k].bytes + 15) / 16 ? units : (c.p[k].bytes + 15) / 16;
    if (units == 0) return hipSuccess;
    uint32_t blocks = (uint32_t)((units + kBlock * kPer - 1) / (kBlock * kPer));
    if (blocks > 64) blocks = 64;
    hipLaunchKernelGGL(copy_in_kernel, dim3(blocks), dim3(kBlock), 0, stream, c);
    return hipGetLastError();
}

}  // namespace l7
