// Protocol split of a mixed batch (product code).
//
// l7g_classify launches one classifier per protocol present in the batch.
// The Kafka and memcached classifiers are one lane per request, so in a mixed
// stream (cfg5) most of their lanes would only discover "not my protocol" and
// idle while the others decode.  This kernel writes, for each of those two
// protocols, the list of request indices that belong to it; the classifiers
// then walk only their own list.  One block owns 4096 consecutive requests
// (16 per lane, protocol kept in registers between the count and the write
// pass) and takes its slot range with one atomic per protocol.
#include <hip/hip_runtime.h>

#include "../device_tables.h"

namespace l7 {

namespace {
constexpr int kBlock = 256;
constexpr int kPer = 16;
constexpr int kWaves = kBlock / 64;
}  // namespace

__global__ __launch_bounds__(kBlock) void partition_kernel(const uint32_t *__restrict__ conn_ids, uint32_t n,
                                                           const DevConn *__restrict__ conns, uint32_t nconns,
                                                           uint32_t *__restrict__ sel_kafka,
                                                           uint32_t *__restrict__ sel_mc,
                                                           uint32_t *__restrict__ counts) {
    __shared__ uint32_t s_off[kWaves][2];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t start = (uint64_t)blockIdx.x * (kBlock * kPer);
    const uint64_t below = (1ull << lane) - 1;
    uint8_t p[kPer];
    uint32_t ck = 0, cm = 0;
#pragma unroll
    for (int r = 0; r < kPer; r++) {
        const uint64_t idx = start + (uint64_t)r * kBlock + threadIdx.x;
        uint8_t proto = 0;
        if (idx < n) {
            const uint32_t ci = conn_ids[idx];
            if (ci < nconns) proto = conns[ci].proto;
        }
        p[r] = proto;
        ck += __popcll(__ballot(proto == PROTO_KAFKA));
        cm += __popcll(__ballot(proto == PROTO_MEMCACHE));
    }
    if (lane == 0) { s_off[wave][0] = ck; s_off[wave][1] = cm; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tk = 0, tm = 0;
        for (int w = 0; w < kWaves; w++) { tk += s_off[w][0]; tm += s_off[w][1]; }
        uint32_t bk = tk ? atomicAdd(&counts[0], tk) : 0, bm = tm ? atomicAdd(&counts[1], tm) : 0;
        for (int w = 0; w < kWaves; w++) {
            const uint32_t a = s_off[w][0], b = s_off[w][1];
            s_off[w][0] = bk; s_off[w][1] = bm;
            bk += a; bm += b;
        }
    }
    __syncthreads();
    uint32_t ok = s_off[wave][0], om = s_off[wave][1];
#pragma unroll
    for (int r = 0; r < kPer; r++) {
        const uint32_t idx = (uint32_t)(start + (uint64_t)r * kBlock + threadIdx.x);
        const uint64_t mk = __ballot(p[r] == PROTO_KAFKA), mm = __ballot(p[r] == PROTO_MEMCACHE);
        if (p[r] == PROTO_KAFKA) sel_kafka[ok + __popcll(mk & below)] = idx;
        if (p[r] == PROTO_MEMCACHE) sel_mc[om + __popcll(mm & below)] = idx;
        ok += __popcll(mk);
        om += __popcll(mm);
    }
}

// counts[0..1] must be zero on entry (the caller clears them on `stream`).
hipError_t LaunchPartition(const uint32_t *conn_ids, uint32_t n, const DevConn *conns, uint32_t nconns,
                           uint32_t *sel_kafka, uint32_t *sel_mc, uint32_t *counts, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)(((uint64_t)n + kBlock * kPer - 1) / (kBlock * kPer));
    hipLaunchKernelGGL(partition_kernel, dim3(blocks), dim3(kBlock), 0, stream, conn_ids, n, conns, nconns, sel_kafka,
                       sel_mc, counts);
    return hipGetLastError();
}

}  // namespace l7
