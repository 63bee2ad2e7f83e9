// Per-rule allow hits and per-verdict totals of one l7g_classify call
// (product code), counted after the classifiers from their outputs.
//
// The classifiers used to bump the counters themselves: one device-scope
// atomic per allowed request on its rule's counter.  Device-scope atomics on
// MI355X are performed past the (per-XCD, non-coherent) L2s, and a few
// thousand hot counters shared by every CU serialise there: on the 100M-entry
// mixed stream they cost ~15 ms per call, more than the Kafka kernel.  Here
// the outputs are re-read once (5 B per request, streamed) instead:
//   1. histogram_kernel: each workgroup histograms a contiguous slice of
//      rule[] into LDS (u32 bins; verdicts through wave ballots, not atomics)
//      and stores its bins to a [workgroup][bin] scratch matrix -- plain,
//      coalesced stores, no global atomics;
//   2. reduce_kernel: one thread per bin sums its column and adds the sum to
//      the caller's u64 counter (one writer per counter, stream-ordered).
// Rule sets with more bins than fit in LDS are counted in bin ranges, one
// histogram pass per range.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../device_tables.h"

namespace l7 {

namespace {

constexpr int kHistBlock = 1024;
constexpr uint32_t kHistBins = 16384;  // u32 bins per LDS pass (64 KiB)
constexpr uint32_t kHistBlocks = 256;  // workgroups (one per CU)

// One rule bin per lane (key = bin index, ~0u = none) into the LDS bins.
// Lanes hitting one bin in one ds_add serialise on it (a wave of allowed
// requests of one hot rule is 64 adds to one address), so the lanes that share
// the bin of the first lane with a key are added first as one count, twice
// over; whatever keys remain go in as single adds.
__device__ __forceinline__ void bin_add(uint32_t *bins, uint32_t key, uint32_t lane) {
#pragma unroll
    for (int round = 0; round < 2; round++) {
        const uint64_t act = __ballot(key != ~0u);
        if (!act) return;
        const uint32_t lead = (uint32_t)__builtin_ctzll(act);
        const uint32_t kl = (uint32_t)__builtin_amdgcn_readlane((int)key, (int)lead);
        const uint64_t same = __ballot(key == kl);
        if (lane == lead) atomicAdd(&bins[kl], (uint32_t)__popcll(same));
        if (key == kl) key = ~0u;
    }
    if (key != ~0u) atomicAdd(&bins[key], 1u);
}

// rule bins [lo, lo + nb) of this pass; verdict bins counted only when lo == 0.
// A thread takes 4 consecutive entries per step (one 16-byte load of rules, one
// 4-byte load of verdicts), two steps' loads in flight.
constexpr uint32_t kHistPer = 4;
__global__ __launch_bounds__(kHistBlock) void histogram_kernel(const uint8_t *__restrict__ verdict,
                                                               const int32_t *__restrict__ rule, uint32_t n,
                                                               uint32_t lo, uint32_t nb, uint32_t *__restrict__ scratch,
                                                               uint32_t stride) {
    __shared__ uint32_t bins[kHistBins + 8];
    for (uint32_t i = threadIdx.x; i < nb + 8; i += kHistBlock) bins[i] = 0;
    __syncthreads();
    // slices of whole 4-entry groups (16-byte aligned rule loads)
    const uint32_t ngroups = (n + kHistPer - 1) / kHistPer;
    const uint32_t per = (ngroups + gridDim.x - 1) / gridDim.x;
    const uint32_t g0 = blockIdx.x * per, g1 = min(ngroups, g0 + per);
    const uint32_t lane = threadIdx.x & 63;
    uint32_t vc[5] = {0, 0, 0, 0, 0};
    const bool aligned = ((uintptr_t)rule & 15) == 0;
    for (uint32_t gb = g0; gb < g1; gb += 2 * kHistBlock) {
        int4 rr[2];
        uint32_t vv[2];
        bool full[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t g = gb + u * kHistBlock + threadIdx.x;
            const uint32_t i = g * kHistPer;
            full[u] = g < g1 && i + kHistPer <= n;
            rr[u] = make_int4(-1, -1, -1, -1);
            vv[u] = 0xFFFFFFFFu;
            if (full[u] && aligned) {
                rr[u] = *reinterpret_cast<const int4 *>(rule + i);
                vv[u] = (uint32_t)verdict[i] | (uint32_t)verdict[i + 1] << 8 | (uint32_t)verdict[i + 2] << 16 |
                        (uint32_t)verdict[i + 3] << 24;
            } else if (full[u]) {  // (rule[] not 16-byte aligned: four dword loads)
                rr[u] = make_int4(rule[i], rule[i + 1], rule[i + 2], rule[i + 3]);
                vv[u] = (uint32_t)verdict[i] | (uint32_t)verdict[i + 1] << 8 | (uint32_t)verdict[i + 2] << 16 |
                        (uint32_t)verdict[i + 3] << 24;
            } else if (g < g1) {  // the batch's last, partial group
                int32_t t[4] = {-1, -1, -1, -1};
                uint32_t v = 0xFFFFFFFFu;
                for (uint32_t k = 0; k < kHistPer && i + k < n; k++) {
                    t[k] = rule[i + k];
                    v = (v & ~(0xFFu << (8 * k))) | (uint32_t)verdict[i + k] << (8 * k);
                }
                rr[u] = make_int4(t[0], t[1], t[2], t[3]);
                vv[u] = v;
            }
        }
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int32_t r4[4] = {rr[u].x, rr[u].y, rr[u].z, rr[u].w};
#pragma unroll
            for (int k = 0; k < (int)kHistPer; k++) {
                const int32_t r = r4[k];
                bin_add(bins, (uint32_t)(r - (int32_t)lo) < nb ? (uint32_t)(r - (int32_t)lo) : ~0u, lane);
                if (lo == 0) {
                    const uint32_t v = (vv[u] >> (8 * k)) & 0xFF;
#pragma unroll
                    for (uint32_t q = 0; q < 5; q++) vc[q] += (uint32_t)__popcll(__ballot(v == q));
                }
            }
        }
    }
    if (lo == 0 && lane == 0)
        for (uint32_t k = 0; k < 5; k++)
            if (vc[k]) atomicAdd(&bins[nb + k], vc[k]);
    __syncthreads();
    uint32_t *dst = scratch + (size_t)blockIdx.x * stride;
    for (uint32_t i = threadIdx.x; i < nb + 8; i += kHistBlock) dst[i] = bins[i];
}

// 64 bins per block; 4 threads per bin each sum a quarter of the rows with 8
// loads in flight, then LDS combines the quarters (the column sums used to be
// one thread per bin walking all rows serially: ~80 us of load latency)
constexpr int kRedBins = 64, kRedParts = 4;
__global__ __launch_bounds__(kRedBins * kRedParts) void reduce_kernel(const uint32_t *__restrict__ scratch,
                                                                     uint32_t nblocks, uint32_t stride, uint32_t lo,
                                                                     uint32_t nb, uint32_t nrules,
                                                                     uint64_t *__restrict__ counters) {
    __shared__ uint64_t part[kRedParts][kRedBins];
    const uint32_t t = threadIdx.x % kRedBins, q = threadIdx.x / kRedBins;
    const uint32_t b = blockIdx.x * kRedBins + t;
    const uint32_t nbins = nb + (lo == 0 ? 8 : 0);
    uint64_t s = 0;
    if (b < nbins) {
        uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        uint32_t k = q;
        for (; k + 7 * kRedParts < nblocks; k += 8 * kRedParts) {
#pragma unroll
            for (int u = 0; u < 8; u++) acc[u] += scratch[(size_t)(k + u * kRedParts) * stride + b];
        }
        for (; k < nblocks; k += kRedParts) acc[0] += scratch[(size_t)k * stride + b];
#pragma unroll
        for (int u = 0; u < 8; u++) s += acc[u];
    }
    part[q][t] = s;
    __syncthreads();
    if (q != 0 || b >= nbins) return;
    for (uint32_t p = 1; p < kRedParts; p++) s += part[p][t];
    if (!s) return;
    // atomic: calls on different streams may share one counters array
    unsigned long long *dst = (unsigned long long *)(b >= nb ? &counters[nrules + (b - nb)]  // verdict bins (lo == 0)
                                                             : &counters[lo + b]);
    atomicAdd(dst, (unsigned long long)s);
}

// Proxy statistics (pkg/endpoint/endpoint.go:2207-2233 UpdateProxyStatistics):
// per statistics key -- (policy, proto, port, direction), resolved per
// connection on the host -- received / forwarded / denied / error counts of
// the call's requests, added into the engine's u64[nkeys][4] accumulator.
// ALLOW = forwarded, DENY = denied, PARSE_ERROR = error, each also received;
// INCOMPLETE and UNSUPPORTED requests are no flow yet.
constexpr uint32_t kFlowBinsMax = 4096 * 4;  // LDS u32 bins (64 KiB)

__global__ __launch_bounds__(kHistBlock) void flowstats_kernel(Batch B, uint32_t nkeys, uint64_t *__restrict__ acc) {
    __shared__ uint32_t bins[kFlowBinsMax];
    const uint32_t nb = nkeys * 4;
    for (uint32_t i = threadIdx.x; i < nb; i += kHistBlock) bins[i] = 0;
    __syncthreads();
    const uint32_t per = (B.n + gridDim.x - 1) / gridDim.x;
    const uint32_t b0 = blockIdx.x * per, b1 = min(B.n, b0 + per);
    for (uint32_t i = b0 + threadIdx.x; i < b1; i += kHistBlock) {
        const uint32_t v = B.verdict[i];
        if (v > V_PARSE_ERROR) continue;
        const uint32_t ci = B.conn_ids[i];
        const uint32_t k = ci < B.nconns ? B.conns[ci].skey : 0xFFFFu;
        if (k >= nkeys) continue;
        atomicAdd(&bins[4 * k], 1u);
        atomicAdd(&bins[4 * k + (v == V_ALLOW ? 1 : v == V_DENY ? 2 : 3)], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nb; i += kHistBlock)
        if (bins[i]) atomicAdd((unsigned long long *)&acc[i], (unsigned long long)bins[i]);
}

}  // namespace

uint32_t FlowStatsMaxKeys() { return kFlowBinsMax / 4; }

hipError_t LaunchFlowStats(const Batch &B, uint32_t nkeys, uint64_t *acc, hipStream_t stream) {
    if (B.n == 0 || nkeys == 0) return hipSuccess;
    const uint32_t nblocks = std::min<uint32_t>(kHistBlocks, (B.n + kHistBlock - 1) / kHistBlock);
    hipLaunchKernelGGL(flowstats_kernel, dim3(nblocks), dim3(kHistBlock), 0, stream, B, nkeys, acc);
    return hipGetLastError();
}

// Bytes of scratch LaunchCounters needs.
size_t CountersScratchBytes() { return (size_t)kHistBlocks * (kHistBins + 8) * sizeof(uint32_t); }

// counters: u64[nrules + 8] (rules, then verdicts), accumulated into.
hipError_t LaunchCounters(const uint8_t *verdict, const int32_t *rule, uint32_t n, uint32_t nrules,
                          uint64_t *counters, uint32_t *scratch, hipStream_t stream) {
    if (n == 0 || !counters) return hipSuccess;
    const uint32_t nblocks = std::min<uint32_t>(kHistBlocks, (n + kHistBlock - 1) / kHistBlock);
    const uint32_t stride = kHistBins + 8;
    for (uint32_t lo = 0; lo == 0 || lo < nrules; lo += kHistBins) {
        const uint32_t nb = std::min<uint32_t>(kHistBins, nrules - lo);
        hipLaunchKernelGGL(histogram_kernel, dim3(nblocks), dim3(kHistBlock), 0, stream, verdict, rule, n, lo, nb,
                           scratch, stride);
        const uint32_t nbins = nb + (lo == 0 ? 8 : 0);
        hipLaunchKernelGGL(reduce_kernel, dim3((nbins + kRedBins - 1) / kRedBins), dim3(kRedBins * kRedParts), 0,
                           stream, scratch, nblocks, stride, lo, nb, nrules, counters);
    }
    return hipGetLastError();
}

}  // namespace l7
