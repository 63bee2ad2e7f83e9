// HTTP requests grouped by rule set (product code).
//
// The reference evaluates each request against the rule set of its own remote
// identity (envoy/cilium_network_policy.h:90-146: PortNetworkPolicyRules per
// port, each rule's remote-identity set).  With many identities (cfg4: 512
// identities, 10k rules) the requests of one launch use hundreds of rule sets;
// a tile of 64 requests in stream order then mixes many of them, and the HTTP
// kernel can stage none of their images in LDS.  These kernels sort the
// batch's HTTP entries by rule set (a counting sort: per-workgroup LDS
// histograms, one global reservation per workgroup and bin) and cut each rule
// set's run into segments of at most kGroupSegEntries entries, which
// http_grouped_kernel (http_classify.hip) takes one per workgroup: it stages
// the segment's image in LDS once and its waves classify the segment's tiles
// from there.  Rule sets whose image does not fit the LDS budget are listed
// after all the others (the general kernel reads them through L2).  Order
// within a rule set is whatever the reservations make it: every output is
// indexed by request, so it does not matter.
#include <hip/hip_runtime.h>

#include "../device_tables.h"

namespace l7 {

namespace {
constexpr int kBlock = 256;
constexpr int kPer = 8;  // entries per thread
}  // namespace

// The entry -> (request index, HTTP rule set or -1) step shared by the passes:
// entry i of `sel` (the partition's HTTP list) or request i.
__device__ __forceinline__ int32_t group_rs(const Batch &B, const HttpTables &T, uint32_t idx, bool &other) {
    const uint32_t ci = B.conn_ids[idx];
    const DevConn c = ci < B.nconns ? B.conns[ci] : DevConn{-1, PROTO_NONE, 0, 0xFFFF};
    const bool mine = !L7_PROTO_OWNED(c.proto) || c.proto == PROTO_HTTP;
    const bool http = mine && c.proto == PROTO_HTTP && c.ruleset >= 0 && (uint32_t)c.ruleset < T.nrulesets;
    other = mine && !http;
    return http ? c.ruleset : -1;
}

// hist[r] += the entries on rule set r
__global__ __launch_bounds__(kBlock) void http_group_count_kernel(Batch B, HttpTables T, const uint32_t *__restrict__ sel,
                                                                  const uint32_t *__restrict__ sel_count,
                                                                  uint32_t *__restrict__ hist) {
    __shared__ uint32_t h[kMaxGroupRulesets];
    const uint32_t nrs = T.nrulesets, m = sel ? *sel_count : B.n;
    for (uint32_t r = threadIdx.x; r < nrs; r += kBlock) h[r] = 0;
    __syncthreads();
    const uint32_t start = blockIdx.x * (kBlock * kPer);
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const uint32_t i = start + k * kBlock + threadIdx.x;
        if (i < m) {
            bool other;
            const int32_t r = group_rs(B, T, sel ? sel[i] : i, other);
            if (r >= 0) atomicAdd(&h[r], 1u);
        }
    }
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < nrs; r += kBlock)
        if (h[r]) atomicAdd(&hist[r], h[r]);
}

// One workgroup: every rule set's first position in the grouped list (rule
// sets whose image fits the LDS budget first, the others after them), and the
// segment table.  ctl: [0] segments, [1] the grouped kernel's segment counter,
// [2] entries on big-image rule sets, [3] the general kernel's tile counter
// ([1] and [3] zeroed by the caller).
__global__ __launch_bounds__(1024) void http_group_scan_kernel(HttpTables T, const uint32_t *__restrict__ hist,
                                                               uint32_t *__restrict__ cursor, uint32_t *__restrict__ segs,
                                                               uint32_t *__restrict__ ctl) {
    constexpr uint32_t kT = 1024, kBins = kMaxGroupRulesets / kT;
    __shared__ uint32_t part[3][kT];
    const uint32_t t = threadIdx.x, nrs = T.nrulesets;
    uint32_t cs[kBins], cb[kBins], ns[kBins];
    uint32_t sums[3] = {0, 0, 0};  // small-image entries, big-image entries, segments
#pragma unroll
    for (uint32_t k = 0; k < kBins; k++) {
        const uint32_t r = t * kBins + k;
        const uint32_t c = r < nrs ? hist[r] : 0;
        const bool big = r < nrs && T.rulesets[r].image_len > kGroupImageBytes;
        cs[k] = big ? 0 : c;
        cb[k] = big ? c : 0;
        ns[k] = (cs[k] + kGroupSegEntries - 1) / kGroupSegEntries;
        sums[0] += cs[k];
        sums[1] += cb[k];
        sums[2] += ns[k];
    }
    // exclusive block scans of the three per-thread sums (Hillis-Steele over LDS)
    for (int q = 0; q < 3; q++) part[q][t] = sums[q];
    __syncthreads();
    for (uint32_t d = 1; d < kT; d <<= 1) {
        uint32_t v[3];
        for (int q = 0; q < 3; q++) v[q] = t >= d ? part[q][t - d] : 0;
        __syncthreads();
        for (int q = 0; q < 3; q++) part[q][t] += v[q];
        __syncthreads();
    }
    // big-image rule sets: their own list (gbig), flagged by the cursor's top bit
    uint32_t ps = part[0][t] - sums[0], pb = part[1][t] - sums[1], pg = part[2][t] - sums[2];
#pragma unroll
    for (uint32_t k = 0; k < kBins; k++) {
        const uint32_t r = t * kBins + k;
        if (r >= nrs) break;
        if (cb[k]) {
            cursor[r] = pb | 0x80000000u;
            pb += cb[k];
        } else {
            cursor[r] = ps;
            for (uint32_t j = 0; j < ns[k]; j++) {
                const uint32_t e0 = j * kGroupSegEntries;
                segs[3 * pg] = r;
                segs[3 * pg + 1] = ps + e0;
                segs[3 * pg + 2] = min(kGroupSegEntries, cs[k] - e0);
                pg++;
            }
            ps += cs[k];
        }
    }
    if (t == kT - 1) {
        ctl[0] = part[2][kT - 1];
        ctl[2] = part[1][kT - 1];
    }
}

// Every HTTP entry to its rule set's run of the grouped list; with
// answer_other, entries on unknown connections or connections without a parser
// are answered here (UNSUPPORTED), as the HTTP kernel would have.
__global__ __launch_bounds__(kBlock) void http_group_scatter_kernel(Batch B, HttpTables T,
                                                                    const uint32_t *__restrict__ sel,
                                                                    const uint32_t *__restrict__ sel_count,
                                                                    uint32_t *__restrict__ cursor,
                                                                    uint32_t *__restrict__ gsel,
                                                                    uint32_t *__restrict__ gbig, uint32_t answer_other) {
    __shared__ uint32_t h[kMaxGroupRulesets];
    const uint32_t nrs = T.nrulesets, m = sel ? *sel_count : B.n;
    for (uint32_t r = threadIdx.x; r < nrs; r += kBlock) h[r] = 0;
    __syncthreads();
    const uint32_t start = blockIdx.x * (kBlock * kPer);
    uint32_t idx[kPer], rank[kPer];
    int32_t rs[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const uint32_t i = start + k * kBlock + threadIdx.x;
        rs[k] = -1;
        if (i < m) {
            idx[k] = sel ? sel[i] : i;
            bool other;
            rs[k] = group_rs(B, T, idx[k], other);
            if (rs[k] >= 0) rank[k] = atomicAdd(&h[rs[k]], 1u);
            else if (other && answer_other) {
                B.verdict[idx[k]] = V_UNSUPPORTED;
                B.rule[idx[k]] = -1;
                B.consumed[idx[k]] = 0;
            }
        }
    }
    __syncthreads();
    for (uint32_t r = threadIdx.x; r < nrs; r += kBlock)
        if (h[r]) h[r] = atomicAdd(&cursor[r], h[r]);  // this workgroup's run inside the rule set's
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; k++)
        if (rs[k] >= 0) {
            const uint32_t at = h[rs[k]] + rank[k];
            if (at >> 31) gbig[at & 0x7FFFFFFFu] = idx[k];
            else gsel[at] = idx[k];
        }
}

// ctl and hist must be zero on entry ((4 + nrulesets) words); cursor, segs,
// gsel and gbig are written here.  n: entries in the list (an upper bound when
// sel_count is on the device).
hipError_t LaunchHttpGroup(const Batch &B, const HttpTables &T, const uint32_t *sel, const uint32_t *sel_count,
                           uint32_t n, bool answer_other, uint32_t *ctl, uint32_t *hist, uint32_t *cursor,
                           uint32_t *segs, uint32_t *gsel, uint32_t *gbig, hipStream_t stream) {
    if (n == 0 || T.nrulesets == 0 || T.nrulesets > kMaxGroupRulesets) return hipErrorInvalidValue;
    const uint32_t blocks = (n + kBlock * kPer - 1) / (kBlock * kPer);
    hipLaunchKernelGGL(http_group_count_kernel, dim3(blocks), dim3(kBlock), 0, stream, B, T, sel, sel_count, hist);
    hipLaunchKernelGGL(http_group_scan_kernel, dim3(1), dim3(1024), 0, stream, T, hist, cursor, segs, ctl);
    hipLaunchKernelGGL(http_group_scatter_kernel, dim3(blocks), dim3(kBlock), 0, stream, B, T, sel, sel_count, cursor,
                       gsel, gbig, answer_other ? 1u : 0u);
    return hipGetLastError();
}

}  // namespace l7
