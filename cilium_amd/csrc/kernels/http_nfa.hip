// HTTP NFA pre-pass on gfx950 (product code): evaluates the rule sets'
// NFA-fallback matchers (patterns whose DFA alone exceeds the state budget;
// re_dfa.h BitNfa) before the framing kernel runs.
//
// One lane per request.  Only requests whose rule set carries NFA matchers do
// any work: the lane finds the value of each such matcher's header slot --
// the first occurrence, leading and trailing OWS excluded, exactly the bytes
// the framing kernel's DFAs would walk -- and runs the bit-parallel rune NFA
// over it (regex/nfa_walk.h, the same code the host test hook runs).  Bit k of
// nfa_bits[i] = matcher k accepted.  A request that does not frame has its
// bits ignored: the framing kernel answers it before it looks at them.
//
// This is the fallback path: an NFA step costs one table row
// per active 8-position chunk instead of the DFA's single transition.
#include <hip/hip_runtime.h>

#include "../device_tables.h"
#include "../regex/nfa_walk.h"

namespace l7 {

namespace {

constexpr int kNfaBlock = 256;

__device__ __forceinline__ bool name_is(const uint8_t *r, uint32_t p, uint32_t q, const uint8_t *lname, uint32_t n) {
    if (q - p != n) return false;
    for (uint32_t k = 0; k < n; k++) {
        uint32_t c = r[p + k];
        if (c - 'A' < 26u) c += 32;
        if (c != lname[k]) return false;
    }
    return true;
}

// Value span of header slot `slot` in request r[0, len): the request line's
// method / target, or the first header line whose name is the slot's.
__device__ bool value_span(const uint8_t *r, uint32_t len, uint32_t slot, const uint8_t *img, uint32_t *vo,
                           uint32_t *vl) {
    uint32_t i = 0;
    while (i < len && r[i] != ' ') i++;
    if (i >= len) return false;
    if (slot == SLOT_METHOD) { *vo = 0; *vl = i; return true; }
    uint32_t j = i + 1;
    while (j < len && r[j] > 0x20 && r[j] != 0x7F) j++;
    if (slot == SLOT_PATH) { *vo = i + 1; *vl = j - i - 1; return true; }
    const ImgHeader *H = (const ImgHeader *)img;
    const uint8_t *lname = (const uint8_t *)"host";
    uint32_t nlen = 4;
    if (slot >= SLOT_CUSTOM0) {
        const DevHdrName *hn = (const DevHdrName *)(img + H->hdr_off) + (slot - SLOT_CUSTOM0);
        lname = img + hn->name_off;
        nlen = hn->len;
    }
    while (j < len && r[j] != '\n') j++;  // end of the request line
    uint32_t p = j + 1;
    while (p < len && r[p] != '\r') {
        uint32_t q = p;
        while (q < len && r[q] != ':' && r[q] != '\n') q++;
        if (q >= len || r[q] != ':') return false;
        if (name_is(r, p, q, lname, nlen)) {
            uint32_t v = q + 1;
            while (v < len && (r[v] == ' ' || r[v] == '\t')) v++;
            uint32_t e = v;
            while (e < len && r[e] != '\r' && r[e] != '\n') e++;
            while (e > v && (r[e - 1] == ' ' || r[e - 1] == '\t')) e--;
            *vo = v;
            *vl = e - v;
            return true;
        }
        while (q < len && r[q] != '\n') q++;
        p = q + 1;
    }
    return false;
}

__device__ __forceinline__ void nfa_request(const Batch &B, const HttpTables &T, uint32_t i, uint64_t *scratch) {
    const uint32_t ci = B.conn_ids[i];
    if (ci >= B.nconns) return;
    const DevConn conn = B.conns[ci];
    if (conn.proto != PROTO_HTTP || conn.ruleset < 0 || (uint32_t)conn.ruleset >= T.nrulesets) return;
    const uint8_t *img = T.images + T.rulesets[conn.ruleset].image_off;
    const ImgHeader *H = (const ImgHeader *)img;
    const uint32_t nnfa = H->nnfa;
    if (nnfa == 0) return;
    const uint64_t off = B.offs[i];
    const uint32_t len = B.lens[i];
    uint64_t bits = 0;
    if (l7_in_arena(off, len, B.arena_len)) {
        const uint8_t *r = B.arena + off;
        const DevNfaRef *refs = (const DevNfaRef *)(img + H->nfa_off);
        for (uint32_t k = 0; k < nnfa; k++) {
            const DevNfaRef ref = refs[k];
            uint32_t vo, vl;
            if (value_span(r, len, ref.slot, img, &vo, &vl) && nfa_run(T.nfa_pool, ref.nfa, r + vo, vl, scratch))
                bits |= 1ull << k;
        }
    }
    T.nfa_bits[i] = bits;
}

}  // namespace

// grid-stride: a launch with large NFAs has as many lanes as it has scratch for
__global__ __launch_bounds__(kNfaBlock) void http_nfa_kernel(Batch B, HttpTables T) {
    uint64_t *scratch = l7_nfa_lane_scratch(T.nfa_scratch, T.nfa_lane_words);
    for (uint32_t i = blockIdx.x * kNfaBlock + threadIdx.x; i < B.n; i += gridDim.x * kNfaBlock)
        nfa_request(B, T, i, scratch);
}

// scratch_lanes: lanes T.nfa_scratch holds (when it is set)
hipError_t LaunchHttpNfa(const Batch &B, const HttpTables &T, uint32_t scratch_lanes, hipStream_t stream) {
    if (B.n == 0) return hipSuccess;
    uint32_t blocks = (B.n + kNfaBlock - 1) / kNfaBlock;
    if (T.nfa_scratch) blocks = max(1u, min(blocks, scratch_lanes / kNfaBlock));
    hipLaunchKernelGGL(http_nfa_kernel, dim3(blocks), dim3(kNfaBlock), 0, stream, B, T);
    return hipGetLastError();
}

}  // namespace l7
