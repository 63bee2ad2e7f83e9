// r2d2 request classification on gfx950 (product code).
//
// proxylib's r2d2 parser (proxylib/r2d2/r2d2parser.go:140-214), one lane per
// request: the request is the bytes up to the first "\r\n" (none: MORE 1 ->
// INCOMPLETE, consumed 1); its fields are strings.Split on single spaces;
// cmd = field 0, file = field 1 when there are exactly two fields, else "".
// A rule holds iff its cmd is unset or equal and its file regex is unset or
// matches the file (regexp.MatchString, unanchored): the rule set's cmd masks,
// file DFAs (mask rows of the rules whose regex accepts) and NFA-fallback
// regexes decide it.  The verdict is the first rule that holds (ALLOW, frame
// = line + 2), else the rule set's terminal verdict (proxylib policymap).
// The line is short; each lane reads its bytes through its own 16-byte
// register window.
#include <hip/hip_runtime.h>

#include "../device_tables.h"
#include "../regex/nfa_walk.h"

namespace l7 {

namespace {

constexpr int kBlock = 256;

struct Win {  // 16-byte aligned register window
    uint64_t base;
    uint32_t w0, w1, w2, w3;
};
__device__ __forceinline__ uint32_t rd(Win &r, const uint8_t *p) {
    const uint64_t a = (uint64_t)p, base = a & ~(uint64_t)15;
    if (base != r.base) {
        const uint4 v = *(const uint4 *)base;
        r.w0 = v.x; r.w1 = v.y; r.w2 = v.z; r.w3 = v.w;
        r.base = base;
    }
    const uint32_t k = (uint32_t)(a >> 2) & 3;
    const uint32_t a0 = r.w0, a1 = r.w1, a2 = r.w2, a3 = r.w3;
    const uint32_t w = k == 0 ? a0 : k == 1 ? a1 : k == 2 ? a2 : a3;
    return (w >> ((a & 3) * 8)) & 0xFF;
}

}  // namespace

__device__ __forceinline__ void r2d2_one(const Batch &B, const R2Tables &T, uint32_t answer_other, uint32_t i,
                                         uint64_t *scratch) {
    const uint32_t ci = B.conn_ids[i];
    const DevConn conn = ci < B.nconns ? B.conns[ci] : DevConn{-1, PROTO_NONE, 0, 0xFFFF};
    if (conn.proto != PROTO_R2D2 || conn.ruleset < 0 || (uint32_t)conn.ruleset >= T.nrulesets) {
        if (answer_other && !L7_PROTO_OWNED(conn.proto)) {
            B.verdict[i] = V_UNSUPPORTED;
            B.rule[i] = -1;
            B.consumed[i] = 0;
        }
        return;
    }
    const uint64_t off = B.offs[i];
    const uint32_t len = B.lens[i];
    uint8_t verdict = V_UNSUPPORTED;
    int32_t rule = -1;
    uint32_t consumed = 0;
    if (l7_in_arena(off, len, B.arena_len)) {
        const uint8_t *b = B.arena + off;
        Win W{~0ull, 0, 0, 0, 0};
        // first "\r\n", the spaces before it, and the command bytes
        uint32_t lf = 0, sp1 = 0xFFFFFFFFu, nsp = 0, cw0 = 0, cw1 = 0;
        bool found = false;
        uint32_t prev = 0x100;
        for (uint32_t p = 0; p < len; p++) {
            const uint32_t c = rd(W, b + p);
            if (prev == '\r' && c == '\n') { lf = p - 1; found = true; break; }
            if (prev == ' ') { nsp++; if (nsp == 1) sp1 = p - 1; }
            prev = c;
        }
        if (!found) {
            verdict = V_INCOMPLETE;  // MORE, 1
            consumed = 1;
        } else {
            const uint32_t clen = sp1 != 0xFFFFFFFFu ? sp1 : lf;
            for (uint32_t p = 0; p < clen && p < 8; p++) {
                const uint32_t c = rd(W, b + p);
                if (p < 4) cw0 |= c << (8 * p);
                else cw1 |= c << (8 * (p - 4));
            }
            uint32_t cmd = 4;  // R2_OTHER
            if (clen == 4 && cw0 == ('R' | 'E' << 8 | 'A' << 16 | 'D' << 24)) cmd = 0;
            else if (clen == 5 && cw0 == ('W' | 'R' << 8 | 'I' << 16 | 'T' << 24) && cw1 == 'E') cmd = 1;
            else if (clen == 4 && cw0 == ('H' | 'A' << 8 | 'L' << 16 | 'T' << 24)) cmd = 2;
            else if (clen == 5 && cw0 == ('R' | 'E' << 8 | 'S' << 16 | 'E' << 24) && cw1 == 'T') cmd = 3;
            const uint32_t f0 = nsp == 1 ? sp1 + 1 : 0, f1 = nsp == 1 ? lf : 0;  // the file field
            const uint8_t *img = T.images + T.rulesets[conn.ruleset].image_off;
            const R2ImgHeader *H = (const R2ImgHeader *)img;
            const uint32_t nch = H->nchunks;
            const uint64_t *cmdm = (const uint64_t *)(img + H->cmd_off) + cmd * nch;
            const uint64_t *nof = (const uint64_t *)(img + H->nofile_off);
            uint64_t ok[kR2MaxChunks];
#pragma unroll
            for (int c = 0; c < kR2MaxChunks; c++) ok[c] = (uint32_t)c < nch ? nof[c] : 0;
            const DevDfa *dd = (const DevDfa *)(img + H->dfa_off);
            for (uint32_t d = 0; d < H->ndfa; d++) {
                const DevDfa D = dd[d];
                uint32_t st = D.start;
                for (uint32_t p = f0; p < f1 && st; p++)
                    st = ((const uint16_t *)(img + D.trans_off))[st * D.ncls + img[D.cls_off + rd(W, b + p)]];
                const uint64_t *m = (const uint64_t *)(img + D.mask_off) + (size_t)st * nch;
#pragma unroll
                for (int c = 0; c < kR2MaxChunks; c++)
                    if ((uint32_t)c < nch) ok[c] |= m[c];
            }
            const DevNfaRef *refs = (const DevNfaRef *)(img + H->nfa_off);
            for (uint32_t k = 0; k < H->nnfa; k++) {
                const DevNfaRef r = refs[k];
                if (!nfa_run(T.nfa_pool, r.nfa, b + f0, f1 - f0, scratch)) continue;
                const uint64_t *own = (const uint64_t *)(img + r.mask_off);
#pragma unroll
                for (int c = 0; c < kR2MaxChunks; c++)
                    if ((uint32_t)c < nch) ok[c] |= own[c];
            }
            verdict = H->terminal;
            consumed = lf + 2;
            const int32_t *ids = (const int32_t *)(img + H->rule_off);
#pragma unroll
            for (int c = 0; c < kR2MaxChunks; c++) {
                if ((uint32_t)c >= nch) break;
                const uint64_t hit = ok[c] & cmdm[c];
                if (hit) {
                    verdict = V_ALLOW;
                    rule = ids[c * 64 + __builtin_ctzll(hit)];
                    break;
                }
            }
            if (verdict != V_ALLOW && verdict != V_DENY) consumed = 0;
        }
    }
    B.verdict[i] = verdict;
    B.rule[i] = rule;
    B.consumed[i] = consumed;
}

// grid-stride: a launch with large NFAs has as many lanes as it has scratch for
__global__ __launch_bounds__(kBlock) void r2d2_classify_kernel(Batch B, R2Tables T, uint32_t answer_other) {
    uint64_t *scratch = l7_nfa_lane_scratch(T.nfa_scratch, T.nfa_lane_words);
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < B.n; i += gridDim.x * kBlock)
        r2d2_one(B, T, answer_other, i, scratch);
}

// scratch_lanes: lanes T.nfa_scratch holds (when it is set)
hipError_t LaunchR2d2Classify(const Batch &B, const R2Tables &T, bool answer_other, uint32_t scratch_lanes,
                              hipStream_t stream) {
    if (B.n == 0) return hipSuccess;
    uint32_t blocks = (B.n + kBlock - 1) / kBlock;
    if (T.nfa_scratch) blocks = max(1u, min(blocks, scratch_lanes / kBlock));
    hipLaunchKernelGGL(r2d2_classify_kernel, dim3(blocks), dim3(kBlock), 0, stream, B, T, answer_other ? 1u : 0u);
    return hipGetLastError();
}

}  // namespace l7
