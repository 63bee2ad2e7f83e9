// proxylib cassandra request classification on gfx950 (product code).
//
// proxylib/cassandra/cassandraparser.go, one lane per request (a frame at the
// start of the request's bytes):
//   framing (OnData :171-210): < 9 bytes => INCOMPLETE, consumed = the missing
//     header bytes (MORE); body length > 256 MB => PARSE_ERROR, consumed 3
//     (ERROR_INVALID_FRAME_LENGTH); missing body bytes => INCOMPLETE with their
//     count; reply direction bit or compression flag => PARSE_ERROR, consumed
//     2 (ERROR_INVALID_FRAME_TYPE);
//   cassandraParseRequest (:471-581): QUERY / PREPARE => parseQuery
//     (kernels/cass_parse.h; a short body or a trailing FROM is a Go panic =>
//     PARSE_ERROR, consumed 0; an unparsable query => PARSE_ERROR 2); BATCH
//     always panics (:519); EXECUTE => PARSE_ERROR 2, since a batch carries no
//     prepared statements (the proxylib shim answers EXECUTE from its PREPARE
//     cache); any other opcode => a two-part path every rule matches;
//   Connection.Matches over the rule set's image: query_action row AND the
//     query_table automata over parts[3] of the path, which is produced as a
//     stream of lowered bytes straight from the request (and, for an undotted
//     table, from the USE request that set the keyspace).
//
// Keyspace: a batch's requests on one connection are read in batch order, as
// proxylib's OnData reads a connection's frames, so the keyspace of request i
// is the one set by the last USE (a QUERY or PREPARE "use x") before i on the
// same connection; none => "".  cassandra_use_kernel writes one key per
// request, (connection << 32 | index) for a USE request and ~0 otherwise; the
// keys are radix-sorted (hipcub), and a lane whose table needs the keyspace
// finds the last USE on its connection before it by one binary search over
// them: O(n log n) per batch however many USE requests it holds (a scan of an
// unordered USE list per lane was O(n x #USE), quadratic on a USE-heavy batch).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "../device_tables.h"
#include "cass_parse.h"

namespace l7 {

namespace {

constexpr int kBlock = 256;
constexpr uint32_t kCassMaxLen = 268435456u;  // cassMaxLen (:56)

__device__ __forceinline__ uint32_t be32(const uint8_t *b) {
    return (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3];
}
__device__ __forceinline__ uint32_t be16(const uint8_t *b) { return (uint32_t)b[0] << 8 | b[1]; }

// The query of a QUERY / PREPARE frame at b (len bytes of buffer): q / qn, or
// false with *verdict / *consumed set (framing outcome, panic, or not a query).
struct Frame {
    uint8_t verdict;     // V_* when not a query
    uint32_t consumed;
    uint32_t fl;         // frame length
    uint8_t op;
};
__device__ __forceinline__ bool frame_of(const uint8_t *b, uint32_t len, Frame *F) {
    F->consumed = 0;
    F->fl = 0;
    F->op = 0;
    if (len < 9) { F->verdict = V_INCOMPLETE; F->consumed = 9 - len; return false; }
    const uint32_t rl = be32(b + 5);
    if (rl > kCassMaxLen) { F->verdict = V_PARSE_ERROR; F->consumed = 3; return false; }
    const uint32_t fl = 9 + rl;
    if (fl > len) { F->verdict = V_INCOMPLETE; F->consumed = fl - len; return false; }
    F->fl = fl;
    if ((b[0] & 0x80) || (b[1] & 0x01)) { F->verdict = V_PARSE_ERROR; F->consumed = 2; return false; }
    F->op = b[4];
    return true;
}

// QUERY / PREPARE: the long string at 9; false = the slice expressions panic.
// The frame is data[0:fl] of the bytes.Join buffer (cassandraparser.go:174,
// :211); Go bounds data[9:13] and data[13:13+ql] by the slice's capacity, so
// they read on into the bytes after the frame and panic only past the
// buffer's end (cap = the request's buffer length; a single-slice join's
// allocator slack is not restated: parity unpinned, oracle/cassandra_ref.c).
__device__ __forceinline__ bool query_of(const uint8_t *b, uint32_t cap, uint32_t *qn) {
    if (cap < 13) return false;
    const uint32_t ql = be32(b + 9);
    const uint32_t end = 13u + ql;  // uint32 arithmetic, as in Go
    if (end < 13u || end > cap) return false;
    *qn = ql;
    return true;
}

struct CountSink {
    uint32_t n = 0;
    __device__ void raw(uint32_t) { n++; }
    __device__ void rune(uint32_t) { n++; }
};
struct DfaSink {
    const uint8_t *img;
    DevDfa D;
    uint32_t st;
    __device__ void raw(uint32_t c) {
        if (st) st = ((const uint16_t *)(img + D.trans_off))[st * D.ncls + img[D.cls_off + c]];
    }
    __device__ void rune(uint32_t r) {
        uint8_t e[4];
        const uint32_t n = cass_encode(r, e);
        for (uint32_t k = 0; k < n; k++) raw(e[k]);
    }
};
struct NfaSink {
    const uint8_t *pool;
    uint64_t off;
    NfaRun R;
    __device__ void raw(uint32_t c) { nfa_step(pool, off, R, 0xFFFD, c); }
    __device__ void rune(uint32_t r) {
        uint8_t e[4];
        cass_encode(r, e);
        nfa_step(pool, off, R, r, e[0]);
    }
};

}  // namespace

// One key per request: (connection << 32 | index) for a USE request, ~0 otherwise.
__global__ __launch_bounds__(kBlock) void cassandra_use_kernel(Batch B, CassTables T, uint64_t *__restrict__ keys) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= B.n) return;
    keys[i] = ~0ull;
    const uint32_t ci = B.conn_ids[i];
    if (ci >= B.nconns || B.conns[ci].proto != PROTO_CASSANDRA) return;
    const uint64_t off = B.offs[i];
    const uint32_t len = B.lens[i];
    if (!l7_in_arena(off, len, B.arena_len)) return;
    const uint8_t *b = B.arena + off;
    Frame F;
    uint32_t qn;
    if (!frame_of(b, len, &F) || (F.op != 0x07 && F.op != 0x09) || !query_of(b, len, &qn)) return;
    // cheap pre-check: the first token must be "use" (ASCII only: no other rune lowers to u, s or e)
    uint32_t p = 0;
    while (p < qn) {
        uint32_t w;
        const uint32_t r = nfa_decode(b + 13, p, qn, &w);
        if (!cass_space(r)) break;
        p += w;
    }
    if (p + 3 > qn || (b[13 + p] | 0x20) != 'u' || (b[14 + p] | 0x20) != 's' || (b[15 + p] | 0x20) != 'e') return;
    const CassQuery Q = cass_parse_query(b + 13, qn, T.lower, T.nlower);
    if (Q.status == CQ_OK && Q.is_use) keys[i] = (uint64_t)ci << 32 | i;
}

__device__ __forceinline__ void cassandra_one(const Batch &B, const CassTables &T, const uint64_t *__restrict__ use_keys,
                                              uint32_t answer_other, uint32_t i, uint64_t *scratch) {
    const uint32_t ci = B.conn_ids[i];
    const DevConn conn = ci < B.nconns ? B.conns[ci] : DevConn{-1, PROTO_NONE, 0, 0xFFFF};
    if (conn.proto != PROTO_CASSANDRA || conn.ruleset < 0 || (uint32_t)conn.ruleset >= T.nrulesets) {
        if (answer_other && !L7_PROTO_OWNED(conn.proto)) {  // no parser: UNSUPPORTED
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
        const uint8_t *img = T.images + T.rulesets[conn.ruleset].image_off;
        const CassImgHeader *H = (const CassImgHeader *)img;
        const uint32_t nch = H->nchunks;
        const int32_t *ids = (const int32_t *)(img + H->rule_off);
        Frame F;
        bool query_like = false;
        CassQuery Q{};
        uint32_t qn = 0;
        if (!frame_of(b, len, &F)) {
            verdict = F.verdict;
            consumed = F.consumed;
        } else if (F.op == 0x07 || F.op == 0x09) {
            if (!query_of(b, len, &qn)) {
                verdict = V_PARSE_ERROR;  // slice bounds panic
            } else {
                Q = cass_parse_query(b + 13, qn, T.lower, T.nlower);
                if (Q.status == CQ_PANIC) verdict = V_PARSE_ERROR;
                else if (Q.status == CQ_INVALID) { verdict = V_PARSE_ERROR; consumed = 2; }
                else query_like = true;
            }
        } else if (F.op == 0x0D) {
            verdict = V_PARSE_ERROR;  // Uint16(data[10:11]) panics
        } else if (F.op == 0x0A) {
            if (len < 11 || 11u + be16(b + 9) > len) verdict = V_PARSE_ERROR;  // panic (capacity-bounded, as above)
            else { verdict = V_PARSE_ERROR; consumed = 2; }                      // no prepared statement here
        } else {  // "/" + opcode name: every rule matches
            verdict = H->nrules ? V_ALLOW : H->terminal;
            rule = H->nrules ? ids[0] : -1;
            consumed = F.fl;
        }
        if (query_like) {
            // keyspace: the last USE on this connection before request i
            const uint8_t *ks = nullptr;
            CassQuery K{};
            if (Q.seg3 == S3_KS_TABLE) {
                // the largest sorted key below (ci << 32 | i), if it is on connection ci
                const uint64_t probe = (uint64_t)ci << 32 | i;
                uint32_t lo = 0, hi = B.n;  // first key >= probe
                while (lo < hi) {
                    const uint32_t mid = lo + ((hi - lo) >> 1);
                    if (use_keys[mid] < probe) lo = mid + 1; else hi = mid;
                }
                int64_t best = -1;
                if (lo > 0 && (use_keys[lo - 1] >> 32) == ci) best = (int64_t)(use_keys[lo - 1] & 0xFFFFFFFFu);
                if (best >= 0) {
                    const uint8_t *bj = B.arena + B.offs[best];
                    const uint32_t qj = be32(bj + 9);
                    K = cass_parse_query(bj + 13, qj, T.lower, T.nlower);
                    ks = bj + 13;
                }
            }
            const uint8_t *q = b + 13;
            CountSink cnt;
            cass_seg3(Q, q, ks, K.ts, K.te, K.fc, T.lower, T.nlower, cnt);
            uint64_t ok[kCassMaxChunks];
            const uint64_t *act = (const uint64_t *)(img + H->act_off) +
                                  (size_t)(Q.action >= 0 ? Q.action : kCassActions) * nch;
            const uint64_t *notab = (const uint64_t *)(img + H->notab_off);
#pragma unroll
            for (int c = 0; c < kCassMaxChunks; c++) ok[c] = (uint32_t)c < nch ? (cnt.n ? notab[c] : ~0ull) : 0;
            if (cnt.n) {  // parts[3] non-empty: the table regexes decide
                const DevDfa *dd = (const DevDfa *)(img + H->dfa_off);
                for (uint32_t d = 0; d < H->ndfa; d++) {
                    DfaSink S{img, dd[d], dd[d].start};
                    cass_seg3(Q, q, ks, K.ts, K.te, K.fc, T.lower, T.nlower, S);
                    const uint64_t *m = (const uint64_t *)(img + S.D.mask_off) + (size_t)S.st * nch;
#pragma unroll
                    for (int c = 0; c < kCassMaxChunks; c++)
                        if ((uint32_t)c < nch) ok[c] |= m[c];
                }
                const DevNfaRef *refs = (const DevNfaRef *)(img + H->nfa_off);
                for (uint32_t k = 0; k < H->nnfa; k++) {
                    const DevNfaRef r = refs[k];
                    NfaSink S{T.nfa_pool, r.nfa, {}};
                    nfa_begin(S.R, scratch);
                    cass_seg3(Q, q, ks, K.ts, K.te, K.fc, T.lower, T.nlower, S);
                    if (!nfa_end(T.nfa_pool, r.nfa, S.R)) continue;
                    const uint64_t *own = (const uint64_t *)(img + r.mask_off);
#pragma unroll
                    for (int c = 0; c < kCassMaxChunks; c++)
                        if ((uint32_t)c < nch) ok[c] |= own[c];
                }
            }
            verdict = H->terminal;
            consumed = F.fl;
#pragma unroll
            for (int c = 0; c < kCassMaxChunks; c++) {
                if ((uint32_t)c >= nch) break;
                const uint64_t hit = ok[c] & act[c];
                if (hit) {
                    verdict = V_ALLOW;
                    rule = ids[c * 64 + __builtin_ctzll(hit)];
                    break;
                }
            }
        }
    }
    B.verdict[i] = verdict;
    B.rule[i] = rule;
    B.consumed[i] = consumed;
}

// grid-stride: a launch with large NFAs has as many lanes as it has scratch for
__global__ __launch_bounds__(kBlock) void cassandra_classify_kernel(Batch B, CassTables T,
                                                                    const uint64_t *__restrict__ use_keys,
                                                                    uint32_t answer_other) {
    uint64_t *scratch = l7_nfa_lane_scratch(T.nfa_scratch, T.nfa_lane_words);
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < B.n; i += gridDim.x * kBlock)
        cassandra_one(B, T, use_keys, answer_other, i, scratch);
}

// Scratch bytes LaunchCassandraClassify needs for a batch of n requests.
size_t CassandraScratchBytes(uint32_t n) {
    size_t temp = 0;
    if (hipcub::DeviceRadixSort::SortKeys(nullptr, temp, (const uint64_t *)nullptr, (uint64_t *)nullptr, (int)n, 0, 64) !=
        hipSuccess)
        return 0;
    const size_t kb = ((size_t)n * sizeof(uint64_t) + 256 + 255) & ~(size_t)255;  // as LaunchCassandraClassify lays it out
    return 2 * kb + ((temp + 255) & ~(size_t)255);
}

// scratch: CassandraScratchBytes(B.n) bytes (256-byte aligned)
// nfa_lanes: lanes T.nfa_scratch holds (when it is set)
hipError_t LaunchCassandraClassify(const Batch &B, const CassTables &T, void *scratch, size_t scratch_bytes,
                                   bool answer_other, uint32_t nfa_lanes, hipStream_t stream) {
    if (B.n == 0) return hipSuccess;
    const size_t kb = ((size_t)B.n * sizeof(uint64_t) + 256 + 255) & ~(size_t)255;
    uint64_t *keys = (uint64_t *)scratch;
    uint64_t *sorted = (uint64_t *)((uint8_t *)scratch + kb);
    void *temp = (uint8_t *)scratch + 2 * kb;
    if (scratch_bytes < 2 * kb) return hipErrorInvalidValue;
    size_t temp_bytes = scratch_bytes - 2 * kb;
    const dim3 grid((B.n + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(cassandra_use_kernel, grid, dim3(kBlock), 0, stream, B, T, keys);
    hipError_t rc = hipGetLastError();
    if (rc != hipSuccess) return rc;
    // connection ids are < 2^32 and request indices < 2^32: all 64 bits
    rc = hipcub::DeviceRadixSort::SortKeys(temp, temp_bytes, keys, sorted, (int)B.n, 0, 64, stream);
    if (rc != hipSuccess) return rc;
    dim3 cgrid = grid;
    if (T.nfa_scratch) cgrid.x = max(1u, min(cgrid.x, nfa_lanes / kBlock));
    hipLaunchKernelGGL(cassandra_classify_kernel, cgrid, dim3(kBlock), 0, stream, B, T, sorted, answer_other ? 1u : 0u);
    return hipGetLastError();
}

}  // namespace l7
