// HTTP/1 request classification on gfx950 (product code).
//
// One lane per request (grid-stride).  Each lane
//   1. frames its request left to right (request line, header lines, empty
//      line; the grammar and error precedence are DESIGN.md §HTTP framing,
//      restating what Envoy's HTTP/1 codec enforces before
//      cilium.l7policy's decodeHeaders, envoy/cilium_l7policy.cc:127-182),
//      reading 16-byte aligned words and recording the value spans of the
//      header slots its rule set needs (:method, :path, :authority, <= 8
//      custom headers) in LDS;
//   2. evaluates its connection's rule set (envoy/cilium_network_policy.h
//      :50-237 lowered by engine/http_compile.cc): per 64-rule chunk, every
//      referenced field's DFAs are walked over the field bytes and the
//      per-state rule masks are AND-ed; the first surviving rule wins.
// Outputs: verdict (u8), matched global rule id (i32, -1 none), consumed (u32).
#include <hip/hip_runtime.h>

#include "../device_tables.h"

namespace l7 {

namespace {

enum : int {
    ST_METHOD = 0, ST_TARGET, ST_VER, ST_LSTART, ST_NAME, ST_OWS, ST_VALUE, ST_LF, ST_FINAL_LF, ST_DONE, ST_ERR,
};
enum : int { HK_NONE = 0, HK_SLOT, HK_CL, HK_TE };

constexpr int kBlock = 256;
__constant__ uint32_t kVer[10] = {'H', 'T', 'T', 'P', '/', 0x100, '.', 0x100, '\r', '\n'};

__device__ __forceinline__ bool is_tchar(uint32_t c) {
    // tchar = "!#$%&'*+-.^_`|~" / DIGIT / ALPHA  (bitmap over 0x20..0x7F)
    const uint32_t m1 = 0x03FF6CFAu;  // 0x20-0x3F: ! # $ % & ' * + - . 0-9
    const uint32_t m2 = 0xC7FFFFFEu;  // 0x40-0x5F: A-Z ^ _
    const uint32_t m3 = 0x57FFFFFFu;  // 0x60-0x7F: ` a-z | ~
    if (c < 0x20 || c >= 0x80) return false;
    uint32_t w = c < 0x40 ? m1 : (c < 0x60 ? m2 : m3);
    return (w >> (c & 31)) & 1;
}

__device__ __forceinline__ uint32_t fnv_step(uint32_t h, uint32_t c) {  // == l7_fnv_step (host)
    c += (c - 'A' < 26u) ? 32u : 0u;
    return (h ^ c) * 16777619u;
}

// bytes equal ignoring ASCII case (b is already lower-case)
__device__ bool name_eq(const uint8_t *a, const uint8_t *b, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) {
        uint32_t c = a[i];
        if (c >= 'A' && c <= 'Z') c += 32;
        if (c != b[i]) return false;
    }
    return true;
}

__constant__ uint8_t kHost[4] = {'h', 'o', 's', 't'};
__constant__ uint8_t kCL[14] = {'c', 'o', 'n', 't', 'e', 'n', 't', '-', 'l', 'e', 'n', 'g', 't', 'h'};
__constant__ uint8_t kTE[17] = {'t', 'r', 'a', 'n', 's', 'f', 'e', 'r', '-', 'e', 'n', 'c', 'o', 'd', 'i', 'n', 'g'};

constexpr uint32_t fnv_const(const char *s, int n) {
    uint32_t h = kFnvBasis;
    for (int i = 0; i < n; i++) h = (h ^ (uint8_t)s[i]) * 16777619u;
    return h;
}
constexpr uint32_t kHashHost = fnv_const("host", 4);
constexpr uint32_t kHashCL = fnv_const("content-length", 14);
constexpr uint32_t kHashTE = fnv_const("transfer-encoding", 17);

// Walk one DFA over arena[o, o+l); returns the state's rule mask at EOF.
__device__ uint64_t dfa_walk(const HttpTables &T, const DevDfa &d, const uint8_t *p, uint32_t l) {
    const uint16_t *tr = T.trans + d.trans_off;
    const uint8_t *cls = T.cls + d.cls_off;
    const uint32_t ncls = d.ncls;
    uint32_t s = d.start;
    uintptr_t a = (uintptr_t)p;
    uint32_t i = 0;
    while (i < l && s != 0) {
        const uint4 w = *(const uint4 *)((a + i) & ~(uintptr_t)15);
        uint32_t k = (uint32_t)((a + i) & 15);
        uint64_t lo = ((uint64_t)w.y << 32) | w.x, hi = ((uint64_t)w.w << 32) | w.z;
        if (k >= 8) { lo = hi >> (8 * (k - 8)); hi = 0; }
        else if (k > 0) { lo = (lo >> (8 * k)) | (hi << (64 - 8 * k)); hi >>= 8 * k; }
        uint32_t nb = 16 - k;
        if (nb > l - i) nb = l - i;
        for (uint32_t j = 0; j < nb; j++) {
            uint32_t c = (uint32_t)lo & 0xFF;
            lo = (lo >> 8) | (hi << 56);
            hi >>= 8;
            s = tr[s * ncls + cls[c]];
            if (s == 0) break;
        }
        i += nb;
    }
    return T.masks[d.mask_off + s];
}

}  // namespace

__global__ __launch_bounds__(kBlock) void http_classify_kernel(
    const uint8_t *__restrict__ arena, const uint64_t *__restrict__ offs, const uint32_t *__restrict__ lens,
    const uint32_t *__restrict__ conn_ids, uint32_t n, const DevConn *__restrict__ conns, uint32_t nconns,
    HttpTables T, uint8_t *__restrict__ out_verdict, int32_t *__restrict__ out_rule, uint32_t *__restrict__ out_consumed,
    uint64_t *__restrict__ counters, uint32_t ncounters) {
    __shared__ uint2 spans[kNumSlots * kBlock];
    const uint32_t tid = threadIdx.x;
    for (uint32_t idx = blockIdx.x * kBlock + tid; idx < n; idx += gridDim.x * kBlock) {
        const uint64_t off = offs[idx];
        const uint32_t len = lens[idx];
        const uint32_t ci = conn_ids[idx];
        uint8_t verdict = V_PARSE_ERROR;
        int32_t rule = -1;
        uint32_t consumed = 0;
        const DevConn conn = ci < nconns ? conns[ci] : DevConn{-1, PROTO_NONE, {0, 0, 0}};
        // entries of other protocols belong to their own kernels; this kernel
        // also answers entries whose connection is unknown or has no parser
        if (conn.proto == PROTO_KAFKA || conn.proto == PROTO_MEMCACHE) continue;
        if (conn.proto != PROTO_HTTP || conn.ruleset < 0 || (uint32_t)conn.ruleset >= T.nrulesets) {
            verdict = conn.proto == PROTO_HTTP ? V_DENY : V_UNSUPPORTED;
            out_verdict[idx] = verdict; out_rule[idx] = rule; out_consumed[idx] = consumed;
            continue;
        }
        const DevRuleset rs = T.rulesets[conn.ruleset];
        const uint8_t *req = arena + off;

        // ------------------------------------------------------------ framing
        int st = ST_METHOD;
        uint32_t present = 0;
        uint32_t tok = 0;         // start of the current token (method/target/name/value)
        uint32_t vend = 0, vk = 0;
        uint32_t hash = kFnvBasis;
        int hk = HK_NONE, hslot = 0;
        bool have_cl = false, have_te = false, cl_bad = false, cl_ws = false;
        uint64_t cl = 0, clv = 0;  // committed Content-Length / value of the current line
        uint32_t ndig = 0, hdr_end = 0;
        uint32_t pos = 0;
        const uintptr_t base = (uintptr_t)req;
        while (pos < len && st < ST_DONE) {
            const uint4 w = *(const uint4 *)((base + pos) & ~(uintptr_t)15);
            uint32_t k = (uint32_t)((base + pos) & 15);
            uint64_t lo = ((uint64_t)w.y << 32) | w.x, hi = ((uint64_t)w.w << 32) | w.z;
            if (k >= 8) { lo = hi >> (8 * (k - 8)); hi = 0; }
            else if (k > 0) { lo = (lo >> (8 * k)) | (hi << (64 - 8 * k)); hi >>= 8 * k; }
            uint32_t nb = 16 - k;
            if (nb > len - pos) nb = len - pos;
            for (uint32_t j = 0; j < nb && st < ST_DONE; j++, pos++) {
                const uint32_t c = (uint32_t)lo & 0xFF;
                lo = (lo >> 8) | (hi << 56);
                hi >>= 8;
                switch (st) {
                case ST_METHOD:
                    if (c == ' ') {
                        if (pos == 0) { st = ST_ERR; break; }
                        spans[SLOT_METHOD * kBlock + tid] = make_uint2(0, pos);
                        present |= 1u << SLOT_METHOD;
                        st = ST_TARGET; tok = pos + 1;
                    } else if (!is_tchar(c)) st = ST_ERR;
                    break;
                case ST_TARGET:
                    if (c == ' ') {
                        if (pos == tok) { st = ST_ERR; break; }
                        spans[SLOT_PATH * kBlock + tid] = make_uint2(tok, pos - tok);
                        present |= 1u << SLOT_PATH;
                        st = ST_VER; vk = 0;
                    } else if (c <= 0x20 || c == 0x7F) st = ST_ERR;
                    break;
                case ST_VER: {
                    uint32_t want = kVer[vk];
                    bool ok = want == 0x100 ? (c >= '0' && c <= '9') : (c == want);
                    if (!ok) { st = ST_ERR; break; }
                    if (++vk == 10) st = ST_LSTART;
                    break;
                }
                case ST_LSTART:
                    if (c == '\r') { st = ST_FINAL_LF; break; }
                    if (!is_tchar(c)) { st = ST_ERR; break; }  // includes SP/HTAB (obs-fold)
                    tok = pos; hash = fnv_step(kFnvBasis, c); st = ST_NAME;
                    break;
                case ST_NAME:
                    if (c == ':') {
                        const uint32_t nl = pos - tok;
                        hk = HK_NONE;
                        if (hash == kHashHost && nl == 4 && name_eq(req + tok, kHost, 4)) {
                            if (!(present & (1u << SLOT_AUTHORITY))) { hk = HK_SLOT; hslot = SLOT_AUTHORITY; }
                        } else if (hash == kHashCL && nl == 14 && name_eq(req + tok, kCL, 14)) {
                            hk = HK_CL;
                        } else if (hash == kHashTE && nl == 17 && name_eq(req + tok, kTE, 17)) {
                            hk = HK_TE;
                        } else {
                            for (uint32_t q = 0; q < rs.nhdr; q++) {
                                const DevHdrName h = T.hdrs[rs.hdr_first + q];
                                if (h.hash == hash && h.len == nl && !(present & (1u << (SLOT_CUSTOM0 + q))) &&
                                    name_eq(req + tok, T.names + h.name_off, nl)) {
                                    hk = HK_SLOT; hslot = SLOT_CUSTOM0 + q;
                                    break;
                                }
                            }
                        }
                        st = ST_OWS; clv = 0; ndig = 0; cl_bad = false; cl_ws = false;
                        break;
                    }
                    if (!is_tchar(c)) { st = ST_ERR; break; }
                    hash = fnv_step(hash, c);
                    break;
                case ST_OWS:
                    if (c == ' ' || c == '\t') break;
                    tok = pos; vend = pos; st = ST_VALUE;
                    [[fallthrough]];
                case ST_VALUE:
                    if (c == '\r') { st = ST_LF; break; }
                    if ((c < 0x20 && c != '\t') || c == 0x7F) { st = ST_ERR; break; }
                    if (c != ' ' && c != '\t') {
                        vend = pos + 1;
                        if (hk == HK_CL) {
                            if (c >= '0' && c <= '9' && !cl_ws) { clv = clv * 10 + (c - '0'); ndig++; }
                            else cl_bad = true;
                        }
                    } else if (hk == HK_CL) cl_ws = true;
                    break;
                case ST_LF:
                    if (c != '\n') { st = ST_ERR; break; }
                    if (hk == HK_SLOT) {
                        spans[hslot * kBlock + tid] = make_uint2(tok, vend - tok);
                        present |= 1u << hslot;
                    } else if (hk == HK_CL) {
                        if (have_cl || ndig == 0 || ndig > 10 || cl_bad) { st = ST_ERR; break; }
                        have_cl = true;
                        cl = clv;
                    } else if (hk == HK_TE) {
                        have_te = true;
                    }
                    st = ST_LSTART;
                    break;
                case ST_FINAL_LF:
                    if (c != '\n') { st = ST_ERR; break; }
                    hdr_end = pos + 1;
                    st = ST_DONE;
                    break;
                }
            }
        }
        if (st == ST_ERR) verdict = V_PARSE_ERROR;
        else if (st != ST_DONE) verdict = V_INCOMPLETE;
        else if (have_te) verdict = V_UNSUPPORTED;
        else {
            const uint64_t total = (uint64_t)hdr_end + (have_cl ? cl : 0);
            if (total > 0xFFFFFFFFull) verdict = V_PARSE_ERROR;
            else if (total > len) verdict = V_INCOMPLETE;
            else {
                consumed = (uint32_t)total;
                // --------------------------------------------- rule evaluation
                verdict = rs.terminal;
                for (uint32_t c = 0; c < rs.nchunks; c++) {
                    const DevChunk ch = T.chunks[rs.chunk_first + c];
                    uint64_t m = ch.all_mask;
                    for (uint32_t f = 0; f < ch.nfields && m; f++) {
                        const DevField fd = T.fields[ch.field_first + f];
                        if (fd.slot >= kNumSlots || !(present & (1u << fd.slot))) { m &= fd.absent_mask; continue; }
                        const uint2 sp = spans[fd.slot * kBlock + tid];
                        for (uint32_t q = 0; q < fd.ndfa && m; q++) {
                            const DevDfa d = T.dfas[fd.dfa_first + q];
                            m &= dfa_walk(T, d, req + sp.x, sp.y);
                        }
                    }
                    if (m) {
                        verdict = V_ALLOW;
                        rule = T.rule_ids[ch.rule_id_off + (uint32_t)__builtin_ctzll(m)];
                        break;
                    }
                }
            }
        }
        out_verdict[idx] = verdict;
        out_rule[idx] = rule;
        out_consumed[idx] = consumed;
        if (counters) {
            atomicAdd((unsigned long long *)&counters[ncounters - 8 + verdict], 1ull);
            if (rule >= 0 && (uint32_t)rule < ncounters - 8) atomicAdd((unsigned long long *)&counters[rule], 1ull);
        }
    }
}

// Host-side launcher (called from the C-ABI).
hipError_t LaunchHttpClassify(const uint8_t *arena, const uint64_t *offs, const uint32_t *lens, const uint32_t *conn_ids,
                              uint32_t n, const DevConn *conns, uint32_t nconns, const HttpTables &T,
                              uint8_t *verdict, int32_t *rule, uint32_t *consumed, uint64_t *counters,
                              uint32_t ncounters, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    uint32_t blocks = (n + kBlock - 1) / kBlock;
    if (blocks > 65535u * 4) blocks = 65535u * 4;
    hipLaunchKernelGGL(http_classify_kernel, dim3(blocks), dim3(kBlock), 0, stream, arena, offs, lens, conn_ids, n,
                       conns, nconns, T, verdict, rule, consumed, counters, ncounters);
    return hipGetLastError();
}

}  // namespace l7
