// HTTP/1 request classification on gfx950 (product code).
//
// One lane per request, one forward pass over its bytes.  The request is
// read as 64-byte windows (four 16-byte loads, the next window prefetched
// into registers while the current one is consumed); a window is copied to
// the lane's LDS slot only when bytes in it are looked at one by one.
//
//   * request line and header names are framed byte by byte (the grammar and
//     error precedence are DESIGN.md §HTTP framing, restating what Envoy's
//     HTTP/1 codec enforces before cilium.l7policy's decodeHeaders,
//     envoy/cilium_l7policy.cc:127-182);
//   * the values of header slots the connection's rule set constrains
//     (:method, :path, :authority, <= 8 custom headers) are fed through the
//     slot's DFAs while they are framed, and the end state's per-chunk rule
//     masks are AND-ed into <= 4 register accumulators;
//   * every other header value is skipped 64 bytes per step with a SWAR scan
//     for the bytes that end or invalidate it (CTLs, DEL);
//   * at the end, the first rule whose accumulator bit survives wins
//     (envoy/cilium_network_policy.h:50-237 lowered by engine/http_compile.cc).
// Rule sets larger than 4 chunks x 4 DFAs per slot re-frame the request once
// per group (results identical; only the cost grows).
//
// The image of the rule set serving most connections is staged in LDS by each
// workgroup; waves whose lanes all use it read tables from LDS, others from
// HBM/L2 through the same offsets.
#include <hip/hip_runtime.h>

#include <cstddef>

#include "../device_tables.h"

namespace l7 {

namespace {

constexpr int kBlock = 512;
constexpr int kLdsRuleCounters = 1024;
constexpr uint32_t kNoChunk = 0xFFFFFFF0u;  // cursor holds no chunk (never k or k - 1)
constexpr uint32_t kEnd = 0x100;   // "byte" returned past the end of the request

__device__ __forceinline__ bool is_tchar(uint32_t c) {
    // tchar = "!#$%&'*+-.^_`|~" / DIGIT / ALPHA  (bitmap over 0x20..0x7F)
    const uint32_t m1 = 0x03FF6CFAu;  // 0x20-0x3F: ! # $ % & ' * + - . 0-9
    const uint32_t m2 = 0xC7FFFFFEu;  // 0x40-0x5F: A-Z ^ _
    const uint32_t m3 = 0x57FFFFFFu;  // 0x60-0x7F: ` a-z | ~
    uint32_t w = c < 0x40 ? m1 : (c < 0x60 ? m2 : m3);
    return (c - 0x20u < 0x60u) && ((w >> (c & 31)) & 1);
}

__device__ __forceinline__ uint32_t fnv_step(uint32_t h, uint32_t c) {  // == l7_fnv_step (host)
    c += (c - 'A' < 26u) ? 32u : 0u;
    return (h ^ c) * 16777619u;
}

constexpr uint32_t fnv_const(const char *s, int n) {
    uint32_t h = kFnvBasis;
    for (int i = 0; i < n; i++) h = (h ^ (uint8_t)s[i]) * 16777619u;
    return h;
}
constexpr uint32_t kHashHost = fnv_const("host", 4);
constexpr uint32_t kHashCL = fnv_const("content-length", 14);
constexpr uint32_t kHashTE = fnv_const("transfer-encoding", 17);
__constant__ uint32_t kVer[10] = {'H', 'T', 'T', 'P', '/', 0x100, '.', 0x100, '\r', '\n'};
__constant__ uint8_t kHost[4] = {'h', 'o', 's', 't'};
__constant__ uint8_t kCL[14] = {'c', 'o', 'n', 't', 'e', 'n', 't', '-', 'l', 'e', 'n', 'g', 't', 'h'};
__constant__ uint8_t kTE[17] = {'t', 'r', 'a', 'n', 's', 'f', 'e', 'r', '-', 'e', 'n', 'c', 'o', 'd', 'i', 'n', 'g'};

// Per-dword SWAR: bit 7 of byte i set iff byte i < 0x20 or == 0x7F (exact, no
// carries between bytes).  HT is reported too and skipped by the caller.
__device__ __forceinline__ uint32_t stop_bits(uint32_t x) {
    const uint32_t t = x & 0x7F7F7F7Fu;
    return (~(t + 0x60606060u) | (t + 0x01010101u)) & ~x & 0x80808080u;
}
// bit 7 of each byte -> 4-bit nibble
__device__ __forceinline__ uint32_t nib(uint32_t s) { return __builtin_amdgcn_ubfe((s >> 7) * 0x204081u, 21, 4); }

// ---------------------------------------------------------------- tables
// Rule-set image accessor: LDS (hot rule set) or global memory.
template <bool kLds>
struct Img {
    const uint8_t *p;
    __device__ __forceinline__ uint32_t u8(uint32_t o) const { return p[o]; }
    __device__ __forceinline__ uint32_t u16(uint32_t o) const { return *(const uint16_t *)(p + o); }
    __device__ __forceinline__ uint32_t u32(uint32_t o) const { return *(const uint32_t *)(p + o); }
    __device__ __forceinline__ uint64_t u64(uint32_t o) const { return *(const uint64_t *)(p + o); }
};

// ---------------------------------------------------------------- cursor
// Byte-wise reads: the 16-byte chunk holding the current position plus the
// next chunk, prefetched.  Positions are relative to the request start
// rounded down to 64 bytes, so chunks and windows are aligned in memory.
// Loads are never predicated: a chunk past the request end is read from the
// request's last chunk instead (its bytes are never consumed), so every load
// stays inside the request's own 16-byte chunks.
struct Cursor {
    const uint8_t *abase;  // request start rounded down to 64 B
    uint32_t lena;         // request end, relative to abase (> 0)
    uint32_t last;         // offset of the chunk holding the request's last byte
    uint32_t ck;           // chunk index held in cw
    uint4 cw, nw;
};

__device__ __forceinline__ uint4 load16(const Cursor &C, uint32_t k) {
    return *(const uint4 *)(C.abase + min(k * 16, C.last));
}

__device__ __forceinline__ void cursor_init(Cursor &C, const uint8_t *req, uint32_t len) {  // len > 0
    const uint32_t a = (uint32_t)((uintptr_t)req & 63);
    C.abase = req - a;
    C.lena = len + a;
    C.last = (C.lena - 1) & ~15u;
    C.ck = a >> 4;
    C.cw = load16(C, C.ck);
    C.nw = load16(C, C.ck + 1);
}

// Byte at aligned position pa (kEnd past the request).  Positions only move
// forward: usually into the prefetched chunk, after a skip anywhere ahead.
__device__ __forceinline__ uint32_t rd(Cursor &C, uint32_t pa) {
    if (pa >= C.lena) return kEnd;
    const uint32_t k = pa >> 4;
    if (k != C.ck) {
        C.cw = k == C.ck + 1 ? C.nw : load16(C, k);
        C.ck = k;
        C.nw = load16(C, k + 1);
    }
    // two selects + v_perm_b32 (selector 0x0C yields a zero byte); an indexed
    // select over the four dwords would be lowered to a scratch array
    const uint32_t q = pa & 15;
    const bool upper = (q & 8) != 0;
    const uint32_t lo = upper ? C.cw.z : C.cw.x, hi = upper ? C.cw.w : C.cw.y;
    return __builtin_amdgcn_perm(hi, lo, (q & 7) | 0x0C0C0C00u);
}

__device__ __forceinline__ void load64(const Cursor &C, uint32_t k, uint4 &w0, uint4 &w1, uint4 &w2, uint4 &w3) {
    const uint32_t o = k * 64;
    w0 = *(const uint4 *)(C.abase + min(o, C.last));
    w1 = *(const uint4 *)(C.abase + min(o + 16, C.last));
    w2 = *(const uint4 *)(C.abase + min(o + 32, C.last));
    w3 = *(const uint4 *)(C.abase + min(o + 48, C.last));
}

// 64-bit mask of the stop bytes of a window (bit i = byte i).
__device__ __forceinline__ uint32_t mask32(uint4 w) {
    return nib(stop_bits(w.x)) | nib(stop_bits(w.y)) << 4 | nib(stop_bits(w.z)) << 8 | nib(stop_bits(w.w)) << 12;
}
__device__ __forceinline__ uint64_t window_mask(uint4 a0, uint4 a1, uint4 a2, uint4 a3) {
    return (uint64_t)(mask32(a0) | mask32(a1) << 16) | (uint64_t)(mask32(a2) | mask32(a3) << 16) << 32;
}

// First position >= pa whose byte ends or invalidates a header value (CTL,
// DEL, or the request end); HT is reported as well.  Reads 64-byte windows
// (the next one in flight while the current one is tested); windows without
// such a byte cost only the SWAR test.
__device__ __forceinline__ uint32_t skip_value(const Cursor &C, uint32_t pa) {
    if (pa >= C.lena) return C.lena;
    uint32_t k = pa >> 6;
    uint4 a0, a1, a2, a3, b0, b1, b2, b3;
    load64(C, k, a0, a1, a2, a3);
    load64(C, k + 1, b0, b1, b2, b3);
    for (;;) {
        const uint32_t any = stop_bits(a0.x) | stop_bits(a0.y) | stop_bits(a0.z) | stop_bits(a0.w) |
                             stop_bits(a1.x) | stop_bits(a1.y) | stop_bits(a1.z) | stop_bits(a1.w) |
                             stop_bits(a2.x) | stop_bits(a2.y) | stop_bits(a2.z) | stop_bits(a2.w) |
                             stop_bits(a3.x) | stop_bits(a3.y) | stop_bits(a3.z) | stop_bits(a3.w);
        const uint32_t wend = k * 64 + 64;
        if (any != 0 || wend > C.lena) {
            uint64_t m = window_mask(a0, a1, a2, a3);
            if (wend > C.lena) m |= ~0ull << (C.lena & 63);  // request end inside this window
            if (pa > k * 64) m &= ~0ull << (pa & 63);
            if (m) return k * 64 + (uint32_t)__builtin_ctzll(m);
        }
        k++;
        a0 = b0; a1 = b1; a2 = b2; a3 = b3;
        load64(C, k + 1, b0, b1, b2, b3);
    }
}

// Lower-cased comparison of request bytes (global memory) with a table name.
__device__ bool name_eq(const uint8_t *a, const uint8_t *b, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) {
        uint32_t c = a[i];
        if (c - 'A' < 26u) c += 32;
        if (c != b[i]) return false;
    }
    return true;
}

// Image header fields (ImgHeader), read when needed rather than held in
// registers; wave-uniform in the LDS path, so moved to SGPRs there.
template <bool kLds>
__device__ __forceinline__ uint32_t uni(uint32_t v) {
    return kLds ? (uint32_t)__builtin_amdgcn_readfirstlane((int)v) : v;
}
#define HDR_U32(I, field) uni<kLds>((I).u32(offsetof(ImgHeader, field)))
#define HDR_U8(I, field) uni<kLds>((I).u8(offsetof(ImgHeader, field)))

// DFAs of one slot for the current pass.
struct SlotDfas {
    uint32_t nd;
    uint32_t cls[kDfasPerPass], trans[kDfasPerPass], mask[kDfasPerPass], ncls[kDfasPerPass];
    uint32_t st[kDfasPerPass];
};

template <bool kLds>
__device__ __forceinline__ void slot_begin(const Img<kLds> &I, uint32_t slot, uint32_t dgroup,
                                           SlotDfas &S) {
    const uint32_t lo = I.u8(offsetof(ImgHeader, slot_dfa) + slot) + dgroup * kDfasPerPass;
    const uint32_t hi = I.u8(offsetof(ImgHeader, slot_dfa) + slot + 1);
    S.nd = hi > lo ? min(hi - lo, (uint32_t)kDfasPerPass) : 0;
#pragma unroll
    for (int k = 0; k < kDfasPerPass; k++) {
        S.st[k] = 0;
        if ((uint32_t)k < S.nd) {
            const uint32_t d = HDR_U32(I, dfa_off) + (lo + k) * sizeof(DevDfa);
            S.cls[k] = I.u32(d + 0);
            S.trans[k] = I.u32(d + 4);
            S.mask[k] = I.u32(d + 8);
            const uint32_t nc_st = I.u32(d + 12);
            S.ncls[k] = nc_st & 0xFFFF;
            S.st[k] = nc_st >> 16;
        }
    }
}

template <bool kLds>
__device__ __forceinline__ void slot_step(const Img<kLds> &I, SlotDfas &S, uint32_t c) {
#pragma unroll
    for (int k = 0; k < kDfasPerPass; k++)
        if (S.st[k] != 0) S.st[k] = I.u16(S.trans[k] + 2 * (S.st[k] * S.ncls[k] + I.u8(S.cls[k] + c)));
}

// AND the end states' masks of chunks [cg, cg + nc) into acc.
template <bool kLds>
__device__ __forceinline__ void slot_end(const Img<kLds> &I, const SlotDfas &S, uint32_t nchunks, uint32_t cg,
                                         uint32_t nc, uint64_t *acc) {
#pragma unroll
    for (int k = 0; k < kDfasPerPass; k++) {
        if ((uint32_t)k >= S.nd) break;
        const uint32_t base = S.mask[k] + 8 * (S.st[k] * nchunks + cg);
#pragma unroll
        for (int c = 0; c < kChunksPerPass; c++)
            if ((uint32_t)c < nc) acc[c] &= I.u64(base + 8 * c);
    }
}

struct Result {
    uint8_t verdict;
    int32_t rule;
    uint32_t consumed;
};

// One framing pass over the request; on success the accumulators hold the
// chunk group's slot masks and *hdr_end / *cl the framing results.
template <bool kLds>
__device__ __forceinline__ uint8_t frame_pass(const Img<kLds> &I, const uint8_t *names_g, const uint8_t *req,
                              uint32_t len, uint32_t cg, uint32_t nc, uint32_t dgroup, uint64_t *acc,
                              uint32_t *present_out, uint32_t *consumed_out) {
    Cursor C;
    cursor_init(C, req, len);
    const uint32_t a0 = (uint32_t)((uintptr_t)req & 63);  // aligned position of byte 0
    const uint32_t nchunks = HDR_U8(I, nchunks);
    uint32_t present = 0;
    uint32_t pa = a0;
    uint32_t c;
    SlotDfas S;

    // ---- method: 1*tchar SP
    slot_begin(I, SLOT_METHOD, dgroup, S);
    for (;;) {
        c = rd(C, pa);
        if (c == ' ') break;
        if (!is_tchar(c)) return c == kEnd ? V_INCOMPLETE : V_PARSE_ERROR;
        slot_step(I, S, c);
        pa++;
    }
    if (pa == a0) return V_PARSE_ERROR;
    slot_end(I, S, nchunks, cg, nc, acc);
    present |= 1u << SLOT_METHOD;
    pa++;
    // ---- request target: 1*(VCHAR / obs-text) SP
    slot_begin(I, SLOT_PATH, dgroup, S);
    const uint32_t ps = pa;
    for (;;) {
        c = rd(C, pa);
        if (c == ' ') break;
        if (c <= 0x20 || c == 0x7F || c == kEnd) return c == kEnd ? V_INCOMPLETE : V_PARSE_ERROR;
        slot_step(I, S, c);
        pa++;
    }
    if (pa == ps) return V_PARSE_ERROR;
    slot_end(I, S, nchunks, cg, nc, acc);
    present |= 1u << SLOT_PATH;
    pa++;
    // ---- "HTTP/" DIGIT "." DIGIT CRLF
#pragma unroll 1
    for (uint32_t i = 0; i < 10; i++) {
        c = rd(C, pa);
        const uint32_t want = kVer[i];
        if (want == 0x100 ? c - '0' >= 10u : c != want) return c == kEnd ? V_INCOMPLETE : V_PARSE_ERROR;
        pa++;
    }
    // ---- header lines
    bool have_cl = false, have_te = false;
    uint64_t cl = 0;
    const uint8_t *abase = C.abase;
    for (;;) {
        c = rd(C, pa);
        if (c == '\r') {
            c = rd(C, pa + 1);
            if (c != '\n') return c == kEnd ? V_INCOMPLETE : V_PARSE_ERROR;
            pa += 2;
            break;
        }
        // field-name: 1*tchar ":"  (a line starting with SP/HT is obs-fold: error)
        const uint32_t ns = pa;
        uint32_t hash = kFnvBasis;
        for (;;) {
            c = rd(C, pa);
            if (c == ':') break;
            if (!is_tchar(c)) return c == kEnd ? V_INCOMPLETE : V_PARSE_ERROR;
            hash = fnv_step(hash, c);
            pa++;
        }
        const uint32_t nl = pa - ns;
        if (nl == 0) return V_PARSE_ERROR;
        pa++;
        uint32_t slot = ~0u;
        bool is_cl = false, is_te = false;
        if (nl == 4 && hash == kHashHost && name_eq(abase + ns, kHost, 4)) {
            if (!(present & (1u << SLOT_AUTHORITY))) slot = SLOT_AUTHORITY;
        } else {
            if (nl == 14 && hash == kHashCL && name_eq(abase + ns, kCL, 14)) is_cl = true;
            else if (nl == 17 && hash == kHashTE && name_eq(abase + ns, kTE, 17)) is_te = true;
            const uint32_t nhdr = HDR_U8(I, nhdr);
            for (uint32_t q = 0; q < nhdr; q++) {
                const uint32_t ho = HDR_U32(I, hdr_off) + q * sizeof(DevHdrName);
                if (I.u32(ho) == hash && (I.u32(ho + 4) & 0xFFFF) == nl && name_eq(abase + ns, names_g + I.u32(ho + 8), nl)) {
                    if (!(present & (1u << (SLOT_CUSTOM0 + q)))) slot = SLOT_CUSTOM0 + q;
                    break;
                }
            }
        }
        if (slot != ~0u && !((HDR_U32(I, ref_slots) >> slot) & 1)) slot = ~0u;
        // OWS
        for (;;) {
            c = rd(C, pa);
            if (c != ' ' && c != '\t') break;
            pa++;
        }
        uint64_t clv = 0;
        uint32_t ndig = 0;
        bool cl_bad = false, cl_ws = false;
        if (slot == ~0u && !is_cl) {
            // value nobody looks at: SWAR skip to CR, CTL or DEL
            C.ck = kNoChunk;  // the byte cursor's chunks are dead across the skip
            for (;;) {
                pa = skip_value(C, pa);
                c = rd(C, pa);
                if (c != '\t') break;
                pa++;
            }
            if (c != '\r') return c == kEnd ? V_INCOMPLETE : V_PARSE_ERROR;
        } else {
            if (slot != ~0u) slot_begin(I, slot, dgroup, S);
            else {
                S.nd = 0;
#pragma unroll
                for (int k = 0; k < kDfasPerPass; k++) S.st[k] = 0;
            }
            uint32_t saved[kDfasPerPass];
            bool in_ows = false;
            for (;;) {
                c = rd(C, pa);
                if (c == '\r') break;
                if ((c < 0x20 && c != '\t') || c == 0x7F || c == kEnd) return c == kEnd ? V_INCOMPLETE : V_PARSE_ERROR;
                if (c == ' ' || c == '\t') {
                    if (!in_ows) {
#pragma unroll
                        for (int k = 0; k < kDfasPerPass; k++) saved[k] = S.st[k];
                        in_ows = true;
                    }
                    cl_ws = true;
                } else {
                    in_ows = false;
                    if (c - '0' < 10u && !cl_ws) { clv = clv * 10 + (c - '0'); ndig++; }
                    else cl_bad = true;
                }
                if (S.nd) slot_step(I, S, c);
                pa++;
            }
            if (in_ows) {
#pragma unroll
                for (int k = 0; k < kDfasPerPass; k++) S.st[k] = saved[k];
            }
        }
        // CR LF
        c = rd(C, pa + 1);
        if (c != '\n') return c == kEnd ? V_INCOMPLETE : V_PARSE_ERROR;
        pa += 2;
        if (is_cl) {
            if (have_cl || ndig == 0 || ndig > 10 || cl_bad) return V_PARSE_ERROR;
            have_cl = true;
            cl = clv;
        }
        if (is_te) have_te = true;
        if (slot != ~0u) {
            slot_end(I, S, nchunks, cg, nc, acc);
            present |= 1u << slot;
        }
    }
    if (have_te) return V_UNSUPPORTED;
    const uint64_t total = (uint64_t)(pa - a0) + cl;
    if (total > 0xFFFFFFFFull) return V_PARSE_ERROR;
    if (total > len) return V_INCOMPLETE;
    *consumed_out = (uint32_t)total;
    *present_out = present;
    return V_ALLOW;  // framing ok
}

template <bool kLds>
__device__ __forceinline__ Result classify(const Img<kLds> &I, const uint8_t *names_g, const uint8_t *req, uint32_t len) {
    if (len == 0) return Result{V_INCOMPLETE, -1, 0};
    Result R{V_PARSE_ERROR, -1, 0};
    const uint32_t nchunks = HDR_U8(I, nchunks);
    const uint32_t max_dfas = HDR_U8(I, max_slot_dfas);
    const uint32_t ngroups = nchunks ? (nchunks + kChunksPerPass - 1) / kChunksPerPass : 1;
    const uint32_t ndg = max_dfas ? (max_dfas + kDfasPerPass - 1) / kDfasPerPass : 1;
    for (uint32_t g = 0; g < ngroups; g++) {
        const uint32_t cg = g * kChunksPerPass;
        const uint32_t nc = nchunks > cg ? min(nchunks - cg, (uint32_t)kChunksPerPass) : 0;
        uint64_t acc[kChunksPerPass];
#pragma unroll
        for (int c = 0; c < kChunksPerPass; c++) acc[c] = (uint32_t)c < nc ? I.u64(HDR_U32(I, init_off) + 8 * (cg + c)) : 0;
        uint32_t present = 0, consumed = 0;
        for (uint32_t dg = 0; dg < ndg; dg++) {
            const uint8_t v = frame_pass(I, names_g, req, len, cg, nc, dg, acc, &present, &consumed);
            if (v != V_ALLOW) { R.verdict = v; return R; }
        }
        R.consumed = consumed;
        // headers the rule set constrains but the request lacks
        uint32_t missing = HDR_U32(I, ref_slots) & 0xFFFF & ~present;
        while (missing) {
            const uint32_t s = __builtin_ctz(missing);
            missing &= missing - 1;
#pragma unroll
            for (int c = 0; c < kChunksPerPass; c++)
                if ((uint32_t)c < nc) acc[c] &= I.u64(HDR_U32(I, absent_off) + 8 * (s * nchunks + cg + c));
        }
#pragma unroll
        for (int c = 0; c < kChunksPerPass; c++) {
            if ((uint32_t)c < nc && acc[c]) {
                R.verdict = V_ALLOW;
                R.rule = (int32_t)I.u32(HDR_U32(I, rule_off) + 4 * (64 * (cg + c) + (uint32_t)__builtin_ctzll(acc[c])));
                return R;
            }
        }
    }
    R.verdict = (uint8_t)HDR_U8(I, terminal);
    return R;
}

}  // namespace

__global__ __launch_bounds__(kBlock) void http_classify_kernel(
    const uint8_t *__restrict__ arena, const uint64_t *__restrict__ offs, const uint32_t *__restrict__ lens,
    const uint32_t *__restrict__ conn_ids, uint32_t n, const DevConn *__restrict__ conns, uint32_t nconns,
    HttpTables T, uint8_t *__restrict__ out_verdict, int32_t *__restrict__ out_rule, uint32_t *__restrict__ out_consumed,
    uint64_t *__restrict__ counters, uint32_t ncounters) {
    __shared__ __attribute__((aligned(16))) uint8_t s_img[kLdsImageBytes];
    __shared__ uint32_t s_cnt[8 + kLdsRuleCounters];
    const uint32_t tid = threadIdx.x;

    // stage the hot rule set's image; zero the counters
    const int32_t hot = T.hot_ruleset;
    if (hot >= 0 && (uint32_t)hot < T.nrulesets) {
        const DevRuleset r = T.rulesets[hot];
        const uint4 *src = (const uint4 *)(T.images + r.image_off);
        const uint32_t n16 = min(r.image_len, kLdsImageBytes) / 16;
        for (uint32_t i = tid; i < n16; i += kBlock) ((uint4 *)s_img)[i] = src[i];
    }
    if (counters)
        for (uint32_t i = tid; i < 8 + kLdsRuleCounters; i += kBlock) s_cnt[i] = 0;
    __syncthreads();

    const uint32_t nrules = ncounters > 8 ? ncounters - 8 : 0;
    for (uint32_t idx = blockIdx.x * kBlock + tid; idx < n; idx += gridDim.x * kBlock) {
        const uint32_t ci = conn_ids[idx];
        const DevConn conn = ci < nconns ? conns[ci] : DevConn{-1, PROTO_NONE, {0, 0, 0}};
        // entries of other protocols belong to their own kernels; this kernel
        // also answers entries whose connection is unknown or has no parser
        if (conn.proto == PROTO_KAFKA || conn.proto == PROTO_MEMCACHE) continue;
        Result R{V_UNSUPPORTED, -1, 0};
        if (conn.proto == PROTO_HTTP && conn.ruleset >= 0 && (uint32_t)conn.ruleset < T.nrulesets) {
            const uint8_t *req = arena + offs[idx];
            const uint32_t len = lens[idx];
            const DevRuleset rs = T.rulesets[conn.ruleset];
            const uint8_t *gimg = T.images + rs.image_off;
            if (__all(conn.ruleset == hot)) R = classify(Img<true>{s_img}, gimg, req, len);
            else R = classify(Img<false>{gimg}, gimg, req, len);
        }
        out_verdict[idx] = R.verdict;
        out_rule[idx] = R.rule;
        out_consumed[idx] = R.consumed;
        if (counters) {
            atomicAdd(&s_cnt[R.verdict], 1u);
            if (R.rule >= 0 && (uint32_t)R.rule < nrules) {
                if (R.rule < kLdsRuleCounters) atomicAdd(&s_cnt[8 + R.rule], 1u);
                else atomicAdd((unsigned long long *)&counters[R.rule], 1ull);
            }
        }
    }
    if (counters) {
        __syncthreads();
        for (uint32_t i = tid; i < 8 + kLdsRuleCounters; i += kBlock) {
            const uint32_t v = s_cnt[i];
            if (!v) continue;
            if (i < 8) atomicAdd((unsigned long long *)&counters[nrules + i], (unsigned long long)v);
            else if (i - 8 < nrules) atomicAdd((unsigned long long *)&counters[i - 8], (unsigned long long)v);
        }
    }
}

// Host-side launcher (called from the C-ABI): a persistent grid of two
// workgroups per CU (LDS: 40 KiB image + 4 KiB counters each).
hipError_t LaunchHttpClassify(const uint8_t *arena, const uint64_t *offs, const uint32_t *lens, const uint32_t *conn_ids,
                              uint32_t n, const DevConn *conns, uint32_t nconns, const HttpTables &T,
                              uint8_t *verdict, int32_t *rule, uint32_t *consumed, uint64_t *counters,
                              uint32_t ncounters, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    static int num_cus = 0;
    if (num_cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || num_cus <= 0)
            num_cus = 256;
    }
    uint32_t blocks = (n + kBlock - 1) / kBlock;
    blocks = min(blocks, (uint32_t)num_cus * 2);
    hipLaunchKernelGGL(http_classify_kernel, dim3(blocks), dim3(kBlock), 0, stream, arena, offs, lens, conn_ids, n,
                       conns, nconns, T, verdict, rule, consumed, counters, ncounters);
    return hipGetLastError();
}

}  // namespace l7
