// HTTP/1 request classification on gfx950 (product code), v3.
//
// Work split: one wave owns a tile of 64 consecutive requests, one lane per
// request.  The requests' bytes reach the lanes through LDS in rounds:
//
//   * DMA: each round the wave copies, for every lane still working, the next
//     128-byte window of its request (one cache line: windows are 128-byte
//     aligned in memory) into the lane's LDS slot with global_load_lds_dwordx4.
//     Eight lanes cooperate per window, so one wave-instruction moves eight
//     full cache lines (coalesced) and a round is eight instructions for the
//     whole wave.  Chunks outside [current position, request end) are not read.
//     The chunk order inside a slot is XOR-swizzled by the lane index, so the
//     lanes' later ds_read_b128 of "their chunk k" hit 64 distinct banks.
//   * parse: every lane then consumes its window from LDS with the resumable
//     framer below: the request line, header names (through the rule set's
//     name DFA), and the values of header slots the rule set constrains (fed
//     through the slot's DFAs, end-state rule masks AND-ed into <= 4 u64
//     accumulators).  Values nobody constrains are skipped 16 bytes per step
//     with a SWAR test for CTL/DEL.
//
// Sixteen waves per CU (one 1024-thread workgroup, all 160 KiB of LDS: 16 x
// 8 KiB windows + the hot rule-set image + rule counters) keep ~100 KiB of DMA
// in flight per CU while other waves parse.
//
// The grammar, error precedence and policy semantics restate Envoy's HTTP/1
// codec + cilium.l7policy (envoy/cilium_l7policy.cc:127-182,
// envoy/cilium_network_policy.h:50-237); the oracle is
// oracle/http_ref.c.  Rule sets larger than 4 chunks x 2 DFAs per slot are
// evaluated in several framing passes (results identical; only cost grows).
#include <hip/hip_runtime.h>

#include <cstddef>

#include "../device_tables.h"

namespace l7 {

namespace {

constexpr int kWaves = 16;
constexpr int kBlock = 64 * kWaves;
constexpr uint32_t kWin = 128;                 // bytes per lane per round (one cache line)
constexpr uint32_t kWaveLds = 64 * kWin;       // 8 KiB per wave
constexpr int kLdsRuleCounters = 1016;
constexpr uint32_t kOffImg = kWaves * kWaveLds;
constexpr uint32_t kOffCnt = kOffImg + kLdsImageBytes;
constexpr uint32_t kLdsBytes = kOffCnt + (8 + kLdsRuleCounters) * 4;
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");

enum : uint32_t {
    M_METHOD, M_TARGET, M_VERSION, M_LINE, M_NAME, M_OWS, M_VALUE, M_SKIP, M_LF, M_ENDLF, M_DONE
};
constexpr uint32_t kNoSlot = 0xFF;

__constant__ uint32_t kVer[10] = {'H', 'T', 'T', 'P', '/', 0x100, '.', 0x100, '\r', '\n'};

// Per-dword SWAR: bit 7 of byte i set iff byte i < 0x20 or == 0x7F (exact).
__device__ __forceinline__ uint32_t stop_bits(uint32_t x) {
    const uint32_t t = x & 0x7F7F7F7Fu;
    return (~(t + 0x60606060u) | (t + 0x01010101u)) & ~x & 0x80808080u;
}
// bit 7 of each byte -> 4-bit nibble
__device__ __forceinline__ uint32_t nib(uint32_t s) { return __builtin_amdgcn_ubfe((s >> 7) * 0x204081u, 21, 4); }

// Rule-set image accessor: LDS (hot rule set) or global memory.
template <bool kLds>
struct Img {
    const uint8_t *p;
    __device__ __forceinline__ uint32_t u8(uint32_t o) const { return p[o]; }
    __device__ __forceinline__ uint32_t u16(uint32_t o) const { return *(const uint16_t *)(p + o); }
    __device__ __forceinline__ uint32_t u32(uint32_t o) const { return *(const uint32_t *)(p + o); }
    __device__ __forceinline__ uint64_t u64(uint32_t o) const { return *(const uint64_t *)(p + o); }
};

// Header fields: wave-uniform in the LDS path (kept in SGPRs there).
template <bool kLds>
__device__ __forceinline__ uint32_t uni(uint32_t v) {
    return kLds ? (uint32_t)__builtin_amdgcn_readfirstlane((int)v) : v;
}
#define HDR_U32(I, field) uni<kLds>((I).u32(offsetof(ImgHeader, field)))
#define HDR_U16(I, field) uni<kLds>((I).u16(offsetof(ImgHeader, field)))
#define HDR_U8(I, field) uni<kLds>((I).u8(offsetof(ImgHeader, field)))

// ---------------------------------------------------------------- lane state
struct Lane {
    uint64_t wb;        // request start rounded down to 128 B (absolute)
    uint32_t a0;        // position of request byte 0 relative to wb
    uint32_t lena;      // a0 + len
    uint32_t pa;        // next position to look at
    uint32_t mode;
    uint32_t mark;      // token start (method/target/name) or version index
    uint32_t idx;       // request index
    bool done;
    uint8_t verdict;
    int32_t rule;
    uint32_t consumed;
    // framing
    uint32_t present;   // slots seen (first occurrence)
    uint32_t slot;      // slot of the current header value (kNoSlot: none)
    uint32_t nstate;    // name DFA state
    uint32_t ninfo;     // NI_* flags of the current header name
    bool have_cl, have_te, cl_bad, cl_ws, in_ows;
    uint32_t ndig;
    uint64_t clv, cl;
    // DFAs of the current slot
    uint32_t nd;
    uint32_t dcls[kDfasPerPass], dtrans[kDfasPerPass], dmask[kDfasPerPass], dncls[kDfasPerPass];
    uint32_t st[kDfasPerPass], saved[kDfasPerPass];
    // rule accumulators for the current chunk group
    uint64_t acc[kChunksPerPass];
    uint32_t cg, dg;    // chunk group, DFA group of this pass
};

template <bool kLds>
__device__ __forceinline__ void slot_begin(const Img<kLds> &I, Lane &L, uint32_t slot) {
    const uint32_t lo = I.u8(offsetof(ImgHeader, slot_dfa) + slot) + L.dg * kDfasPerPass;
    const uint32_t hi = I.u8(offsetof(ImgHeader, slot_dfa) + slot + 1);
    L.nd = hi > lo ? min(hi - lo, (uint32_t)kDfasPerPass) : 0;
#pragma unroll
    for (int k = 0; k < kDfasPerPass; k++) {
        L.st[k] = 0;
        if ((uint32_t)k < L.nd) {
            const uint32_t d = HDR_U32(I, dfa_off) + (lo + k) * sizeof(DevDfa);
            L.dcls[k] = I.u32(d + 0);
            L.dtrans[k] = I.u32(d + 4);
            L.dmask[k] = I.u32(d + 8);
            const uint32_t nc_st = I.u32(d + 12);
            L.dncls[k] = nc_st & 0xFFFF;
            L.st[k] = nc_st >> 16;
        }
    }
}

template <bool kLds>
__device__ __forceinline__ void slot_step(const Img<kLds> &I, Lane &L, uint32_t c) {
#pragma unroll
    for (int k = 0; k < kDfasPerPass; k++)
        if (L.st[k] != 0) L.st[k] = I.u16(L.dtrans[k] + 2 * (L.st[k] * L.dncls[k] + I.u8(L.dcls[k] + c)));
}

// AND the end states' masks of the pass's chunks into the accumulators.
template <bool kLds>
__device__ __forceinline__ void slot_end(const Img<kLds> &I, Lane &L) {
    const uint32_t nchunks = HDR_U8(I, nchunks);
    const uint32_t nc = nchunks > L.cg ? min(nchunks - L.cg, (uint32_t)kChunksPerPass) : 0;
#pragma unroll
    for (int k = 0; k < kDfasPerPass; k++) {
        if ((uint32_t)k >= L.nd) break;
        const uint32_t base = L.dmask[k] + 8 * (L.st[k] * nchunks + L.cg);
#pragma unroll
        for (int c = 0; c < kChunksPerPass; c++)
            if ((uint32_t)c < nc) L.acc[c] &= I.u64(base + 8 * c);
    }
}

template <bool kLds>
__device__ __forceinline__ void acc_init(const Img<kLds> &I, Lane &L) {
    const uint32_t nchunks = HDR_U8(I, nchunks);
#pragma unroll
    for (int c = 0; c < kChunksPerPass; c++)
        L.acc[c] = L.cg + c < nchunks ? I.u64(HDR_U32(I, init_off) + 8 * (L.cg + c)) : 0;
}

template <bool kLds>
__device__ __forceinline__ void frame_reset(const Img<kLds> &I, Lane &L) {
    L.pa = L.a0;
    L.mode = M_METHOD;
    L.mark = L.a0;
    L.present = 0;
    L.have_cl = L.have_te = false;
    L.cl = 0;
    slot_begin(I, L, SLOT_METHOD);
}

__device__ __forceinline__ void finish(Lane &L, uint8_t v, int32_t rule = -1) {
    L.done = true;
    L.mode = M_DONE;
    L.verdict = v;
    L.rule = rule;
    if (v != V_ALLOW && v != V_DENY) L.consumed = 0;
}

// Headers complete (framing succeeded for this pass): next pass or verdict.
template <bool kLds>
__device__ __forceinline__ void headers_done(const Img<kLds> &I, Lane &L) {
    const uint64_t total = (uint64_t)(L.pa - L.a0) + L.cl;
    if (L.have_te) {
        finish(L, V_UNSUPPORTED);
    } else if (total > 0xFFFFFFFFull) {
        finish(L, V_PARSE_ERROR);
    } else if (total > (uint64_t)(L.lena - L.a0)) {
        finish(L, V_INCOMPLETE);
    } else {
        L.consumed = (uint32_t)total;
        const uint32_t max_dfas = HDR_U8(I, max_slot_dfas);
        const uint32_t ndg = max_dfas ? (max_dfas + kDfasPerPass - 1) / kDfasPerPass : 1;
        const uint32_t nchunks = HDR_U8(I, nchunks);
        if (L.dg + 1 < ndg) {  // more DFAs of this chunk group: frame again
            L.dg++;
            frame_reset(I, L);
        } else {
            const uint32_t nc = nchunks > L.cg ? min(nchunks - L.cg, (uint32_t)kChunksPerPass) : 0;
            // headers the rule set constrains but the request lacks
            uint32_t missing = HDR_U32(I, ref_slots) & 0xFFFF & ~L.present;
            while (missing) {
                const uint32_t s = __builtin_ctz(missing);
                missing &= missing - 1;
#pragma unroll
                for (int c = 0; c < kChunksPerPass; c++)
                    if ((uint32_t)c < nc) L.acc[c] &= I.u64(HDR_U32(I, absent_off) + 8 * (s * nchunks + L.cg + c));
            }
            int32_t hit = -1;
#pragma unroll
            for (int c = kChunksPerPass - 1; c >= 0; c--)
                if ((uint32_t)c < nc && L.acc[c]) hit = (int32_t)(64 * (L.cg + c) + (uint32_t)__builtin_ctzll(L.acc[c]));
            if (hit >= 0) {
                finish(L, V_ALLOW, (int32_t)I.u32(HDR_U32(I, rule_off) + 4 * (uint32_t)hit));
            } else if (L.cg + kChunksPerPass < nchunks) {  // next chunk group
                L.cg += kChunksPerPass;
                L.dg = 0;
                acc_init(I, L);
                frame_reset(I, L);
            } else {
                finish(L, (uint8_t)HDR_U8(I, terminal));
            }
        }
    }
}

// Header line complete (CRLF seen); false = Content-Length framing error.
template <bool kLds>
__device__ __forceinline__ bool line_done(const Img<kLds> &I, Lane &L) {
    bool ok = true;
    if (L.ninfo & NI_CL) {
        ok = !(L.have_cl || L.ndig == 0 || L.ndig > 10 || L.cl_bad);
        L.have_cl = true;
        L.cl = L.clv;
    }
    if (L.ninfo & NI_TE) L.have_te = true;
    if (L.slot != kNoSlot) {
        slot_end(I, L);
        L.present |= 1u << L.slot;
    }
    return ok;
}

// ---------------------------------------------------------------- parse one window
// Consumes [L.pa, min(window end, request end)) from the lane's LDS slot.
// Every loop has a single exit; errors set the mode to M_DONE, so later
// blocks fall through (keeps the control flow shallow for the register
// allocator).
template <bool kLds>
__device__ __forceinline__ void parse_window(const Img<kLds> &I, Lane &L, const uint8_t *slot, uint32_t swz) {
    const uint32_t lim = min((L.pa & ~(kWin - 1)) + kWin, L.lena);
    // byte at p (p < lim): chunk (p >> 4) & 7 sits at position ((p >> 4) & 7) ^ sw
    auto B = [&](uint32_t p) -> uint32_t { return slot[(p & (kWin - 1)) ^ swz]; };
    const uint32_t ncls_name = HDR_U16(I, name_ncls);
    const uint32_t name_cls = HDR_U32(I, name_cls_off), name_trans = HDR_U32(I, name_trans_off);

    // ---- request line
    if (L.mode == M_METHOD) {  // 1*tchar SP
        uint32_t c = 0;
        for (; L.pa < lim; L.pa++) {
            c = B(L.pa);
            if (I.u8(name_cls + c) == 0) break;  // not a tchar (SP included)
            slot_step(I, L, c);
        }
        if (L.pa < lim) {
            if (c != ' ' || L.pa == L.mark) {
                finish(L, V_PARSE_ERROR);
            } else {
                slot_end(I, L);
                L.present |= 1u << SLOT_METHOD;
                L.pa++;
                L.mark = L.pa;
                L.mode = M_TARGET;
                slot_begin(I, L, SLOT_PATH);
            }
        }
    }
    if (L.mode == M_TARGET) {  // 1*(VCHAR / obs-text) SP
        uint32_t c = 0;
        for (; L.pa < lim; L.pa++) {
            c = B(L.pa);
            if (c <= 0x20 || c == 0x7F) break;
            slot_step(I, L, c);
        }
        if (L.pa < lim) {
            if (c != ' ' || L.pa == L.mark) {
                finish(L, V_PARSE_ERROR);
            } else {
                slot_end(I, L);
                L.present |= 1u << SLOT_PATH;
                L.pa++;
                L.mark = 0;
                L.mode = M_VERSION;
            }
        }
    }
    if (L.mode == M_VERSION) {  // "HTTP/" DIGIT "." DIGIT CRLF
        for (; L.pa < lim && L.mark < 10; L.pa++, L.mark++) {
            const uint32_t c = B(L.pa);
            const uint32_t want = kVer[L.mark];
            if (want == 0x100 ? c - '0' >= 10u : c != want) break;
        }
        if (L.mark == 10) L.mode = M_LINE;
        else if (L.pa < lim) finish(L, V_PARSE_ERROR);
    }
    // ---- header lines
    while (L.mode >= M_LINE && L.mode < M_DONE && L.pa < lim) {
        if (L.mode == M_LINE) {
            if (B(L.pa) == '\r') {
                L.pa++;
                L.mode = M_ENDLF;
            } else {
                L.mode = M_NAME;
                L.mark = L.pa;
                L.nstate = kNameStart;
            }
        }
        if (L.mode == M_ENDLF && L.pa < lim) {
            if (B(L.pa) != '\n') {
                finish(L, V_PARSE_ERROR);
            } else {
                L.pa++;
                headers_done(I, L);  // done, or a new pass from the request start
            }
        }
        if (L.mode == M_NAME) {  // 1*tchar ":"  (obs-fold SP/HT is not a tchar)
            uint32_t c = 0;
            for (; L.pa < lim; L.pa++) {
                c = B(L.pa);
                const uint32_t k = I.u8(name_cls + c);
                if (k == 0) break;
                L.nstate = I.u16(name_trans + 2 * (L.nstate * ncls_name + k));
            }
            if (L.pa < lim) {
                if (c != ':' || L.pa == L.mark) {
                    finish(L, V_PARSE_ERROR);
                } else {
                    L.pa++;
                    L.ninfo = L.nstate >= kNameStart ? I.u8(HDR_U32(I, name_info_off) + L.nstate) : 0;
                    uint32_t s = kNoSlot;
                    if (L.ninfo & NI_HOST) s = SLOT_AUTHORITY;
                    else if (L.ninfo & NI_CUSTOM) s = SLOT_CUSTOM0 + (L.ninfo & NI_CUSTOM) - 1;
                    if (s != kNoSlot && ((L.present >> s) & 1)) s = kNoSlot;                // first occurrence only
                    if (s != kNoSlot && !((HDR_U32(I, ref_slots) >> s) & 1)) s = kNoSlot;  // nobody looks at it
                    L.slot = s;
                    L.mode = M_OWS;
                }
            }
        }
        if (L.mode == M_OWS) {
            for (; L.pa < lim; L.pa++) {
                const uint32_t c = B(L.pa);
                if (c != ' ' && c != '\t') break;
            }
            if (L.pa < lim) {
                if (L.slot == kNoSlot && !(L.ninfo & NI_CL)) {
                    L.mode = M_SKIP;
                } else {
                    L.mode = M_VALUE;
                    if (L.slot != kNoSlot) {
                        slot_begin(I, L, L.slot);
                    } else {
                        L.nd = 0;
#pragma unroll
                        for (int k = 0; k < kDfasPerPass; k++) L.st[k] = 0;
                    }
                    L.in_ows = false;
                    L.clv = 0;
                    L.ndig = 0;
                    L.cl_bad = L.cl_ws = false;
                }
            }
        }
        if (L.mode == M_VALUE) {  // a value some rule (or Content-Length framing) looks at
            uint32_t c = 0;
            for (; L.pa < lim; L.pa++) {
                c = B(L.pa);
                if ((c < 0x20 && c != '\t') || c == 0x7F) break;  // CR ends it; other CTLs are errors
                const bool ws = c == ' ' || c == '\t';
                if (ws && !L.in_ows) {
#pragma unroll
                    for (int k = 0; k < kDfasPerPass; k++) L.saved[k] = L.st[k];
                }
                L.in_ows = ws;
                L.cl_ws |= ws;
                if (!ws) {
                    if (c - '0' < 10u && !L.cl_ws) {
                        L.clv = L.clv * 10 + (c - '0');
                        L.ndig++;
                    } else {
                        L.cl_bad = true;
                    }
                }
                slot_step(I, L, c);
            }
            if (L.pa < lim) {
                if (c != '\r') {
                    finish(L, V_PARSE_ERROR);
                } else {
                    if (L.in_ows) {  // trailing OWS is not part of the value
#pragma unroll
                        for (int k = 0; k < kDfasPerPass; k++) L.st[k] = L.saved[k];
                    }
                    L.pa++;
                    L.mode = M_LF;
                }
            }
        }
        if (L.mode == M_SKIP) {  // a value nobody looks at: find CR (or a CTL / DEL) 16 bytes a step
            uint32_t stop = 0;
            while (L.pa < lim) {
                const uint32_t k = L.pa >> 4;
                const uint4 w = *(const uint4 *)(slot + ((L.pa & (kWin - 16)) ^ swz));
                uint32_t m = nib(stop_bits(w.x)) | nib(stop_bits(w.y)) << 4 | nib(stop_bits(w.z)) << 8 |
                             nib(stop_bits(w.w)) << 12;
                m &= 0xFFFFu << (L.pa & 15);
                const uint32_t cend = (k + 1) * 16;
                if (cend > lim) m &= (1u << (lim & 15)) - 1u;  // lim inside this chunk
                const uint32_t p = k * 16 + (uint32_t)__builtin_ctz(m | 0x10000u);
                L.pa = min(p, lim);
                if (p < cend) {
                    const uint32_t c = B(p);
                    if (c != '\t') {
                        stop = c | 0x100;
                        break;
                    }
                    L.pa++;
                }
            }
            if (stop) {
                if (stop != ('\r' | 0x100)) {
                    finish(L, V_PARSE_ERROR);
                } else {
                    L.pa++;
                    L.mode = M_LF;
                }
            }
        }
        if (L.mode == M_LF && L.pa < lim) {
            if (B(L.pa) != '\n') {
                finish(L, V_PARSE_ERROR);
            } else {
                L.pa++;
                if (line_done(I, L)) L.mode = M_LINE;
                else finish(L, V_PARSE_ERROR);
            }
        }
    }
}

// ---------------------------------------------------------------- DMA
// Copies, for every working lane t, chunks [lo, hi] of the 128-byte window at
// `win` into LDS slot t (chunk c stored at position c ^ s(t)).  packed =
// window address | hi << 4 | lo << 1 | 1 (addresses are 128-byte aligned).
__device__ __forceinline__ void dma_windows(uint8_t *wave_lds, uint64_t packed, uint32_t lane) {
    const uint32_t plo = (uint32_t)packed, phi = (uint32_t)(packed >> 32);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's earlier LDS reads have landed
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const int t = 8 * j + (int)(lane >> 3);
        const uint32_t tlo = __shfl(plo, t), thi = __shfl(phi, t);
        const uint32_t c = (lane & 7) ^ (((uint32_t)t >> 1) & 7);
        const uint32_t clo = (tlo >> 1) & 7, chi = (tlo >> 4) & 7;
        if ((tlo & 1) && c >= clo && c <= chi) {
            const uint8_t *src = (const uint8_t *)((((uint64_t)thi) << 32) | (tlo & ~127u)) + 16 * c;
            __builtin_amdgcn_global_load_lds((const void *)src,
                                             (__attribute__((address_space(3))) void *)(wave_lds + j * 1024), 16, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

struct Out {
    uint8_t *verdict;
    int32_t *rule;
    uint32_t *consumed;
    uint32_t *s_cnt;
    uint64_t *counters;
    uint32_t nrules;
};

__device__ __forceinline__ void emit(const Lane &L, const Out &O) {
    O.verdict[L.idx] = L.verdict;
    O.rule[L.idx] = L.rule;
    O.consumed[L.idx] = L.consumed;
    if (O.counters) {
        atomicAdd(&O.s_cnt[L.verdict], 1u);
        if (L.rule >= 0 && (uint32_t)L.rule < O.nrules) {
            if (L.rule < kLdsRuleCounters) atomicAdd(&O.s_cnt[8 + L.rule], 1u);
            else atomicAdd((unsigned long long *)&O.counters[L.rule], 1ull);
        }
    }
}

// All rounds of one tile.
template <bool kLds>
__device__ __forceinline__ void run_tile(Lane &L, const uint8_t *img, uint8_t *wave_lds, uint32_t lane, const Out &O) {
    const Img<kLds> I{img};
    if (!L.done) {
        L.cg = 0;
        L.dg = 0;
        acc_init(I, L);
        frame_reset(I, L);
        if (L.lena == L.a0) {
            finish(L, V_INCOMPLETE);
            emit(L, O);
        }
    }
    const uint8_t *slot = wave_lds + lane * kWin;
    const uint32_t swz = ((lane >> 1) & 7) << 4;
    while (__any(!L.done)) {
        uint64_t packed = 0;
        if (!L.done) {
            const uint32_t w = L.pa & ~(kWin - 1);
            const uint32_t lo = (L.pa - w) >> 4;
            const uint32_t hi = min(L.lena - 1 - w, kWin - 1) >> 4;
            packed = (L.wb + w) | (hi << 4) | (lo << 1) | 1u;
        }
        dma_windows(wave_lds, packed, lane);
        if (!L.done) {
            parse_window(I, L, slot, swz);
            if (!L.done && L.pa >= L.lena) finish(L, V_INCOMPLETE);
            if (L.done) emit(L, O);
        }
    }
}

}  // namespace

// kHot = true : requests whose connection uses the hot rule set (image in LDS),
//               plus entries on connections without an HTTP parser.
// kHot = false: every other HTTP request (images read through L2); all of
//               them when no hot kernel runs (T.hot_ruleset < 0).
template <bool kHot>
__global__ __launch_bounds__(kBlock) void http_classify_kernel(
    const uint8_t *__restrict__ arena, const uint64_t *__restrict__ offs, const uint32_t *__restrict__ lens,
    const uint32_t *__restrict__ conn_ids, uint32_t n, const DevConn *__restrict__ conns, uint32_t nconns,
    HttpTables T, uint8_t *__restrict__ out_verdict, int32_t *__restrict__ out_rule, uint32_t *__restrict__ out_consumed,
    uint64_t *__restrict__ counters, uint32_t ncounters) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63, wave = tid >> 6;
    uint8_t *s_img = lds + kOffImg;
    uint32_t *s_cnt = (uint32_t *)(lds + kOffCnt);

    const int32_t hot = T.hot_ruleset;
    const bool hot_ok = hot >= 0 && (uint32_t)hot < T.nrulesets && T.rulesets[hot].image_len <= kLdsImageBytes;
    if (kHot && !hot_ok) return;
    // stage the hot rule set's image; zero the counters
    if (kHot) {
        const DevRuleset r = T.rulesets[hot];
        const uint4 *src = (const uint4 *)(T.images + r.image_off);
        const uint32_t n16 = (r.image_len + 15) / 16;
        for (uint32_t i = tid; i < n16; i += kBlock) ((uint4 *)s_img)[i] = src[i];
    }
    if (counters)
        for (uint32_t i = tid; i < 8 + kLdsRuleCounters; i += kBlock) s_cnt[i] = 0;
    __syncthreads();

    const Out O{out_verdict, out_rule, out_consumed, s_cnt, counters, ncounters > 8 ? ncounters - 8 : 0};
    uint8_t *wave_lds = lds + wave * kWaveLds;
    const uint32_t ntiles = (n + 63) / 64;
    for (uint32_t tile = blockIdx.x * kWaves + wave; tile < ntiles; tile += gridDim.x * kWaves) {
        Lane L;
        L.idx = tile * 64 + lane;
        L.done = true;
        L.verdict = V_UNSUPPORTED;
        L.rule = -1;
        L.consumed = 0;
        L.mode = M_DONE;
        L.wb = 0;
        L.a0 = L.lena = L.pa = 0;
        const uint8_t *img = kHot ? s_img : nullptr;
        if (L.idx < n) {
            const uint32_t ci = conn_ids[L.idx];
            const DevConn conn = ci < nconns ? conns[ci] : DevConn{-1, PROTO_NONE, {0, 0, 0}};
            // entries of other protocols belong to their own kernels; the HTTP
            // kernel answers entries whose connection is unknown or has no parser
            const bool mine = !(conn.proto == PROTO_KAFKA || conn.proto == PROTO_MEMCACHE);
            const bool http = mine && conn.proto == PROTO_HTTP && conn.ruleset >= 0 && (uint32_t)conn.ruleset < T.nrulesets;
            const bool is_hot = http && hot_ok && conn.ruleset == hot;
            if (mine && !http && (kHot || !hot_ok)) emit(L, O);  // unsupported connection: answered now
            if (http && is_hot == kHot) {
                const uint64_t off = offs[L.idx];
                const uint32_t len = lens[L.idx];
                const uint64_t a = (uint64_t)(arena + off);
                L.wb = a & ~(uint64_t)127;
                L.a0 = (uint32_t)(a & 127);
                L.lena = L.a0 + len;
                if (L.lena < L.a0) L.lena = 0xFFFFFFFFu;  // len > 4 GiB - 128: framing stops there
                if (!kHot) img = T.images + T.rulesets[conn.ruleset].image_off;
                L.done = false;
            }
        }
        run_tile<kHot>(L, img, wave_lds, lane, O);
    }
    if (counters) {
        __syncthreads();
        const uint32_t nrules = O.nrules;
        for (uint32_t i = tid; i < 8 + kLdsRuleCounters; i += kBlock) {
            const uint32_t v = s_cnt[i];
            if (!v) continue;
            if (i < 8) atomicAdd((unsigned long long *)&counters[nrules + i], (unsigned long long)v);
            else if (i - 8 < nrules) atomicAdd((unsigned long long *)&counters[i - 8], (unsigned long long)v);
        }
    }
}

// Host-side launcher (called from the C-ABI): persistent grids of one
// 1024-thread workgroup per CU; the hot-rule-set kernel, then (only if some
// HTTP connection uses another rule set) the general one.
hipError_t LaunchHttpClassify(const uint8_t *arena, const uint64_t *offs, const uint32_t *lens, const uint32_t *conn_ids,
                              uint32_t n, const DevConn *conns, uint32_t nconns, const HttpTables &T, bool any_cold,
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
    const uint32_t ntiles = (n + 63) / 64;
    uint32_t blocks = (ntiles + kWaves - 1) / kWaves;
    blocks = min(blocks, (uint32_t)num_cus);
    const bool hot = T.hot_ruleset >= 0;
    if (hot)
        hipLaunchKernelGGL(http_classify_kernel<true>, dim3(blocks), dim3(kBlock), 0, stream, arena, offs, lens, conn_ids,
                           n, conns, nconns, T, verdict, rule, consumed, counters, ncounters);
    if (!hot || any_cold)
        hipLaunchKernelGGL(http_classify_kernel<false>, dim3(blocks), dim3(kBlock), 0, stream, arena, offs, lens,
                           conn_ids, n, conns, nconns, T, verdict, rule, consumed, counters, ncounters);
    return hipGetLastError();
}

}  // namespace l7
