// HTTP/1 request classification on gfx950 (product code), v4.
//
// One wave owns a tile of 64 consecutive requests, one lane per request.
// Work proceeds in rounds, each made of three wave-wide steps:
//
//   1. window DMA: for every lane that needs bytes, the wave copies the next
//      256-byte window of the lane's request (16-byte aligned, clipped to the
//      request) into the lane's LDS slot with global_load_lds_dwordx4.
//      Sixteen lanes cooperate per window (one wave-instruction moves four
//      windows); chunk c of lane t's window is stored at position c ^ (t & 15)
//      so the lanes' later ds_read_b128 of "their chunk k" hit 64 distinct
//      banks.
//   2. parse: each lane runs the resumable framer over its window: request
//      line, header names (name DFA), header values of slots the rule set
//      constrains (slot DFAs; end-state rule masks AND-ed into u64
//      accumulators), Content-Length digits.  Bytes come from a two-chunk
//      register cursor (16-byte LDS reads, next chunk prefetched); tchar and
//      CTL tests are ALU; on the long tokens the DFA class of the next byte is
//      fetched while the current transition is in flight, so a byte costs one
//      dependent LDS round trip.  Values nobody constrains are skipped 16
//      bytes a step (SWAR CTL/DEL test).
//   3. skip: before its first window the wave streams its tile's byte span
//      once (coalesced LDS-DMA, 16 pieces of 1 KiB in flight) and keeps a
//      bit per 16-byte chunk holding a value-stop byte (< 0x20 other than HT,
//      or DEL) in registers.  A lane whose unconstrained value runs past its
//      window finds the first marked chunk after it by ds_bpermute and reads
//      just that chunk; when the stop is the CR of "\r\n\r\n" the request
//      finishes there, otherwise the next window starts at the stop.
//
// For the benchmark stream a tile takes the span stream, one window per
// request (the head) and one map lookup (the long pad header); constrained
// values stop being walked once their DFA state is absorbing.
//
// One 512-thread workgroup per CU: 8 waves x 16 KiB windows + the hot rule
// set's image (<= 32 KiB) = 160 KiB of LDS.
//
// Grammar, error precedence and policy semantics: Envoy's HTTP/1 codec +
// cilium.l7policy (envoy/cilium_l7policy.cc:127-182,
// envoy/cilium_network_policy.h:50-237); the oracle is
// oracle/http_ref.c.  Rule sets larger than kChunksPerPass chunks x
// kDfasPerPass DFAs per slot are evaluated in several framing passes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>

#include "../device_tables.h"
#include "copy_in.h"
#include "gmem.h"
#include "service.h"

// OCKL's DPP wave reductions (64-bit forms are not declared by hip_runtime.h)
extern "C" __device__ __attribute__((const)) unsigned long long __ockl_wfred_min_u64(unsigned long long);
extern "C" __device__ __attribute__((const)) unsigned long long __ockl_wfred_max_u64(unsigned long long);
extern "C" __device__ __attribute__((const)) unsigned long long __ockl_wfred_and_u64(unsigned long long);

namespace l7 {

namespace {

// (Round 6: 16 waves with 128-byte windows, 128 VGPRs, 4 waves per SIMD:
// 22.8 ms on cfg5 against 17.0 -- the spills and twice the window rounds cost
// more than the occupancy gains; 12 waves 23.2 ms; profiles/r6/ab6d_*.)
constexpr int kWaves = 8;
constexpr int kBlock = 64 * kWaves;
constexpr uint32_t kWin = 256;                 // bytes per lane window
constexpr uint32_t kWinChunks = kWin / 16;
constexpr uint32_t kWaveLds = 64 * kWin;       // 16 KiB per wave
constexpr uint32_t kOffImg = kWaves * kWaveLds;
constexpr uint32_t kLdsBytes = kOffImg + kLdsImageBytes;
static_assert(kLdsBytes <= 160 * 1024, "LDS budget");
constexpr uint32_t kLanesPerWin = kWinChunks;  // DMA: one lane per 16-byte chunk of a window
constexpr uint32_t kWinPerInst = 64 / kLanesPerWin;
static_assert(kWinChunks == 8 || kWinChunks == 16, "window size");
// Chunk swizzle of lane t's slot, chosen so that the 16 lanes of each
// ds_read_b128 bank group reading "their chunk k" cover all 64 banks.
__device__ __forceinline__ uint32_t win_swizzle(uint32_t t) {
    return kWinChunks == 16 ? (t & 15) : ((t >> 1) & 7);
}

// Optional per-phase cycle accounting (debug builds with -DL7G_PHASE_TIMING:
// libl7gpu_timing.so, used by tools/exp_http.py).  Slots: 0 dma, 1 parse,
// 2 tile map + skips, 3 emit/other, 4 rounds, 5 skips, 6 tiles.
#ifdef L7G_PHASE_TIMING
__device__ unsigned long long g_phase[16];
#define PH_DECL uint64_t ph_t = __builtin_amdgcn_s_memtime(); uint64_t ph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define PH_MARK(slot) do { const uint64_t ph_n = __builtin_amdgcn_s_memtime(); ph_acc[slot] += ph_n - ph_t; ph_t = ph_n; } while (0)
#define PH_COUNT(slot, v) (ph_acc[slot] += (v))
#define PH_FLUSH(lane) do { if ((lane) == 0) for (int ph_i = 0; ph_i < 8; ph_i++) atomicAdd(&g_phase[ph_i], (unsigned long long)ph_acc[ph_i]); } while (0)
#else
#define PH_DECL
#define PH_MARK(slot) do {} while (0)
#define PH_COUNT(slot, v) do {} while (0)
#define PH_FLUSH(lane) do {} while (0)
#endif
// latency path: cycles of a section, added to g_phase[slot] by lane 0
#ifdef L7G_PHASE_TIMING
#define LAT_T0 uint64_t lat_t = __builtin_amdgcn_s_memtime();
#define LAT_T(slot) do { const uint64_t lat_n = __builtin_amdgcn_s_memtime(); if ((threadIdx.x & 63) == 0) atomicAdd(&g_phase[slot], (unsigned long long)(lat_n - lat_t)); lat_t = lat_n; } while (0)
#define LAT_N(slot) do { if ((threadIdx.x & 63) == 0) atomicAdd(&g_phase[slot], 1ull); } while (0)
#else
#define LAT_T0
#define LAT_T(slot) do {} while (0)
#define LAT_N(slot) do {} while (0)
#endif

enum : uint32_t {
    M_METHOD, M_TARGET, M_VERSION, M_LINE, M_NAME, M_OWS, M_VALUE, M_SKIP, M_LF, M_ENDLF, M_DONE,
    // chunked body (Transfer-Encoding: chunked), after the verdict is known
    M_CHSIZE, M_CHEXT, M_CHLF, M_CHDATA, M_CHDCR, M_CHDLF, M_TRL, M_TRLSCAN, M_TRLLF, M_TRLEND
};
constexpr uint32_t kNoSlot = 0xFF;

__constant__ uint32_t kVer[10] = {'H', 'T', 'T', 'P', '/', 0x100, '.', 0x100, '\r', '\n'};

__device__ __forceinline__ bool is_tchar(uint32_t c) {
    // tchar = "!#$%&'*+-.^_`|~" / DIGIT / ALPHA  (bitmap over 0x20..0x7F)
    const uint32_t m1 = 0x03FF6CFAu;  // 0x20-0x3F
    const uint32_t m2 = 0xC7FFFFFEu;  // 0x40-0x5F
    const uint32_t m3 = 0x57FFFFFFu;  // 0x60-0x7F
    const uint32_t w = c < 0x40 ? m1 : (c < 0x60 ? m2 : m3);
    return (c - 0x20u < 0x60u) && ((w >> (c & 31)) & 1);
}

// Per-dword SWAR: bit 7 of byte i set iff byte i < 0x20 or == 0x7F (exact).
__device__ __forceinline__ uint32_t stop_bits(uint32_t x) {
    const uint32_t t = x & 0x7F7F7F7Fu;
    return (~(t + 0x60606060u) | (t + 0x01010101u)) & ~x & 0x80808080u;
}
// bit 7 of each byte -> 4-bit nibble
__device__ __forceinline__ uint32_t nib(uint32_t s) { return __builtin_amdgcn_ubfe((s >> 7) * 0x204081u, 21, 4); }
// 16-bit mask of the stop bytes of a chunk
__device__ __forceinline__ uint32_t stop_mask(uint4 w) {
    return nib(stop_bits(w.x)) | nib(stop_bits(w.y)) << 4 | nib(stop_bits(w.z)) << 8 | nib(stop_bits(w.w)) << 12;
}
// bit 7 of byte i set iff byte i <= 0x20 or == 0x7F (ends a request target)
__device__ __forceinline__ uint32_t tstop_bits(uint32_t x) {
    const uint32_t t = x & 0x7F7F7F7Fu;
    return (~(t + 0x5F5F5F5Fu) | (t + 0x01010101u)) & ~x & 0x80808080u;
}
// bit 7 of byte i set iff byte i ends a header value: < 0x20 other than HT, or DEL
__device__ __forceinline__ uint32_t vstop_bits(uint32_t x) {
    const uint32_t t = x ^ 0x09090909u;  // HT -> 0
    const uint32_t ht = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
    return stop_bits(x) & ~ht;
}
// nonzero iff some byte of the chunk is < 0x20 or DEL (HT included: a superset
// of the value stops, for the tile map)
__device__ __forceinline__ uint32_t stop_any(uint4 w) {
    const uint32_t a = w.x & 0x7F7F7F7Fu, b = w.y & 0x7F7F7F7Fu, c = w.z & 0x7F7F7F7Fu, d = w.w & 0x7F7F7F7Fu;
    const uint32_t s = ((~(a + 0x60606060u) | (a + 0x01010101u)) & ~w.x) | ((~(b + 0x60606060u) | (b + 0x01010101u)) & ~w.y) |
                       ((~(c + 0x60606060u) | (c + 0x01010101u)) & ~w.z) | ((~(d + 0x60606060u) | (d + 0x01010101u)) & ~w.w);
    return s & 0x80808080u;
}
// bit 7 of byte i set iff byte i is one of [0-9A-Za-z-] (a subset of tchar)
__device__ __forceinline__ uint32_t alnum_bits(uint32_t x) {
    const uint32_t h = x | 0x80808080u;
    const uint32_t l = x | 0xA0A0A0A0u;  // letters folded to lower case, bit 7 set
    const uint32_t dig = (h - 0x30303030u) & ~(h - 0x3A3A3A3Au);
    const uint32_t let = (l - 0x61616161u) & ~(l - 0x7B7B7B7Bu);
    const uint32_t t = x ^ 0x2D2D2D2Du;  // '-' -> 0
    const uint32_t dash = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t);
    return (dig | let | dash) & ~x & 0x80808080u;
}
// 16-bit mask of the bytes of a chunk that are not [0-9A-Za-z-]
__device__ __forceinline__ uint32_t nonalnum_mask(uint4 w) {
    return (nib(~alnum_bits(w.x) & 0x80808080u) | nib(~alnum_bits(w.y) & 0x80808080u) << 4 |
            nib(~alnum_bits(w.z) & 0x80808080u) << 8 | nib(~alnum_bits(w.w) & 0x80808080u) << 12);
}
__device__ __forceinline__ uint32_t tstop_mask(uint4 w) {
    return nib(tstop_bits(w.x)) | nib(tstop_bits(w.y)) << 4 | nib(tstop_bits(w.z)) << 8 | nib(tstop_bits(w.w)) << 12;
}
__device__ __forceinline__ uint32_t vstop_mask(uint4 w) {
    return nib(vstop_bits(w.x)) | nib(vstop_bits(w.y)) << 4 | nib(vstop_bits(w.z)) << 8 | nib(vstop_bits(w.w)) << 12;
}
__device__ __forceinline__ uint32_t byte_of(uint4 w, uint32_t q) {
    // two selects + v_perm_b32 (an indexed select would be lowered to scratch)
    const bool upper = (q & 8) != 0;
    const uint32_t lo = upper ? w.z : w.x, hi = upper ? w.w : w.y;
    return __builtin_amdgcn_perm(hi, lo, (q & 7) | 0x0C0C0C00u);
}

// Rule-set image accessor: LDS (hot rule set) or global memory.
template <bool kLds>
struct Img {
    const uint8_t *p;
    __device__ __forceinline__ uint32_t u8(uint32_t o) const { return p[o]; }
    __device__ __forceinline__ uint32_t u16(uint32_t o) const { return *(const uint16_t *)(p + o); }
    __device__ __forceinline__ uint32_t u32(uint32_t o) const { return *(const uint32_t *)(p + o); }
    __device__ __forceinline__ uint64_t u64(uint32_t o) const { return *(const uint64_t *)(p + o); }
    __device__ __forceinline__ uint4 u128(uint32_t o) const { return *(const uint4 *)(p + o); }  // o 16-byte aligned
};
template <bool kLds>
__device__ __forceinline__ uint32_t uni(uint32_t v) {
    return kLds ? (uint32_t)__builtin_amdgcn_readfirstlane((int)v) : v;
}
#define HDR_U32(I, field) uni<kLds>((I).u32(offsetof(ImgHeader, field)))
#define HDR_U16(I, field) uni<kLds>((I).u16(offsetof(ImgHeader, field)))
#define HDR_U8(I, field) uni<kLds>((I).u8(offsetof(ImgHeader, field)))

// ---------------------------------------------------------------- lane state
struct Lane {
    uint64_t base;      // request start rounded down to 16 B (absolute address)
    uint32_t a0;        // position of request byte 0 relative to base
    uint32_t lena;      // a0 + len
    uint32_t pa;        // next position to look at
    uint32_t w;         // position of the window held in the lane's LDS slot
    uint32_t mode;
    uint32_t mark;      // token start (method/target/name) or version index
    uint32_t idx;       // request index
    bool done;          // verdict known
    bool owed;          // verdict not yet written out
    bool scan;          // an unconstrained value continues past the window
    bool tail;          // the skipped value ends in "\r\n\r\n" (end of the header block)
    uint8_t verdict;
    int32_t rule;
    uint32_t consumed;
    // framing
    uint32_t present;   // slots seen (first occurrence)
    uint32_t slot;      // slot of the current header value (kNoSlot: none)
    uint32_t nstate;    // name DFA state
    uint32_t ninfo;     // NI_* flags of the current header name
    bool have_cl, chunked, cl_bad, cl_ws, in_ows;
    uint32_t ndig;      // Content-Length digits; Transfer-Encoding: bytes of "chunked" matched (0xFF: no)
    uint64_t clv, cl;   // clv: Content-Length value; in the chunked body: the chunk size
    // DFA of the current slot (kDfasPerPass == 1); dtrans == 0: none
    uint32_t dcls, dtrans, dmask, dncls, st, saved;
    uint32_t dabs;      // states >= dabs (and 0) are absorbing
    uint64_t acc[kChunksPerPass];
    uint32_t cg, dg;    // chunk group, DFA group of this pass
};
static_assert(kDfasPerPass == 1, "one DFA per slot per framing pass");

template <bool kLds>
__device__ __forceinline__ void slot_begin(const Img<kLds> &I, Lane &L, uint32_t slot) {
    const uint32_t lo = I.u8(offsetof(ImgHeader, slot_dfa) + slot) + L.dg;
    const uint32_t hi = I.u8(offsetof(ImgHeader, slot_dfa) + slot + 1);
    L.st = 0;
    L.dcls = L.dtrans = L.dmask = L.dncls = L.dabs = 0;
    if (lo < hi) {
        const uint32_t d = HDR_U32(I, dfa_off) + lo * sizeof(DevDfa);
        L.dcls = I.u32(d + 0);
        L.dtrans = I.u32(d + 4);
        L.dmask = I.u32(d + 8);
        const uint32_t nc_st = I.u32(d + 12);
        L.dncls = nc_st & 0xFFFF;
        L.st = nc_st >> 16;
        L.dabs = I.u32(d + 16);
    }
}

template <bool kLds>
__device__ __forceinline__ void dfa_step(const Img<kLds> &I, Lane &L, uint32_t c) {
    if (L.st) L.st = I.u16(L.dtrans + 2 * (L.st * L.dncls + I.u8(L.dcls + c)));
}

// AND the end state's masks of the pass's chunks into the accumulators.
template <bool kLds>
__device__ __forceinline__ void slot_end(const Img<kLds> &I, Lane &L) {
    if (L.dtrans == 0) return;  // no DFA of this pass on the slot
    const uint32_t nchunks = HDR_U8(I, nchunks);
    const uint32_t nc = nchunks > L.cg ? min(nchunks - L.cg, (uint32_t)kChunksPerPass) : 0;
    const uint32_t base = L.dmask + 8 * (L.st * nchunks + L.cg);
#pragma unroll
    for (int c = 0; c < kChunksPerPass; c++)
        if ((uint32_t)c < nc) L.acc[c] &= I.u64(base + 8 * c);
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
    L.have_cl = L.chunked = false;
    L.cl = 0;
    slot_begin(I, L, SLOT_METHOD);
}

__device__ __forceinline__ void finish(Lane &L, uint8_t v, int32_t rule = -1) {
    L.done = true;
    L.scan = false;
    L.mode = M_DONE;
    L.verdict = v;
    L.rule = rule;
    if (v != V_ALLOW && v != V_DENY) L.consumed = 0;
}

// Headers complete (framing succeeded for this pass): next pass or verdict.
// The verdict of a request whose body is chunked: the chunks (and trailers)
// are walked after it to find where the request ends.
__device__ __forceinline__ void verdict_then_body(Lane &L, uint8_t v, int32_t rule) {
    if (!L.chunked) {
        finish(L, v, rule);
        return;
    }
    L.verdict = v;
    L.rule = rule;
    L.mode = M_CHSIZE;
    L.mark = L.pa;
    L.clv = 0;
}

template <bool kLds>
__device__ __forceinline__ void headers_done(const Img<kLds> &I, Lane &L, const uint64_t *nfa_bits) {
    const uint64_t total = L.chunked ? (uint64_t)(L.pa - L.a0) : (uint64_t)(L.pa - L.a0) + L.cl;
    if (total > 0xFFFFFFFFull) {
        finish(L, V_PARSE_ERROR);
    } else if (total > (uint64_t)(L.lena - L.a0)) {
        finish(L, V_INCOMPLETE);
    } else {
        L.consumed = (uint32_t)total;
        const uint32_t ndg = max((uint32_t)HDR_U8(I, max_slot_dfas), 1u);
        const uint32_t nchunks = HDR_U8(I, nchunks);
        if (L.dg + 1 < ndg) {  // more DFAs on some slot: frame again for this chunk group
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
            // matchers the NFA pre-pass evaluated (present slots; an absent one
            // is covered by the absent masks above)
            const uint32_t nnfa = HDR_U8(I, nnfa);
            if (nnfa) {
                const uint64_t bits = nfa_bits[L.idx];
                const uint32_t refs = HDR_U32(I, nfa_off);
                for (uint32_t k = 0; k < nnfa; k++) {
                    const uint32_t ref = refs + k * (uint32_t)sizeof(DevNfaRef);
                    if (!((L.present >> I.u8(ref + offsetof(DevNfaRef, slot))) & 1)) continue;
                    const uint32_t mo = I.u32(ref + offsetof(DevNfaRef, mask_off)) +
                                        8 * ((uint32_t)((bits >> k) & 1) * nchunks + L.cg);
#pragma unroll
                    for (int c = 0; c < kChunksPerPass; c++)
                        if ((uint32_t)c < nc) L.acc[c] &= I.u64(mo + 8 * c);
                }
            }
            int32_t hit = -1;
#pragma unroll
            for (int c = kChunksPerPass - 1; c >= 0; c--)
                if ((uint32_t)c < nc && L.acc[c]) hit = (int32_t)(64 * (L.cg + c) + (uint32_t)__builtin_ctzll(L.acc[c]));
            if (hit >= 0) {
                verdict_then_body(L, V_ALLOW, (int32_t)I.u32(HDR_U32(I, rule_off) + 4 * (uint32_t)hit));
            } else if (L.cg + kChunksPerPass < nchunks) {  // next chunk group
                L.cg += kChunksPerPass;
                L.dg = 0;
                acc_init(I, L);
                frame_reset(I, L);
            } else {
                verdict_then_body(L, (uint8_t)HDR_U8(I, terminal), -1);
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
    if ((L.ninfo & NI_TE) && L.ndig == 7) L.chunked = true;  // the value is "chunked" (case-insensitive)
    if (L.slot != kNoSlot) {
        slot_end(I, L);
        L.present |= 1u << L.slot;
    }
    return ok;
}

// ---------------------------------------------------------------- byte cursor
// Bytes of the lane's window, read from LDS one at a time (branch-free; the
// long-token loops below fetch them ahead of use).
struct Cursor {
    const uint8_t *slot;
    uint32_t swz;       // chunk swizzle of this lane, << 4
    uint32_t w;         // window start position
    __device__ __forceinline__ uint4 chunk(uint32_t k) const {
        return *(const uint4 *)(slot + (((k << 4) & (kWin - 16)) ^ swz));
    }
    // byte at position p (w <= p < w + kWin)
    __device__ __forceinline__ uint32_t at(uint32_t p) const { return slot[((p - w) & (kWin - 1)) ^ swz]; }
};

// First byte at or after pa (and before lim, inside the window) that ends a
// token, 16 bytes a step: kKind 0 = request target (<= 0x20 or DEL), 1 =
// header value (CTL other than HT, or DEL), 2 = simple header name (not
// [0-9A-Za-z-]).  lim if none.
template <int kKind>
__device__ __forceinline__ uint32_t find_stop(const Cursor &C, uint32_t pa, uint32_t lim) {
    while (pa < lim) {
        const uint4 w = C.chunk((pa - C.w) >> 4);
        uint32_t m = (kKind == 0 ? tstop_mask(w) : kKind == 1 ? vstop_mask(w) : nonalnum_mask(w)) & (0xFFFFu << (pa & 15));
        const uint32_t cend = (pa & ~15u) + 16;
        if (cend > lim) m &= (1u << (lim & 15)) - 1u;
        if (m) return (pa & ~15u) + (uint32_t)__builtin_ctz(m);
        pa = cend;
    }
    return lim;
}

// OWS after a header name is over (L.pa at the value's first byte, inside the
// window): a value nobody looks at is skipped, anything else is walked.
template <bool kLds>
__device__ __forceinline__ void ows_done(const Img<kLds> &I, Lane &L) {
    if (L.slot == kNoSlot && !(L.ninfo & (NI_CL | NI_TE))) {
        L.mode = M_SKIP;
    } else {
        L.mode = M_VALUE;
        if (L.slot != kNoSlot) {
            slot_begin(I, L, L.slot);
        } else {
            L.st = 0;
            L.dcls = L.dtrans = 0;
        }
        L.in_ows = false;
        L.clv = 0;
        L.ndig = 0;
        L.cl_bad = L.cl_ws = false;
    }
}

// Header name -> slot, as at the end of M_NAME (L.ninfo set).
template <bool kLds>
__device__ __forceinline__ void name_slot(const Img<kLds> &I, Lane &L) {
    uint32_t s = kNoSlot;
    if (L.ninfo & NI_HOST) s = SLOT_AUTHORITY;
    else if (L.ninfo & NI_CUSTOM) s = SLOT_CUSTOM0 + (L.ninfo & NI_CUSTOM) - 1;
    if (s != kNoSlot && ((L.present >> s) & 1)) s = kNoSlot;                // first occurrence only
    if (s != kNoSlot && !((HDR_U32(I, ref_slots) >> s) & 1)) s = kNoSlot;  // nobody looks at it
    L.slot = s;
}

// bit i (0..15) set iff byte i of the 16 bytes is SP or HT
__device__ __forceinline__ uint32_t ws_mask(uint4 w) {
    auto eq = [](uint32_t x, uint32_t b) {  // bit 7 of byte i set iff byte i == b
        const uint32_t t = x ^ b;
        return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
    };
    return nib(eq(w.x, 0x20202020u) | eq(w.x, 0x09090909u)) | nib(eq(w.y, 0x20202020u) | eq(w.y, 0x09090909u)) << 4 |
           nib(eq(w.z, 0x20202020u) | eq(w.z, 0x09090909u)) << 8 | nib(eq(w.w, 0x20202020u) | eq(w.w, 0x09090909u)) << 12;
}

// A header line's start, 16 bytes at a time (L.mode == M_LINE, L.pa + 16 <=
// lim): the 16 bytes at L.pa are cut out of two window chunks at once.
//   "\r\n"                        -> end of the header block (M_ENDLF's work);
//   name of 1..15 [0-9A-Za-z-] + ":" -> the name's flags from the image's name
//                                    table in one probe (instead of a DFA step
//                                    per byte), its slot, and OWS over when it
//                                    ends inside the 16 bytes;
//   anything else                 -> left to the byte-wise framer (M_LINE).
// The outcome is exactly the byte-wise one's (DevNameEnt).
template <bool kLds>
__device__ __forceinline__ void fast_line(const Img<kLds> &I, Lane &L, const Cursor &C, const uint64_t *nfa_bits) {
    const uint32_t k0 = (L.pa - C.w) >> 4, o = L.pa & 15, i = o >> 2, sh = (o & 3) * 8;
    const uint4 a = C.chunk(k0), b = C.chunk(k0 + 1);  // (b unused when o == 0)
    const uint32_t d1 = i == 0 ? a.y : i == 1 ? a.z : i == 2 ? a.w : b.x;
    const uint32_t d0 = i == 0 ? a.x : i == 1 ? a.y : i == 2 ? a.z : a.w;
    const uint32_t d2 = i == 0 ? a.z : i == 1 ? a.w : i == 2 ? b.x : b.y;
    const uint32_t d3 = i == 0 ? a.w : i == 1 ? b.x : i == 2 ? b.y : b.z;
    const uint32_t d4 = i == 0 ? b.x : i == 1 ? b.y : i == 2 ? b.z : b.w;
    uint4 f;
    f.x = (uint32_t)((((uint64_t)d1 << 32) | d0) >> sh);
    f.y = (uint32_t)((((uint64_t)d2 << 32) | d1) >> sh);
    f.z = (uint32_t)((((uint64_t)d3 << 32) | d2) >> sh);
    f.w = (uint32_t)((((uint64_t)d4 << 32) | d3) >> sh);
    const uint32_t b0 = f.x & 0xFF;
    if (b0 == '\r') {  // M_LINE -> M_ENDLF -> headers_done
        if (((f.x >> 8) & 0xFF) != '\n') {
            finish(L, V_PARSE_ERROR);
        } else {
            L.pa += 2;
            headers_done(I, L, nfa_bits);
        }
        return;
    }
    const uint32_t e = (uint32_t)__builtin_ctz(nonalnum_mask(f) | 0x10000u);
    if (e == 0 || e == 16 || byte_of(f, e) != ':') return;  // the byte-wise framer decides
    const uint32_t nb = HDR_U8(I, ntab_bits);
    if (nb == 0) return;
    // lower-cased name bytes (OR 0x20 is exact on [0-9A-Za-z-]), zero past e
    auto keep = [e](uint32_t j) { return e >= 4 * j + 4 ? 0xFFFFFFFFu : e <= 4 * j ? 0u : (1u << (8 * (e - 4 * j))) - 1u; };
    const uint32_t w0 = (f.x | 0x20202020u) & keep(0), w1 = (f.y | 0x20202020u) & keep(1);
    const uint32_t w2 = (f.z | 0x20202020u) & keep(2), w3 = (f.w | 0x20202020u) & keep(3);
    const uint32_t h = l7_name_hash(w0, w1, w2, w3, e, HDR_U32(I, ntab_mul), nb);
    const uint32_t ent = HDR_U32(I, ntab_off) + h * (uint32_t)sizeof(DevNameEnt);
    const uint4 n = I.u128(ent);
    const uint32_t meta = I.u32(ent + 16);
    const bool hit = (meta & 0xFF) == e && n.x == w0 && n.y == w1 && n.z == w2 && n.w == w3;
    L.mark = L.pa;
    L.ninfo = hit ? (meta >> 8) & 0xFF : 0u;
    name_slot(I, L);
    // OWS: the first byte after ':' that is not SP / HT, if among the 16
    const uint32_t v = (uint32_t)__builtin_ctz((~ws_mask(f) & (0xFFFFu << (e + 1)) & 0xFFFFu) | 0x10000u);
    if (v < 16) {
        L.pa += v;
        ows_done(I, L);
    } else {
        L.pa += e + 1;
        L.mode = M_OWS;
    }
}

// ---------------------------------------------------------------- parse one window
// Consumes [L.pa, min(window end, request end)).  Every loop has a single
// exit; errors set the mode to M_DONE so later blocks fall through.
template <bool kLds>
__device__ __forceinline__ void parse_window(const Img<kLds> &I, Lane &L, Cursor &C, const uint64_t *nfa_bits) {
    const uint32_t lim = min(L.w + kWin, L.lena);
    C.w = L.w;
    const uint32_t ncls_name = HDR_U16(I, name_ncls);
    const uint32_t name_cls = HDR_U32(I, name_cls_off), name_trans = HDR_U32(I, name_trans_off);

    // ---- request line
    if (L.mode == M_METHOD) {  // 1*tchar SP
        // software pipeline as for the target: byte p+2 and the class of byte
        // p+1 are read while the transition on byte p is in flight
        uint32_t c = 0;
        if (L.pa < lim) {
            c = C.at(L.pa);
            uint32_t k = L.dcls ? I.u8(L.dcls + c) : 0;
            uint32_t c1 = L.pa + 1 < lim ? C.at(L.pa + 1) : 0;
            while (is_tchar(c)) {
                const uint32_t p1 = L.pa + 1;
                const uint32_t c2 = p1 + 1 < lim ? C.at(p1 + 1) : 0;
                const uint32_t k1 = L.dcls ? I.u8(L.dcls + c1) : 0;
                if (L.st) L.st = I.u16(L.dtrans + 2 * (L.st * L.dncls + k));
                L.pa = p1;
                if (p1 >= lim) break;
                c = c1;
                c1 = c2;
                k = k1;
            }
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
        if (L.pa < lim) {
            // software pipeline: byte p+2 and the class of byte p+1 are read
            // while the transition on byte p is in flight
            c = C.at(L.pa);
            uint32_t k = L.dcls ? I.u8(L.dcls + c) : 0;
            uint32_t c1 = L.pa + 1 < lim ? C.at(L.pa + 1) : 0;
            while (c > 0x20 && c != 0x7F && L.st != 0 && L.st < L.dabs) {
                const uint32_t p1 = L.pa + 1;
                const uint32_t c2 = p1 + 1 < lim ? C.at(p1 + 1) : 0;
                const uint32_t k1 = L.dcls ? I.u8(L.dcls + c1) : 0;
                if (L.st) L.st = I.u16(L.dtrans + 2 * (L.st * L.dncls + k));
                L.pa = p1;
                if (p1 >= lim) break;
                c = c1;
                c1 = c2;
                k = k1;
            }
        }
        if (L.pa < lim && c > 0x20 && c != 0x7F) {  // absorbing state: the rest of the target cannot change it
            L.pa = find_stop<0>(C, L.pa, lim);
            c = L.pa < lim ? C.at(L.pa) : 0;
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
        if (L.mark == 0 && L.pa + 10 <= lim) {  // all ten bytes in the window: compare them at once
            const uint32_t k0 = (L.pa - L.w) >> 4, o = L.pa & 15, i = o >> 2, sh = o & 3;
            const uint4 a = C.chunk(k0), b = C.chunk(k0 + 1);  // (b unused when the bytes end in a)
            const uint32_t e0 = i == 0 ? a.x : i == 1 ? a.y : i == 2 ? a.z : a.w;
            const uint32_t e1 = i == 0 ? a.y : i == 1 ? a.z : i == 2 ? a.w : b.x;
            const uint32_t e2 = i == 0 ? a.z : i == 1 ? a.w : i == 2 ? b.x : b.y;
            const uint32_t e3 = i == 0 ? a.w : i == 1 ? b.x : i == 2 ? b.y : b.z;
            const uint32_t r0 = __builtin_amdgcn_alignbyte(e1, e0, sh);
            const uint32_t r1 = __builtin_amdgcn_alignbyte(e2, e1, sh);
            const uint32_t r2 = __builtin_amdgcn_alignbyte(e3, e2, sh);
            if (r0 == 0x50545448u && (r1 & 0x00FF00FFu) == 0x002E002Fu && ((r1 >> 8) & 0xFF) - '0' < 10u &&
                (r1 >> 24) - '0' < 10u && (r2 & 0xFFFFu) == 0x0A0Du) {
                L.pa += 10;
                L.mark = 10;
            }
        }
        for (; L.pa < lim && L.mark < 10; L.pa++, L.mark++) {
            const uint32_t c = C.at(L.pa);
            const uint32_t want = kVer[L.mark];
            if (want == 0x100 ? c - '0' >= 10u : c != want) break;
        }
        if (L.mark == 10) L.mode = M_LINE;
        else if (L.pa < lim) finish(L, V_PARSE_ERROR);
    }
    // ---- header lines
    while (L.mode >= M_LINE && L.mode < M_DONE && L.pa < lim) {
        if (L.mode == M_LINE && L.pa + 16 <= lim) fast_line(I, L, C, nfa_bits);
        if (L.mode == M_LINE) {
            if (C.at(L.pa) == '\r') {
                L.pa++;
                L.mode = M_ENDLF;
            } else {
                L.mode = M_NAME;
                L.mark = L.pa;
                L.nstate = kNameStart;
            }
        }
        if (L.mode == M_ENDLF && L.pa < lim) {
            if (C.at(L.pa) != '\n') {
                finish(L, V_PARSE_ERROR);
            } else {
                L.pa++;
                headers_done(I, L, nfa_bits);  // done, or a new pass from the request start
            }
        }
        if (L.mode == M_NAME) {  // 1*tchar ":"  (obs-fold SP/HT is not a tchar)
            uint32_t c = 0;
            if (L.pa < lim) {
                c = C.at(L.pa);
                uint32_t k = I.u8(name_cls + c);  // 0 = not a tchar
                uint32_t c1 = L.pa + 1 < lim ? C.at(L.pa + 1) : 0;
                while (k != 0 && L.nstate != kNameOther) {
                    const uint32_t p1 = L.pa + 1;
                    const uint32_t c2 = p1 + 1 < lim ? C.at(p1 + 1) : 0;
                    const uint32_t k1 = I.u8(name_cls + c1);
                    L.nstate = I.u16(name_trans + 2 * (L.nstate * ncls_name + k));
                    L.pa = p1;
                    if (p1 >= lim) break;
                    c = c1;
                    c1 = c2;
                    k = k1;
                }
                if (L.pa < lim && k != 0) {
                    // a name the rule set does not know (the DFA state loops on
                    // every tchar): only where it ends matters.  [0-9A-Za-z-]
                    // runs are skipped 16 bytes a step, other tchars one by one.
                    L.pa = find_stop<2>(C, L.pa, lim);
                    c = L.pa < lim ? C.at(L.pa) : 0;
                    while (L.pa < lim && c != ':' && is_tchar(c)) {
                        L.pa++;
                        c = L.pa < lim ? C.at(L.pa) : 0;
                    }
                }
            }
            if (L.pa < lim) {
                if (c != ':' || L.pa == L.mark) {
                    finish(L, V_PARSE_ERROR);
                } else {
                    L.pa++;
                    L.ninfo = L.nstate >= kNameStart ? I.u8(HDR_U32(I, name_info_off) + L.nstate) : 0;
                    name_slot(I, L);
                    L.mode = M_OWS;
                }
            }
        }
        if (L.mode == M_OWS) {
            for (; L.pa < lim; L.pa++) {
                const uint32_t c = C.at(L.pa);
                if (c != ' ' && c != '\t') break;
            }
            if (L.pa < lim) ows_done(I, L);
        }
        if (L.mode == M_VALUE && !(L.ninfo & (NI_CL | NI_TE))) {  // a value some rule looks at: DFA walk only
            // software pipeline as for the target: byte p+1 and its class are
            // read while the transition on byte p is in flight
            uint32_t c = 0, nx = 0;  // nx: the byte after c when in hand (| 0x100)
            if (L.pa < lim) {
                c = C.at(L.pa);
                uint32_t k = L.dcls ? I.u8(L.dcls + c) : 0;
                uint32_t c1 = L.pa + 1 < lim ? C.at(L.pa + 1) : 0;
                // CR ends it, other CTLs are errors; an absorbing state outside an
                // OWS run ends the walk (trailing OWS needs the state before it)
                while (!((c < 0x20 && c != '\t') || c == 0x7F) && (L.in_ows || (L.st != 0 && L.st < L.dabs))) {
                    const uint32_t p1 = L.pa + 1;
                    const uint32_t c2 = p1 + 1 < lim ? C.at(p1 + 1) : 0;
                    const uint32_t k1 = L.dcls ? I.u8(L.dcls + c1) : 0;
                    const bool ws = c == ' ' || c == '\t';
                    if (ws && !L.in_ows) L.saved = L.st;
                    L.in_ows = ws;
                    if (L.st) L.st = I.u16(L.dtrans + 2 * (L.st * L.dncls + k));
                    L.pa = p1;
                    if (p1 >= lim) break;
                    c = c1;
                    c1 = c2;
                    k = k1;
                }
                if (L.pa + 1 < lim) nx = c1 | 0x100;
            }
            if (L.pa < lim && !((c < 0x20 && c != '\t') || c == 0x7F)) {  // absorbing: skip to the value's end
                L.pa = find_stop<1>(C, L.pa, lim);
                c = L.pa < lim ? C.at(L.pa) : 0;
                nx = 0;
            }
            if (L.pa < lim) {
                if (c != '\r') {
                    finish(L, V_PARSE_ERROR);
                } else {
                    if (L.in_ows) L.st = L.saved;  // trailing OWS is not part of the value
                    if (nx) {  // M_LF's work on the byte in hand
                        L.pa += 2;
                        if (nx != ('\n' | 0x100)) finish(L, V_PARSE_ERROR);
                        else if (line_done(I, L)) L.mode = M_LINE;
                        else finish(L, V_PARSE_ERROR);
                    } else {
                        L.pa++;
                        L.mode = M_LF;
                    }
                }
            }
        }
        if (L.mode == M_VALUE) {  // Content-Length / Transfer-Encoding (and possibly a rule's DFA on it)
            uint32_t c = 0;
            const bool te = (L.ninfo & NI_TE) != 0;
            for (; L.pa < lim; L.pa++) {
                c = C.at(L.pa);
                if ((c < 0x20 && c != '\t') || c == 0x7F) break;  // CR ends it; other CTLs are errors
                const bool ws = c == ' ' || c == '\t';
                if (ws && !L.in_ows) L.saved = L.st;
                L.in_ows = ws;
                if (!ws) {
                    if (te) {  // "chunked", case-insensitive, then trailing OWS only
                        const uint32_t want = (uint32_t)(0x64656B6E756863ull >> (8 * min(L.ndig, 7u))) & 0xFF;
                        L.ndig = (!L.cl_ws && L.ndig < 7 && (c | 0x20) == want) ? L.ndig + 1 : 0xFF;
                    } else if (c - '0' < 10u && !L.cl_ws) {
                        L.clv = L.clv * 10 + (c - '0');
                        L.ndig++;
                    } else {
                        L.cl_bad = true;
                    }
                }
                L.cl_ws |= ws;
                dfa_step(I, L, c);
            }
            if (L.pa < lim) {
                if (c != '\r') {
                    finish(L, V_PARSE_ERROR);
                } else {
                    if (L.in_ows) L.st = L.saved;  // trailing OWS is not part of the value
                    L.pa++;
                    L.mode = M_LF;
                }
            }
        }
        if (L.mode == M_SKIP) {  // a value nobody looks at: find CR (or a CTL / DEL) 16 bytes a step
            uint32_t stop = 0, next = 0;  // next: the byte after the stop when the chunk holds it (| 0x100)
            while (L.pa < lim) {
                const uint4 w = C.chunk((L.pa - L.w) >> 4);
                const uint32_t any = stop_bits(w.x) | stop_bits(w.y) | stop_bits(w.z) | stop_bits(w.w);
                uint32_t m = any ? stop_mask(w) & (0xFFFFu << (L.pa & 15)) : 0;
                const uint32_t cend = L.pa - (L.pa & 15) + 16;
                if (cend > lim) m &= (1u << (lim & 15)) - 1u;  // lim inside this chunk
                const uint32_t p = cend - 16 + (uint32_t)__builtin_ctz(m | 0x10000u);
                L.pa = min(p, lim);
                if (p < cend) {
                    const uint32_t c = byte_of(w, p & 15);
                    if (c != '\t') {
                        stop = c | 0x100;
                        if (p + 1 < cend && p + 1 < lim) next = byte_of(w, (p + 1) & 15) | 0x100;
                        break;
                    }
                    L.pa++;
                }
            }
            if (stop) {
                if (stop != ('\r' | 0x100)) {
                    finish(L, V_PARSE_ERROR);
                } else if (next) {  // M_LF's work on the byte in hand
                    L.pa += 2;
                    if (next != ('\n' | 0x100)) finish(L, V_PARSE_ERROR);
                    else if (line_done(I, L)) L.mode = M_LINE;
                    else finish(L, V_PARSE_ERROR);
                } else {
                    L.pa++;
                    L.mode = M_LF;
                }
            } else if (L.pa < L.lena) {
                L.scan = true;  // the value continues past the window: the wave scans it
            }
        }
        if (L.mode == M_LF && L.pa < lim) {
            if (C.at(L.pa) != '\n') {
                finish(L, V_PARSE_ERROR);
            } else {
                L.pa++;
                if (line_done(I, L)) L.mode = M_LINE;
                else finish(L, V_PARSE_ERROR);
            }
        }
    }
    // ---- chunked body: chunk = 1*HEXDIG [";" ext] CRLF data CRLF; size 0 ends
    // the chunks, then trailer lines up to an empty line (oracle/http_ref.c)
    while (L.mode > M_DONE && L.pa < lim) {
        const uint32_t c = C.at(L.pa);
        switch (L.mode) {
        case M_CHSIZE: {
            const uint32_t d = c - '0' < 10u ? c - '0' : (c | 0x20) - 'a' < 6u ? (c | 0x20) - 'a' + 10 : 0xFF;
            if (d != 0xFF) {
                L.clv = L.clv * 16 + d;
                L.pa++;
                if (L.clv > 0xFFFFFFFFull) finish(L, V_PARSE_ERROR);
            } else if (L.pa == L.mark) {
                finish(L, V_PARSE_ERROR);
            } else if (c == ';') {
                L.pa++;
                L.mode = M_CHEXT;
            } else if (c == '\r') {
                L.pa++;
                L.mode = M_CHLF;
            } else {
                finish(L, V_PARSE_ERROR);
            }
            break;
        }
        case M_CHEXT:
            if (c == '\n') finish(L, V_PARSE_ERROR);
            else if (c == '\r') L.mode = M_CHLF;
            L.pa++;
            break;
        case M_CHLF:
            if (c != '\n') { finish(L, V_PARSE_ERROR); break; }
            L.pa++;
            L.mode = L.clv ? M_CHDATA : M_TRL;
            break;
        case M_CHDATA:  // skip the data by its length
            if ((uint64_t)(L.pa - L.a0) + L.clv > 0xFFFFFFFFull) {
                finish(L, V_PARSE_ERROR);
            } else if ((uint64_t)L.pa + L.clv > L.lena) {
                L.pa = L.lena;
                finish(L, V_INCOMPLETE);
            } else {
                L.pa += (uint32_t)L.clv;
                L.mode = M_CHDCR;
            }
            break;
        case M_CHDCR:
            if (c != '\r') { finish(L, V_PARSE_ERROR); break; }
            L.pa++;
            L.mode = M_CHDLF;
            break;
        case M_CHDLF:
            if (c != '\n') { finish(L, V_PARSE_ERROR); break; }
            L.pa++;
            L.mode = M_CHSIZE;
            L.mark = L.pa;
            L.clv = 0;
            break;
        case M_TRL:
            if (c == '\n') { finish(L, V_PARSE_ERROR); break; }
            L.mode = c == '\r' ? M_TRLEND : M_TRLSCAN;
            L.pa++;
            break;
        case M_TRLSCAN:
            if (c == '\n') finish(L, V_PARSE_ERROR);
            else if (c == '\r') L.mode = M_TRLLF;
            L.pa++;
            break;
        case M_TRLLF:
            if (c != '\n') { finish(L, V_PARSE_ERROR); break; }
            L.pa++;
            L.mode = M_TRL;
            break;
        default:  // M_TRLEND
            if (c != '\n') { finish(L, V_PARSE_ERROR); break; }
            L.pa++;
            finish(L, L.verdict, L.rule);
            L.consumed = L.pa - L.a0;
            break;
        }
    }
}

// ---------------------------------------------------------------- window DMA
// For every lane t with a window to load: chunks [0, hi] of the 256-byte
// window at address `win` into LDS slot t (chunk c stored at position
// c ^ (t & 15)).  packed = window address | hi (addresses are 16-byte aligned;
// 0 = nothing to load).
__device__ __forceinline__ void dma_windows_issue(uint8_t *wave_lds, uint64_t packed, uint32_t lane) {
    const uint32_t plo = (uint32_t)packed, phi = (uint32_t)(packed >> 32);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's earlier LDS reads have landed
    // every window address first, one wait, then the loads: issued one per
    // load, the compiler waits on each ds_bpermute in turn (16 serial LDS
    // round trips per round)
    uint32_t tlo[kWinChunks], thi[kWinChunks];
#pragma unroll
    for (int j = 0; j < (int)kWinChunks; j++) {
        const int t = (int)(kWinPerInst * j + lane / kLanesPerWin);
        tlo[j] = __shfl(plo, t);
        thi[j] = __shfl(phi, t);
    }
#pragma unroll
    for (int j = 0; j < (int)kWinChunks; j++) {
        const uint32_t t = kWinPerInst * j + lane / kLanesPerWin;
        const uint32_t c = (lane % kLanesPerWin) ^ win_swizzle(t);
        if ((tlo[j] | thi[j]) && c <= (tlo[j] & 15)) {
            const uint8_t *src = (const uint8_t *)((((uint64_t)thi[j]) << 32) | (tlo[j] & ~15u)) + 16 * c;
            __builtin_amdgcn_global_load_lds((const void *)src,
                                             (__attribute__((address_space(3))) void *)(wave_lds + j * 1024), 16, 0, 0);
        }
    }
}
__device__ __forceinline__ void dma_windows(uint8_t *wave_lds, uint64_t packed, uint32_t lane) {
    dma_windows_issue(wave_lds, packed, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
// the DMA word of a lane's next window (0: nothing to load)
__device__ __forceinline__ uint64_t window_packed(Lane &L) {
    if (L.done) return 0;
    L.w = L.pa & ~15u;
    const uint32_t hi = min(L.lena - 1 - L.w, kWin - 1) >> 4;
    return (L.base + L.w) | hi;
}

// ---------------------------------------------------------------- value-stop map of a tile
// A value nobody constrains ends at its first "value stop" byte (< 0x20 other
// than HT, or DEL: CR normally, anything else is an error).  Before its first
// window the wave streams its tile's bytes, and each lane keeps, for its own
// request, one bit per 16-byte chunk -- "holds a value stop" -- in registers.
// A step moves 128 bytes of every request of the tile into VGPRs: load q of
// step j covers requests 8q..8q+7, lane l reading chunk 8j + (l & 7) of
// request 8q + (l >> 3), so one load instruction touches 8 full lines; a
// ballot per load hands each lane its request's eight bits; three steps are in
// flight.  (Four lanes per request and 64-byte steps: 2.42 -> 2.18 ms on 4M
// mixed-stream HTTP requests against one line per lane; eight lanes and VGPRs
// instead of an LDS ring went further, DESIGN.md.)  So every 16-byte chunk of
// a request is read once, whatever lies between the tile's requests (packed
// streams, the HTTP list of a mixed batch, scattered offsets), and a lane
// searches only its own bits.  A long value is then skipped by finding the
// lane's first marked chunk at or after L.pa and reading only that chunk and
// the next.  Chunks past the mapped range (kMapChunks, 3 KiB) continue window
// by window.  The head windows' DMA is issued before the map, into the window
// area, so it overlaps the map's stream.
//
// The bits enter a per-lane shift register eight at a time (one step), so
// after smax8 steps (the tile's longest request) chunk c sits at bit
// c + T.off with T.off = kMapChunks - 8 smax8, the same for every lane.
//
// Packed tiles (the 64 requests side by side, their span at most 9/8 of their
// own chunks) take the span mode instead: the span streams as coalesced 1 KiB
// pieces (lane l loads the piece's chunk l), a ballot gives every lane the
// piece's 64 stop bits, and each lane keeps the (at most four) pieces that
// overlap its request and finally shifts its own chunks into place (T.off = 0).
// One 1 KiB piece is 8 full cache lines per load instruction where the
// per-lane steps touch 64 lines: 0.48 vs 0.64 ms on cfg2's packed 1M stream;
// on the mixed stream's HTTP list the per-lane steps win (2.35 vs 2.61 ms per
// 4M requests) since no foreign byte is read.
constexpr uint32_t kMapWords = 6;
constexpr uint32_t kMapChunks = kMapWords * 32;             // chunks mapped per request
constexpr int kRing = (int)(kWaveLds / 1024);               // span mode: 1 KiB pieces in flight
constexpr uint64_t kSpanChunksMax = 256 * 64;               // span mode: at most 256 KiB

// Lane mode leaves out each request's first kWin bytes: map_skip only ever
// searches from the end of a window (a value still open there), so the first
// window's chunks are never looked up, and the head window reads them anyway.
constexpr uint32_t kSkipSteps = kWin / 64;

struct TileMap {
    uint32_t off;              // bit position of chunk 0 (uniform)
    uint32_t from;             // first chunk the map holds (uniform)
    uint32_t m[kMapWords];     // this lane's request: chunk bits (shift register)
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ uint4 u4(gm_u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }

__device__ __forceinline__ uint32_t byte_at32(uint4 a, uint4 b, uint32_t i) {
    // byte i (0..31) of the 32 bytes a, b (little endian)
    const uint32_t d = i < 16 ? (i < 8 ? (i < 4 ? a.x : a.y) : (i < 12 ? a.z : a.w))
                              : (i < 24 ? (i < 20 ? b.x : b.y) : (i < 28 ? b.z : b.w));
    return (d >> (8 * (i & 3))) & 0xFF;
}

// a lane's chunk count (lanes without a request or with an empty one: 0)
__device__ __forceinline__ uint32_t map_nch(const Lane &L) { return L.lena > L.a0 ? (L.lena + 15u) >> 4 : 0u; }

// Span mode (packed tiles): see above.  The lane's request covers span chunks
// [vs, vs + nch); pieces j0..j0+3 (j0 = vs / 64) hold them.
__device__ __forceinline__ void map_span(TileMap &T, const Lane &L, uint32_t lane, uint8_t *wave_lds, uint64_t lo,
                                         uint32_t vtot, uint32_t nch) {
    const uint32_t npieces = (vtot + 63) >> 6;
    const uint32_t vs = nch ? (uint32_t)((L.base - lo) >> 4) : 0u;
    const uint32_t j0 = vs >> 6;
    uint32_t pc[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // pieces j0..j0+3, 2 words each
    // piece j -> slot j % kRing; an idle slot still issues its load (at the span
    // start), so a slot is examined with exactly kRing-1 loads behind it
#define MAP_PIECE(s, j)                                                                                   \
    do {                                                                                                  \
        const uint64_t a_ = lo + ((uint64_t)(j) << 10) + 16 * lane;                                       \
        __builtin_amdgcn_global_load_lds((const void *)((j) < npieces && ((j) << 6) + lane < vtot ? a_ : lo), \
                                         (__attribute__((address_space(3))) void *)(wave_lds + (s) * 1024), \
                                         16, 0, 0);                                                       \
    } while (0)
#pragma unroll
    for (int s = 0; s < kRing; s++) MAP_PIECE(s, (uint32_t)s);
    for (uint32_t jb = 0; jb < npieces; jb += kRing) {
#pragma unroll
        for (int s = 0; s < kRing; s++) {
            const uint32_t j = jb + s;
            wait_vmcnt<kRing - 1>();
            if (j < npieces) {
                // inline asm: a plain LDS read here would make hipcc drain every
                // in-flight LDS-DMA first (vmcnt(0)), serialising the ring
                uint4 v;
                asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                             : "=v"(v)
                             : "v"((uint32_t)(uintptr_t)(wave_lds + s * 1024 + 16 * lane))
                             : "memory");
                const bool ok = (j << 6) + lane < vtot;
                const uint64_t M = __ballot(ok && stop_any(v) != 0);  // HT marks too: map_skip sorts it out
                const uint32_t q = j - j0;  // which of the lane's pieces (>= 4 or wrapped: none)
#pragma unroll
                for (int t = 0; t < 4; t++)
                    if (q == (uint32_t)t) {
                        pc[2 * t] = (uint32_t)M;
                        pc[2 * t + 1] = (uint32_t)(M >> 32);
                    }
            }
            MAP_PIECE(s, j + kRing);
        }
    }
    wait_vmcnt<0>();
#undef MAP_PIECE
    // own chunk c = bit (vs & 63) + c of pc[]: shift right by vs & 63
    const uint32_t sh = vs & 63, wsh = sh >> 5, bsh = sh & 31;
#pragma unroll
    for (int w = 0; w < (int)kMapWords; w++) {
        const uint32_t a0 = wsh ? pc[w + 1] : pc[w];
        const uint32_t a1 = wsh ? (w + 2 < 8 ? pc[w + 2] : 0u) : pc[w + 1];
        T.m[w] = __builtin_amdgcn_alignbit(a1, a0, bsh);
    }
    T.off = 0;
}

// Returns true when the lane-mode map also DMA'd the tile's first head
// windows (window_packed of every lane) into the window area.
__device__ __forceinline__ bool build_tile_map(TileMap &T, Lane &L, uint32_t lane, uint8_t *wave_lds) {
#pragma unroll
    for (int q = 0; q < (int)kMapWords; q++) T.m[q] = 0;
    T.off = kMapChunks;
    T.from = 0;
    const uint32_t nch = min(map_nch(L), kMapChunks);
    const uint32_t nseg = (nch + 3) >> 2;  // 64-byte steps of this lane
    // wave reductions by DPP (__ockl_wfred_*): no LDS round trips
    const uint32_t smax = (uint32_t)__builtin_amdgcn_readfirstlane((int)__ockl_wfred_max_u32(nseg));
    if (smax == 0) return false;
    const uint64_t act = __ballot(nch > 0);
    const uint64_t dummy = (uint64_t)__shfl((unsigned long long)L.base, (int)__builtin_ctzll(act));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // earlier LDS reads of the window area have landed
    {
        uint64_t lo = __ockl_wfred_min_u64(nch ? L.base : ~0ull);
        uint64_t hi = __ockl_wfred_max_u64(nch ? L.base + ((uint64_t)nch << 4) : 0ull);
        uint32_t own = __ockl_wfred_add_u32(nch);
        lo = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(lo >> 32)) << 32) |
             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)lo);
        hi = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(hi >> 32)) << 32) |
             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)hi);
        own = (uint32_t)__builtin_amdgcn_readfirstlane((int)own);
        const uint64_t span = (hi - lo) >> 4;
        if (span <= kSpanChunksMax && span <= (uint64_t)own + (own >> 3)) {
            map_span(T, L, lane, wave_lds, lo, (uint32_t)span, nch);
            return false;
        }
    }
    T.off = kMapChunks - 4 * smax;
    T.from = 4 * kSkipSteps;
    if (smax <= kSkipSteps) return false;  // every request fits its head window
    // Lanes with nothing (more) to load still issue theirs, at a chunk of the
    // tile, so every step is eight loads and vmcnt counts stay exact.  Eight
    // lanes per request: a step is 128 bytes (a whole line) per request, load q
    // of step j covers requests 8q..8q+7, lane l reading chunk 8j + (l & 7) of
    // request 8q + (l >> 3), so every load instruction touches 8 full lines.
    // The head windows go into the window area now (the map does not use it),
    // so their DMA overlaps the map stream; the map's steps land in VGPRs,
    // kMapDepth of them in flight.  Loads and waits are written out (inline
    // asm): the compiler's own wait placement drains every load at the loop
    // head (vmcnt(0)), which leaves one memory latency per kMapDepth steps.
    {
        dma_windows_issue(wave_lds, window_packed(L), lane);
        const uint32_t smax8 = (smax + 1) >> 1, skip8 = kWin / 128;
        T.off = kMapChunks - 8 * smax8;
        const uint32_t sub8 = lane & 7, grp8 = lane >> 3;
        uint64_t qb8[8];
        uint32_t qn8[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            qb8[q] = (uint64_t)__shfl((unsigned long long)L.base, 8 * q + (int)grp8);
            qn8[q] = (uint32_t)__shfl((int)nch, 8 * q + (int)grp8);
        }
        constexpr int kMapDepth = 3;  // 128-byte-per-lane steps in flight
        gm_u32x4 buf[kMapDepth][8];
#define MAP_LOAD8(s, j)                                                                                        \
    do {                                                                                                       \
        _Pragma("unroll") for (int q_ = 0; q_ < 8; q_++) {                                                     \
            const uint32_t c_ = 8 * (uint32_t)(j) + sub8;                                                      \
            const uint64_t a_ = c_ < qn8[q_] ? qb8[q_] + ((uint64_t)c_ << 4) : dummy;                          \
            asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(buf[s][q_]) : "v"(a_) : "memory");           \
        }                                                                                                      \
    } while (0)
#pragma unroll
        for (int s = 0; s < kMapDepth; s++) MAP_LOAD8(s, skip8 + (uint32_t)s);
        for (uint32_t j0 = skip8; j0 < smax8; j0 += kMapDepth) {
#pragma unroll
            for (int s = 0; s < kMapDepth; s++) {
                const uint32_t j = j0 + s;
                asm volatile("s_waitcnt vmcnt(%8)"
                             : "+v"(buf[s][0]), "+v"(buf[s][1]), "+v"(buf[s][2]), "+v"(buf[s][3]), "+v"(buf[s][4]),
                               "+v"(buf[s][5]), "+v"(buf[s][6]), "+v"(buf[s][7])
                             : "n"(8 * (kMapDepth - 1)));
                // block q, bit l: request 8q + (l >> 3), chunk 8j + (l & 7)
                uint64_t M[8];
#pragma unroll
                for (int q = 0; q < 8; q++) M[q] = __ballot(stop_any(u4(buf[s][q])) != 0);
                MAP_LOAD8(s, j + kMapDepth);
                if (j < smax8) {
                    const uint32_t qo = lane >> 3;
                    uint64_t Mq = M[0];
#pragma unroll
                    for (int q = 1; q < 8; q++) Mq = qo == (uint32_t)q ? M[q] : Mq;
                    uint32_t nb = (uint32_t)(Mq >> (8 * (lane & 7))) & 0xFFu;
                    if (8 * j >= nch) nb = 0;
#pragma unroll
                    for (int q = 0; q < (int)kMapWords - 1; q++) T.m[q] = __builtin_amdgcn_alignbit(T.m[q + 1], T.m[q], 8);
                    T.m[kMapWords - 1] = (T.m[kMapWords - 1] >> 8) | (nb << 24);
                }
            }
        }
#undef MAP_LOAD8
        wait_vmcnt<0>();
        return true;
    }
}

// Lanes with L.scan set: skip the rest of the value with the lane's map.
__device__ __forceinline__ void map_skip(Lane &L, const TileMap &T) {
    if (!__any(L.scan)) return;
    if (!L.scan) return;
    const uint32_t nch = map_nch(L);
    const uint32_t mapped = min(nch, kMapChunks);
    for (;;) {
        const uint32_t k = L.pa >> 4;
        if (k < T.from) {  // (not reached: a scan starts at a window's end) window by window
            L.scan = false;
            return;
        }
        // first marked chunk in [k, mapped): bit positions [k + off, mapped + off)
        uint32_t found = 0xFFFFFFFFu;
        if (k < mapped) {
            const uint32_t p0 = k + T.off, p1 = mapped + T.off;
#pragma unroll
            for (int w = (int)kMapWords - 1; w >= 0; w--) {
                const uint32_t lo = 32u * (uint32_t)w;
                uint32_t bits = T.m[w];
                if (p0 > lo) bits = p0 - lo >= 32 ? 0u : bits & (0xFFFFFFFFu << (p0 - lo));
                if (p1 < lo + 32) bits = p1 <= lo ? 0u : bits & (0xFFFFFFFFu >> (lo + 32 - p1));
                if (bits) found = lo + (uint32_t)__builtin_ctz(bits) - T.off;
            }
        }
        if (found == 0xFFFFFFFFu) {
            if (mapped < nch) {  // no stop in the mapped chunks: on window by window after them
                L.pa = max(L.pa, mapped << 4);
                L.scan = false;
            } else {             // no value stop before the request's end
                L.pa = L.lena;
                finish(L, V_INCOMPLETE);
            }
            return;
        }
        const uint32_t cpos = found << 4;  // the marked chunk, request-relative
        const uint64_t ca = L.base + cpos;
        const uint4 w0 = gload16(ca);  // global, not flat (gmem.h)
        const uint4 w1 = cpos + 16 < L.lena ? gload16(ca + 16) : make_uint4(0, 0, 0, 0);
        const uint32_t lo_b = L.pa > cpos ? L.pa - cpos : 0;
        const uint32_t hi_b = min(L.lena - cpos, 16u);
        const uint32_t m = vstop_mask(w0) & (0xFFFFu << lo_b) & ((1u << hi_b) - 1u);
        if (m) {
            const uint32_t b = (uint32_t)__builtin_ctz(m);
            L.pa = cpos + b;
            L.scan = false;
            // "\r\n\r\n" here ends the header block: no window needed for it
            if (L.pa + 4 <= L.lena) {
                const uint32_t t4 = byte_at32(w0, w1, b) | byte_at32(w0, w1, b + 1) << 8 |
                                    byte_at32(w0, w1, b + 2) << 16 | byte_at32(w0, w1, b + 3) << 24;
                L.tail = t4 == 0x0A0D0A0Du;
            }
            return;
        }
        // the chunk's stops lie before pa (or are HT): search on
        L.pa = cpos + 16;
        if (L.pa >= L.lena) {
            L.pa = L.lena;
            finish(L, V_INCOMPLETE);
            return;
        }
    }
}

// The skipped value ended at the CR of "\r\n\r\n": what parse_window does for
// those four bytes (M_SKIP -> M_LF -> line_done -> M_LINE -> M_ENDLF ->
// headers_done), without another window.
template <bool kLds>
__device__ __forceinline__ void finish_tail(const Img<kLds> &I, Lane &L, const uint64_t *nfa_bits) {
    L.tail = false;
    L.pa += 4;
    if (line_done(I, L)) {
        L.mode = M_LINE;
        headers_done(I, L, nfa_bits);
    } else {
        finish(L, V_PARSE_ERROR);
    }
}

struct Out {
    uint8_t *verdict;
    int32_t *rule;
    uint32_t *consumed;
    const uint64_t *nfa_bits;  // NFA pre-pass results (HttpTables::nfa_bits)
};

__device__ __forceinline__ void emit(const Lane &L, const Out &O) {
    O.verdict[L.idx] = L.verdict;
    O.rule[L.idx] = L.rule;
    O.consumed[L.idx] = L.consumed;
}

// All rounds of one tile.
// kInit = false: the lanes' framing state is set up by the caller (latency path).
// pre: the tile's map, already built (latency path); null: built here.
template <bool kLds, bool kFlush = true, bool kInit = true>
__device__ __forceinline__ void run_tile(Lane &L, const uint8_t *img, uint8_t *wave_lds, uint32_t lane, const Out &O,
                                         const TileMap *pre = nullptr) {
    const Img<kLds> I{img};
    L.scan = false;
    L.tail = false;
    if (kInit && !L.done) {
        L.cg = 0;
        L.dg = 0;
        acc_init(I, L);
        frame_reset(I, L);
        if (L.lena == L.a0) finish(L, V_INCOMPLETE);
    }
    PH_DECL
    TileMap TM;
    bool loaded = false;  // true: the first windows are in
    if (pre) TM = *pre;
    else loaded = build_tile_map(TM, L, lane, wave_lds);
    PH_MARK(2);
    Cursor C;
    C.slot = wave_lds + lane * kWin;
    C.swz = win_swizzle(lane) << 4;
    while (__any(!L.done)) {
        const uint64_t packed = window_packed(L);
        PH_MARK(3);
        if (!loaded) dma_windows(wave_lds, packed, lane);
        loaded = false;
        PH_MARK(0);
        if (!L.done) {
            parse_window(I, L, C, O.nfa_bits);
            if (!L.done && !L.scan && L.pa >= L.lena) finish(L, V_INCOMPLETE);
        }
        PH_MARK(1);
        PH_COUNT(5, __builtin_popcountll(__ballot(L.scan)));
        map_skip(L, TM);
        if (L.tail) finish_tail(I, L, O.nfa_bits);
        PH_MARK(2);
        if (L.done && L.owed) {
            emit(L, O);
            L.owed = false;
        }
        PH_COUNT(4, 1);
    }
    if (L.done && L.owed) {  // answered before any round
        emit(L, O);
        L.owed = false;
    }
    PH_MARK(3);
    PH_COUNT(6, 1);
    if (kFlush) PH_FLUSH(lane);
}


// ---------------------------------------------------------------- latency path
// bit i (0..15) set iff byte i of the chunk is CR
__device__ __forceinline__ uint32_t cr_mask(uint4 w) {
    auto eq = [](uint32_t x) {
        const uint32_t t = x ^ 0x0D0D0D0Du;
        return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
    };
    return nib(eq(w.x)) | nib(eq(w.y)) << 4 | nib(eq(w.z)) << 8 | nib(eq(w.w)) << 12;
}

constexpr uint32_t kLatLines = 63;  // header lines one wave frames side by side (lane k: line k)

// One request per wave, for the small calls of the synchronous drop-ins (one
// Allowed(), a few requests): the tile kernel's one lane walks a request's
// lines one after the other, every byte a chain of dependent LDS reads (a
// 1.1 KB cfg2 request: ~43k cycles of framing on one lane, the same with
// warm caches).  Here the request's lines are framed side by side.
//
// Every line of a request ends at its first CR: the method, target, name and
// value walks all stop there, and anything but LF after it is an error.  So
// the wave first finds the CRs (a ballot scan, 1 KiB per step, up to the
// empty line that ends the header block), then lane k runs the ordinary
// framer over line k alone -- lane 0 the request line from the request's
// start, lane k >= 1 from line k's first byte in M_LINE, each with L.lena at
// its line's end (its CR + 2) -- and what the lines leave behind is merged
// the way the sequential walk accumulates it: any error makes the request
// PARSE_ERROR; a slot counts at its first occurrence only (the lowest line),
// and its masks AND into the rule accumulators, which start at the init masks
// on lane 0 and at all ones on the other lanes; two Content-Length lines are
// an error and the first one's value counts; a chunked Transfer-Encoding line
// makes the body chunked.  (A repeated slot's value is walked by its DFA where
// the sequential framer skips it: both stop at the same bytes and fail on the
// same ones, and the walk's masks are dropped.)  Lane 0 then ends the header
// block as the framer does (headers_done on the merged state) and, when the
// answer needs more -- a chunked body, another framing pass of a large rule
// set -- carries on sequentially from there.  A header block of more than
// kLatLines lines is framed sequentially from the start by lane 0.
// All lanes enter with the same L (the request; done = false, owed = true).
template <bool kLds>
__device__ __forceinline__ void lat_request(const Lane &L, const uint8_t *img, uint8_t *wave_lds, uint32_t lane,
                                            const Out &O) {
    const Img<kLds> I{img};
    const uint32_t a0 = L.a0, lena = L.lena;
    if (lena == a0) {  // nothing yet
        if (lane == 0) {
            Lane W = L;
            finish(W, V_INCOMPLETE);
            emit(W, O);
        }
        return;
    }
    LAT_T0
    // ---- the CRs, in order, until the empty line (crpos: kLatLines + 2 entries)
    const uint32_t nch = (lena + 15) >> 4;
    uint32_t *crpos = reinterpret_cast<uint32_t *>(wave_lds);
    const uint64_t below = (1ull << lane) - 1;
    uint32_t ncr = 0;
    int hend = -1;     // index of the empty line that ends the header block
    bool all = false;  // every byte scanned
    // The scan also yields the tile map run_tile would stream (span mode: every
    // lane's request has this base, so chunk c is bit c): the value-stop bits of
    // the first kMapChunks chunks, one ballot per 64.
    TileMap TM;
#pragma unroll
    for (int q = 0; q < (int)kMapWords; q++) TM.m[q] = 0;
    TM.off = 0;
    TM.from = 0;
    // crpos[r]: the r-th CR's position | kLfKnown (the byte after it was in the
    // scan's registers) | kLfYes (and it is LF)
    constexpr uint32_t kLfKnown = 1u << 31, kLfYes = 1u << 30, kPos = kLfYes - 1;
    for (uint32_t c0 = 0;; c0 += 64) {
        const uint32_t c = c0 + lane;
        uint32_t m = 0;
        uint4 w = make_uint4(0, 0, 0, 0);
        if (c < nch) {
            w = gload16(L.base + 16ull * c);
            m = cr_mask(w);
            const uint32_t p0 = 16 * c;
            if (p0 < a0) m &= 0xFFFFu << (a0 - p0);
            if (p0 + 16 > lena) m &= (1u << (lena - p0)) - 1u;
        }
        const uint64_t sb = __ballot(c < nch && stop_any(w) != 0);
        if (c0 < kMapChunks) {
#pragma unroll
            for (int q = 0; q < (int)kMapWords; q += 2)
                if ((uint32_t)q == c0 / 32) {
                    TM.m[q] = (uint32_t)sb;
                    TM.m[q + 1] = (uint32_t)(sb >> 32);
                }
        }
        const uint32_t nb0 = (uint32_t)__shfl_down((int)(w.x & 0xFF), 1);  // the next chunk's first byte
        const uint32_t cnt = (uint32_t)__builtin_popcount(m);
        uint32_t ex = 0;  // exclusive prefix of cnt over the lanes (cnt <= 16: five ballots)
#pragma unroll
        for (int b = 0; b < 5; b++) ex += (uint32_t)__popcll(__ballot((cnt >> b) & 1) & below) << b;
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readfirstlane((int)__ockl_wfred_add_u32(cnt));
        for (uint32_t r = ncr + ex; m; m &= m - 1, r++) {
            const uint32_t b = (uint32_t)__builtin_ctz(m);
            const bool known = b < 15 || (lane < 63 && c + 1 < nch);
            const uint32_t nx = b < 15 ? byte_of(w, b + 1) : nb0;
            if (r < kLatLines + 2) crpos[r] = (16 * c + b) | (known ? kLfKnown : 0u) | (known && nx == '\n' ? kLfYes : 0u);
        }
        ncr += tot;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t have = min(ncr, kLatLines + 1);
        const uint64_t eb =
            __ballot(lane >= 1 && lane < have && (crpos[lane] & kPos) == (crpos[lane - 1] & kPos) + 2);
        if (eb) {
            hend = (int)__builtin_ctzll(eb);
            break;
        }
        if (c0 + 64 >= nch) {
            all = true;
            break;
        }
        if (ncr > kLatLines) break;
    }
    LAT_T(9);
    if (!(hend > 0 || (all && ncr <= kLatLines))) {  // too many lines: sequentially, lane 0
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        Lane W = L;
        if (lane != 0) {
            W.done = true;
            W.owed = false;
            W.base = 0;
            W.a0 = W.pa = W.lena = 0;
        }
        run_tile<kLds>(W, img, wave_lds, lane, O);
        return;
    }
    // ---- lane k: line k
    uint32_t nl;
    if (hend > 0) {
        nl = (uint32_t)hend;
    } else {
        const uint32_t sp = ncr ? (crpos[ncr - 1] & kPos) + 2 : a0;  // an unterminated last line
        nl = ncr + (sp < lena ? 1u : 0u);
    }
    uint32_t start = a0, cr = 0;
    const bool has_cr = lane < nl && lane < ncr;
    if (lane < nl && lane > 0) start = (crpos[lane - 1] & kPos) + 2;
    if (has_cr) cr = crpos[lane] & kPos;
    const uint32_t lend = has_cr ? min(cr + 2, lena) : lena;
    // (a line that would start at the request's end follows "\r\r" there: the
    // line before it fails on its LF, and this one has no byte to frame)
    const bool act = lane < nl && start < lend;
    const uint32_t cr_end_w = hend > 0 ? crpos[hend] : 0u, cr_end = cr_end_w & kPos;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // crpos read: the window area is the lanes' again
    __builtin_amdgcn_wave_barrier();
    const bool complete = has_cr && cr + 2 <= lena;
    Lane W = L;
    W.owed = false;
    W.cg = 0;
    W.dg = 0;
    acc_init(I, W);
    frame_reset(I, W);
    if (act) {
        W.lena = lend;
        if (lane > 0) {
#pragma unroll
            for (int c = 0; c < kChunksPerPass; c++) W.acc[c] = ~0ull;
            W.pa = W.mark = start;
            W.mode = M_LINE;
            W.st = 0;
            W.dcls = W.dtrans = W.dmask = W.dncls = W.dabs = 0;
            W.slot = kNoSlot;
        }
    } else {
        W.done = true;
        W.base = 0;
        W.a0 = W.pa = W.lena = 0;
    }
    run_tile<kLds, true, false>(W, img, wave_lds, lane, O, &TM);
    LAT_T(10);
    // ---- merge (a line that reached its end finished INCOMPLETE there)
    const bool bad = act && W.verdict == V_PARSE_ERROR;
    const bool inc = act && !bad && !complete;
    const uint64_t clb = __ballot(act && W.have_cl);
    const bool err = __ballot(bad) != 0 || __popcll(clb) > 1;
    const bool any_inc = __ballot(inc) != 0;
    const uint64_t cl = clb ? (uint64_t)__shfl((unsigned long long)W.cl, (int)__builtin_ctzll(clb)) : 0ull;
    const bool chunked = __ballot(act && W.chunked) != 0;
    const uint32_t pres = act ? W.present : 0u;
    bool keep = act;
#pragma unroll
    for (int sl = 0; sl < 16; sl++) {
        const bool mine = lane >= 1 && act && pres == (1u << sl);
        const uint64_t mk = __ballot(mine);
        if (mine && lane != (uint32_t)__builtin_ctzll(mk)) keep = false;
    }
    const uint32_t present = __ockl_wfred_or_u32(keep ? pres : 0u);
    uint64_t acc[kChunksPerPass];
#pragma unroll
    for (int c = 0; c < kChunksPerPass; c++) acc[c] = __ockl_wfred_and_u64(keep ? W.acc[c] : ~0ull);
    if (lane != 0) {
        W.done = true;
        W.owed = false;
        W.base = 0;
        W.a0 = W.pa = W.lena = 0;
    } else {
        W.done = false;
        W.owed = true;
        W.scan = W.tail = false;
        W.lena = lena;
        if (err) {
            finish(W, V_PARSE_ERROR);
        } else if (hend <= 0 || any_inc || cr_end + 1 >= lena) {
            finish(W, V_INCOMPLETE);
        } else if ((cr_end_w & kLfKnown) ? !(cr_end_w & kLfYes) : *(const uint8_t *)(L.base + cr_end + 1) != '\n') {
            finish(W, V_PARSE_ERROR);
        } else {
            W.pa = cr_end + 2;
            W.mode = M_LINE;
            W.present = present;
#pragma unroll
            for (int c = 0; c < kChunksPerPass; c++) W.acc[c] = acc[c];
            W.have_cl = clb != 0;
            W.cl = cl;
            W.chunked = chunked;
            headers_done(I, W, O.nfa_bits);
        }
    }
    if (__ballot(lane == 0 && !W.done)) run_tile<kLds, true, false>(W, img, wave_lds, lane, O);  // body / next pass
    else if (lane == 0) emit(W, O);
    LAT_T(11);
}

// ---------------------------------------------------------------- latency path: well-formed heads
// lat_request runs the general framer on each lane's line, and on one wave its
// instruction path -- every mode of the resumable state machine, per byte --
// is what a synchronous call waits for (cfg2's 1.1 KB request: ~38k cycles of
// parse_window for six lines).  Most requests a proxy sees are well formed,
// and for those the framer's outcome has a short closed form, computed here
// with the bytes in LDS, the token boundaries from wave-wide masks, one lane
// per header line and one lane per DFA walk:
//
//   the header block [a0, H) ends at the first empty line; in it, no byte is a
//   CTL other than HT / CR / LF or DEL, every CR is followed by LF and every
//   LF follows a CR; line 0 is  method SP target SP "HTTP/" DIGIT "." DIGIT
//   with a method of 1..16 tchars and a target of >= 1 bytes (no SP: the
//   second SP ends it); every other line is  name ":" value  with a name of
//   1..15 [0-9A-Za-z-] (the image's name table: fast_line's lookup) and no
//   Content-Length or Transfer-Encoding header (their framing stays with the
//   framer); the rule set needs one framing pass (one DFA per slot, at most
//   kChunksPerPass chunks, no NFA matchers); at most 62 header lines.
//
// Under those conditions the framer walks the method and the target through
// their slot DFAs (the target until its state is absorbing), gives each
// header line its name's slot at the slot's first occurrence when a rule
// looks at it, walks that value from its first non-OWS byte through the
// slot's DFA with the trailing OWS excluded (until absorbing outside OWS),
// ANDs the end states' masks and the absent slots' masks into the init masks,
// and answers the first rule left (else the terminal verdict) with consumed =
// H - a0 (no Content-Length) -- which is what this computes.  Anything else,
// or a request longer than 4 KiB, returns false and goes to lat_request
// (envoy/cilium_l7policy.cc:127-182, envoy/cilium_network_policy.h:128-192).
constexpr uint32_t kFastMaxChunks = 256;  // 4 KiB of request bytes in the wave's LDS area
constexpr uint32_t kFastOffCr = kFastMaxChunks * 16, kFastOffLf = kFastOffCr + 2 * kFastMaxChunks;
constexpr uint32_t kFastOffBad = kFastOffLf + 2 * kFastMaxChunks, kFastOffPos = kFastOffBad + 2 * kFastMaxChunks;
static_assert(kFastOffPos + 4 * 64 <= kWaveLds, "fast path LDS layout");

// bit i (0..15) set iff byte i of the chunk is b
__device__ __forceinline__ uint32_t byte_mask(uint4 w, uint32_t b) {
    const uint32_t bb = b * 0x01010101u;
    auto eq = [bb](uint32_t x) {
        const uint32_t t = x ^ bb;
        return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
    };
    return nib(eq(w.x)) | nib(eq(w.y)) << 4 | nib(eq(w.z)) << 8 | nib(eq(w.w)) << 12;
}
// bytes the fast path refuses anywhere in a header block: < 0x20 other than
// HT / CR / LF, or DEL
__device__ __forceinline__ uint32_t fast_bad_mask(uint4 w) {
    return stop_mask(w) & ~(byte_mask(w, '\t') | byte_mask(w, '\r') | byte_mask(w, '\n'));
}

template <bool kLds>
__device__ __forceinline__ bool lat_fast(const Lane &L, const uint8_t *img, uint8_t *wave_lds, uint32_t lane,
                                         const Out &O) {
    const Img<kLds> I{img};
    LAT_T0
    const uint32_t a0 = L.a0, lena = L.lena;
    const uint32_t nch = (lena + 15) >> 4;
    // the rule set: one framing pass, no NFA matchers, a name table
    const uint32_t nchunks = HDR_U8(I, nchunks);
    if (lena <= a0 || nch > kFastMaxChunks || HDR_U8(I, nnfa) != 0 || HDR_U8(I, max_slot_dfas) > 1 ||
        nchunks > (uint32_t)kChunksPerPass || HDR_U8(I, ntab_bits) == 0)
        return false;
    uint16_t *crm = reinterpret_cast<uint16_t *>(wave_lds + kFastOffCr);
    uint16_t *lfm = reinterpret_cast<uint16_t *>(wave_lds + kFastOffLf);
    uint16_t *badm = reinterpret_cast<uint16_t *>(wave_lds + kFastOffBad);
    uint32_t *crpos = reinterpret_cast<uint32_t *>(wave_lds + kFastOffPos);
    const uint64_t below = (1ull << lane) - 1;
    // ---- the request into LDS, its CR / LF / refused-byte masks, the first 64 CRs in order
    uint32_t ncr = 0;
    for (uint32_t c0 = 0; c0 < nch; c0 += 64) {
        const uint32_t c = c0 + lane;
        uint32_t m = 0;
        if (c < nch) {
            const uint4 w = gload16(L.base + 16ull * c);
            *reinterpret_cast<uint4 *>(wave_lds + 16 * c) = w;
            const uint32_t p0 = 16 * c;
            uint32_t in = 0xFFFFu;  // bytes of [a0, lena)
            if (p0 < a0) in &= 0xFFFFu << (a0 - p0);
            if (p0 + 16 > lena) in &= (1u << (lena - p0)) - 1u;
            m = byte_mask(w, '\r') & in;
            crm[c] = (uint16_t)m;
            lfm[c] = (uint16_t)(byte_mask(w, '\n') & in);
            badm[c] = (uint16_t)(fast_bad_mask(w) & in);
        }
        const uint32_t cnt = (uint32_t)__builtin_popcount(m);
        uint32_t ex = 0;
#pragma unroll
        for (int b = 0; b < 5; b++) ex += (uint32_t)__popcll(__ballot((cnt >> b) & 1) & below) << b;
        for (uint32_t r = ncr + ex; m; m &= m - 1, r++)
            if (r < 64) crpos[r] = 16 * c + (uint32_t)__builtin_ctz(m);
        ncr += (uint32_t)__builtin_amdgcn_readfirstlane((int)__ockl_wfred_add_u32(cnt));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    LAT_T(13);
    // the empty line: the first CR two bytes after the one before it
    const uint32_t have = min(ncr, 64u);
    const uint32_t mycr = lane < have ? crpos[lane] : 0u;
    const uint32_t prevcr = lane >= 1 && lane < have ? crpos[lane - 1] : 0u;
    const uint64_t eb = __ballot(lane >= 1 && lane < have && mycr == prevcr + 2);
    if (!eb) return false;
    const uint32_t hend = (uint32_t)__builtin_ctzll(eb);  // lines 0 .. hend-1, then the empty line
    if (hend > 62) return false;
    const uint32_t H = (uint32_t)__shfl((int)mycr, (int)hend) + 2;  // end of the header block
    if (H > lena) return false;
    // ---- the block's bytes: nothing refused, CR and LF only as CRLF
    bool bad = false;
    for (uint32_t c = lane; 16 * c < H; c += 64) {
        const uint32_t p0 = 16 * c;
        uint32_t in = 0xFFFFu;
        if (p0 < a0) in &= 0xFFFFu << (a0 - p0);
        if (p0 + 16 > H) in &= (1u << (H - p0)) - 1u;
        const uint32_t cr = crm[c], prev = c ? (uint32_t)crm[c - 1] >> 15 : 0u;
        bad |= (badm[c] & in) != 0 || (lfm[c] & in) != (((cr << 1) | prev) & in);
    }
    if (__ballot(bad)) return false;
    LAT_T(9);
    // ---- lane k: line k = [s, e), e its CR
    const uint32_t s = lane == 0 ? a0 : prevcr + 2, e = mycr;
    const bool line = lane < hend;
    auto chunk = [&](uint32_t k) { return *reinterpret_cast<const uint4 *>(wave_lds + 16 * k); };
    // the 16 bytes at p (p + 16 may pass the copy's end only inside its last chunk's area)
    auto bytes16 = [&](uint32_t p) {
        const uint32_t k0 = p >> 4, o = p & 15, i = o >> 2, sh = (o & 3) * 8;
        const uint4 a = chunk(k0), b = k0 + 1 < kFastMaxChunks ? chunk(k0 + 1) : make_uint4(0, 0, 0, 0);
        const uint32_t d0 = i == 0 ? a.x : i == 1 ? a.y : i == 2 ? a.z : a.w;
        const uint32_t d1 = i == 0 ? a.y : i == 1 ? a.z : i == 2 ? a.w : b.x;
        const uint32_t d2 = i == 0 ? a.z : i == 1 ? a.w : i == 2 ? b.x : b.y;
        const uint32_t d3 = i == 0 ? a.w : i == 1 ? b.x : i == 2 ? b.y : b.z;
        const uint32_t d4 = i == 0 ? b.x : i == 1 ? b.y : i == 2 ? b.z : b.w;
        uint4 f;
        f.x = (uint32_t)((((uint64_t)d1 << 32) | d0) >> sh);
        f.y = (uint32_t)((((uint64_t)d2 << 32) | d1) >> sh);
        f.z = (uint32_t)((((uint64_t)d3 << 32) | d2) >> sh);
        f.w = (uint32_t)((((uint64_t)d4 << 32) | d3) >> sh);
        return f;
    };
    auto byte_at = [&](uint32_t p) { return (uint32_t)wave_lds[p]; };
    bool refuse = false;
    // request line (lane 0): exactly two SPs and no HT (HT ends a target, and
    // not SP after it is an error), a method of 1..15 [0-9A-Za-z-], the version
    uint32_t sp1 = 0, sp2 = 0;
    if (lane == 0) {
        uint32_t nsp = 0;
        bool ht = false;
        for (uint32_t p = s & ~15u; p < e; p += 16) {
            const uint4 w = chunk(p >> 4);
            uint32_t in = 0xFFFFu;
            if (p < s) in &= 0xFFFFu << (s - p);
            if (p + 16 > e) in &= (1u << (e - p)) - 1u;
            uint32_t m = byte_mask(w, ' ') & in;
            ht |= (byte_mask(w, '\t') & in) != 0;
            const uint32_t q1 = p + (uint32_t)__builtin_ctz(m | 0x10000u);
            const uint32_t m2 = m & (m - 1);
            const uint32_t q2 = p + (uint32_t)__builtin_ctz(m2 | 0x10000u);
            sp2 = nsp == 0 ? q2 : nsp == 1 ? q1 : sp2;
            sp1 = nsp == 0 ? q1 : sp1;
            nsp += (uint32_t)__builtin_popcount(m);
        }
        const uint4 f = bytes16(s), v = bytes16(sp2 + 1);
        refuse = nsp != 2 || ht || sp1 == s || sp1 - s > 15 || sp2 == sp1 + 1 || e - sp2 != 9 ||
                 (uint32_t)__builtin_ctz(nonalnum_mask(f) | 0x10000u) != sp1 - s ||
                 !(v.x == 0x50545448u && (v.y & 0x00FF00FFu) == 0x002E002Fu && ((v.y >> 8) & 0xFF) - '0' < 10u &&
                   (v.y >> 24) - '0' < 10u);
    }
    // header lines (lanes 1 .. hend-1): the name's flags from the name table
    uint32_t ninfo = 0, vs = 0;
    if (line && lane > 0) {
        const uint4 f = bytes16(s);
        const uint32_t en = (uint32_t)__builtin_ctz(nonalnum_mask(f) | 0x10000u);
        if (en == 0 || en == 16 || s + en >= e || byte_of(f, en) != ':') {
            refuse = true;
        } else {
            auto keep = [en](uint32_t j) { return en >= 4 * j + 4 ? 0xFFFFFFFFu : en <= 4 * j ? 0u : (1u << (8 * (en - 4 * j))) - 1u; };
            const uint32_t w0 = (f.x | 0x20202020u) & keep(0), w1 = (f.y | 0x20202020u) & keep(1);
            const uint32_t w2 = (f.z | 0x20202020u) & keep(2), w3 = (f.w | 0x20202020u) & keep(3);
            const uint32_t h = l7_name_hash(w0, w1, w2, w3, en, HDR_U32(I, ntab_mul), HDR_U8(I, ntab_bits));
            const uint32_t ent = HDR_U32(I, ntab_off) + h * (uint32_t)sizeof(DevNameEnt);
            const uint4 n = I.u128(ent);
            const uint32_t meta = I.u32(ent + 16);
            const bool hit = (meta & 0xFF) == en && n.x == w0 && n.y == w1 && n.z == w2 && n.w == w3;
            ninfo = hit ? (meta >> 8) & 0xFF : 0u;
            if (ninfo & (NI_CL | NI_TE)) refuse = true;  // body framing: the framer's
            vs = s + en + 1;  // then past the OWS (M_OWS)
            const uint32_t o = (uint32_t)__builtin_ctz((~ws_mask(bytes16(vs)) & 0xFFFFu) | 0x10000u);
            vs += o;
            if (o == 16)
                while (vs < e && (byte_at(vs) == ' ' || byte_at(vs) == '\t')) vs++;
        }
    }
    if (__ballot(refuse)) return false;
    LAT_T(10);
    // slots: a header's at its first occurrence when some rule looks at it
    const uint32_t ref = HDR_U32(I, ref_slots);
    uint32_t slot = kNoSlot;
    if (line && lane > 0) {
        if (ninfo & NI_HOST) slot = SLOT_AUTHORITY;
        else if (ninfo & NI_CUSTOM) slot = SLOT_CUSTOM0 + (ninfo & NI_CUSTOM) - 1;
        if (slot != kNoSlot && !((ref >> slot) & 1)) slot = kNoSlot;
    }
#pragma unroll
    for (uint32_t sl = SLOT_AUTHORITY; sl < (uint32_t)kNumSlots; sl++) {
        const uint64_t mk = __ballot(slot == sl);
        if (slot == sl && lane != (uint32_t)__builtin_ctzll(mk)) slot = kNoSlot;
    }
    LAT_T(14);
    // ---- the DFA walks: lane 0 the target, lane 63 the method, lane k its value
    sp1 = (uint32_t)__shfl((int)sp1, 0);
    sp2 = (uint32_t)__shfl((int)sp2, 0);
    uint32_t wslot = slot, from = vs, to = e, kind = 2;  // kind: 0 method, 1 target, 2 value
    if (lane == 0) { wslot = SLOT_PATH; from = sp1 + 1; to = sp2; kind = 1; }
    if (lane == 63) { wslot = SLOT_METHOD; from = a0; to = sp1; kind = 0; }
    uint64_t acc[kChunksPerPass];
#pragma unroll
    for (int c = 0; c < kChunksPerPass; c++) acc[c] = ~0ull;
    const uint32_t nc = min(nchunks, (uint32_t)kChunksPerPass);
    if (wslot != kNoSlot) {
        const uint32_t lo = I.u8(offsetof(ImgHeader, slot_dfa) + wslot);
        const uint32_t hi = I.u8(offsetof(ImgHeader, slot_dfa) + wslot + 1);
        if (lo < hi) {
            const uint32_t d = HDR_U32(I, dfa_off) + lo * sizeof(DevDfa);
            const uint32_t dcls = I.u32(d + 0), dtrans = I.u32(d + 4), dmask = I.u32(d + 8);
            const uint32_t nc_st = I.u32(d + 12), dncls = nc_st & 0xFFFF, dabs = I.u32(d + 16);
            uint32_t st = nc_st >> 16, saved = 0;
            bool in_ows = false;
            uint32_t p = from;
            // the framer's walks (parse_window M_METHOD / M_TARGET / M_VALUE), 16
            // bytes a step: their classes read together, then the transitions
            bool go = p < to && (kind == 0 || (st != 0 && st < dabs));
            while (go) {
                const uint4 f = bytes16(p);
                uint32_t k[16];
#pragma unroll
                for (uint32_t j = 0; j < 16; j++) k[j] = I.u8(dcls + byte_of(f, j));
#pragma unroll
                for (uint32_t j = 0; j < 16; j++) {
                    if (go) {
                        if (kind == 2) {
                            const uint32_t c = byte_of(f, j);
                            const bool ws = c == ' ' || c == '\t';
                            if (ws && !in_ows) saved = st;
                            in_ows = ws;
                        }
                        if (st) st = I.u16(dtrans + 2 * (st * dncls + k[j]));
                        p++;
                        go = p < to && (kind == 0 || in_ows || (st != 0 && st < dabs));
                    }
                }
            }
            if (kind == 2 && p >= to && in_ows) st = saved;  // trailing OWS is not part of the value
            const uint32_t base = dmask + 8 * (st * nchunks);
#pragma unroll
            for (int cc = 0; cc < kChunksPerPass; cc++)
                if ((uint32_t)cc < nc) acc[cc] = I.u64(base + 8 * cc);
        }
    }
    LAT_T(15);
    // ---- merge (headers_done on one pass)
    const uint32_t present = __ockl_wfred_or_u32(lane > 0 && lane < 63 && slot != kNoSlot ? 1u << slot : 0u) |
                             (1u << SLOT_METHOD) | (1u << SLOT_PATH);
    uint64_t a[kChunksPerPass];
#pragma unroll
    for (int c = 0; c < kChunksPerPass; c++) a[c] = __ockl_wfred_and_u64(acc[c]);
    if (lane == 0) {
#pragma unroll
        for (int c = 0; c < kChunksPerPass; c++)
            a[c] &= (uint32_t)c < nchunks ? I.u64(HDR_U32(I, init_off) + 8 * c) : 0ull;
        uint32_t missing = ref & 0xFFFF & ~present;
        while (missing) {
            const uint32_t sl = __builtin_ctz(missing);
            missing &= missing - 1;
#pragma unroll
            for (int c = 0; c < kChunksPerPass; c++)
                if ((uint32_t)c < nc) a[c] &= I.u64(HDR_U32(I, absent_off) + 8 * (sl * nchunks + c));
        }
        int32_t hit = -1;
#pragma unroll
        for (int c = kChunksPerPass - 1; c >= 0; c--)
            if ((uint32_t)c < nc && a[c]) hit = (int32_t)(64 * c + (uint32_t)__builtin_ctzll(a[c]));
        Lane W = L;
        W.consumed = H - a0;
        if (hit >= 0) finish(W, V_ALLOW, (int32_t)I.u32(HDR_U32(I, rule_off) + 4 * (uint32_t)hit));
        else finish(W, (uint8_t)HDR_U8(I, terminal), -1);
        emit(W, O);
    }
    LAT_T(11);
    return true;
}

}  // namespace

// kHot = true : requests whose connection uses the hot rule set (image in LDS),
//               plus entries on connections without an HTTP parser.
// kHot = false: every other HTTP request (images read through L2); all of
//               them when no hot kernel runs (T.hot_ruleset < 0).
// answer_other: also answer the entries no classifier owns (unknown connection,
// no parser) UNSUPPORTED; false when partition_kernel has answered them.
// sel: the HTTP requests of a mixed batch (partition_kernel), tiles of 64
// list entries; null: the whole batch, tiles of 64 consecutive requests.
// kGrab: tiles taken from the counter per atomic (1, or 4 for short requests;
// the launcher's note).  Separate instantiations keep kGrab == 1 the round-4
// code (+1-2 % on cfg2 when the grab size was a runtime value).
template <bool kHot, uint32_t kGrab = 1>
__global__ __launch_bounds__(kBlock) void http_classify_kernel(Batch B, HttpTables T, const uint32_t *__restrict__ sel,
                                                               const uint32_t *__restrict__ sel_count,
                                                               uint32_t answer_other, uint32_t *__restrict__ tile_ctr) {
    const uint8_t *__restrict__ arena = B.arena;
    const uint32_t n = B.n, nconns = B.nconns;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63, wave = tid >> 6;
    uint8_t *s_img = lds + kOffImg;

    const int32_t hot = T.hot_ruleset;
    const bool hot_ok = hot >= 0 && (uint32_t)hot < T.nrulesets && T.rulesets[hot].image_len <= kLdsImageBytes;
    if (kHot && !hot_ok) return;
#ifdef L7G_PHASE_TIMING
    const uint64_t ph_k0 = __builtin_amdgcn_s_memtime();
#endif
    // stage the hot rule set's image
    if (kHot) {
        const DevRuleset r = T.rulesets[hot];
        const uint4 *src = (const uint4 *)(T.images + r.image_off);
        const uint32_t n16 = (r.image_len + 15) / 16;
        // every load issued before the first store: one memory round trip, not
        // one per 8 KiB (a small launch -- one request -- waits on this)
        constexpr uint32_t kIters = (kLdsImageBytes / 16 + kBlock - 1) / kBlock;
        uint4 t[kIters];
#pragma unroll
        for (uint32_t k = 0; k < kIters; k++)
            if (tid + k * kBlock < n16) t[k] = src[tid + k * kBlock];
#pragma unroll
        for (uint32_t k = 0; k < kIters; k++)
            if (tid + k * kBlock < n16) ((uint4 *)s_img)[tid + k * kBlock] = t[k];
    }
    __syncthreads();
#ifdef L7G_PHASE_TIMING
    if (tid == 0) atomicAdd(&g_phase[7], (unsigned long long)(__builtin_amdgcn_s_memtime() - ph_k0));
#endif

    const Out O{B.verdict, B.rule, B.consumed, T.nfa_bits};
    uint8_t *wave_lds = lds + wave * kWaveLds;
    const uint32_t m = sel ? *sel_count : n;
    const uint32_t ntiles = (m + 63) / 64;
    // Tiles: the first by position, the rest (when the launcher passes a zeroed
    // counter) taken one at a time by whichever wave is free, so the waves of
    // the persistent grid finish together whatever their tiles cost; else a
    // fixed stride.
    const uint32_t stride = gridDim.x * kWaves;
    uint32_t grab_next = 0, grab_left = 0;  // tiles taken from the counter, not started yet (wave-uniform)
    for (uint32_t tile = blockIdx.x * kWaves + wave, next; tile < ntiles; tile = next) {
        next = tile + stride;
        Lane L;
        const uint32_t slot = tile * 64 + lane;
        L.idx = sel ? (slot < m ? sel[slot] : n) : slot;
        L.done = true;
        L.owed = false;
        L.verdict = V_UNSUPPORTED;
        L.rule = -1;
        L.consumed = 0;
        L.mode = M_DONE;
        L.base = 0;
        L.a0 = L.pa = L.w = L.lena = 0;
        const uint8_t *img = kHot ? s_img : nullptr;
        if (L.idx < n) {
            const uint32_t ci = B.conn_ids[L.idx];
            const DevConn conn = ci < nconns ? B.conns[ci] : DevConn{-1, PROTO_NONE, 0, 0xFFFF};
            // entries of other protocols belong to their own kernels; the HTTP
            // kernel answers entries whose connection is unknown or has no parser
            const bool mine = !L7_PROTO_OWNED(conn.proto) || conn.proto == PROTO_HTTP;
            const bool http = mine && conn.proto == PROTO_HTTP && conn.ruleset >= 0 && (uint32_t)conn.ruleset < T.nrulesets;
            const bool is_hot = http && hot_ok && conn.ruleset == hot;
            if (mine && !http && answer_other && (kHot || !hot_ok)) L.owed = true;  // unsupported connection: answered as is
            if (http && is_hot == kHot) {
                const uint64_t off = B.offs[L.idx];
                const uint32_t len = B.lens[L.idx];
                if (!l7_in_arena(off, len, B.arena_len)) {  // outside the arena: out of contract
                    L.owed = true;
                } else {
                const uint64_t a = (uint64_t)(arena + off);
                L.base = a & ~(uint64_t)15;
                L.a0 = (uint32_t)(a & 15);
                L.lena = len > 0xFFFFFF00u ? 0xFFFFFF00u + L.a0 : L.a0 + len;  // > 4 GiB - 256: framing stops there
                if (!kHot) img = T.images + T.rulesets[conn.ruleset].image_off;
                L.done = false;
                L.owed = true;
                }
            }
        }
        run_tile<kHot>(L, img, wave_lds, lane, O);
        if (tile_ctr) {  // taken at the tile's end: a wave asks for work only when it is free
            if (kGrab == 1) {
                uint32_t t = 0;
                if (lane == 0) t = atomicAdd(tile_ctr, 1u);
                next = stride + __builtin_amdgcn_readfirstlane(t);
            } else {
                if (grab_left == 0) {
                    uint32_t t = 0;
                    if (lane == 0) t = atomicAdd(tile_ctr, kGrab);
                    grab_next = stride + __builtin_amdgcn_readfirstlane(t);
                    grab_left = kGrab;
                }
                next = grab_next++;
                grab_left--;
            }
        }
    }
}


// One request per wave (lat_request above) for small calls; the image
// staging, the request's checks and the answers for entries no parser owns are
// the tile kernel's.  stage: copy the hot rule set's image into LDS (the
// resident service stages it once for its lifetime).  Ends with a barrier.
template <bool kHot>
__device__ __forceinline__ void lat_body(const Batch &B, const HttpTables &T, const uint32_t *__restrict__ sel,
                                         const uint32_t *__restrict__ sel_count, uint32_t answer_other, uint8_t *lds,
                                         bool stage) {
    const uint8_t *__restrict__ arena = B.arena;
    const uint32_t n = B.n, nconns = B.nconns;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63, wave = tid >> 6;
    uint8_t *s_img = lds + kOffImg;
#ifdef L7G_PHASE_TIMING
    const uint64_t ph_k0 = __builtin_amdgcn_s_memtime();
#endif
    const int32_t hot = T.hot_ruleset;
    const bool hot_ok = hot >= 0 && (uint32_t)hot < T.nrulesets && T.rulesets[hot].image_len <= kLdsImageBytes;
    if (kHot && !hot_ok) return;
    if (kHot && stage) {
        const DevRuleset r = T.rulesets[hot];
        const uint4 *src = (const uint4 *)(T.images + r.image_off);
        const uint32_t n16 = (r.image_len + 15) / 16;
        constexpr uint32_t kIters = (kLdsImageBytes / 16 + kBlock - 1) / kBlock;
        uint4 t[kIters];
#pragma unroll
        for (uint32_t k = 0; k < kIters; k++)
            if (tid + k * kBlock < n16) t[k] = src[tid + k * kBlock];
#pragma unroll
        for (uint32_t k = 0; k < kIters; k++)
            if (tid + k * kBlock < n16) ((uint4 *)s_img)[tid + k * kBlock] = t[k];
    }
    __syncthreads();
#ifdef L7G_PHASE_TIMING
    if (tid == 0) atomicAdd(&g_phase[7], (unsigned long long)(__builtin_amdgcn_s_memtime() - ph_k0));
#endif
    const Out O{B.verdict, B.rule, B.consumed, T.nfa_bits};
    uint8_t *wave_lds = lds + wave * kWaveLds;
    const uint32_t m = sel ? *sel_count : n;
    for (uint32_t r = blockIdx.x * kWaves + wave; r < m; r += gridDim.x * kWaves) {
        LAT_T0
        Lane L;
        L.idx = sel ? sel[r] : r;
        L.done = true;
        L.owed = false;
        L.verdict = V_UNSUPPORTED;
        L.rule = -1;
        L.consumed = 0;
        L.mode = M_DONE;
        L.base = 0;
        L.a0 = L.pa = L.w = L.lena = 0;
        const uint8_t *img = kHot ? s_img : nullptr;
        if (L.idx < n) {
            const uint32_t ci = B.conn_ids[L.idx];
            const DevConn conn = ci < nconns ? B.conns[ci] : DevConn{-1, PROTO_NONE, 0, 0xFFFF};
            const bool mine = !L7_PROTO_OWNED(conn.proto) || conn.proto == PROTO_HTTP;
            const bool http = mine && conn.proto == PROTO_HTTP && conn.ruleset >= 0 && (uint32_t)conn.ruleset < T.nrulesets;
            const bool is_hot = http && hot_ok && conn.ruleset == hot;
            if (mine && !http && answer_other && (kHot || !hot_ok)) L.owed = true;
            if (http && is_hot == kHot) {
                const uint64_t off = B.offs[L.idx];
                const uint32_t len = B.lens[L.idx];
                if (!l7_in_arena(off, len, B.arena_len)) {
                    L.owed = true;
                } else {
                    const uint64_t a = (uint64_t)(arena + off);
                    L.base = a & ~(uint64_t)15;
                    L.a0 = (uint32_t)(a & 15);
                    L.lena = len > 0xFFFFFF00u ? 0xFFFFFF00u + L.a0 : L.a0 + len;
                    if (!kHot) img = T.images + T.rulesets[conn.ruleset].image_off;
                    L.done = false;
                    L.owed = true;
                }
            }
        }
        LAT_T(8);
        LAT_N(12);
        if (!L.done) {
            if (!lat_fast<kHot>(L, img, wave_lds, lane, O)) lat_request<kHot>(L, img, wave_lds, lane, O);
        } else if (L.owed && lane == 0) {
            emit(L, O);
        }
    }
    __syncthreads();
}

template <bool kHot>
// ci: the call's inputs to copy first (a one-workgroup launch), or none.
__global__ __launch_bounds__(kBlock) void http_latency_kernel(Batch B, HttpTables T, const uint32_t *__restrict__ sel,
                                                              const uint32_t *__restrict__ sel_count,
                                                              uint32_t answer_other, CopyIn ci) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
    copy_in_block(ci);
    lat_body<kHot>(B, T, sel, sel_count, answer_other, lds, true);
    signal_done_block(ci);
}

// The resident service (kernels/service.h): one workgroup serves the
// synchronous HTTP calls (one Envoy Allowed(), a few requests) the host posts
// to the box, each as the launched path would run it -- the inputs copied
// into HBM, the hot pass and / or the general pass of lat_body, the answers to
// pinned memory, then the done word -- with the hot rule set's image staged
// in LDS once for the service's lifetime.  The box's first word holds the
// poll's result (wave 0's window area: free between calls).
__global__ __launch_bounds__(kBlock) void http_service_kernel(SvcBox *box, SvcStatic S, HttpTables T, uint32_t seen0,
                                                              uint64_t idle) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
    uint32_t *word = reinterpret_cast<uint32_t *>(lds);
    uint32_t seen = seen0;
    uint64_t t_last = __builtin_amdgcn_s_memtime();
    bool staged = false;
    if (threadIdx.x == 0) svc_store(&box->state, kSvcRunning);
    for (;;) {
        const SvcCall c = svc_next(box, seen, t_last, idle, word);
        if (!c.seq) break;
        const Batch B = svc_batch(S, c);
        const CopyIn ci = svc_copy(S, box, c);
        copy_in_block(ci);
        const uint32_t other = (c.flags & kSvcAnswerOther) ? 1u : 0u;
        if (c.flags & kSvcHttpHot) {
            lat_body<true>(B, T, nullptr, nullptr, other, lds, !staged);
            staged = true;
        }
        if (c.flags & kSvcHttpGeneral) lat_body<false>(B, T, nullptr, nullptr, other, lds, false);
        signal_done_block(ci);
        __syncthreads();
        t_last = __builtin_amdgcn_s_memtime();
    }
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        svc_store(&box->state, kSvcStopped);
    }
}

// Requests grouped by rule set (http_group.hip): a workgroup takes one segment
// of the grouped list at a time (all of it on one rule set), stages that rule
// set's image in LDS, and its waves take the segment's tiles of 64 entries
// from a counter in LDS; the image-in-LDS framer runs them (a tile never mixes
// rule sets, so image-derived values are wave-uniform as in the hot kernel).
// ctl: [0] segments, [1] the segment counter (zeroed by the launcher).
__global__ __launch_bounds__(kBlock) void http_grouped_kernel(Batch B, HttpTables T, const uint32_t *__restrict__ gsel,
                                                              const uint32_t *__restrict__ segs,
                                                              uint32_t *__restrict__ ctl) {
    const uint8_t *__restrict__ arena = B.arena;
    const uint32_t n = B.n;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63, wave = tid >> 6;
    uint8_t *s_img = lds + kOffImg;
    uint32_t *s_ctl = reinterpret_cast<uint32_t *>(lds + kOffImg + kGroupImageBytes);  // segment, tile counter
    const Out O{B.verdict, B.rule, B.consumed, T.nfa_bits};
    uint8_t *wave_lds = lds + wave * kWaveLds;
    const uint32_t nsegs = ctl[0];
    for (;;) {
        if (tid == 0) {
            s_ctl[0] = atomicAdd(&ctl[1], 1u);
            s_ctl[1] = 0;
        }
        __syncthreads();
        const uint32_t sg = s_ctl[0];
        if (sg >= nsegs) break;
        const uint32_t rs = segs[3 * sg], e0 = segs[3 * sg + 1], cnt = segs[3 * sg + 2];
        {
            const DevRuleset r = T.rulesets[rs];
            const uint4 *src = (const uint4 *)(T.images + r.image_off);
            const uint32_t n16 = (r.image_len + 15) / 16;
            constexpr uint32_t kIters = (kGroupImageBytes / 16 + kBlock - 1) / kBlock;
            uint4 t[kIters];
#pragma unroll
            for (uint32_t k = 0; k < kIters; k++)
                if (tid + k * kBlock < n16) t[k] = src[tid + k * kBlock];
#pragma unroll
            for (uint32_t k = 0; k < kIters; k++)
                if (tid + k * kBlock < n16) ((uint4 *)s_img)[tid + k * kBlock] = t[k];
        }
        __syncthreads();
        for (;;) {
            uint32_t tile = 0;
            if (lane == 0) tile = atomicAdd(&s_ctl[1], 1u);
            tile = (uint32_t)__builtin_amdgcn_readfirstlane((int)tile);
            if (tile * 64 >= cnt) break;
            Lane L;
            const uint32_t slot = tile * 64 + lane;
            L.idx = slot < cnt ? gsel[e0 + slot] : n;
            L.done = true;
            L.owed = false;
            L.verdict = V_UNSUPPORTED;
            L.rule = -1;
            L.consumed = 0;
            L.mode = M_DONE;
            L.base = 0;
            L.a0 = L.pa = L.w = L.lena = 0;
            if (L.idx < n) {  // (every grouped entry is an HTTP request on rule set rs)
                L.owed = true;
                const uint64_t off = B.offs[L.idx];
                const uint32_t len = B.lens[L.idx];
                if (l7_in_arena(off, len, B.arena_len)) {  // else out of contract: answered UNSUPPORTED
                    const uint64_t a = (uint64_t)(arena + off);
                    L.base = a & ~(uint64_t)15;
                    L.a0 = (uint32_t)(a & 15);
                    L.lena = len > 0xFFFFFF00u ? 0xFFFFFF00u + L.a0 : L.a0 + len;
                    L.done = false;
                }
            }
            run_tile<true>(L, s_img, wave_lds, lane, O);
        }
        __syncthreads();  // every wave is done with the image before the next segment's
    }
}

// Host-side launcher (called from the C-ABI): persistent grids of one
// 512-thread workgroup per CU; the hot-rule-set kernel, then (only if some
// HTTP connection uses another rule set) the general one.
// latency: a small call, one request per wave (http_latency_kernel)
// (ci: latency only, with one workgroup: copied by the first kernel launched)
hipError_t LaunchHttpClassify(const Batch &B, const HttpTables &T, const uint32_t *sel, const uint32_t *sel_count,
                              bool any_cold, bool answer_other, uint32_t *tile_ctr, bool latency, const CopyIn *ci,
                              hipStream_t stream) {
    if (B.n == 0) return hipSuccess;
    static int num_cus = 0;
    if (num_cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || num_cus <= 0)
            num_cus = 256;
    }
    const bool hot = T.hot_ruleset >= 0;
    const uint32_t other = answer_other ? 1u : 0u;
    if (latency) {
        const uint32_t lblocks = min((B.n + kWaves - 1) / kWaves, (uint32_t)num_cus);
        if (ci && lblocks != 1) return hipErrorInvalidValue;
        // the copy in the first kernel, the done word from the last
        const bool gen = !hot || any_cold;
        CopyIn first = ci ? *ci : CopyIn{};
        if (hot) {
            CopyIn k = first;
            if (gen) k.done = nullptr;
            hipLaunchKernelGGL(http_latency_kernel<true>, dim3(lblocks), dim3(kBlock), 0, stream, B, T, sel, sel_count,
                               other, k);
            first.n = 0;
        }
        if (gen)
            hipLaunchKernelGGL(http_latency_kernel<false>, dim3(lblocks), dim3(kBlock), 0, stream, B, T, sel, sel_count,
                               other, first);
        return hipGetLastError();
    }
    if (ci) return hipErrorInvalidValue;
    const uint32_t ntiles = (B.n + 63) / 64;
    uint32_t blocks = (ntiles + kWaves - 1) / kWaves;
    blocks = min(blocks, (uint32_t)num_cus);
    // tile_ctr: two zeroed counters (hot, general launch) or null (fixed stride).
    // Tiles taken from a counter one at a time serialise on its atomic when
    // they are quick (short requests: 4M 34-byte requests 0.74 ms, taken four at
    // a time 0.36 ms), and cost a longer tail when they are not (cfg2's 1.1 KB
    // requests: 1.59 vs 1.63 ms), so a batch of short requests takes four.
    // A wave with many tiles to run (a long batch: cfg5's 50M HTTP requests are
    // ~380 tiles per wave) also takes two per atomic: the tail grows by half a
    // tile, the counter's queue shrinks (cfg5 HTTP 16.94 -> 16.87 ms, profiles/r5/ab5e_work_grab.log).
    const uint32_t per_wave = ntiles / (blocks * kWaves);
    const uint32_t grab = B.arena_len / B.n < 512 ? 4u : per_wave >= 64 ? 2u : 1u;
    using Kern = void (*)(Batch, HttpTables, const uint32_t *, const uint32_t *, uint32_t, uint32_t *);
    const Kern kHot = grab == 4 ? http_classify_kernel<true, 4> : grab == 2 ? http_classify_kernel<true, 2>
                                                                         : http_classify_kernel<true, 1>;
    const Kern kGen = grab == 4 ? http_classify_kernel<false, 4> : grab == 2 ? http_classify_kernel<false, 2>
                                                                          : http_classify_kernel<false, 1>;
    if (hot)
        hipLaunchKernelGGL(kHot, dim3(blocks), dim3(kBlock), 0, stream, B, T, sel, sel_count, other, tile_ctr);
    if (!hot || any_cold)
        hipLaunchKernelGGL(kGen, dim3(blocks), dim3(kBlock), 0, stream, B, T, sel, sel_count, other,
                           tile_ctr ? tile_ctr + 1 : nullptr);
    return hipGetLastError();
}

// The grouped list (LaunchHttpGroup's outputs): the grouped kernel over the
// segments, then the general kernel over the entries on rule sets whose image
// exceeds the LDS budget (gbig, ctl[2] of them; ctl[3] its tile counter).
hipError_t LaunchHttpGrouped(const Batch &B, const HttpTables &T, const uint32_t *gsel, const uint32_t *segs,
                             const uint32_t *gbig, uint32_t *ctl, bool any_big, hipStream_t stream) {
    if (B.n == 0) return hipSuccess;
    static int num_cus = 0;
    if (num_cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&num_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || num_cus <= 0)
            num_cus = 256;
    }
    const uint32_t ntiles = (B.n + 63) / 64;
    const uint32_t blocks = min((ntiles + kWaves - 1) / kWaves, (uint32_t)num_cus);
    hipLaunchKernelGGL(http_grouped_kernel, dim3(blocks), dim3(kBlock), 0, stream, B, T, gsel, segs, ctl);
    if (any_big)
        hipLaunchKernelGGL(http_classify_kernel<false>, dim3(blocks), dim3(kBlock), 0, stream, B, T, gbig, ctl + 2, 0u,
                           ctl + 3);
    return hipGetLastError();
}

// The HTTP service: one workgroup on `stream` until it leaves (idle cycles
// without a call, or stop).
hipError_t LaunchHttpService(SvcBox *box, const SvcStatic &S, const HttpTables &T, uint32_t seen0, uint64_t idle,
                             hipStream_t stream) {
    hipLaunchKernelGGL(http_service_kernel, dim3(1), dim3(kBlock), 0, stream, box, S, T, seen0, idle);
    return hipGetLastError();
}

#ifdef L7G_PHASE_TIMING
hipError_t HttpPhaseTimes(uint64_t *out, bool reset) {
    hipError_t rc = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(unsigned long long) * 16);
    if (rc == hipSuccess && reset) {
        static const unsigned long long z[16] = {};
        rc = hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof z);
    }
    return rc;
}
#else
hipError_t HttpPhaseTimes(uint64_t *, bool) { return hipErrorNotSupported; }
#endif

}  // namespace l7
