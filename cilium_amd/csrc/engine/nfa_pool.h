// Device layout of bit-parallel NFAs (product code): BitNfa (re_dfa.h) ->
// DevNfa + its tables appended to a pool (device_tables.h).
#pragma once
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../device_tables.h"
#include "../regex/re_dfa.h"

namespace l7 {

// Appends n's device tables to pool (16-byte aligned); returns the DevNfa
// offset, or ~0ull with *err when the pool would pass 4 GiB.
inline uint64_t AppendDevNfa(const re::BitNfa &n, std::vector<uint8_t> *pool, std::string *err) {
    const size_t W = (size_t)n.W, K = (size_t)n.K, m = (size_t)n.m;
    auto align = [&](size_t bytes) {
        size_t off = (pool->size() + 15) & ~(size_t)15;
        pool->resize(off + bytes, 0);
        return off;
    };
    if (n.sparse != (W > (size_t)kNfaMaxWords)) {
        *err = "NFA table form does not match its size";
        return ~0ull;
    }
    const size_t t_bytes = n.sparse ? sizeof(DevNfaSparse) + K * m * 4 + n.row_ptr.size() * 4 + n.pair_w.size() * 12 + 64
                                    : K * 8 * W * 256 * W * 8;
    const size_t niv = n.ivl_lo.size();
    if (pool->size() + t_bytes + niv * (W * 8 + 4) + K * W * 8 + 512 > (1ull << 32)) {
        *err = "NFA tables exceed 4 GiB";
        return ~0ull;
    }
    DevNfa d{};
    const size_t doff = align(sizeof(DevNfa));
    d.m = (uint32_t)n.m;
    d.W = (uint32_t)W;
    d.K = (uint32_t)K;
    d.nivl = (uint32_t)niv;
    memcpy(d.condmap, n.condmap, sizeof d.condmap);
    if (n.sparse) {
        d.t_off = align(sizeof(DevNfaSparse));
        DevNfaSparse sp{};
        sp.row_of_off = align(K * m * 4);
        memcpy(pool->data() + sp.row_of_off, n.row_of.data(), K * m * 4);
        sp.row_ptr_off = align(n.row_ptr.size() * 4);
        memcpy(pool->data() + sp.row_ptr_off, n.row_ptr.data(), n.row_ptr.size() * 4);
        sp.pair_w_off = align(n.pair_w.size() * 4);
        memcpy(pool->data() + sp.pair_w_off, n.pair_w.data(), n.pair_w.size() * 4);
        sp.pair_m_off = align(n.pair_m.size() * 8);
        memcpy(pool->data() + sp.pair_m_off, n.pair_m.data(), n.pair_m.size() * 8);
        memcpy(pool->data() + d.t_off, &sp, sizeof sp);
    } else {
        d.t_off = align(t_bytes);
        uint64_t *T = (uint64_t *)(pool->data() + d.t_off);
        for (size_t k = 0; k < K; k++)
            for (size_t j = 0; j < 8 * W; j++) {
                uint64_t *tab = T + (k * 8 * W + j) * 256 * W;  // [v][W]
                for (size_t v = 1; v < 256; v++) {
                    const size_t b = (size_t)__builtin_ctz((unsigned)v), p = 8 * j + b;
                    const uint64_t *rest = tab + (v & (v - 1)) * W;
                    uint64_t *dst = tab + v * W;
                    for (size_t u = 0; u < W; u++)
                        dst[u] = rest[u] | (p < (size_t)n.m ? n.follow[(k * n.m + p) * W + u] : 0);
                }
            }
    }
    d.ivl_off = align(niv * 4);
    memcpy(pool->data() + d.ivl_off, n.ivl_lo.data(), niv * 4);
    d.b_off = align(niv * W * 8);
    memcpy(pool->data() + d.b_off, n.b.data(), niv * W * 8);
    d.ascii_off = align(128 * 2);
    {
        uint16_t *a = (uint16_t *)(pool->data() + d.ascii_off);
        for (size_t r = 0, iv = 0; r < 128; r++) {
            while (iv + 1 < niv && (size_t)n.ivl_lo[iv + 1] <= r) iv++;
            a[r] = (uint16_t)iv;
        }
    }
    d.acc_off = align(K * W * 8);
    memcpy(pool->data() + d.acc_off, n.acc.data(), K * W * 8);
    memcpy(pool->data() + doff, &d, sizeof d);
    align(16);  // aligned tail: 16-byte reads of the last table stay inside
    return doff;
}

// A pattern past the register NFA (m > kNfaMaxWords * 64 positions) is tried
// as one large DFA first (faster to walk), but the subset construction costs
// about states x positions: its state budget shrinks as the NFA grows, so that
// a pattern whose DFA explodes (.{1000}x.{1000} unanchored) falls through to
// the large NFA in well under a second instead of minutes.
inline int LargeNfaDfaBudget(int m, int cap) { return std::min(cap, std::max(2048, (8 << 20) / std::max(m, 1))); }

// The largest state set (u64 words) among the pool's NFAs (offsets: a
// compiler's pattern -> DevNfa offset map).
template <class Map>
inline uint32_t NfaPoolMaxWords(const std::vector<uint8_t> &pool, const Map &offsets) {
    uint32_t w = 0;
    for (const auto &kv : offsets) w = std::max(w, ((const DevNfa *)(pool.data() + kv.second))->W);
    return w;
}

// An imported tables image (engine/serial.h) is trusted only as far as these
// checks go: every pattern's DevNfa lies inside the pool, 16-byte aligned,
// with its tables inside the pool too; every rule set's image lies inside the
// image bytes.  A well-framed but inconsistent image is refused instead of
// sending the host or the kernels out of bounds.
template <class Map>
inline bool NfaOffsetsValid(const std::vector<uint8_t> &pool, const Map &offsets) {
    const uint64_t size = pool.size();
    auto in = [&](uint64_t off, uint64_t bytes) { return off % 16 == 0 && off <= size && bytes <= size - off; };
    for (const auto &kv : offsets) {
        const uint64_t off = kv.second;
        if (!in(off, sizeof(DevNfa))) return false;
        DevNfa d;
        memcpy(&d, pool.data() + off, sizeof d);
        const uint64_t W = d.W, K = d.K, niv = d.nivl;
        if (W == 0 || W > (1u << 16) || K == 0 || K > 64 || niv > (1u << 24)) return false;
        if (!in(d.ivl_off, niv * 4) || !in(d.b_off, niv * W * 8) || !in(d.acc_off, K * W * 8) ||
            !in(d.ascii_off, 128 * 2) || !in(d.t_off, W > (uint64_t)kNfaMaxWords ? sizeof(DevNfaSparse) : K * 8 * W * 256 * W * 8))
            return false;
        if (W > (uint64_t)kNfaMaxWords) {
            // the sparse rows (nfa_walk.h nfa_big_step): every position's row
            // index, each row's pair range and every pair inside the pool
            const uint64_t m = d.m;
            if (m == 0 || m > W * 64) return false;
            DevNfaSparse sp;
            memcpy(&sp, pool.data() + d.t_off, sizeof sp);
            if (!in(sp.row_of_off, K * m * 4) || !in(sp.row_ptr_off, 4)) return false;
            const uint32_t *row_of = (const uint32_t *)(pool.data() + sp.row_of_off);
            uint64_t rows = 0;
            for (uint64_t i = 0; i < K * m; i++) rows = std::max(rows, (uint64_t)row_of[i] + 1);
            if (!in(sp.row_ptr_off, (rows + 1) * 4)) return false;
            const uint32_t *row_ptr = (const uint32_t *)(pool.data() + sp.row_ptr_off);
            for (uint64_t r = 0; r < rows; r++)
                if (row_ptr[r] > row_ptr[r + 1]) return false;
            const uint64_t pairs = row_ptr[rows];
            if (!in(sp.pair_w_off, pairs * 4) || !in(sp.pair_m_off, pairs * 8)) return false;
            const uint32_t *pair_w = (const uint32_t *)(pool.data() + sp.pair_w_off);
            for (uint64_t q = 0; q < pairs; q++)
                if (pair_w[q] >= W) return false;
        }
    }
    return true;
}
template <class R>
inline bool RulesetImagesValid(const std::vector<R> &rulesets, const std::vector<uint8_t> &images) {
    for (const auto &r : rulesets)
        if ((uint64_t)r.image_off + r.image_len > images.size()) return false;
    return true;
}
// The NFA references a rule-set image holds (header Hdr at the image's
// offset 0: nchunks, nnfa, nfa_off -> DevNfaRef[nnfa]): the reference table
// and each mask row inside the image, each NFA offset one the pool's checked
// map holds (mask rows: HTTP u64[2][nchunks], the others u64[nchunks]).
// Checked after RulesetImagesValid.
template <class Hdr, class R, class Map>
inline bool ImageNfaRefsValid(const std::vector<R> &rulesets, const std::vector<uint8_t> &images, const Map &offsets,
                              uint64_t mask_bytes_per_chunk) {
    for (const auto &r : rulesets) {
        if (r.image_len < sizeof(Hdr)) return false;
        Hdr h;
        memcpy(&h, images.data() + r.image_off, sizeof h);
        const uint64_t nnfa = h.nnfa;
        if (nnfa == 0) continue;
        if ((uint64_t)h.nfa_off + nnfa * sizeof(DevNfaRef) > r.image_len) return false;
        for (uint64_t k = 0; k < nnfa; k++) {
            DevNfaRef ref;
            memcpy(&ref, images.data() + r.image_off + h.nfa_off + k * sizeof(DevNfaRef), sizeof ref);
            if ((uint64_t)ref.mask_off + mask_bytes_per_chunk * h.nchunks > r.image_len) return false;
            bool known = false;
            for (const auto &kv : offsets)
                if ((uint64_t)kv.second == ref.nfa) { known = true; break; }
            if (!known) return false;
        }
    }
    return true;
}

}  // namespace l7
