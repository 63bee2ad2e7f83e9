// Library-internal entry points shared by the C-ABI (capi.cc) and the
// proxylib shim (proxylib/shim.cc); not part of include/l7gpu.h.
#pragma once
#include <cstddef>
#include <cstdint>

struct l7g_engine;

// One policy version, JSON (proto_form 0) or an NPDS DiscoveryResponse
// (proto_form 1).  proxylib != 0: the proxylib instance's update, which also
// NACKs what only proxylib's policymap rejects -- mismatching L7 types on one
// port (proxylib/proxylib/policymap.go:135-143, recovered as an update error
// in instance.go:168-176); the previous version then stays in force.
int l7g_policy_update_view(l7g_engine *e, const uint8_t *buf, size_t len, int proto_form, int proxylib, char *err,
                           size_t errlen);

// l7g_classify_host in two steps (the batcher's flushers, csrc/batcher.cc):
// l7g_host_stage returns the calling thread's pinned staging for a call of n
// requests over arena_len bytes (grown as needed; valid until the thread's
// next stage); the caller fills it in place, then l7g_host_run classifies it
// exactly as l7g_classify_host would and waits.  0 = ok, else a hipError_t.
int l7g_host_stage(l7g_engine *e, uint32_t n, uint64_t arena_len, uint8_t **arena, uint64_t **off, uint32_t **len,
                   uint32_t **conn);
int l7g_host_run(l7g_engine *e, uint32_t n, uint64_t arena_len, uint8_t *verdict, int32_t *rule, uint32_t *consumed);
// The same with inputs already in pinned host memory (hipHostMalloc: a
// batcher slot filled in place by its submitters): off[0..n), then len and
// conn `stride` entries further on (len = (u8 *)off + stride * 8, conn =
// (u8 *)off + stride * 12; stride >= n), and the request bytes as nseg
// blocks that the device sees concatenated (off[] indexes the concatenation);
// a block is `rows` rows of `width` bytes, `pitch` bytes apart in host memory
// (one 2-D copy).  Copied to the device (or, one single-row block and a small
// call, read in place), classified, waited for.
struct l7g_host_seg {
    const uint8_t *p;
    uint64_t width, pitch;
    uint32_t rows;
};
int l7g_host_run_pinned(l7g_engine *e, uint32_t n, const uint64_t *off, size_t stride, const l7g_host_seg *seg,
                        int nseg, uint8_t *verdict, int32_t *rule, uint32_t *consumed);
// Sizes the calling thread's stream and staging for calls of up to n requests
// over arena_len bytes now, so that no such call reallocates them.
int l7g_host_reserve(l7g_engine *e, uint32_t n, uint64_t arena_len);
void *l7g_pinned_alloc(size_t bytes);  // hipHostMalloc (NULL on failure)
int l7g_engine_has_device(const l7g_engine *e);  // 1: the engine launches on a GPU; 0: host-only (tables only)
void l7g_pinned_free(void *p);
