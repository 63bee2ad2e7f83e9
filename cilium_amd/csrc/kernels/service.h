// The resident service kernels' mailbox loop (product code; the box layout is
// service_types.h, the host side capi.cc Service).  One workgroup polls
// pinned host memory for the synchronous drop-in calls (one Allowed(), one
// OnData), so such a call costs no launch and no completion signal: the host
// writes the call's inputs and a sequence number, the workgroup copies the
// inputs into HBM, classifies them with the same code the launched
// one-workgroup kernels run, writes the answers to pinned memory and stores
// the sequence number to the box's done word.
//
// Every exit is bounded: the workgroup leaves after `idle` cycles without a
// job or when the host sets stop, through a handshake (state EXITING, a
// system-scope fence, req_seq read once more) that cannot lose a job the host
// posted meanwhile -- the host, which writes req_seq and then reads state with
// a fence in between, either sees EXITING / STOPPED and relaunches, or the
// workgroup sees the new req_seq and serves it.
#pragma once
#include <hip/hip_runtime.h>

#include "service_types.h"

namespace l7 {

__device__ __forceinline__ uint32_t svc_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void svc_store(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the box's first 16 bytes, read past every cache (system scope: sc0 sc1)
__device__ __forceinline__ uint4 svc_load_head(const SvcBox *box) {
    uint4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(box) : "memory");
    return v;
}

struct SvcCall {
    uint32_t seq, n, arena_len, flags;
};

// The next job (every thread gets it; seq 0: leave).  Thread 0 polls while
// the others wait at the barrier; word: 4 u32 of LDS the call may use.
__device__ __forceinline__ SvcCall svc_next(SvcBox *box, uint32_t &seen, uint64_t &t_last, uint64_t idle,
                                            uint32_t *word) {
    if (threadIdx.x == 0) {
        uint4 h = make_uint4(0, 0, 0, 0);
        for (;;) {
            h = svc_load_head(box);
            if (h.x != seen) break;
            if (svc_load(&box->stop) || __builtin_amdgcn_s_memtime() - t_last > idle) {
                svc_store(&box->state, kSvcExiting);
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
                h = svc_load_head(box);
                if (h.x != seen) {
                    svc_store(&box->state, kSvcRunning);
                    break;
                }
                h.x = 0;  // leave (the caller stores STOPPED)
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        word[0] = h.x;
        word[1] = h.y;
        word[2] = h.z;
        word[3] = h.w;
    }
    __syncthreads();
    SvcCall c;
    c.seq = (uint32_t)__builtin_amdgcn_readfirstlane((int)word[0]);
    c.n = (uint32_t)__builtin_amdgcn_readfirstlane((int)word[1]);
    c.arena_len = (uint32_t)__builtin_amdgcn_readfirstlane((int)word[2]);
    c.flags = (uint32_t)__builtin_amdgcn_readfirstlane((int)word[3]);
    __syncthreads();  // (thread 0 writes the words again only after every thread read them)
    if (c.seq) {
        seen = c.seq;
        // system-scope acquire in every wave: the call's pinned inputs are read fresh
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    return c;
}

// The call's Batch over the service's staging (layout: service_types.h).
__device__ __forceinline__ Batch svc_batch(const SvcStatic &S, const SvcCall &c) {
    const uint32_t nn = c.n ? c.n : 1;
    const size_t a_off = SvcArenaOff(c.n);
    Batch B;
    B.arena = S.dev_in + a_off;
    B.arena_len = c.arena_len;
    B.offs = (const uint64_t *)S.dev_in;
    B.lens = (const uint32_t *)(S.dev_in + (size_t)nn * 8);
    B.conn_ids = (const uint32_t *)(S.dev_in + (size_t)nn * 12);
    B.conns = S.conns;
    B.nconns = S.nconns;
    B.verdict = S.pin_out;
    B.rule = (int32_t *)(S.pin_out + ((nn + 3) & ~3u));
    B.consumed = (uint32_t *)(S.pin_out + ((nn + 3) & ~3u) + (size_t)nn * 4);
    B.n = c.n;
    return B;
}
// The copy of the call's inputs (pinned -> HBM), and the done word after its answers.
__device__ __forceinline__ CopyIn svc_copy(const SvcStatic &S, SvcBox *box, const SvcCall &c) {
    CopyIn ci{};
    ci.p[0].src = S.pin_in;
    ci.p[0].dst = S.dev_in;
    ci.p[0].bytes = SvcArenaOff(c.n) + c.arena_len;
    ci.n = 1;
    ci.done = &box->done;
    ci.seq = c.seq;
    return ci;
}

}  // namespace l7
