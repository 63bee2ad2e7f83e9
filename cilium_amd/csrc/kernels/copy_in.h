// The copy of a small call's inputs done by the call's first kernel when that
// kernel is a single workgroup (a one-request Allowed(), one OnData): every
// thread's loads before its stores, then a fence and a barrier, so the
// workgroup's waves read the copy -- one launch fewer than copy_in_kernel.
#pragma once
#include <hip/hip_runtime.h>

#include "copy_in_types.h"
#include "gmem.h"

namespace l7 {

__device__ __forceinline__ void copy_in_block(const CopyIn &c) {
    if (c.n == 0) return;
    constexpr int kPer = 4;
#pragma unroll
    for (int k = 0; k < 4; k++) {  // (unrolled: an indexed kernel argument would live in scratch)
        if (k >= c.n) break;
        const uint64_t units = (c.p[k].bytes + 15) / 16;
        const uint4 *s = reinterpret_cast<const uint4 *>(c.p[k].src);
        uint4 *d = reinterpret_cast<uint4 *>(c.p[k].dst);
        for (uint64_t u0 = 0; u0 < units; u0 += (uint64_t)blockDim.x * kPer) {
            uint4 v[kPer];
#pragma unroll
            for (int j = 0; j < kPer; j++) {
                const uint64_t u = u0 + (uint64_t)j * blockDim.x + threadIdx.x;
                if (u < units) v[j] = gload16((uint64_t)(uintptr_t)(s + u));
            }
#pragma unroll
            for (int j = 0; j < kPer; j++) {
                const uint64_t u = u0 + (uint64_t)j * blockDim.x + threadIdx.x;
                if (u < units) d[u] = v[j];
            }
        }
    }
    __threadfence();
    __syncthreads();
}

// The call's last kernel, one workgroup: every output stored, then seq to
// the host's done word (system scope, vector store); all threads call it.
__device__ __forceinline__ void signal_done_block(const CopyIn &c) {
    if (c.done == nullptr) return;
    // every thread fences its own stores (answers in pinned host memory on the
    // zero-copy path) at system scope before the barrier, so all waves'
    // answers are visible to the host before thread 0's release of the word
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(c.done, c.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace l7
