// Global-memory loads from integer addresses (product code).  A load through
// a pointer made from an integer, or one that may point to LDS, compiles to a
// flat load; flat loads count against lgkmcnt as well as vmcnt, so every wait
// for an LDS read (DFA tables, CRC tables, staged windows) would also wait for
// them.  These helpers name the global address space explicitly.
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>

namespace l7 {

typedef uint32_t gm_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 gload16(uint64_t a) {
    const gm_u32x4 v = *(const __attribute__((address_space(1))) gm_u32x4 *)a;
    return make_uint4(v.x, v.y, v.z, v.w);
}

}  // namespace l7
