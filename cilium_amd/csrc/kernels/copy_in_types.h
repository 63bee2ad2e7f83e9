// A small call's input pieces, copied from pinned host memory into HBM before
// the classifiers read them (capi.cc HostRun; kernels/copy_in.hip, or the
// first kernel of the call when it runs as one workgroup).  Plain types: the
// host side includes this too.
#pragma once
#include <stdint.h>

namespace l7 {

struct CopyPiece {
    const uint8_t *src;  // 16-byte aligned, readable to the next multiple of 16
    uint8_t *dst;        // 16-byte aligned
    uint64_t bytes;
};
struct CopyIn {
    CopyPiece p[4];
    int n;  // pieces (0: nothing to copy)
    // with done: the kernel that ends the call (one workgroup) stores seq there
    // (pinned host memory) after its outputs, and the host waits on that word
    // instead of on the stream
    uint32_t *done;
    uint32_t seq;
};

}  // namespace l7
