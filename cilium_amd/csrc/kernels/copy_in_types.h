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
};

}  // namespace l7
