// The resident service kernels' mailbox (product code; capi.cc Service,
// kernels http_service_kernel / memcache_service_kernel): a synchronous
// drop-in call (one Allowed(), one OnData) is posted here instead of being
// launched.  Plain types: the host side includes this too.  The box lives in
// pinned, coherent host memory; the host writes a job and then req_seq, the
// kernel (one workgroup, polling) serves it and stores the job's CopyIn.seq to
// its done word, as the launched one-workgroup kernel does.
#pragma once
#include <stdint.h>

#include "../device_tables.h"
#include "copy_in_types.h"

namespace l7 {

enum : uint32_t { kSvcStopped = 0, kSvcRunning = 1, kSvcExiting = 2 };

// The service's own staging (allocated with it; kernel arguments for its
// lifetime): a call's inputs in the layout of l7g_classify_host's staging --
// [off u64[nn] | len u32[nn] | conn u32[nn] | arena at a_off], nn = max(n, 1),
// a_off = (16 nn + 255) & ~255 -- in pinned memory, copied by the kernel into
// dev_in; its answers [verdict u8[(nn + 3) & ~3] | rule i32[nn] | consumed
// u32[nn]] written to pinned memory in place.  conns / tables: the engine's
// as they were when the kernel was launched (a policy or connection update
// stops the service first).
struct SvcStatic {
    const uint8_t *pin_in;  // device view of the pinned inputs
    uint8_t *dev_in;
    uint8_t *pin_out;       // device view of the pinned outputs
    const DevConn *conns;
    uint32_t nconns;
    uint32_t pad;
};

// flags of a job
enum : uint32_t {
    kSvcHttpHot = 1,      // HTTP: the hot rule set's pass (image staged once, in LDS)
    kSvcHttpGeneral = 2,  // HTTP: the general pass (other rule sets' images through L2)
    kSvcAnswerOther = 4,  // answer entries no parser owns (UNSUPPORTED)
};

struct SvcBox {
    // one 16-byte read per poll brings a new req_seq with its job's words (the
    // host writes them first; a read of one line returns them as of one moment)
    uint32_t req_seq;    // host: the last job posted (served when it differs from the last one seen)
    uint32_t n, arena_len, flags;  // host: the job
    uint32_t stop;       // host: exit at the next poll (a throughput launch wants every CU; an update)
    uint32_t state;      // kernel: kSvcRunning / kSvcExiting / kSvcStopped
    uint32_t done;       // kernel: req_seq of the last job answered (after its answers)
    uint32_t pad[9];
};
static_assert(sizeof(SvcBox) == 64, "one line");

L7_HD constexpr inline size_t SvcArenaOff(uint32_t n) { return ((size_t)(n ? n : 1) * 16 + 255) & ~(size_t)255; }

}  // namespace l7
