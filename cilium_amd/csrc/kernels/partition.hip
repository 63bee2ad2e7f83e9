// Protocol split of a mixed batch (product code).
//
// l7g_classify launches one classifier per protocol present in the batch.
// The Kafka and memcached classifiers are one lane per request, so in a mixed
// stream (cfg5) most of their lanes would only discover "not my protocol" and
// idle while the others decode.  This kernel writes, for each of those two
// protocols, the list of request indices that belong to it; the classifiers
// then walk only their own list.  Kafka requests are further grouped by length
// class, so a wave of the one-lane-per-request Kafka kernel holds requests
// that take the same decode path for about as long, and no longer waits on one
// long produce request among short fetches (a wave runs as long as its longest
// lane, and divergent paths run one after the other).  The class comes from
// the request's length, and only where the length cannot tell a fetch from a
// produce from the api key: round 3 read each Kafka request's api key and each
// memcached request's first byte, one HBM line per request, 5 of its 7 GB per
// cfg5 launch; the memcached kernel now splits text from binary itself, from
// bytes it reads anyway.  HTTP entries stay one list, but a block writes its
// HTTP entries length class by length class (round 6), so the HTTP kernel's
// tiles hold requests of about one length (http_class below).  One block owns
// 4096 consecutive requests (8 per lane, protocol kept in registers between
// the count and the write pass) and takes its slot range with one atomic per
// list.
#include <hip/hip_runtime.h>

#include "../device_tables.h"

namespace l7 {

namespace {
// 512 threads x 8 rows: a workgroup's 4096 requests keep stream order in every
// list, so a Kafka wave's 64 entries lie closer together than with 2048
// (cfg5: partition 0.69 -> 0.65 ms and Kafka 16.69 -> 16.49 ms; 16 rows of 256:
// partition 0.79; 1024 threads: 0.97; profiles/r5/ab5h_partition_block.log)
constexpr int kBlock = 512;
constexpr int kPer = 8;  // rows (of kBlock requests) per workgroup
constexpr int kWaves = kBlock / 64;
// list classes: 0..kKafkaClasses-1 Kafka by kind / length, then memcached
// text, memcached binary, other memcached text, then HTTP by length
// (kHttpSub classes, one list).  counts[] keeps one word per list: the Kafka
// classes, memcached retrievals, memcached binary, HTTP, other memcached text.
constexpr int kKafkaClasses = L7_KAFKA_CLASSES;
constexpr int kMcText = kKafkaClasses, kMcBinary = kKafkaClasses + 1;
constexpr int kMcText2 = kKafkaClasses + 2;  // text commands not starting with 'g' (storage, delete, ...)
constexpr int kHttp0 = kKafkaClasses + 3;    // HTTP by length class: kHttp0 .. kHttp0 + kHttpSub - 1
constexpr int kHttpSub = 4;  // (2 classes: cfg5 36.23 ms, 8: 36.25, 4: 36.06-36.16, none: 36.52-36.60)
constexpr int kClasses = kHttp0 + kHttpSub;
constexpr int kCntHttp = kKafkaClasses + 2, kCntMcText2 = kKafkaClasses + 3;  // their counts[] words
__device__ __forceinline__ int count_word(int c) { return c < kMcText2 ? c : c == kMcText2 ? kCntMcText2 : kCntHttp; }

static_assert(kKafkaClasses == 1 || kKafkaClasses == 8, "length classes");
static_assert(kKafkaClasses + 4 <= 26, "counts[26..31] hold the work counters and the compressed-Kafka count");
// HTTP length classes: within a workgroup's 4096 requests the HTTP entries are
// written class by class (stream order within a class), so an HTTP tile of 64
// entries mostly holds requests of about one length, and the kernel's
// value-stop map, which steps as far as the tile's longest request, runs about
// as long as its requests (cfg5: 256..2048-byte requests)
// (cfg5 step, profiles/r6/ab6r_http_length_classes.txt)
__device__ __forceinline__ int http_class(uint32_t len) { return len < 704 ? 0 : len < 1152 ? 1 : len < 1600 ? 2 : 3; }
// Kafka list class: the decode path a lane takes is set by the request kind
// and, for produce, by how many message bytes it hashes.  The length tells the
// kinds apart well enough to schedule by (requests without message sets --
// metadata, offsets, heartbeats -- are tens of bytes, a fetch of a few topics
// and partitions a hundred or two, a produce carries its messages); a request
// in the "wrong" class only shares a wave with a different path: every class
// takes every kind, so this is scheduling, not semantics.
// Lengths in [kKafkaAmbLo, kKafkaAmbHi) are where a fetch of many partitions
// and a produce of one small message overlap: there (only there) the api key
// (bytes 4-5) is read.  kind: that key, 0xFFFF when not read.
constexpr uint32_t kKafkaAmbLo = 147, kKafkaAmbHi = 256;
__device__ __forceinline__ uint8_t kafka_class(uint32_t len, uint32_t kind) {
    if (kKafkaClasses == 1) return 0;
    if (len < 67) return 1;   // no message set
    if (len < kKafkaAmbLo) return 0;  // fetch
    if (len < kKafkaAmbHi && kind != 0) return kind == 1 ? 0 : 1;
    return len < 384 ? 2 : len < 640 ? 3 : len < 896 ? 4 : len < 1280 ? 5 : len < 2048 ? 6 : 7;  // produce
}
}  // namespace

// Lists: Kafka class c at sel_kafka + c * n; memcached text retrievals from
// the start of sel_mc, binary requests from its end (n slots hold both); HTTP
// from the start of sel_http, the other memcached text commands from its end;
// counts[c] entries each (Kafka classes, memcached retrievals, memcached
// binary, HTTP, other memcached text).  Within a
// block's 4096 requests every list keeps stream order, so an HTTP tile of 64
// list entries is, but for the tiles that straddle two blocks, a window of
// the stream (the HTTP kernel's value-stop map streams that window).  Requests no classifier owns (unknown connection index, a
// connection without a parser) are answered here: UNSUPPORTED, rule -1,
// consumed 0, so every request of the batch gets a verdict whichever
// classifiers run (the HTTP kernel is then told not to answer them again).
__global__ __launch_bounds__(kBlock) void partition_kernel(Batch B, uint32_t *__restrict__ sel_kafka,
                                                           uint32_t *__restrict__ sel_mc,
                                                           uint32_t *__restrict__ sel_http,
                                                           uint32_t *__restrict__ counts) {
    const uint32_t n = B.n;
    __shared__ uint32_t s_off[kWaves][kClasses];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t start = (uint64_t)blockIdx.x * (kBlock * kPer);
    const uint64_t below = (1ull << lane) - 1;
    uint8_t p[kPer];  // class + 1, 0 = none
    uint32_t cnt[kClasses] = {};
    // The rows' loads go out phase by phase (connection ids, connections,
    // Kafka lengths, offsets, api keys), so a block waits five memory
    // latencies, not five per row.
    uint32_t ci[kPer], pw[kPer];
#pragma unroll
    for (int r = 0; r < kPer; r++) {
        const uint64_t idx = start + (uint64_t)r * kBlock + threadIdx.x;
        ci[r] = idx < n ? B.conn_ids[idx] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int r = 0; r < kPer; r++) {  // proto | flags << 8 of the connection, PROTO_NONE if unknown
        pw[r] = PROTO_NONE;
        if (ci[r] < B.nconns) {
            const DevConn c = B.conns[ci[r]];
            pw[r] = (uint32_t)c.proto | (uint32_t)c.flags << 8;
        }
    }
    // Kafka: the length; the offset only where the api key is read (the
    // classes are scheduling: the Kafka kernel checks every request's bytes
    // against the arena itself)
    uint32_t len[kPer];
#pragma unroll
    for (int r = 0; r < kPer; r++) {
        const uint64_t idx = start + (uint64_t)r * kBlock + threadIdx.x;
        len[r] = (pw[r] & 0xFF) == PROTO_KAFKA || (pw[r] & 0xFF) == PROTO_HTTP ? B.lens[idx] : 0;
    }
    uint64_t off[kPer];
#pragma unroll
    for (int r = 0; r < kPer; r++) {
        const uint64_t idx = start + (uint64_t)r * kBlock + threadIdx.x;
        off[r] = (pw[r] & 0xFF) == PROTO_KAFKA && len[r] >= kKafkaAmbLo && len[r] < kKafkaAmbHi ? B.offs[idx] : ~0ull;
    }
    uint32_t kd[kPer];  // Kafka api key where the length does not settle the class
#pragma unroll
    for (int r = 0; r < kPer; r++) {
        kd[r] = 0xFFFFu;
        if (off[r] != ~0ull && l7_in_arena(off[r], len[r], B.arena_len))
            kd[r] = (uint32_t)B.arena[off[r] + 4] << 8 | B.arena[off[r] + 5];
    }
#pragma unroll
    for (int r = 0; r < kPer; r++) {
        const uint64_t idx = start + (uint64_t)r * kBlock + threadIdx.x;
        uint8_t cls = 0;
        if (idx < n) {
            const uint32_t proto = pw[r] & 0xFF;
            if (proto == PROTO_KAFKA) {
                cls = 1 + kafka_class(len[r], kd[r]);
            }
            else if (proto == PROTO_MEMCACHE) {
                cls = 1 + kMcText;  // one list: the memcached kernel splits it by parser itself
            }
            else if (proto == PROTO_HTTP) cls = 1 + kHttp0 + http_class(len[r]);
            else if (!L7_PROTO_OWNED(proto)) {  // (r2d2, cassandra: their kernels walk the whole batch)
                B.verdict[idx] = V_UNSUPPORTED;
                B.rule[idx] = -1;
                B.consumed[idx] = 0;
            }
        }
        p[r] = cls;
#pragma unroll
        for (int c = 0; c < kClasses; c++) cnt[c] += __popcll(__ballot(cls == c + 1));
    }
    if (lane == 0)
        for (int c = 0; c < kClasses; c++) s_off[wave][c] = cnt[c];
    __syncthreads();
    if (threadIdx.x < kHttp0) {
        const int c = threadIdx.x;
        uint32_t t = 0;
        for (int w = 0; w < kWaves; w++) t += s_off[w][c];
        uint32_t b = t ? atomicAdd(&counts[count_word(c)], t) : 0;
        for (int w = 0; w < kWaves; w++) {
            const uint32_t a = s_off[w][c];
            s_off[w][c] = b;
            b += a;
        }
    } else if (threadIdx.x == kHttp0) {  // the HTTP classes: one range of the list, class by class
        uint32_t t = 0;
        for (int c = kHttp0; c < kClasses; c++)
            for (int w = 0; w < kWaves; w++) t += s_off[w][c];
        uint32_t b = t ? atomicAdd(&counts[kCntHttp], t) : 0;
        for (int c = kHttp0; c < kClasses; c++)
            for (int w = 0; w < kWaves; w++) {
                const uint32_t a = s_off[w][c];
                s_off[w][c] = b;
                b += a;
            }
    }
    __syncthreads();
    uint32_t lo[kClasses];
#pragma unroll
    for (int c = 0; c < kClasses; c++) lo[c] = s_off[wave][c];
#pragma unroll
    for (int r = 0; r < kPer; r++) {
        const uint32_t idx = (uint32_t)(start + (uint64_t)r * kBlock + threadIdx.x);
#pragma unroll
        for (int c = 0; c < kClasses; c++) {
            const uint64_t mk = __ballot(p[r] == c + 1);
            if (p[r] == c + 1) {
                const uint32_t pos = lo[c] + __popcll(mk & below);
                if (c < kKafkaClasses) sel_kafka[(size_t)c * n + pos] = idx;
                else if (c == kMcText) sel_mc[pos] = idx;
                else if (c == kMcBinary) sel_mc[n - 1 - pos] = idx;  // binary from the list's end
                else if (c == kMcText2) sel_http[n - 1 - pos] = idx;  // other text commands from the HTTP list's end
                else sel_http[pos] = idx;
            }
            lo[c] += __popcll(mk);
        }
    }
}

// counts[0..kKafkaClasses + 4) must be zero on entry (the caller clears them on `stream`).
hipError_t LaunchPartition(const Batch &B, uint32_t *sel_kafka, uint32_t *sel_mc, uint32_t *sel_http, uint32_t *counts,
                           hipStream_t stream) {
    if (B.n == 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)(((uint64_t)B.n + kBlock * kPer - 1) / (kBlock * kPer));
    hipLaunchKernelGGL(partition_kernel, dim3(blocks), dim3(kBlock), 0, stream, B, sel_kafka, sel_mc, sel_http, counts);
    return hipGetLastError();
}

}  // namespace l7
