/*
 * l7gpu.h — C-ABI of the MI355X-native batched L7 policy classifier.
 *
 * This is the drop-in boundary for the reference's L7 verdict path.  Every
 * entry point is plain C (pointers + sizes, no C++/torch types) so a Go cgo
 * package, Envoy's dlopen loader, or ctypes can bind it.  What each entry
 * replaces in the reference (file:line):
 *
 *   l7g_policy_update   proxylib Instance.PolicyUpdate            proxylib/proxylib/instance.go:168-219
 *                       Envoy NetworkPolicyMap::onConfigUpdate     envoy/cilium_network_policy.h:240-250
 *                       (policies in the cilium.NetworkPolicy shape, envoy/cilium/npds.proto:31-182,
 *                        as JSON; see DESIGN.md §Policy JSON)
 *   l7g_policy_index    NetworkPolicyMap::GetPolicyInstance        envoy/cilium_network_policy.h:213-221
 *   l7g_conns_set,      proxylib OnNewConnection / Close           proxylib/proxylib.go:57-74,112-116
 *   l7g_conn_update
 *                       Cilium::SocketOption (identity, port, dir) envoy/cilium_l7policy.cc:133-150
 *   l7g_classify        per request: AccessFilter::decodeHeaders -> NetworkPolicyMap::Allowed
 *                                                                  envoy/cilium_l7policy.cc:127-182,
 *                                                                  envoy/cilium_network_policy.h:223-237
 *                       kafka.ReadRequest + canAccess/MatchesRule  pkg/kafka/request.go:186-229,
 *                                                                  pkg/proxy/kafka.go:117-153,
 *                                                                  pkg/kafka/policy.go:200-225
 *                       proxylib OnData (memcache parser) -> Connection.Matches
 *                                                                  proxylib/proxylib.go:97-110,
 *                                                                  proxylib/memcached/parser.go:186-202,
 *                                                                  proxylib/proxylib/policymap.go:210-236
 *   l7g_frame_streams   the parsers' framing of a connection's input: proto.ReadReq's size prefix
 *                                                                  vendor/github.com/optiopay/kafka/proto/messages.go:124-165,
 *                       memcached text line / binary header        proxylib/memcached/text/parser.go:72-262,
 *                                                                  proxylib/memcached/binary/parser.go:72-139
 *   counters argument   Endpoint.UpdateProxyStatistics counters    pkg/endpoint/endpoint.go:2207-2233
 *   of l7g_classify     (per-rule allow hits + per-verdict totals, accumulated on the device)
 *
 * Verdict codes match the oracle (oracle/l7ref.h) and DESIGN.md.
 */
#ifndef L7GPU_H
#define L7GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct l7g_engine l7g_engine;

enum { L7G_PROTO_HTTP = 1, L7G_PROTO_KAFKA = 2, L7G_PROTO_MEMCACHE = 3, L7G_PROTO_R2D2 = 4, L7G_PROTO_CASSANDRA = 5 };
/* L7G_PROTO_CASSANDRA keeps no state between l7g_classify calls: a request's
 * keyspace comes only from the last USE on its connection earlier in the same
 * batch (a USE from an earlier batch is not remembered, so "t" stays ".t"
 * rather than "ks.t"), and an EXECUTE is never resolved to its prepared query
 * (answered L7G_PARSE_ERROR, consumed 2).  The proxylib shim keeps both per
 * connection (USE keyspace, PREPARE ids) and replays them into each batch, as
 * cassandraparser.go does; a direct caller that needs the reference's
 * cross-batch behaviour must do the same. */
enum {
    L7G_DENY = 0,        /* policy denies (HTTP 403 / Kafka ErrTopicAuthorizationFailed) */
    L7G_ALLOW = 1,       /* policy allows; rule = matched global rule id or -1 */
    L7G_PARSE_ERROR = 2, /* malformed request (connection is closed by the caller) */
    L7G_INCOMPLETE = 3,  /* more bytes are needed (proxylib MORE) */
    L7G_UNSUPPORTED = 4, /* no parser for the connection, a request outside the arena, a nested compressed
                            Kafka set beyond the decode space (kafka_inflate.hip) */
};

/* memcached: proxylib picks the text or binary parser from the first byte a
 * connection carries and keeps it (proxylib/memcached/parser.go:186-202).
 * L7G_CONN_PROXYLIB: an HTTP or Kafka connection served by the proxylib
 * "http" / "kafka" parser: proxylib's policymap semantics apply (no port entry
 * => DENY, SrcId is the remote in both directions; policymap.go:208-236,
 * connection.go:176-179) instead of Envoy's / the in-agent Kafka proxy's. */
enum { L7G_CONN_MC_TEXT = 1, L7G_CONN_MC_BINARY = 2, L7G_CONN_PROXYLIB = 4 };

/* Connection attributes (20 bytes; identical layout to the oracle's ref_conn_t). */
typedef struct {
    int32_t policy;   /* l7g_policy_index(name), -1 = no policy for this endpoint (deny) */
    uint32_t port;    /* destination port */
    uint8_t ingress;  /* 1 = ingress */
    uint8_t proto;    /* L7G_PROTO_* */
    uint16_t flags;   /* L7G_CONN_MC_*: memcached parser chosen for the connection (0 = by first byte) */
    uint32_t src_id;  /* source security identity */
    uint32_t dst_id;  /* destination security identity */
} l7g_conn_t;

typedef struct {
    uint32_t policies, rules, http_rulesets, http_chunks, http_dfas, http_dfa_states;
    uint32_t kafka_rulesets, kafka_rules, kafka_topics;
    uint64_t table_bytes;       /* device table blob (0 until first upload) */
    uint64_t http_image_bytes;  /* all HTTP rule-set images */
    int32_t hot_ruleset;        /* HTTP rule set staged in LDS, -1 none */
    uint32_t hot_image_bytes;
    uint32_t mc_rulesets, mc_rules, mc_dfas, mc_dfa_states;
    uint32_t http_nfas;         /* distinct patterns on the bit-parallel NFA fallback */
    uint32_t mc_nfas;
    uint64_t nfa_pool_bytes;    /* their device tables */
    uint32_t r2d2_rulesets, r2d2_rules;
} l7g_stats_t;

/* Engine bound to one HIP device.  err receives a message on failure.
 * device == L7G_HOST_ONLY creates a compile-only engine (policy validation and
 * rule-table statistics; classification returns hipErrorNoDevice). */
#define L7G_HOST_ONLY (-1)
l7g_engine *l7g_engine_create(int device, char *err, size_t errlen);
void l7g_engine_destroy(l7g_engine *e);

/* Atomically replaces the policy set (0 = ok).  On error the previous policy
 * set stays in force (like an NPDS NACK).  Existing connections are re-resolved. */
int l7g_policy_update(l7g_engine *e, const char *json, size_t len, char *err, size_t errlen);
/* The same policy delivery as the NPDS stream carries it: buf is a serialized
 * envoy.api.v2.DiscoveryResponse whose resources are google.protobuf.Any of
 * type.googleapis.com/cilium.NetworkPolicy (envoy/cilium/npds.proto:31-182),
 * decoded by the library's own proto3 wire-format reader.  Same atomic swap and
 * NACK as l7g_policy_update; a response the JSON path would express the same
 * way compiles to identical tables. */
int l7g_policy_update_proto(l7g_engine *e, const uint8_t *buf, size_t len, char *err, size_t errlen);
int32_t l7g_policy_index(l7g_engine *e, const char *name, size_t len);
int32_t l7g_policy_nrules(l7g_engine *e);

/* Compiled tables across GPUs (the NPDS receiver is rank 0,
 * proxylib/proxylib/instance.go:168-219): one rank compiles, the others install.
 * l7g_tables_export writes the current policy version -- its source bytes and
 * every compiler's rule sets (device images plus the rule-list -> rule-set
 * cache) -- into buf; *len = the bytes needed.  Returns 0, or -2 when buf is
 * NULL or cap is too small (only *len is set).  l7g_tables_import installs such
 * an image: the policy is parsed, not compiled, and the connections are
 * re-resolved against the imported rule sets (one the exporter did not compile
 * is compiled here).  Same atomic swap / NACK as l7g_policy_update. */
int l7g_tables_export(l7g_engine *e, uint8_t *buf, size_t cap, size_t *len);
int l7g_tables_import(l7g_engine *e, const uint8_t *buf, size_t len, char *err, size_t errlen);
/* Rule sets this engine compiled itself since its policy version was installed
 * (0 on a rank that imported every rule set it uses). */
uint64_t l7g_tables_compiled(l7g_engine *e);
/* FNV-1a 64 of the device table blob the engine installs (equal digests <=>
 * byte-identical tables). */
uint64_t l7g_tables_digest(l7g_engine *e);

/* Replaces the connection table (connection i = conns[i]); compiles the rule
 * sets the connections need.  0 = ok. */
int l7g_conns_set(l7g_engine *e, const l7g_conn_t *conns, uint32_t n, char *err, size_t errlen);

/* Sets (or adds, growing the table) connection `index` alone; rule sets are
 * compiled on first use.  The proxylib shim calls it from OnNewConnection /
 * Close and when a memcached connection's parser is chosen.  0 = ok. */
int l7g_conn_update(l7g_engine *e, uint32_t index, const l7g_conn_t *conn, char *err, size_t errlen);

/* Classifies n requests resident in device memory: request i is
 * arena[off[i] .. off[i]+len[i]) on connection conn[i], inside
 * [arena, arena + arena_len) (an HTTP request reaching past it is answered
 * UNSUPPORTED).  The arena must stay readable up to the next 16-byte boundary
 * past its last byte (true of every hipMalloc / torch allocation); the kernels
 * read aligned 16-byte words.  Writes verdict[i],
 * rule[i] (global rule id, -1 = none) and consumed[i]: for ALLOW/DENY the
 * bytes of the first request (proxylib's PASS/DROP length, which may exceed
 * len[i] for memcached data blocks); for memcached INCOMPLETE the proxylib
 * MORE byte count (0 = NOP) and for memcached PARSE_ERROR the OpError code
 * (2 = INVALID_FRAME_TYPE; 0 = parser error); 0 otherwise.  Asynchronous on `stream`
 * (a hipStream_t, NULL = default stream).  counters may be NULL, else a
 * device array of (rules + 8) uint64 that accumulates per-rule allow hits
 * followed by per-verdict totals (added atomically, so calls on different
 * streams may share one array).  Batches with Kafka requests or with more
 * than one protocol use a scratch of 32 + (L7_KAFKA_CLASSES + 3) n uint32 (the
 * partition lists and work counters; 32 + 11 n with 8 classes), HTTP-only
 * batches of 2^18 or more requests 4 words (tile counters); scratch is kept per stream (up to
 * 16 streams, then handed over least recently used first), so calls on
 * different streams run concurrently and calls on one stream are ordered by
 * it.  With Kafka rules the engine also holds ONE 1 GiB decode region for
 * compressed message sets, allocated with the first Kafka batch and shared by
 * all streams: the decode kernels of calls on different streams run one after
 * the other (each waits for the previous one's completion event).  Returns 0
 * or a HIP error code. */
int l7g_classify(l7g_engine *e, const uint8_t *arena, uint64_t arena_len, const uint64_t *off, const uint32_t *len,
                 const uint32_t *conn, uint32_t n, uint8_t *verdict, int32_t *rule, uint32_t *consumed,
                 uint64_t *counters, void *stream);

/* Device framing of connection streams (replaces the host scan that proposes
 * where a connection's frames start: Kafka's BE int32 size prefix,
 * proto.ReadReq vendor/github.com/optiopay/kafka/proto/messages.go:124-165;
 * memcached text lines + storage data blocks and binary 24-byte header + body,
 * proxylib/memcached/{text,binary}/parser.go; HTTP/1 head + Content-Length;
 * r2d2 lines; cassandra 9-byte header + body).  Stream s is arena[s_off[s],
 * s_off[s] + s_len[s]) on connection s_conn[s] (a memcached connection without
 * a chosen parser takes the one the stream's first byte picks).  One device
 * lane walks each stream; output slots [s * max_frames, (s + 1) * max_frames):
 * frame k of stream s starts at frame_off (an arena offset) and is handed
 * frame_len = the bytes from there to the stream's end, as proxylib hands a
 * parser the joined input; frame_conn = s_conn[s]; nframes[s] frames.  The
 * walk stops at a frame whose end is not in the stream or cannot be known
 * before parsing it (a chunked HTTP body, an unreadable size): that frame is
 * the last, with the rest of the stream, and the classifier's consumed length
 * says where the next one starts.  Empty slots: length 0, connection ~0.  All
 * pointers are device memory; asynchronous on `stream`.  0 or a hipError_t. */
int l7g_frame_streams(l7g_engine *e, const uint8_t *arena, uint64_t arena_len, const uint64_t *s_off,
                      const uint32_t *s_len, const uint32_t *s_conn, uint32_t n, uint32_t max_frames,
                      uint64_t *frame_off, uint32_t *frame_len, uint32_t *frame_conn, uint32_t *nframes, void *stream);
/* l7g_frame_streams, then l7g_classify over all n * max_frames slots (the
 * empty ones answer L7G_UNSUPPORTED): a batch of connection streams in, one
 * verdict per frame out, with no host pass over the bytes.  A frame is
 * confirmed when its consumed length equals the distance to the next frame
 * (or, for the last, when the caller accepts a partial one). */
int l7g_classify_streams(l7g_engine *e, const uint8_t *arena, uint64_t arena_len, const uint64_t *s_off,
                         const uint32_t *s_len, const uint32_t *s_conn, uint32_t n, uint32_t max_frames,
                         uint64_t *frame_off, uint32_t *frame_len, uint32_t *frame_conn, uint32_t *nframes,
                         uint8_t *verdict, int32_t *rule, uint32_t *consumed, uint64_t *counters, void *stream);

/* Same with host buffers: copies in, classifies, copies out, synchronises.
 * Each calling thread gets its own stream and device staging, so calls from
 * several threads overlap (the engine lock covers only the enqueue). */
int l7g_classify_host(l7g_engine *e, const uint8_t *arena, uint64_t arena_len, const uint64_t *off,
                      const uint32_t *len, const uint32_t *conn, uint32_t n, uint8_t *verdict, int32_t *rule,
                      uint32_t *consumed);

int l7g_stats(l7g_engine *e, l7g_stats_t *out);

/* Resident services: the synchronous drop-in calls of l7g_classify_host (and
 * so the Envoy adapter's Allowed() and proxylib's OnData) whose requests are
 * all HTTP (at most 8) or all memcached (at most 64) are posted to one polling
 * workgroup per protocol instead of launched: no launch and no completion
 * signal per call.  A service starts with the first such call, stays while
 * calls keep coming and leaves after ~50 ms without one, when a batch of
 * 4096 or more requests wants every CU, or before a policy or connection
 * update.  Answers are those of the launched path (the same device code); a
 * kernel fault is reported by the call that was waiting.  On by default
 * (L7G_SERVICE=0 at engine creation turns it off).  Returns the previous
 * setting. */
int l7g_service_enable(l7g_engine *e, int on);
/* [0] HTTP calls served, [1] HTTP workgroup launches, [2] memcached calls,
 * [3] memcached launches. */
void l7g_service_stats(l7g_engine *e, uint64_t out[4]);

/* Asynchronous batching for callers that decide one request at a time on an
 * event loop -- Envoy's cilium.l7policy decodeHeaders
 * (envoy/cilium_l7policy.cc:127-182), which would return StopIteration and
 * resume (continueDecoding / sendLocalReply) from the callback.  Submitters
 * copy their request straight into the open batch slot (pinned host memory in
 * the layout the device copy reads; a fetch-and-add on one of the slot's eight
 * lane words reserves the place, no lock).  Two flusher threads each seal the open slot once max_requests are in
 * it, its first request has waited max_wait_us, or a flush is asked for
 * (under load a batch can hold up to twice max_requests: requests keep coming
 * while the slot is sealed), classify it in place with one launch on their own
 * stream (so one batch is on the device while the next fills), and call each
 * request's callback from the flusher thread -- batches in the order they
 * were sealed, a thread's requests in submission order.  A device failure
 * answers every request of that batch L7G_UNSUPPORTED.  A callback must not
 * call l7g_batcher_flush or l7g_batcher_destroy (from a flusher thread both
 * return at once, doing nothing). */
typedef void (*l7g_done_fn)(void *ctx, uint8_t verdict, int32_t rule, uint32_t consumed);
typedef struct l7g_batcher l7g_batcher;
/* Slots hold max(2 x max_requests, 1024) requests and 2 KiB of request bytes
 * per request each; four slots are allocated (pinned) up front.  max_requests
 * is capped at 65536 (4 x 256 MiB pinned).  NULL when the engine has a device
 * and the slots cannot be pinned (the device path needs pinned slots). */
l7g_batcher *l7g_batcher_create(l7g_engine *e, uint32_t max_requests, uint32_t max_wait_us);
/* The batch size the batcher flushes at: max_requests as created, or 65536
 * when create capped it (a caller that asked for more learns it here). */
uint32_t l7g_batcher_max_requests(const l7g_batcher *b);
/* 0 = queued; -1 = the batcher is shutting down; -2 = backpressure: both
 * flushers are busy and the open slot is full, or the request is larger than
 * one of a slot's eight lanes (max(2 x max_requests, 1024) x 256 bytes) (the
 * callback is not called; the caller decides the request itself or retries). */
int l7g_batcher_submit(l7g_batcher *b, const uint8_t *req, uint32_t len, uint32_t conn, l7g_done_fn done, void *ctx);
/* Flushes now and returns once every request submitted before the call has
 * had its callback (0); -1 when called from a callback. */
int l7g_batcher_flush(l7g_batcher *b);
/* Flushes what is pending, then stops the flusher threads. */
void l7g_batcher_destroy(l7g_batcher *b);
/* Requests classified and launches made so far (for latency accounting). */
void l7g_batcher_stats(l7g_batcher *b, uint64_t *requests, uint64_t *launches);
/* Where the flusher threads' time went, summed over both, in ns: [0] waiting
 * for a sealed slot's entries to be published, [1] the device round trip (copy, launch, wait),
 * [2] callbacks, [3] waiting for the previous batch's callbacks (ordering);
 * [4] the largest batch. */
void l7g_batcher_timing(l7g_batcher *b, uint64_t out[5]);

/* Measurement hook (bench.py): with profiling on, l7g_classify records HIP
 * events on its stream around each kernel it launches; l7g_profile_last waits
 * for the last call and returns the device time in ms of its four stages
 * (partition, HTTP, Kafka, memcached; 0 = not launched).  Off by default. */
int l7g_profile_enable(l7g_engine *e, int on);

/* Proxy statistics (pkg/endpoint/endpoint.go:2207-2233 UpdateProxyStatistics,
 * the policy_l7_received/forwarded/denied/parse_errors_total counters of
 * pkg/metrics/metrics.go:269-296): while enabled, every l7g_classify adds, per
 * (policy, protocol, port, direction) of its connections, the requests that
 * completed a flow -- ALLOW = forwarded, DENY = denied, PARSE_ERROR = error,
 * each also received -- into a device accumulator.  l7g_flow_stats copies the
 * non-zero entries out (at most cap; *n = how many there are) and, with reset,
 * zeroes the accumulator.  Off by default. */
typedef struct {
    int32_t policy;
    uint8_t proto;     /* L7G_PROTO_* */
    uint8_t ingress;
    uint16_t port;
    uint64_t received, forwarded, denied, error;
} l7g_flow_stat_t;
int l7g_flow_stats_enable(l7g_engine *e, int on);
int l7g_flow_stats(l7g_engine *e, l7g_flow_stat_t *out, uint32_t cap, uint32_t *n, int reset);
int l7g_profile_last(l7g_engine *e, float out_ms[4]);

/* Profiling hook: per-phase cycle totals of the HTTP kernels, 16 slots (0
 * window DMA, 1 parse, 2 long-value scan, 3 other, 4 rounds, 5 scanned values,
 * 6 tiles, 7 rule-set image staging; latency kernel: 8 request fetch, 9 CR
 * scan, 10 lines framed, 11 merge + end of the header block, 12 requests),
 * summed over waves since the last reset.  Only a timing build
 * (-DL7G_PHASE_TIMING) records them; the product build returns
 * hipErrorNotSupported. */
int l7g_debug_phase_times(l7g_engine *e, uint64_t *out16, int reset);
/* The same for the Kafka kernel (-DL7G_KX_TIMING builds; slots: 0 framing,
 * 1 walk, 2 CRC pass, 3 topic lookups, 4 verdict + output, 5 walk rounds,
 * 6 window refills, 7 tiles). */
int l7g_debug_kafka_phase_times(l7g_engine *e, uint64_t *out8, int reset);
/* Per-phase cycle totals of the text-stream framer (-DL7G_FRAME_PHASES builds only; else an error). */
int l7g_debug_frame_phase_times(l7g_engine *e, uint64_t *out8, int reset);

/* Kafka correlation-ID rewriting of the in-agent Kafka proxy's forwarding
 * path (pkg/kafka/correlation_cache.go:97-213; one cache per client
 * connection, pkg/proxy/kafka.go:335).  Host code.
 *   l7g_kafka_corr_requests: HandleRequest for a batch of forwarded (allowed)
 *     request frames, in order: each frame's correlation id (bytes 8..12) is
 *     replaced in place by the cache's next sequence number (from 1), written
 *     to new_ids (may be null), and the original remembered.
 *   l7g_kafka_corr_responses: CorrelateResponse for a batch of broker
 *     response frames: a known id (bytes 4..8) is replaced in place by the
 *     original and forgotten; found[i] = 1 then, else 0 (frame untouched).
 *   l7g_kafka_corr_gc: drop entries at least lifetime_ms old (the reference
 *     runs this every RequestLifetime = 5 min); returns how many. */
typedef struct l7g_kafka_corr l7g_kafka_corr;
l7g_kafka_corr *l7g_kafka_corr_create(void);
void l7g_kafka_corr_destroy(l7g_kafka_corr *c);
int l7g_kafka_corr_requests(l7g_kafka_corr *c, uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t n,
                            uint32_t *new_ids);
int l7g_kafka_corr_responses(l7g_kafka_corr *c, uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t n,
                             uint8_t *found);
uint64_t l7g_kafka_corr_gc(l7g_kafka_corr *c, uint64_t lifetime_ms);
uint64_t l7g_kafka_corr_size(l7g_kafka_corr *c);

/* Test hook: compile one Go regexp with the product's DFA compiler and run
 * the compiled tables on the host.  Returns 1 match, 0 no match, -1 compile
 * error (err set).  anchored: 1 = full match, 0 = Go regexp.Match. */
int l7g_debug_regex(const char *pat, size_t patlen, int anchored, const uint8_t *s, size_t slen, char *err,
                    size_t errlen);
/* The same through the bit-parallel NFA fallback (the DevNfa tables and the
 * walk the device pre-pass runs); -1 also when the pattern needs more than
 * 1024 NFA positions. */
int l7g_debug_regex_nfa(const char *pat, size_t patlen, int anchored, const uint8_t *s, size_t slen, char *err,
                        size_t errlen);

#ifdef __cplusplus
}
#endif
#endif
