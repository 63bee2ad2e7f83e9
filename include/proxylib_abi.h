/*
 * proxylib_abi.h — the proxylib C-ABI (libcilium.so) exported by libl7gpu.so.
 *
 * Envoy's Cilium Go filter dlopen()s the proxylib shared object and binds five
 * symbols (envoy/cilium_proxylib.cc:14-66); their C types are those cgo emits
 * for proxylib/proxylib.go:57-155 (proxylib/libcilium.h:13-115) and the enums
 * of proxylib/proxylib/types.h:22-50.  This header declares the same ABI so
 * that libl7gpu.so (or a copy named libcilium.so) is a drop-in: the request
 * verdicts of every parser step run on the GPU through l7gpu.h, the op loop,
 * reply bookkeeping and inject buffers stay on the host exactly as in
 * proxylib/proxylib/connection.go:118-174.
 *
 * Registered parsers (the registry of proxylib/proxylib/parserfactory.go:68-71
 * and each parser's init()): "memcache" (proxylib/memcached), "r2d2"
 * (proxylib/r2d2/r2d2parser.go: a denied request is answered "ERROR\r\n"),
 * "cassandra" (proxylib/cassandra/cassandraparser.go: denials answered with
 * the unauthorized error frame 0x2100; the host keeps the parser's keyspace /
 * prepared-statement state), and "http" and "kafka"
 * (the Envoy-filter protocols run through proxylib's policymap semantics:
 * policymap.go:150-236 -- installed entries only, no port entry => drop, SrcId
 * as the remote in both directions).  HTTP: a denied request is DROPped and
 * the 403 of the HTTP filter injected on the reply side; Kafka: a denied
 * request is DROPped and CreateResponse(ErrTopicAuthorizationFailed) injected
 * (pkg/proxy/kafka.go:249-261).  Every complete request frame of one OnData
 * call is decided in ONE device launch.  Any other proto name =>
 * FILTER_UNKNOWN_PARSER.  Policies: the NPDS stream (xds-path) is replaced
 * by l7g_proxylib_policy_update (same cilium.NetworkPolicy shape as JSON).
 */
#ifndef L7G_PROXYLIB_ABI_H
#define L7G_PROXYLIB_ABI_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int64_t GoInt;
typedef struct { const char *p; ptrdiff_t n; } GoString;
typedef struct { void *data; GoInt len; GoInt cap; } GoSlice;

typedef enum {
    FILTEROP_MORE,
    FILTEROP_PASS,
    FILTEROP_DROP,
    FILTEROP_INJECT,
    FILTEROP_ERROR,
} FilterOpType;

typedef enum {
    FILTEROP_ERROR_INVALID_OP_LENGTH = 1,
    FILTEROP_ERROR_INVALID_FRAME_TYPE,
    FILTEROP_ERROR_INVALID_FRAME_LENGTH,
} FilterOpError;

typedef struct {
    uint64_t op;     /* FilterOpType */
    int64_t n_bytes; /* > 0 */
} FilterOp;

typedef enum {
    FILTER_OK,
    FILTER_POLICY_DROP,
    FILTER_PARSER_ERROR,
    FILTER_UNKNOWN_PARSER,
    FILTER_UNKNOWN_CONNECTION,
    FILTER_INVALID_ADDRESS,
    FILTER_INVALID_INSTANCE,
    FILTER_UNKNOWN_ERROR,
} FilterResult;

/* params: GoSlice of [2]GoString (keys access-log-path, xds-path, node-id).
 * Returns the instance id (same parameters => same instance), 0 on error. */
uint64_t OpenModule(GoSlice params, uint8_t debug);
void CloseModule(uint64_t id);
/* orig_buf / reply_buf: caller-owned inject buffers ([]byte headers), kept
 * for the connection's lifetime and appended to within their capacity. */
FilterResult OnNewConnection(uint64_t instance_id, GoString proto, uint64_t connection_id, uint8_t ingress,
                             uint32_t src_id, uint32_t dst_id, GoString src_addr, GoString dst_addr,
                             GoString policy_name, GoSlice *orig_buf, GoSlice *reply_buf);
/* data: GoSlice of []byte (GoSlice) buffers; ops: GoSlice of [2]int64, len
 * grown by the callee up to cap. */
FilterResult OnData(uint64_t connection_id, uint8_t reply, uint8_t end_stream, GoSlice *data, GoSlice *ops);
void Close(uint64_t connection_id);

/* Policy delivery for an instance (replaces the NPDS client): the
 * cilium.NetworkPolicy list as JSON, swapped atomically; 0 = ok, else the
 * previous policies stay in force and err says why (an NPDS NACK). */
int l7g_proxylib_policy_update(uint64_t instance_id, const char *json, size_t len, char *err, size_t errlen);
/* The same from the NPDS wire form (a serialized DiscoveryResponse; see
 * l7g_policy_update_proto in l7gpu.h). */
int l7g_proxylib_policy_update_proto(uint64_t instance_id, const uint8_t *buf, size_t len, char *err, size_t errlen);
/* Number of open connections (all instances). */
uint64_t l7g_proxylib_connections(void);

/* The Kafka deny response for one request frame: what pkg/proxy/kafka.go:
 * 249-261 sends for a denied request -- req.CreateResponse(proto.
 * ErrTopicAuthorizationFailed) (pkg/kafka/request.go:158-182,
 * response.go:81-315) in the request's kind/version encoding.  Host code.
 * Returns 0 (out[0..*outlen) written), -1 (no response: an untyped kind or an
 * undecodable request, request == nil in the reference), -2 (cap too small;
 * *outlen says how much is needed). */
int l7g_kafka_deny_response(const uint8_t *req, size_t len, uint8_t *out, size_t cap, size_t *outlen);

#ifdef __cplusplus
}
#endif
#endif
