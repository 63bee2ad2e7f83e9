/*
 * l7ref — CPU restatement of the reference's L7 verdict path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker (or the timed CPU baseline), never as the product path.
 * The product (cilium_amd/libl7gpu.so) never links or calls anything here.
 *
 * Pinned against the reference's own known-answer tests, see
 * tests/golden/ and tests/test_oracle_*.py:
 *   - Go regexp:   pkg/policy/api/rule_validation_test.go:155-205,
 *                  proxylib/proxylib_memcached_test.go:626-640,
 *                  proxylib/r2d2/r2d2parser_test.go:150-178
 *   - HTTP policy: envoy/cilium_integration_test.cc:165-199,738-856
 *   - Kafka:       pkg/kafka/policy_test.go:52-127, pkg/proxy/kafka_test.go:167-265
 */
#ifndef L7REF_H
#define L7REF_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- Go regexp (regexp/syntax + regexp, Go 1.10.3) ------------- */
typedef struct ref_re ref_re;
/* Compile `pat` with Go's syntax.Perl flags.  On error returns NULL and writes
 * Go's error text ("error parsing regexp: <code>: `<expr>`") into err. */
ref_re *ref_re_compile(const char *pat, size_t patlen, char *err, size_t errlen);
void ref_re_free(ref_re *re);
/* anchored != 0: full match, i.e. regexp.MustCompile("^(?:"+p+")$").Match(s).
 * anchored == 0: Go regexp.Match(s) (match anywhere). */
int ref_re_match(const ref_re *re, const uint8_t *s, size_t n, int anchored);

/* ---------------- policies (JSON, NPDS NetworkPolicy shape) ----------------- */
typedef struct ref_policy ref_policy;
ref_policy *ref_policy_load(const char *json, size_t len, char *err, size_t errlen);
void ref_policy_free(ref_policy *p);

/* Connection attributes, as passed to proxylib OnNewConnection
 * (proxylib/proxylib.go:57-74) / Envoy SocketOption (envoy/cilium_l7policy.cc:133-150). */
/* memcached parser selection (proxylib/memcached/parser.go:186-202): the
 * first byte a connection carries picks text or binary for its lifetime.
 * 0 = not chosen yet (this buffer's first byte decides). */
enum { L7_CONN_MC_TEXT = 1, L7_CONN_MC_BINARY = 2, L7_CONN_PROXYLIB = 4 };

typedef struct {
    int32_t policy;     /* index of the NetworkPolicy in the loaded set, -1 = unknown */
    uint32_t port;      /* destination port */
    uint8_t ingress;    /* 1 = ingress */
    uint8_t proto;      /* L7_PROTO_* */
    uint16_t flags;     /* L7_CONN_MC_*: memcached framing chosen for the connection */
    uint32_t src_id;    /* source identity */
    uint32_t dst_id;    /* destination identity */
} ref_conn_t;

enum { L7_PROTO_HTTP = 1, L7_PROTO_KAFKA = 2, L7_PROTO_MEMCACHE = 3, L7_PROTO_R2D2 = 4, L7_PROTO_CASSANDRA = 5 };

/* verdict codes (shared meaning with the product, see include/l7gpu.h) */
enum {
    L7_DENY = 0,
    L7_ALLOW = 1,
    L7_PARSE_ERROR = 2,
    L7_INCOMPLETE = 3,
    L7_UNSUPPORTED = 4,
};

/* Classify n requests.  Request i is arena[off[i] .. off[i]+len[i]) on
 * connection conn[i].  Outputs per request: verdict, matched rule index
 * (global rule id, -1 = none), consumed bytes. nthreads <= 1: single thread. */
int ref_classify(const ref_policy *p, const ref_conn_t *conns, uint32_t nconns,
                 const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                 const uint32_t *conn, uint32_t n, uint8_t *verdict, int32_t *rule,
                 uint32_t *consumed, int nthreads);

/* proxylib cassandra parser (proxylib/cassandra/cassandraparser.go), one
 * parser state per connection: keyspace of the last USE, prepared paths by
 * stream id and by prepared id. */
typedef struct ref_cass ref_cass;
ref_cass *ref_cass_new(void);
void ref_cass_free(ref_cass *st);
/* Request direction, one CassandraParser.OnData step on the joined input:
 * returns the op (0 MORE, 1 PASS, 2 DROP, 4 ERROR; -1 = a Go panic, i.e.
 * PARSER_ERROR) and *n; *rule = matched rule id; *path (malloc'd or NULL) =
 * the request's path; inject[*inject_len] = the reply-direction injection
 * (unauthorized / unprepared message).  inject needs 65600 bytes. */
int ref_cass_request(ref_cass *st, const ref_policy *pol, const ref_conn_t *c, const uint8_t *d, uint32_t n,
                     int64_t *nout, int32_t *rule, char **path, uint8_t *inject, uint32_t *inject_len);
/* Reply direction: framing, cassandraParseReply (prepared ids), PASS. */
int ref_cass_reply(ref_cass *st, const uint8_t *d, uint32_t n, int64_t *nout);
/* parseQuery test hook: 0 ok (action / table written), 1 invalid, 2 panic. */
int ref_cass_parse_query(ref_cass *st, const uint8_t *q, size_t n, char *action, size_t alen, char *table, size_t tlen);
const char *ref_cass_keyspace(const ref_cass *st);

/* HTTP/1 framing restatement (debug/test helper): returns status and fills
 * the spans of :method, :path, :authority (offsets relative to buf, -1 = absent). */
typedef struct {
    int32_t status;        /* L7_ALLOW(=ok)/L7_PARSE_ERROR/L7_INCOMPLETE/L7_UNSUPPORTED */
    int32_t method_off, method_len;
    int32_t path_off, path_len;
    int32_t host_off, host_len;
    uint32_t consumed;
    int32_t nheaders;
} ref_http_info_t;
int ref_http_parse(const uint8_t *buf, uint32_t len, ref_http_info_t *info);

#ifdef __cplusplus
}
#endif
#endif
