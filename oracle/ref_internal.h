/* ref_internal.h — TEST INFRASTRUCTURE ONLY (parity oracle internals). */
#ifndef REF_INTERNAL_H
#define REF_INTERNAL_H
#include <stddef.h>
#include <stdint.h>
#include "l7ref.h"

/* ---------------- minimal JSON ---------------- */
enum { JN_NULL, JN_BOOL, JN_NUM, JN_STR, JN_ARR, JN_OBJ };
typedef struct jnode {
    int type;
    double num; int64_t inum; int is_int;
    char *str; size_t slen;        /* JN_STR (UTF-8, NUL-terminated) */
    struct jnode **items; char **keys; size_t *keylens; int n, cap; /* ARR/OBJ */
    int b;
} jnode;
jnode *jparse(const char *s, size_t n, char *err, size_t errlen);
void jfree(jnode *j);
jnode *jget(const jnode *obj, const char *key);

/* ---------------- policy model (NPDS NetworkPolicy, envoy/cilium/npds.proto) ---- */
enum { HM_EXACT, HM_REGEX, HM_PRESENT, HM_PREFIX, HM_SUFFIX, HM_RANGE };
typedef struct {
    char *name; size_t namelen;   /* lower-cased (Envoy LowerCaseString) */
    int type;
    char *value; size_t vlen;
    ref_re *re;
    int invert;
    int64_t rstart, rend;
} ref_hmatch;

typedef struct { ref_hmatch *m; int n; int id; } ref_http_rule;

typedef struct {
    uint64_t keymask;       /* api keys 0..63 allowed; 0 = any (apiKeyInt empty) */
    int any_key;
    int has_version; int16_t version;
    char *topic; size_t topiclen;
    char *client; size_t clientlen;
    int id;
} ref_kafka_rule;

typedef struct {  /* memcache.Rule (proxylib/memcached/parser.go:35-44) */
    const void *group;                 /* MemcacheOpCodeMap entry, NULL = command not found */
    char *key_exact; size_t key_exact_len;
    char *key_prefix; size_t key_prefix_len;
    ref_re *key_re;
    int empty; int id;
    /* r2d2.R2d2Rule (proxylib/r2d2/r2d2parser.go:31-34), for l7_proto "r2d2" */
    char *r2_cmd; size_t r2_cmd_len;   /* NULL = any */
    ref_re *r2_file;                   /* NULL = any */
    /* cassandra.CassandraRule (proxylib/cassandra/cassandraparser.go:50-53) */
    char *cass_action;                 /* query_action, NULL = any */
    ref_re *cass_table;                /* query_table, NULL = any */
} ref_mc_rule;

enum { L7T_NONE = 0, L7T_HTTP, L7T_KAFKA, L7T_L7 };
typedef struct {
    uint64_t *remotes; int nremotes;
    int l7type;
    ref_http_rule *http; int nhttp;
    ref_kafka_rule *kafka; int nkafka;
    char *l7proto;
    ref_mc_rule *l7; int nl7;
} ref_pnp_rule;

typedef struct { uint32_t port; int tcp; ref_pnp_rule *rules; int nrules; int has_http; } ref_port;
typedef struct { char *name; uint64_t id; ref_port *in; int nin; ref_port *eg; int neg; } ref_netpolicy;
struct ref_policy { ref_netpolicy *p; int np; int nrules_total; };

/* ---------------- per-protocol verdict functions ---------------- */
typedef struct { uint8_t verdict; int32_t rule; uint32_t consumed; } ref_out_t;
void ref_http_verdict(const ref_policy *pol, const ref_conn_t *c, const uint8_t *buf, uint32_t len, ref_out_t *o);
void ref_kafka_verdict(const ref_policy *pol, const ref_conn_t *c, const uint8_t *buf, uint32_t len, ref_out_t *o);
void ref_memcache_verdict(const ref_policy *pol, const ref_conn_t *c, const uint8_t *buf, uint32_t len, ref_out_t *o);
void ref_r2d2_verdict(const ref_policy *pol, const ref_conn_t *c, const uint8_t *buf, uint32_t len, ref_out_t *o);
void ref_cassandra_verdict(ref_cass *st, const ref_policy *pol, const ref_conn_t *c, const uint8_t *buf, uint32_t len,
                           ref_out_t *o);
const void *ref_mc_group(const char *name, size_t n);

int ref_port_lookup(const ref_netpolicy *np, int ingress, uint32_t port, const ref_port **exact, const ref_port **wild);
int ref_remote_ok(const ref_pnp_rule *r, uint64_t id);
/* proxylib's view of a port entry (proxylib/proxylib/policymap.go:58-206) with
 * the rule parsers "memcache", "r2d2", PortNetworkPolicyRule_HttpRules and
 * PortNetworkPolicyRule_KafkaRules registered */
int ref_px_nl7(const ref_pnp_rule *r);          /* len(L7Rules) of a rule */
int ref_px_installed(const ref_port *pp);       /* entry kept in PortNetworkPolicies */
int ref_px_have_l7(const ref_port *pp);         /* HaveL7Rules */

#endif
