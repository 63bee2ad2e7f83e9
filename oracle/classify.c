/*
 * classify.c — TEST INFRASTRUCTURE ONLY (parity oracle, see l7ref.h).
 *
 * Policy loading (JSON in the shape of cilium.NetworkPolicy,
 * envoy/cilium/npds.proto:31-182) and the batch classify driver.
 *
 * Validation follows what the reference rejects:
 *   - duplicate TCP port in one direction: envoy/cilium_network_policy.h:158-160
 *   - only TCP entries are installed:      envoy/cilium_network_policy.h:154-165
 *   - HTTP regex must compile (Go syntax):  pkg/policy/api/http.go:66-84
 *   - PortRuleKafka.Sanitize:               pkg/policy/api/rule_validation.go:232-275
 *   - one L7 oneof per rule:                npds.proto:91-106
 * Global rule ids: the i-th L7 rule object in document order
 * (policies -> ingress ports -> rules -> l7 rules, then egress), see DESIGN.md.
 */
#include <ctype.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "ref_internal.h"

typedef struct { char *err; size_t errlen; int failed; int next_id; int mc_stop; } ld;

static int lerr(ld *l, const char *fmt, const char *a) {
    if (!l->failed) { snprintf(l->err, l->errlen, fmt, a ? a : ""); l->failed = 1; }
    return -1;
}
static char *dupn(const char *s, size_t n) { char *d = malloc(n + 1); memcpy(d, s, n); d[n] = 0; return d; }
static const jnode *jlist(const jnode *v, const char *inner) {
    /* accepts {"inner": [...]} (NPDS nesting) or a bare array */
    if (!v) return NULL;
    if (v->type == JN_ARR) return v;
    if (v->type == JN_OBJ) { const jnode *a = jget(v, inner); if (a && a->type == JN_ARR) return a; }
    return NULL;
}
static int jstr(const jnode *o, const char *k, const char **s, size_t *n) {
    const jnode *v = jget(o, k);
    if (!v || v->type != JN_STR) return 0;
    *s = v->str; *n = v->slen; return 1;
}

static int load_hmatch(ld *l, const jnode *j, ref_hmatch *h) {
    memset(h, 0, sizeof *h);
    const char *s; size_t n;
    if (!jstr(j, "name", &s, &n)) return lerr(l, "header matcher without name%s", NULL);
    h->name = dupn(s, n); h->namelen = n;
    for (size_t i = 0; i < n; i++) h->name[i] = (char)tolower((unsigned char)h->name[i]);
    const jnode *inv = jget(j, "invert_match");
    h->invert = inv && inv->type == JN_BOOL && inv->b;
    const jnode *v;
    if (jstr(j, "exact_match", &s, &n)) { h->type = HM_EXACT; h->value = dupn(s, n); h->vlen = n; }
    else if (jstr(j, "regex_match", &s, &n)) { h->type = HM_REGEX; h->value = dupn(s, n); h->vlen = n; }
    else if (jstr(j, "prefix_match", &s, &n)) { h->type = HM_PREFIX; h->value = dupn(s, n); h->vlen = n; }
    else if (jstr(j, "suffix_match", &s, &n)) { h->type = HM_SUFFIX; h->value = dupn(s, n); h->vlen = n; }
    else if ((v = jget(j, "present_match")) && v->type == JN_BOOL) { h->type = HM_PRESENT; }
    else if ((v = jget(j, "range_match")) && v->type == JN_OBJ) {
        const jnode *a = jget(v, "start"), *b = jget(v, "end");
        h->type = HM_RANGE; h->rstart = a ? a->inum : 0; h->rend = b ? b->inum : 0;
    } else if (jstr(j, "value", &s, &n)) { /* deprecated value + regex */
        const jnode *r = jget(j, "regex");
        h->type = (r && r->type == JN_BOOL && r->b) ? HM_REGEX : HM_EXACT;
        h->value = dupn(s, n); h->vlen = n;
    } else {
        h->type = HM_EXACT; h->value = dupn("", 0); h->vlen = 0; /* empty value: presence */
    }
    if (h->type == HM_REGEX) {
        char e[256];
        h->re = ref_re_compile(h->value, h->vlen, e, sizeof e);
        if (!h->re) return lerr(l, "%s", e);
    }
    return 0;
}

static const char *KAFKA_KEYS[] = {
    "produce", "fetch", "offsets", "metadata", "leaderandisr", "stopreplica", "updatemetadata",
    "controlledshutdown", "offsetcommit", "offsetfetch", "findcoordinator", "joingroup", "heartbeat",
    "leavegroup", "syncgroup", "describegroups", "listgroups", "saslhandshake", "apiversions",
    "createtopics", "deletetopics", "deleterecords", "initproducerid", "offsetforleaderepoch",
    "addpartitionstotxn", "addoffsetstotxn", "endtxn", "writetxnmarkers", "txnoffsetcommit",
    "describeacls", "createacls", "deleteacls", "describeconfigs", "alterconfigs",
};

static int ieq(const char *a, size_t n, const char *b) {
    if (strlen(b) != n) return 0;
    for (size_t i = 0; i < n; i++) if (tolower((unsigned char)a[i]) != b[i]) return 0;
    return 1;
}

/* strconv.ParseInt(s, 10, 16) */
static int parse_int16(const char *s, size_t n, int16_t *out) {
    size_t i = 0; int neg = 0;
    if (n == 0) return 0;
    if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
    if (i >= n) return 0;
    long v = 0;
    for (; i < n; i++) {
        if (s[i] < '0' || s[i] > '9') return 0;
        v = v * 10 + (s[i] - '0');
        if (v > 40000) return 0;
    }
    if (neg) v = -v;
    if (v < -32768 || v > 32767) return 0;
    *out = (int16_t)v;
    return 1;
}

static int topic_ok(const char *t, size_t n) { /* KafkaTopicValidChar ^[a-zA-Z0-9\\._\\-]+$ */
    if (n == 0) return 0;
    for (size_t i = 0; i < n; i++) {
        unsigned char c = (unsigned char)t[i];
        if (!(isalnum(c) || c == '\\' || c == '.' || c == '_' || c == '-')) return 0;
    }
    return 1;
}

static int load_kafka(ld *l, const jnode *j, ref_kafka_rule *k) {
    memset(k, 0, sizeof *k);
    k->any_key = 1;
    const char *s; size_t n;
    const char *role = NULL, *key = NULL; size_t rolen = 0, keyn = 0;
    jstr(j, "role", &role, &rolen);
    jstr(j, "apiKey", &key, &keyn);
    if (rolen > 0 && keyn > 0) return lerr(l, "kafka: cannot set both Role and APIKey%s", NULL);
    if (keyn > 0) {
        int found = -1;
        for (int i = 0; i < (int)(sizeof KAFKA_KEYS / sizeof KAFKA_KEYS[0]); i++) if (ieq(key, keyn, KAFKA_KEYS[i])) found = i;
        if (found < 0) return lerr(l, "invalid Kafka APIKey%s", NULL);
        k->any_key = 0; k->keymask |= 1ull << found;
    }
    if (rolen > 0) {
        k->any_key = 0;
        if (ieq(role, rolen, "produce")) k->keymask = (1ull << 0) | (1ull << 3) | (1ull << 18);
        else if (ieq(role, rolen, "consume")) {
            static const int C[] = {1, 2, 3, 8, 9, 10, 11, 12, 13, 14, 18};
            for (size_t i = 0; i < sizeof C / sizeof C[0]; i++) k->keymask |= 1ull << C[i];
        } else return lerr(l, "invalid Kafka APIRole%s", NULL);
    }
    if (jstr(j, "apiVersion", &s, &n) && n > 0) {
        if (!parse_int16(s, n, &k->version)) return lerr(l, "invalid Kafka APIVersion%s", NULL);
        k->has_version = 1;
    }
    if (jstr(j, "topic", &s, &n) && n > 0) {
        if (n > 255) return lerr(l, "kafka topic exceeds maximum len%s", NULL);
        if (!topic_ok(s, n)) return lerr(l, "invalid Kafka Topic name%s", NULL);
        k->topic = dupn(s, n); k->topiclen = n;
    }
    if ((jstr(j, "clientID", &s, &n) || jstr(j, "client_id", &s, &n)) && n > 0) { k->client = dupn(s, n); k->clientlen = n; }
    const jnode *v;
    if ((v = jget(j, "api_key")) && v->type == JN_NUM && v->inum >= 0) {
        if (v->inum > 63) return lerr(l, "kafka api_key out of range%s", NULL);
        k->any_key = 0; k->keymask = 1ull << v->inum;
    }
    if ((v = jget(j, "api_version")) && v->type == JN_NUM && v->inum >= 0) { k->has_version = 1; k->version = (int16_t)v->inum; }
    return 0;
}

/* memcache.L7RuleParser (proxylib/memcached/parser.go:114-148): keys command /
 * keyExact / keyPrefix / keyRegex; anything else, or a key match without a
 * known command, is a ParseError (policy NACK).  An unknown command without
 * key matches leaves an "empty" rule that matches everything. */
static int load_mc_rule(ld *l, const jnode *j, ref_mc_rule *m) {
    const jnode *kv = jget(j, "rule");
    if (!kv) kv = j;
    if (kv->type != JN_OBJ) return 0;
    int found = 0;
    for (int i = 0; i < kv->n; i++) {
        const char *k = kv->keys[i];
        const jnode *v = kv->items[i];
        if (v->type != JN_STR) return lerr(l, "NPDS: memcache rule value is not a string%s", NULL);
        if (!strcmp(k, "command")) { m->group = ref_mc_group(v->str, v->slen); found = m->group != NULL; }
        else if (!strcmp(k, "keyExact")) { free(m->key_exact); m->key_exact = dupn(v->str, v->slen); m->key_exact_len = v->slen; }
        else if (!strcmp(k, "keyPrefix")) { free(m->key_prefix); m->key_prefix = dupn(v->str, v->slen); m->key_prefix_len = v->slen; }
        else if (!strcmp(k, "keyRegex")) {
            char e[256];
            ref_re_free(m->key_re);
            m->key_re = ref_re_compile(v->str, v->slen, e, sizeof e);
            if (!m->key_re) return lerr(l, "%s", e);
        } else return lerr(l, "NPDS: Unsupported key: %s", k);
    }
    if (!found) {
        if (m->key_exact_len > 0 || m->key_prefix_len > 0 || m->key_re)
            return lerr(l, "NPDS: command not specified but key was provided%s", NULL);
        m->empty = 1;
    }
    return 0;
}

/* r2d2.R2d2RuleParser (proxylib/r2d2/r2d2parser.go:69-107): keys cmd / file;
 * an invalid cmd, a file regex with HALT / RESET, an unknown key or a regex
 * that does not compile (regexp.MustCompile) NACKs the policy. */
static int load_r2_rule(ld *l, const jnode *j, ref_mc_rule *m) {
    const jnode *kv = jget(j, "rule");
    if (!kv) kv = j;
    if (kv->type != JN_OBJ) return 0;
    for (int i = 0; i < kv->n; i++) {
        const char *k = kv->keys[i];
        const jnode *v = kv->items[i];
        if (v->type != JN_STR) return lerr(l, "NPDS: r2d2 rule value is not a string%s", NULL);
        if (!strcmp(k, "cmd")) { free(m->r2_cmd); m->r2_cmd = v->slen ? dupn(v->str, v->slen) : NULL; m->r2_cmd_len = v->slen; }
        else if (!strcmp(k, "file")) {
            if (v->slen == 0) continue;
            char e[256];
            ref_re_free(m->r2_file);
            m->r2_file = ref_re_compile(v->str, v->slen, e, sizeof e);
            if (!m->r2_file) return lerr(l, "regexp: Compile(`%s`)", v->str);
        } else return lerr(l, "NPDS: Unsupported key: %s", k);
    }
    const char *c = m->r2_cmd;
    if (c && strcmp(c, "READ") && strcmp(c, "WRITE") && strcmp(c, "HALT") && strcmp(c, "RESET"))
        return lerr(l, "NPDS: Unable to parse L7 r2d2 rule with invalid cmd: '%s'", c);
    if (m->r2_file && c && strcmp(c, "READ") && strcmp(c, "WRITE"))
        return lerr(l, "NPDS: Unable to parse L7 r2d2 rule, cmd '%s' is not compatible with 'file'", c);
    return 0;
}

/* cassandra.CassandraRuleParser (proxylib/cassandra/cassandraparser.go:99-134):
 * keys query_action / query_table; an unknown key, a query_action outside
 * queryActionMap (:319-366), a query_table with a table-less action, or a
 * regex that does not compile (regexp.MustCompile) NACKs the policy. */
static const char *kCassActions[] = {
    "select", "delete", "insert", "update", "create-table", "drop-table", "alter-table", "truncate-table", "use",
    "create-keyspace", "alter-keyspace", "drop-keyspace", "drop-index", "create-index", "create-materialized-view",
    "drop-materialized-view", "create-role", "alter-role", "drop-role", "grant-role", "revoke-role", "list-roles",
    "grant-permission", "revoke-permission", "list-permissions", "create-user", "alter-user", "drop-user",
    "list-users", "create-function", "drop-function", "create-aggregate", "drop-aggregate", "create-type",
    "alter-type", "drop-type", "create-trigger", "drop-trigger"};
static int cass_action_kind(const char *a) {  /* 0 invalid, 1 with table, 2 without */
    for (size_t i = 0; i < sizeof kCassActions / sizeof kCassActions[0]; i++)
        if (!strcmp(a, kCassActions[i])) return i < 12 ? 1 : 2;
    return 0;
}
static int load_cass_rule(ld *l, const jnode *j, ref_mc_rule *m) {
    const jnode *kv = jget(j, "rule");
    if (!kv) kv = j;
    if (kv->type != JN_OBJ) return 0;
    for (int i = 0; i < kv->n; i++) {
        const char *k = kv->keys[i];
        const jnode *v = kv->items[i];
        if (v->type != JN_STR) return lerr(l, "NPDS: cassandra rule value is not a string%s", NULL);
        if (!strcmp(k, "query_action")) { free(m->cass_action); m->cass_action = v->slen ? dupn(v->str, v->slen) : NULL; }
        else if (!strcmp(k, "query_table")) {
            if (v->slen == 0) continue;
            char e[256];
            ref_re_free(m->cass_table);
            m->cass_table = ref_re_compile(v->str, v->slen, e, sizeof e);
            if (!m->cass_table) return lerr(l, "regexp: Compile(`%s`)", v->str);
        } else return lerr(l, "NPDS: Unsupported key: %s", k);
    }
    if (m->cass_action) {
        const int kind = cass_action_kind(m->cass_action);
        if (kind == 0) return lerr(l, "NPDS: Unable to parse L7 cassandra rule with invalid query_action: '%s'", m->cass_action);
        if (kind == 2 && m->cass_table)
            return lerr(l, "NPDS: query_action '%s' is not compatible with a query_table match", m->cass_action);
    }
    return 0;
}

static int load_rule(ld *l, const jnode *j, ref_pnp_rule *r) {
    memset(r, 0, sizeof *r);
    const jnode *rp = jget(j, "remote_policies");
    if (rp && rp->type == JN_ARR) {
        r->nremotes = rp->n;
        r->remotes = calloc((size_t)rp->n + 1, sizeof(uint64_t));
        for (int i = 0; i < rp->n; i++) {
            r->remotes[i] = (uint64_t)rp->items[i]->inum;
            for (int k = 0; k < i; k++) if (r->remotes[k] == r->remotes[i]) return lerr(l, "remote_policies must be unique%s", NULL);
        }
    }
    const char *s; size_t n;
    if (jstr(j, "l7_proto", &s, &n) && n > 0) r->l7proto = dupn(s, n);
    const jnode *h = jlist(jget(j, "http_rules"), "http_rules");
    const jnode *kf = jlist(jget(j, "kafka_rules"), "kafka_rules");
    const jnode *l7 = jlist(jget(j, "l7_rules"), "l7_rules");
    if ((h != NULL) + (kf != NULL) + (l7 != NULL) > 1) return lerr(l, "more than one L7 rule type in a rule%s", NULL);
    if (h) {
        r->l7type = L7T_HTTP; r->nhttp = h->n;
        r->http = calloc((size_t)h->n + 1, sizeof(ref_http_rule));
        for (int i = 0; i < h->n; i++) {
            const jnode *hr = h->items[i];
            const jnode *hs = jget(hr, "headers");
            r->http[i].id = l->next_id++;
            if (hs && hs->type == JN_ARR) {
                r->http[i].n = hs->n;
                r->http[i].m = calloc((size_t)hs->n + 1, sizeof(ref_hmatch));
                for (int q = 0; q < hs->n; q++) if (load_hmatch(l, hs->items[q], &r->http[i].m[q]) < 0) return -1;
            }
        }
    } else if (kf) {
        r->l7type = L7T_KAFKA; r->nkafka = kf->n;
        r->kafka = calloc((size_t)kf->n + 1, sizeof(ref_kafka_rule));
        for (int i = 0; i < kf->n; i++) {
            if (load_kafka(l, kf->items[i], &r->kafka[i]) < 0) return -1;
            r->kafka[i].id = l->next_id++;
        }
    } else if (l7) {
        r->l7type = L7T_L7; r->nl7 = l7->n;
        r->l7 = calloc((size_t)l7->n + 1, sizeof(ref_mc_rule));
        int mc = !l->mc_stop && r->l7proto && !strcmp(r->l7proto, "memcache");
        int r2 = !l->mc_stop && r->l7proto && !strcmp(r->l7proto, "r2d2");
        int cs = !l->mc_stop && r->l7proto && !strcmp(r->l7proto, "cassandra");
        for (int i = 0; i < l7->n; i++) {
            r->l7[i].id = l->next_id++;
            if (mc && load_mc_rule(l, l7->items[i], &r->l7[i]) < 0) return -1;
            if (r2 && load_r2_rule(l, l7->items[i], &r->l7[i]) < 0) return -1;
            if (cs && load_cass_rule(l, l7->items[i], &r->l7[i]) < 0) return -1;
        }
    }
    return 0;
}

static int load_ports(ld *l, const jnode *arr, ref_port **out, int *nout) {
    *out = NULL; *nout = 0;
    if (!arr || arr->type != JN_ARR) return 0;
    ref_port *ps = calloc((size_t)arr->n + 1, sizeof(ref_port));
    *out = ps; *nout = arr->n;
    for (int i = 0; i < arr->n; i++) {
        const jnode *pj = arr->items[i];
        const jnode *pv = jget(pj, "port");
        int64_t port = pv ? pv->inum : 0;
        if (port < 0 || port > 65535) return lerr(l, "port out of range%s", NULL);
        ps[i].port = (uint32_t)port;
        const jnode *pr = jget(pj, "protocol");
        ps[i].tcp = 1;
        if (pr && pr->type == JN_STR && !strcmp(pr->str, "UDP")) ps[i].tcp = 0;
        if (pr && pr->type == JN_NUM && pr->inum != 0) ps[i].tcp = 0;
        const jnode *rs = jget(pj, "rules");
        if (rs && rs->type == JN_ARR) {
            ps[i].nrules = rs->n;
            ps[i].rules = calloc((size_t)rs->n + 1, sizeof(ref_pnp_rule));
            /* proxylib parses a port's rules in order and stops at the first rule
             * whose L7 parser is not registered (policymap.go:118-131): later
             * memcache rules are never parsed, so they raise no ParseError.  With
             * "memcache" the only registered parser, the "Mismatching L7 types"
             * panic (:135-140) cannot fire. */
            l->mc_stop = 0;
            for (int k = 0; k < rs->n; k++) {
                if (load_rule(l, rs->items[k], &ps[i].rules[k]) < 0) return -1;
                if (ps[i].rules[k].l7type == L7T_HTTP) ps[i].has_http = 1;
                const ref_pnp_rule *pr = &ps[i].rules[k];
                /* unregistered parser: an l7_proto no linked parser registers
                 * (proxylib/proxylib.go:24-29), or generic L7 rules */
                if ((pr->l7proto && *pr->l7proto && strcmp(pr->l7proto, "memcache") && strcmp(pr->l7proto, "r2d2") &&
                     strcmp(pr->l7proto, "cassandra") && strcmp(pr->l7proto, "test.headerparser")) ||
                    ((!pr->l7proto || !*pr->l7proto) && pr->l7type == L7T_L7))
                    l->mc_stop = 1;
            }
        }
        if (ps[i].tcp)
            for (int k = 0; k < i; k++)
                if (ps[k].tcp && ps[k].port == ps[i].port) return lerr(l, "PortNetworkPolicy: Duplicate port number%s", NULL);
    }
    return 0;
}

static void free_ports(ref_port *ps, int n) {
    for (int i = 0; i < n; i++) {
        for (int k = 0; k < ps[i].nrules; k++) {
            ref_pnp_rule *r = &ps[i].rules[k];
            for (int q = 0; q < r->nhttp; q++) {
                for (int m = 0; m < r->http[q].n; m++) { free(r->http[q].m[m].name); free(r->http[q].m[m].value); ref_re_free(r->http[q].m[m].re); }
                free(r->http[q].m);
            }
            for (int q = 0; q < r->nkafka; q++) { free(r->kafka[q].topic); free(r->kafka[q].client); }
            for (int q = 0; q < r->nl7; q++) {
                free(r->l7[q].key_exact); free(r->l7[q].key_prefix); ref_re_free(r->l7[q].key_re);
                free(r->l7[q].r2_cmd); ref_re_free(r->l7[q].r2_file);
                free(r->l7[q].cass_action); ref_re_free(r->l7[q].cass_table);
            }
            free(r->http); free(r->kafka); free(r->l7); free(r->remotes); free(r->l7proto);
        }
        free(ps[i].rules);
    }
    free(ps);
}

void ref_policy_free(ref_policy *p) {
    if (!p) return;
    for (int i = 0; i < p->np; i++) { free(p->p[i].name); free_ports(p->p[i].in, p->p[i].nin); free_ports(p->p[i].eg, p->p[i].neg); }
    free(p->p); free(p);
}

ref_policy *ref_policy_load(const char *json, size_t len, char *err, size_t errlen) {
    char dummy[8];
    ld l = {err ? err : dummy, err ? errlen : sizeof dummy, 0, 0, 0};
    if (l.errlen) l.err[0] = 0;
    jnode *root = jparse(json, len, l.err, l.errlen);
    if (!root) return NULL;
    const jnode *arr = root;
    if (root->type == JN_OBJ) {
        const jnode *ps = jget(root, "policies");
        arr = ps;
    }
    ref_policy *p = calloc(1, sizeof(ref_policy));
    if (!arr || arr->type != JN_ARR) { lerr(&l, "expected a list of policies%s", NULL); jfree(root); free(p); return NULL; }
    p->np = arr->n;
    p->p = calloc((size_t)arr->n + 1, sizeof(ref_netpolicy));
    for (int i = 0; i < arr->n && !l.failed; i++) {
        const jnode *pj = arr->items[i];
        const char *s; size_t n;
        p->p[i].name = jstr(pj, "name", &s, &n) ? dupn(s, n) : dupn("", 0);
        const jnode *id = jget(pj, "policy");
        p->p[i].id = id ? (uint64_t)id->inum : 0;
        if (load_ports(&l, jget(pj, "ingress_per_port_policies"), &p->p[i].in, &p->p[i].nin) < 0) break;
        if (load_ports(&l, jget(pj, "egress_per_port_policies"), &p->p[i].eg, &p->p[i].neg) < 0) break;
    }
    jfree(root);
    if (l.failed) { ref_policy_free(p); return NULL; }
    p->nrules_total = l.next_id;
    return p;
}

int ref_port_lookup(const ref_netpolicy *np, int ingress, uint32_t port, const ref_port **exact, const ref_port **wild) {
    const ref_port *ps = ingress ? np->in : np->eg;
    int n = ingress ? np->nin : np->neg;
    *exact = NULL; *wild = NULL;
    for (int i = 0; i < n; i++) {
        if (!ps[i].tcp) continue;
        if (ps[i].port == port) *exact = &ps[i];
        if (ps[i].port == 0 && port != 0) *wild = &ps[i];
    }
    return *exact || *wild;
}

static const char *px_parser(const ref_pnp_rule *r) {  /* policymap.go:68-75 */
    if (r->l7proto && *r->l7proto) return r->l7proto;
    switch (r->l7type) {
    case L7T_HTTP: return "PortNetworkPolicyRule_HttpRules";
    case L7T_KAFKA: return "PortNetworkPolicyRule_KafkaRules";
    case L7T_L7: return "PortNetworkPolicyRule_L7Rules";
    default: return "";
    }
}

int ref_px_nl7(const ref_pnp_rule *r) {
    if (r->l7type == L7T_HTTP) return r->nhttp;
    if (r->l7type == L7T_KAFKA) return r->nkafka;
    if (r->l7type == L7T_L7 && r->l7proto &&
        (!strcmp(r->l7proto, "memcache") || !strcmp(r->l7proto, "r2d2") || !strcmp(r->l7proto, "cassandra") ||
         !strcmp(r->l7proto, "test.headerparser")))
        return r->nl7;
    return 0;
}

int ref_px_installed(const ref_port *pp) {
    const char *first = NULL;
    for (int r = 0; r < pp->nrules; r++) {
        const char *n = px_parser(&pp->rules[r]);
        if (!*n) continue;
        if (strcmp(n, "memcache") && strcmp(n, "r2d2") && strcmp(n, "cassandra") && strcmp(n, "test.headerparser") &&
            strcmp(n, "PortNetworkPolicyRule_HttpRules") &&
            strcmp(n, "PortNetworkPolicyRule_KafkaRules"))
            return 0;  /* no such parser: port skipped (:128-134, 200-203) */
        (void)first;  /* mismatching L7 types NACK the whole proxylib update
                       * (:135-143): such a version is never installed */
    }
    return 1;
}

int ref_px_have_l7(const ref_port *pp) {
    for (int r = 0; r < pp->nrules; r++) if (ref_px_nl7(&pp->rules[r]) > 0) return 1;
    return 0;
}

int ref_remote_ok(const ref_pnp_rule *r, uint64_t id) {
    if (r->nremotes == 0) return 1;
    for (int i = 0; i < r->nremotes; i++) if (r->remotes[i] == id) return 1;
    return 0;
}

typedef struct {
    const ref_policy *p; const ref_conn_t *conns; uint32_t nconns;
    const uint8_t *arena; const uint64_t *off; const uint32_t *len; const uint32_t *conn;
    uint32_t lo, hi; uint8_t *verdict; int32_t *rule; uint32_t *consumed;
} job_t;

static void *run(void *arg) {
    job_t *j = arg;
    for (uint32_t i = j->lo; i < j->hi; i++) {
        ref_out_t o = {L7_UNSUPPORTED, -1, 0}; /* unknown connection / no parser */
        uint32_t ci = j->conn[i];
        if (ci < j->nconns) {
            const ref_conn_t *c = &j->conns[ci];
            const uint8_t *b = j->arena + j->off[i];
            if (c->proto == L7_PROTO_HTTP) ref_http_verdict(j->p, c, b, j->len[i], &o);
            else if (c->proto == L7_PROTO_KAFKA) ref_kafka_verdict(j->p, c, b, j->len[i], &o);
            else if (c->proto == L7_PROTO_MEMCACHE) ref_memcache_verdict(j->p, c, b, j->len[i], &o);
            else if (c->proto == L7_PROTO_R2D2) ref_r2d2_verdict(j->p, c, b, j->len[i], &o);
            else if (c->proto == L7_PROTO_CASSANDRA) continue;  /* answered in order by ref_classify */
            else o.verdict = L7_UNSUPPORTED;
        }
        j->verdict[i] = o.verdict; j->rule[i] = o.rule; j->consumed[i] = o.consumed;
    }
    return NULL;
}

int ref_classify(const ref_policy *p, const ref_conn_t *conns, uint32_t nconns,
                 const uint8_t *arena, const uint64_t *off, const uint32_t *len,
                 const uint32_t *conn, uint32_t n, uint8_t *verdict, int32_t *rule,
                 uint32_t *consumed, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    /* cassandra: requests in batch order, one parser state (keyspace) per
     * connection, as proxylib's OnData walks a connection's frames */
    ref_cass **cs = NULL;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t ci = conn[i];
        if (ci >= nconns || conns[ci].proto != L7_PROTO_CASSANDRA) continue;
        if (!cs) cs = calloc(nconns, sizeof *cs);
        if (!cs[ci]) cs[ci] = ref_cass_new();
        ref_out_t o = {L7_UNSUPPORTED, -1, 0};
        ref_cassandra_verdict(cs[ci], p, &conns[ci], arena + off[i], len[i], &o);
        verdict[i] = o.verdict; rule[i] = o.rule; consumed[i] = o.consumed;
    }
    if (cs) {
        for (uint32_t k = 0; k < nconns; k++) ref_cass_free(cs[k]);
        free(cs);
    }
    job_t jobs[256]; pthread_t th[256];
    uint32_t per = (n + (uint32_t)nthreads - 1) / (uint32_t)nthreads;
    int used = 0;
    for (int t = 0; t < nthreads; t++) {
        uint32_t lo = (uint32_t)t * per, hi = lo + per;
        if (lo >= n) break;
        if (hi > n) hi = n;
        jobs[t] = (job_t){p, conns, nconns, arena, off, len, conn, lo, hi, verdict, rule, consumed};
        used++;
    }
    if (used <= 1) { if (used) run(&jobs[0]); return 0; }
    for (int t = 0; t < used; t++) pthread_create(&th[t], NULL, run, &jobs[t]);
    for (int t = 0; t < used; t++) pthread_join(th[t], NULL);
    return 0;
}
