/* cassandra (proxylib/cassandra/cassandraparser.go) -- oracle restatement
 * (TEST INFRASTRUCTURE: only tests/, smoke() and bench.py's cpu_baseline use
 * it).  A direct, string-building restatement of the Go code, kept deliberately
 * different in shape from the device kernel (which works on token spans):
 *
 *   OnData framing (:171-262): < 9 bytes => MORE 9-len; body length > 256 MB
 *     => ERROR INVALID_FRAME_LENGTH; missing body bytes => MORE; then
 *     cassandraParseRequest on the frame.
 *   cassandraParseRequest (:471-581): reply direction bit or compression flag
 *     => ERROR INVALID_FRAME_TYPE; QUERY / PREPARE => parseQuery of the long
 *     string at 9 (a short body is a Go slice panic); BATCH always panics
 *     (binary.BigEndian.Uint16 of the 1-byte slice data[10:11], :519); EXECUTE
 *     => the path cached for its prepared id (no entry: ERROR
 *     INVALID_FRAME_TYPE); other opcodes => "/" + opcode name.
 *   parseQuery (:368-469): TrimRight(";"), strings.ToLower (Go 1.10
 *     strings.Map: unicode.ToLower per rune; an invalid UTF-8 byte stays as it
 *     is until the first rune that ToLower changes, and becomes U+FFFD after
 *     it), strings.Fields (unicode.IsSpace), comment tokens (prefix "--",
 *     slash-star or "//") reject the query, then the action / table grammar and the
 *     keyspace of the last USE for undotted tables.
 *   CassandraRule.Matches (:58-95) over the proxylib policymap (exact port then
 *     port 0, installed entries only, SrcId as the remote, no entry => drop):
 *     path split on "/", <= 2 parts => match, query_action exact (or any),
 *     query_table regexp.MatchString on parts[3] when that is non-empty.
 *
 * The invalid-UTF-8 behaviour of strings.Map and the Unicode data (Unicode
 * 10.0 assigned set, unicode_tables.h) are not covered by any reference test:
 * parity unpinned there.  The KATs of cassandraparser_test.go:79-282 pin the
 * rest (tests/golden/reference_kats.json "cassandra"). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ref_internal.h"
#include "unicode_tables.h"

/* ---------------- strings ---------------- */
typedef struct { uint8_t *p; size_t n, cap; } sbuf;
static void sb_put(sbuf *b, const void *d, size_t n) {
    if (b->n + n + 1 > b->cap) {
        b->cap = (b->n + n + 1) * 2;
        b->p = realloc(b->p, b->cap);
    }
    memcpy(b->p + b->n, d, n);
    b->n += n;
    b->p[b->n] = 0;
}
static void sb_byte(sbuf *b, uint8_t c) { sb_put(b, &c, 1); }
static void sb_rune(sbuf *b, int32_t r) {  /* utf8.EncodeRune */
    uint8_t e[4];
    if (r < 0x80) { e[0] = (uint8_t)r; sb_put(b, e, 1); }
    else if (r < 0x800) { e[0] = (uint8_t)(0xC0 | r >> 6); e[1] = (uint8_t)(0x80 | (r & 0x3F)); sb_put(b, e, 2); }
    else if (r < 0x10000) {
        e[0] = (uint8_t)(0xE0 | r >> 12); e[1] = (uint8_t)(0x80 | ((r >> 6) & 0x3F)); e[2] = (uint8_t)(0x80 | (r & 0x3F));
        sb_put(b, e, 3);
    } else {
        e[0] = (uint8_t)(0xF0 | r >> 18); e[1] = (uint8_t)(0x80 | ((r >> 12) & 0x3F));
        e[2] = (uint8_t)(0x80 | ((r >> 6) & 0x3F)); e[3] = (uint8_t)(0x80 | (r & 0x3F));
        sb_put(b, e, 4);
    }
}


/* utf8.DecodeRuneInString: (rune, width); invalid => U+FFFD width 1 */
static int dec(const uint8_t *s, size_t n, int32_t *r) {
    uint8_t b0 = s[0];
    if (b0 < 0x80) { *r = b0; return 1; }
    int sz; uint8_t lo = 0x80, hi = 0xBF;
    if (b0 >= 0xC2 && b0 <= 0xDF) sz = 2;
    else if (b0 >= 0xE0 && b0 <= 0xEF) { sz = 3; if (b0 == 0xE0) lo = 0xA0; if (b0 == 0xED) hi = 0x9F; }
    else if (b0 >= 0xF0 && b0 <= 0xF4) { sz = 4; if (b0 == 0xF0) lo = 0x90; if (b0 == 0xF4) hi = 0x8F; }
    else { *r = 0xFFFD; return 1; }
    if (n < (size_t)sz || s[1] < lo || s[1] > hi) { *r = 0xFFFD; return 1; }
    int32_t v = b0 & (0x7F >> (sz + 1));
    v = v << 6 | (s[1] & 0x3F);
    for (int k = 2; k < sz; k++) {
        if (s[k] < 0x80 || s[k] > 0xBF) { *r = 0xFFFD; return 1; }
        v = v << 6 | (s[k] & 0x3F);
    }
    *r = v;
    return sz;
}

/* unicode.ToLower */
static int32_t to_lower(int32_t r) {
    if (r < 0x80) return (r >= 'A' && r <= 'Z') ? r + 32 : r;
    int lo = 0, hi = UNI_LOWER_NPAIRS;
    while (lo < hi) {
        int m = (lo + hi) / 2;
        if ((int32_t)UNI_LOWER_PAIRS[m][0] < r) lo = m + 1; else hi = m;
    }
    if (lo < UNI_LOWER_NPAIRS && (int32_t)UNI_LOWER_PAIRS[lo][0] == r) return (int32_t)UNI_LOWER_PAIRS[lo][1];
    return r;
}

/* strings.ToLower (Go 1.10): ASCII fast path, else strings.Map(unicode.ToLower):
 * the input is returned as is up to the first rune the mapping changes; from
 * there every rune is re-encoded (an invalid byte, decoded as U+FFFD, becomes
 * the 3-byte encoding of U+FFFD). */
static void go_to_lower(const uint8_t *s, size_t n, sbuf *out) {
    size_t i = 0;
    int changed = 0;
    while (i < n) {
        int32_t r;
        int w = dec(s + i, n - i, &r);
        int32_t l = to_lower(r);
        if (!changed && l == r) { sb_put(out, s + i, (size_t)w); i += (size_t)w; continue; }
        changed = 1;
        sb_rune(out, l);
        i += (size_t)w;
    }
    if (!out->p) sb_put(out, "", 0);
}

/* unicode.IsSpace at s (byte length of the space rune, 0 if none) */
static int space_len(const uint8_t *s, size_t n) {
    uint8_t c = s[0];
    if (c == ' ' || (c >= 0x09 && c <= 0x0D)) return 1;
    int32_t r;
    int w = dec(s, n, &r);
    if (r == 0x85 || r == 0xA0 || r == 0x1680 || (r >= 0x2000 && r <= 0x200A) || r == 0x2028 || r == 0x2029 ||
        r == 0x202F || r == 0x205F || r == 0x3000)
        return w;
    return 0;
}

typedef struct { char **f; size_t *len; int n; } fields_t;
static void fields_free(fields_t *f) {
    for (int i = 0; i < f->n; i++) free(f->f[i]);
    free(f->f); free(f->len);
}
/* strings.Fields */
static fields_t go_fields(const uint8_t *s, size_t n) {
    fields_t f = {NULL, NULL, 0};
    int cap = 0;
    size_t i = 0, start = 0;
    int in = 0;
    while (i <= n) {
        int sp = i < n ? space_len(s + i, n - i) : 1;
        if (sp) {
            if (in) {
                if (f.n == cap) { cap = cap ? 2 * cap : 8; f.f = realloc(f.f, cap * sizeof *f.f); f.len = realloc(f.len, cap * sizeof *f.len); }
                f.f[f.n] = malloc(i - start + 1);
                memcpy(f.f[f.n], s + start, i - start);
                f.f[f.n][i - start] = 0;
                f.len[f.n] = i - start;
                f.n++;
                in = 0;
            }
            if (i == n) break;
            i += (size_t)sp;
        } else {
            if (!in) { start = i; in = 1; }
            int32_t r;
            i += (size_t)dec(s + i, n - i, &r);
        }
    }
    return f;
}

static int feq(const fields_t *f, int i, const char *w) { return f->len[i] == strlen(w) && !memcmp(f->f[i], w, f->len[i]); }

/* ---------------- per-connection parser state ---------------- */
/* Paths are Go strings: bytes with a length (a keyspace or table token may
 * hold any byte, NUL included, e.g. a USE whose query runs on past its frame),
 * NUL-terminated only for convenience. */
typedef struct { uint16_t stream; char *path; size_t plen; } by_stream_t;
typedef struct { char *id; size_t idlen; char *path; size_t plen; } by_id_t;
struct ref_cass {
    sbuf keyspace;
    by_stream_t *bs; int nbs;
    by_id_t *bi; int nbi;
};

ref_cass *ref_cass_new(void) {
    ref_cass *c = calloc(1, sizeof *c);
    sb_put(&c->keyspace, "", 0);
    return c;
}
void ref_cass_free(ref_cass *c) {
    if (!c) return;
    free(c->keyspace.p);
    for (int i = 0; i < c->nbs; i++) free(c->bs[i].path);
    for (int i = 0; i < c->nbi; i++) { free(c->bi[i].path); free(c->bi[i].id); }
    free(c->bs); free(c->bi); free(c);
}

enum { Q_OK = 0, Q_INVALID = 1, Q_PANIC = 2 };

/* parseQuery (cassandraparser.go:368-469); on Q_OK *action / *table are
 * malloc'd strings. */
static int parse_query(ref_cass *st, const uint8_t *q, size_t qn, char **action, size_t *alen, char **table,
                       size_t *tlen) {
    while (qn > 0 && q[qn - 1] == ';') qn--;  /* strings.TrimRight(query, ";") */
    sbuf low = {0};
    go_to_lower(q, qn, &low);
    fields_t f = go_fields(low.p, low.n);
    free(low.p);
    int rc = Q_INVALID;
    sbuf act = {0}, tab = {0};
    for (int i = 0; i < f.n; i++)
        if (f.len[i] >= 2 && ((f.f[i][0] == '-' && f.f[i][1] == '-') || (f.f[i][0] == '/' && f.f[i][1] == '*') ||
                              (f.f[i][0] == '/' && f.f[i][1] == '/')))
            goto out;  /* comments: "Unable to safely parse query" */
    if (f.n < 2) goto out;
    sb_put(&act, f.f[0], f.len[0]);
    if (feq(&f, 0, "select") || feq(&f, 0, "delete")) {
        for (int i = 1; i < f.n; i++)
            if (feq(&f, i, "from")) {
                if (i + 1 >= f.n) { rc = Q_PANIC; goto out; }  /* fields[i+1]: index out of range */
                tab.n = 0;
                sb_put(&tab, f.f[i + 1], f.len[i + 1]);  /* strings.ToLower of a lowered token: itself */
            }
        if (tab.n == 0) goto out;
    } else if (feq(&f, 0, "insert")) {
        if (f.n < 3) goto out;
        sb_put(&tab, f.f[2], f.len[2]);
    } else if (feq(&f, 0, "update")) {
        sb_put(&tab, f.f[1], f.len[1]);
    } else if (feq(&f, 0, "use")) {
        size_t a = 0, b = f.len[1];  /* strings.Trim(fields[1], "\"\\'") */
        const char *k = f.f[1];
        while (a < b && (k[a] == '"' || k[a] == '\\' || k[a] == '\'')) a++;
        while (b > a && (k[b - 1] == '"' || k[b - 1] == '\\' || k[b - 1] == '\'')) b--;
        st->keyspace.n = 0;
        sb_put(&st->keyspace, k + a, b - a);
        sb_put(&tab, k + a, b - a);
    } else if (feq(&f, 0, "alter") || feq(&f, 0, "create") || feq(&f, 0, "drop") || feq(&f, 0, "truncate") ||
               feq(&f, 0, "list")) {
        sb_byte(&act, '-');
        sb_put(&act, f.f[1], f.len[1]);
        if (feq(&f, 1, "table") || feq(&f, 1, "keyspace")) {
            if (f.n < 3) goto out;
            sb_put(&tab, f.f[2], f.len[2]);
            if (feq(&f, 2, "if")) {
                if (!strcmp((char *)act.p, "create-table")) {
                    if (f.n < 6) goto out;
                    tab.n = 0;
                    sb_put(&tab, f.f[5], f.len[5]);
                } else if (!strcmp((char *)act.p, "drop-table") || !strcmp((char *)act.p, "drop-keyspace")) {
                    if (f.n < 5) goto out;
                    tab.n = 0;
                    sb_put(&tab, f.f[4], f.len[4]);
                }
            }
        }
        /* (the `action == "truncate" && len(fields) == 2` case of :447 can
         * never hold: action is "truncate-<fields[1]>" by then) */
        if (feq(&f, 1, "materialized")) sb_put(&act, "-view", 5);
        else if (feq(&f, 1, "custom")) { act.n = 0; sb_put(&act, "create-index", 12); }
    } else {
        goto out;
    }
    if (!tab.p) sb_put(&tab, "", 0);
    if (tab.n > 0 && !memchr(tab.p, '.', tab.n) && !(act.n == 3 && !memcmp(act.p, "use", 3))) {
        sbuf t2 = {0};
        sb_put(&t2, st->keyspace.p, st->keyspace.n);
        sb_byte(&t2, '.');
        sb_put(&t2, tab.p, tab.n);
        free(tab.p);
        tab = t2;
    }
    rc = Q_OK;
out:
    fields_free(&f);
    if (rc == Q_OK) { *action = (char *)act.p; *alen = act.n; *table = (char *)tab.p; *tlen = tab.n; }
    else { free(act.p); free(tab.p); }
    return rc;
}

static const char *kOpcodes[17] = {"error", "startup", "ready", "authenticate", "", "options", "supported", "query",
                                   "result", "prepare", "execute", "register", "event", "batch", "auth_challenge",
                                   "auth_response", "auth_success"};

static uint32_t be32(const uint8_t *b) { return (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3]; }
static uint16_t be16(const uint8_t *b) { return (uint16_t)(b[0] << 8 | b[1]); }

/* "/" + op + "/" + action + "/" + table, with its length */
static char *join_path(const char *op, const char *action, size_t alen, const char *table, size_t tlen,
                       size_t *plen) {
    const size_t ol = strlen(op);
    *plen = 3 + ol + alen + tlen;
    char *p = malloc(*plen + 1), *w = p;
    *w++ = '/'; memcpy(w, op, ol); w += ol;
    *w++ = '/'; memcpy(w, action, alen); w += alen;
    *w++ = '/'; memcpy(w, table, tlen); w += tlen;
    *w = 0;
    return p;
}
static char *bdup(const char *s, size_t n) {
    char *d = malloc(n + 1);
    memcpy(d, s, n);
    d[n] = 0;
    return d;
}

/* cassandraParseRequest on a complete frame; returns 0 (ok, *path set),
 * FILTEROP error code 2 (INVALID_FRAME_TYPE, *unprepared set for an EXECUTE
 * without a cached path) or -1 (panic).  The frame is data[0:fl] of the
 * bytes.Join buffer (:174, :211): a Go slice expression is bounded by the
 * slice's capacity, not its length, so data[9:13] and data[13:13+ql] read on
 * into the bytes that follow the frame in the buffer and panic only past its
 * end (cap = the buffer length n; bytes.Join of two or more slices allocates
 * exactly n -- a single slice is copied by append, whose capacity Go rounds
 * up to its allocator's size class; reads into that zeroed slack are not
 * restated: parity unpinned there, no reference test reaches it). */
static int parse_request(ref_cass *st, const uint8_t *d, uint32_t cap, char **path, size_t *plen, int *unprepared) {
    *path = NULL;
    *plen = 0;
    *unprepared = 0;
    if (d[0] & 0x80) return 2;
    if (d[1] & 0x01) return 2;
    const uint8_t op = d[4];
    const char *name = op < 17 ? kOpcodes[op] : "";
    if (op == 0x07 || op == 0x09) {
        if (cap < 13) return -1;
        const uint32_t ql = be32(d + 9);
        const uint32_t end = 13u + ql;  /* uint32 arithmetic, as in Go */
        if (end < 13u || end > cap) return -1;
        char *action, *table;
        size_t alen, tlen;
        int rc = parse_query(st, d + 13, ql, &action, &alen, &table, &tlen);
        if (rc == Q_PANIC) return -1;
        if (rc == Q_INVALID) return 2;
        *path = join_path(name, action, alen, table, tlen, plen);
        free(action); free(table);
        if (op == 0x09) {  /* stash, "prepare" -> "execute" (strings.Replace, first occurrence) */
            const uint16_t sid = be16(d + 2);
            char *x = malloc(*plen + 8);
            size_t xl = *plen, pre = 0;
            while (pre + 7 <= *plen && memcmp(*path + pre, "prepare", 7)) pre++;
            if (pre + 7 <= *plen) {
                memcpy(x, *path, pre);
                memcpy(x + pre, "execute", 7);
                memcpy(x + pre + 7, *path + pre + 7, *plen - pre - 7);
            } else {
                memcpy(x, *path, *plen);
            }
            x[xl] = 0;
            int k;
            for (k = 0; k < st->nbs; k++) if (st->bs[k].stream == sid) break;
            if (k == st->nbs) { st->bs = realloc(st->bs, (size_t)(st->nbs + 1) * sizeof *st->bs); st->bs[k].stream = sid; st->nbs++; }
            else free(st->bs[k].path);
            st->bs[k].path = x;
            st->bs[k].plen = xl;
        }
        return 0;
    }
    if (op == 0x0D) return -1;  /* Uint16(data[10:11]) */
    if (op == 0x0A) {
        if (cap < 11) return -1;
        const uint16_t il = be16(d + 9);
        if (11u + il > cap) return -1;
        for (int k = 0; k < st->nbi; k++)
            if (st->bi[k].idlen == il && !memcmp(st->bi[k].id, d + 11, il) && st->bi[k].plen) {
                *path = bdup(st->bi[k].path, st->bi[k].plen);
                *plen = st->bi[k].plen;
                return 0;
            }
        *unprepared = 1;
        return 2;
    }
    *path = malloc(strlen(name) + 2);
    strcpy(*path, "/"); strcat(*path, name);
    *plen = strlen(*path);
    return 0;
}

/* cassandraParseReply (:605-642) on a complete frame; -1 = panic.  n: the
 * capacity its slices are bounded by (the joined buffer's length, as in
 * parse_request). */
static int parse_reply(ref_cass *st, const uint8_t *d, uint32_t n) {
    if ((d[0] & 0x80) != 0x80) return 0;
    if (d[1] & 0x01) return 0;
    const uint16_t sid = be16(d + 2);
    if (d[4] != 0x08) return 0;
    if (n < 13) return -1;
    if (be32(d + 9) != 4) return 0;
    if (n < 15) return -1;
    const uint16_t il = be16(d + 13);
    if (15u + il > n) return -1;
    for (int k = 0; k < st->nbs; k++)
        if (st->bs[k].stream == sid && st->bs[k].plen) {
            int j;
            for (j = 0; j < st->nbi; j++) if (st->bi[j].idlen == il && !memcmp(st->bi[j].id, d + 15, il)) break;
            if (j == st->nbi) {
                st->bi = realloc(st->bi, (size_t)(st->nbi + 1) * sizeof *st->bi);
                st->bi[j].id = malloc(il + 1u); memcpy(st->bi[j].id, d + 15, il); st->bi[j].idlen = il;
                st->nbi++;
            } else free(st->bi[j].path);
            st->bi[j].path = bdup(st->bs[k].path, st->bs[k].plen);
            st->bi[j].plen = st->bs[k].plen;
        }
    return 0;
}

/* ---------------- policy ---------------- */
/* CassandraRule.Matches (:58-95) */
static int cass_rule_matches(const ref_mc_rule *r, const char *path, size_t plen) {
    /* strings.Split(path, "/") */
    int nparts = 1;
    for (size_t i = 0; i < plen; i++) if (path[i] == '/') nparts++;
    if (nparts <= 2) return 1;
    if (nparts < 4) return 0;
    const char *end = path + plen;
    const char *s1 = (const char *)memchr(path, '/', plen) + 1;
    const char *s2 = (const char *)memchr(s1, '/', (size_t)(end - s1)) + 1;  /* parts[2] */
    const char *s3 = (const char *)memchr(s2, '/', (size_t)(end - s2)) + 1;  /* parts[3] */
    const char *e3 = (const char *)memchr(s3, '/', (size_t)(end - s3));
    size_t l2 = (size_t)(s3 - 1 - s2), l3 = e3 ? (size_t)(e3 - s3) : (size_t)(end - s3);
    if (r->cass_action && (strlen(r->cass_action) != l2 || memcmp(r->cass_action, s2, l2))) return 0;
    if (l3 > 0 && r->cass_table && !ref_re_match(r->cass_table, (const uint8_t *)s3, l3, 0)) return 0;
    return 1;
}

static int cass_port_rules_match(const ref_port *pp, uint64_t remote, const char *path, size_t plen, int32_t *rule) {
    *rule = -1;
    if (!ref_px_have_l7(pp)) return 1;
    if (pp->nrules == 0) return 1;
    for (int r = 0; r < pp->nrules; r++) {
        const ref_pnp_rule *pr = &pp->rules[r];
        if (!ref_remote_ok(pr, remote)) continue;
        if (ref_px_nl7(pr) == 0) return 1;
        if (pr->l7type != L7T_L7 || !pr->l7proto || strcmp(pr->l7proto, "cassandra")) continue;
        for (int k = 0; k < pr->nl7; k++)
            if (cass_rule_matches(&pr->l7[k], path, plen)) { *rule = pr->l7[k].id; return 1; }
    }
    return 0;
}

/* Connection.Matches over the proxylib policymap */
static int cass_matches(const ref_policy *pol, const ref_conn_t *c, const char *path, size_t plen, int32_t *rule) {
    *rule = -1;
    if (c->policy < 0 || c->policy >= pol->np) return 0;
    const ref_port *ex, *wc;
    ref_port_lookup(&pol->p[c->policy], c->ingress, c->port, &ex, &wc);
    const ref_port *cands[2] = {ex, wc};
    for (int k = 0; k < 2; k++) {
        if (!cands[k] || !ref_px_installed(cands[k])) continue;
        if (cass_port_rules_match(cands[k], c->src_id, path, plen, rule)) return 1;
    }
    return 0;
}

/* One request-direction step of CassandraParser.OnData (:171-262) on the
 * joined input.  Returns the op (FILTEROP_*: 0 MORE, 1 PASS, 2 DROP, 4 ERROR;
 * -1 = panic) and *n; *rule = matched rule; *path_out (malloc'd, may be
 * NULL) = the request's path; *inject / *inject_len = what the parser
 * injects in the reply direction (unauthorized / unprepared message). */
int ref_cass_request(ref_cass *st, const ref_policy *pol, const ref_conn_t *c, const uint8_t *d, uint32_t n,
                     int64_t *nout, int32_t *rule, char **path_out, uint8_t *inject, uint32_t *inject_len) {
    *rule = -1;
    *inject_len = 0;
    if (path_out) *path_out = NULL;
    if (n < 9) { *nout = 9 - (int64_t)n; return 0; }
    const uint32_t rl = be32(d + 5);
    if (rl > 268435456u) { *nout = 3; return 4; }  /* ERROR_INVALID_FRAME_LENGTH */
    const int64_t missing = 9 + (int64_t)rl - (int64_t)n;
    if (missing > 0) { *nout = missing; return 0; }
    const uint32_t fl = 9 + rl;
    char *path;
    size_t plen;
    int unprepared;
    int rc = parse_request(st, d, n, &path, &plen, &unprepared);
    if (rc < 0) return -1;
    if (rc > 0) {
        if (unprepared) {  /* sendUnpreparedMsg (:586-601): header + [short bytes] id */
            static const uint8_t base[13] = {0, 0, 0, 0, 0, 0, 0, 0, 0x1a, 0, 0, 0x25, 0};
            memcpy(inject, base, 13);
            inject[0] = (uint8_t)(0x80 | (d[0] & 0x07));
            inject[2] = d[2]; inject[3] = d[3];
            const uint32_t il = be16(d + 9);
            memcpy(inject + 13, d + 9, 2 + il);
            *inject_len = 13 + 2 + il;
        }
        *nout = rc;
        return 4;
    }
    const int ok = cass_matches(pol, c, path, plen, rule);
    if (path_out) *path_out = path; else free(path);
    *nout = fl;
    if (ok) return 1;
    static const uint8_t unauth[35] = {0, 0, 0, 0, 0, 0, 0, 0, 0x1a, 0, 0, 0x21, 0, 0, 0x14, 'R', 'e', 'q',
                                       'u', 'e', 's', 't', ' ', 'U', 'n', 'a', 'u', 't', 'h', 'o', 'r', 'i', 'z',
                                       'e', 'd'};
    memcpy(inject, unauth, sizeof unauth);
    inject[0] = (uint8_t)(0x80 | (d[0] & 0x07));
    inject[2] = d[2]; inject[3] = d[3];
    *inject_len = sizeof unauth;
    *rule = -1;
    return 2;
}

/* Reply-direction step: MORE / ERROR framing as for requests, then
 * cassandraParseReply and PASS the frame; -1 = panic. */
int ref_cass_reply(ref_cass *st, const uint8_t *d, uint32_t n, int64_t *nout) {
    if (n < 9) { *nout = 9 - (int64_t)n; return 0; }
    const uint32_t rl = be32(d + 5);
    if (rl > 268435456u) { *nout = 3; return 4; }
    const int64_t missing = 9 + (int64_t)rl - (int64_t)n;
    if (missing > 0) { *nout = missing; return 0; }
    if (parse_reply(st, d, n) < 0) return -1;
    *nout = 9 + (int64_t)rl;
    return 1;
}

/* parseQuery as a test hook: action / table of a query under `keyspace`
 * (updated by a USE); returns Q_OK / Q_INVALID / Q_PANIC. */
int ref_cass_parse_query(ref_cass *st, const uint8_t *q, size_t n, char *action, size_t alen, char *table, size_t tlen) {
    char *a, *t;
    size_t al, tl;
    int rc = parse_query(st, q, n, &a, &al, &t, &tl);
    if (rc == Q_OK) {
        snprintf(action, alen, "%s", a);
        snprintf(table, tlen, "%s", t);
        free(a); free(t);
    }
    return rc;
}

const char *ref_cass_keyspace(const ref_cass *st) { return (const char *)st->keyspace.p; }

/* Batch-API verdict of one cassandra request (include/l7gpu.h): its
 * connection's keyspace is the one the earlier requests of the batch left in
 * `st` (ref_classify walks a batch's cassandra requests in order, one state
 * per connection); the batch API holds no prepared statements, so EXECUTE is
 * PARSE_ERROR / INVALID_FRAME_TYPE (the proxylib shim resolves it). */
void ref_cassandra_verdict(ref_cass *st, const ref_policy *pol, const ref_conn_t *c, const uint8_t *b, uint32_t len,
                           ref_out_t *o) {
    uint8_t inj[64 + 65536];
    uint32_t il;
    int64_t n;
    int32_t rule;
    const int op = ref_cass_request(st, pol, c, b, len, &n, &rule, NULL, inj, &il);
    o->rule = -1;
    if (op < 0) { o->verdict = L7_PARSE_ERROR; o->consumed = 0; }
    else if (op == 0) { o->verdict = L7_INCOMPLETE; o->consumed = (uint32_t)n; }
    else if (op == 4) { o->verdict = L7_PARSE_ERROR; o->consumed = (uint32_t)n; }
    else { o->verdict = op == 1 ? L7_ALLOW : L7_DENY; o->rule = rule; o->consumed = (uint32_t)n; }
}
