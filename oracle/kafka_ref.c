/*
 * kafka_ref.c — TEST INFRASTRUCTURE ONLY (parity oracle, see l7ref.h).
 *
 * Sequential restatement of the reference's Kafka request path:
 *   vendor/github.com/optiopay/kafka/proto/messages.go
 *     ReadReq                 :124-165   (frame: int32 size, int16 kind)
 *     readMessageSet          :363-494   (LimitReader, CRC32-IEEE, stop w/o drain)
 *     ReadMetadataReq         :504-537   ReadFetchReq        :767-824
 *     ReadConsumerMetadataReq :1033-1054 ReadOffsetCommitReq :1173-1228
 *     ReadOffsetFetchReq      :1389-1430 ReadProduceReq      :1591-1647
 *     ReadOffsetReq           :1810-1858
 *   vendor/.../proto/serialization.go decoder :19-203 (io.ReadFull semantics)
 *   vendor/.../proto/utils.go maxParseBufSize = 6,553,500        :9-24
 *   pkg/kafka/request.go  ReadRequest :186-229, GetTopics :88-153
 *   pkg/kafka/policy.go   isTopicAPIKey :27-52, matchNonTopicRequests :54-70,
 *                         ruleMatches :144-195, MatchesRule :200-225
 *   pkg/policy/api/kafka.go CheckAPIKeyRole :248-261, GetAPIVersion :265-271
 *   pkg/proxy/kafka.go canAccess :117-153 (rules.Kafka == nil => deny)
 * Compressed messages (gzip / snappy, messages.go:460-489) are decoded by
 * kafka_inflate.c and their inner message set read recursively; any decode
 * error fails the request (parity for these is pinned by fixtures built with
 * Python's zlib/gzip and a test snappy encoder, not by reference vectors).
 */
#include <stdlib.h>
#include <string.h>
#include "ref_internal.h"

#define MAX_PARSE_BUF 6553500
enum { KE_NONE = 0, KE_EOF, KE_UNEXPECTED_EOF, KE_OTHER };

typedef struct { const uint8_t *b; size_t pos, end; } kbuf;            /* bytes.Buffer */
typedef struct { kbuf *r; int64_t limit; int err; } kdec;               /* decoder (+LimitReader) */

/* io.ReadFull(r, buf[:n]) */
static int kread(kdec *d, size_t n, size_t *at) {
    size_t avail = d->r->end - d->r->pos;
    if (d->limit >= 0 && (size_t)d->limit < avail) avail = (size_t)d->limit;
    *at = d->r->pos;
    if (n == 0) return KE_NONE;
    if (avail == 0) return KE_EOF;
    size_t take = avail < n ? avail : n;
    d->r->pos += take;
    if (d->limit >= 0) d->limit -= (int64_t)take;
    return take < n ? KE_UNEXPECTED_EOF : KE_NONE;
}
static uint64_t be(const uint8_t *p, int n) { uint64_t v = 0; for (int i = 0; i < n; i++) v = (v << 8) | p[i]; return v; }
static int64_t dec_int(kdec *d, int n) {
    if (d->err) return 0;
    size_t at; int e = kread(d, (size_t)n, &at);
    if (e) { d->err = e; return 0; }
    uint64_t v = be(d->r->b + at, n);
    switch (n) { case 1: return (int8_t)v; case 2: return (int16_t)v; case 4: return (int32_t)v; default: return (int64_t)v; }
}
/* DecodeString: returns offset (into the buffer) / len; len<1 => "" */
static void dec_string(kdec *d, int32_t *off, int32_t *len) {
    *off = 0; *len = 0;
    if (d->err) return;
    int16_t sl = (int16_t)dec_int(d, 2);
    if (d->err) return;
    if (sl < 1) return;
    size_t at; int e = kread(d, (size_t)sl, &at);
    if (e) { d->err = e; return; }
    *off = (int32_t)at; *len = sl;
}
/* DecodeArrayLen(nullable): returns -1 null, >=0 len; *bad set on error */
static int64_t dec_arraylen(kdec *d, int nullable, int *bad) {
    int64_t l = (int32_t)dec_int(d, 4);
    *bad = 0;
    if (l < 0) { if (nullable) return -1; *bad = 1; return 0; }
    if (l > MAX_PARSE_BUF) { *bad = 1; return 0; }
    return l;
}
/* DecodeBytes: the bytes' position (len 0: nil) */
static void dec_bytes_at(kdec *d, size_t *at, size_t *len) {
    *at = 0; *len = 0;
    if (d->err) return;
    int32_t sl = (int32_t)dec_int(d, 4);
    if (d->err) return;
    if (sl < 1) return;
    if (sl > MAX_PARSE_BUF) { d->err = KE_OTHER; return; }
    int e = kread(d, (size_t)sl, at);
    if (e) d->err = e;
    else *len = (size_t)sl;
}
static void dec_bytes(kdec *d) { size_t a, l; dec_bytes_at(d, &a, &l); }

static uint32_t crc_table[256];
static void crc_init(void) {
    static int done = 0;
    if (done) return;
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crc_table[i] = c;
    }
    done = 1;
}
static uint32_t crc32_ieee(const uint8_t *p, size_t n) {
    uint32_t c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; i++) c = crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return c ^ 0xFFFFFFFFu;
}

int ref_gunzip(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *outlen);
int ref_unsnappy(const uint8_t *b, size_t n, uint8_t *out, size_t cap, size_t *outlen);

/* readMessageSet; returns 0 ok, -1 error */
static int read_message_set(kbuf *r, int32_t size, int16_t version) {
    if (size < 0) return 0;
    if (size > MAX_PARSE_BUF) return -1;
    kdec dec = {r, size, 0};
    for (;;) {
        (void)dec_int(&dec, 8); /* offset */
        if (dec.err) return 0;  /* EOF / ErrUnexpectedEOF => return set, nil */
        int32_t msize = (int32_t)dec_int(&dec, 4);
        if (dec.err) return 0;
        if (msize <= 0) return 0;
        if (msize > MAX_PARSE_BUF) return -1;
        size_t at; int e = kread(&dec, (size_t)msize, &at);
        if (e) return 0;
        kbuf mb = {r->b + at, 0, (size_t)msize};
        kdec md = {&mb, -1, 0};
        uint32_t crc = (uint32_t)dec_int(&md, 4);
        if (msize <= 4) return 0; /* MessageSet with no payload: append, return */
        if (crc != crc32_ieee(r->b + at + 4, (size_t)msize - 4)) return 0; /* stop, no drain */
        (void)dec_int(&md, 1); /* magic */
        int8_t attr = (int8_t)dec_int(&md, 1);
        if (version >= 1) (void)dec_int(&md, 8); /* timestamp (keyed on API version) */
        int codec = attr & 3;
        if (codec == 0) {
            dec_bytes(&md); dec_bytes(&md);
            if (md.err) return -1;
        } else if (codec == 1 || codec == 2) {
            size_t vat, vlen;
            dec_bytes(&md); dec_bytes_at(&md, &vat, &vlen);
            if (md.err) return -1;
            uint8_t *dec = malloc(MAX_PARSE_BUF + 1);
            size_t dlen = 0;
            const uint8_t *val = r->b + at + vat;
            int bad = codec == 1 ? ref_gunzip(val, vlen, dec, MAX_PARSE_BUF, &dlen)
                                 : ref_unsnappy(val, vlen, dec, MAX_PARSE_BUF, &dlen);
            if (!bad) {
                kbuf inner = {dec, 0, dlen};
                bad = read_message_set(&inner, (int32_t)dlen, version);
            }
            free(dec);
            if (bad) return -1;
        } else {
            return 0; /* `return nil, err` with err == nil */
        }
    }
}

typedef struct { int32_t off, len; } span_t;
typedef struct {
    int16_t kind, version;
    int typed;       /* 0 = nil request, 1 = typed (has ClientID), 2 = ConsumerMetadata */
    int32_t client_off, client_len;
    span_t *topics; int ntopics, cap;
    int topics_nil;
} kreq;

static void add_topic(kreq *q, int32_t off, int32_t len) {
    if (q->ntopics == q->cap) { q->cap = q->cap ? 2 * q->cap : 8; q->topics = realloc(q->topics, sizeof(span_t) * q->cap); }
    q->topics[q->ntopics++] = (span_t){off, len};
}

/* decoders: return 0 ok, -1 error */
static int read_body(kreq *q, const uint8_t *raw, size_t rawlen) {
    kbuf buf = {raw, 0, rawlen};
    kdec d = {&buf, -1, 0};
    int bad;
    (void)dec_int(&d, 4); (void)dec_int(&d, 2);
    int16_t ver = (int16_t)dec_int(&d, 2);
    (void)dec_int(&d, 4);
    dec_string(&d, &q->client_off, &q->client_len);
    int64_t nt, np;
    switch (q->kind) {
    case 0: /* Produce */
        if (ver >= 3) { int32_t o, l; dec_string(&d, &o, &l); }
        (void)dec_int(&d, 2); (void)dec_int(&d, 4);
        nt = dec_arraylen(&d, 0, &bad); if (bad) return -1;
        for (int64_t t = 0; t < nt; t++) {
            int32_t o, l; dec_string(&d, &o, &l);
            if (d.err) break; /* every later read is a no-op; result is an error */
            add_topic(q, o, l);
            np = dec_arraylen(&d, 0, &bad); if (bad) return -1;
            for (int64_t p = 0; p < np; p++) {
                (void)dec_int(&d, 4); if (d.err) return -1;
                int32_t ss = (int32_t)dec_int(&d, 4); if (d.err) return -1;
                int e = read_message_set(&buf, ss, ver);
                if (e) return e;
            }
        }
        break;
    case 1: /* Fetch */
        (void)dec_int(&d, 4); (void)dec_int(&d, 4); (void)dec_int(&d, 4);
        if (ver >= 3) (void)dec_int(&d, 4);
        if (ver >= 4) (void)dec_int(&d, 1);
        nt = dec_arraylen(&d, 0, &bad); if (bad) return -1;
        for (int64_t t = 0; t < nt; t++) {
            int32_t o, l; dec_string(&d, &o, &l); add_topic(q, o, l);
            np = dec_arraylen(&d, 0, &bad); if (bad) return -1;
            for (int64_t p = 0; p < np; p++) {
                (void)dec_int(&d, 4); (void)dec_int(&d, 8);
                if (ver >= 5) (void)dec_int(&d, 8);
                (void)dec_int(&d, 4);
                if (d.err) break; /* every later read is a no-op */
            }
            if (d.err) break;
        }
        break;
    case 2: /* Offset */
        (void)dec_int(&d, 4);
        if (ver >= 2) (void)dec_int(&d, 1);
        nt = dec_arraylen(&d, 0, &bad); if (bad) return -1;
        for (int64_t t = 0; t < nt; t++) {
            int32_t o, l; dec_string(&d, &o, &l); add_topic(q, o, l);
            np = dec_arraylen(&d, 0, &bad); if (bad) return -1;
            for (int64_t p = 0; p < np; p++) {
                (void)dec_int(&d, 4); (void)dec_int(&d, 8);
                if (ver == 0) (void)dec_int(&d, 4);
                if (d.err) break;
            }
            if (d.err) break;
        }
        break;
    case 3: /* Metadata */
        nt = dec_arraylen(&d, 1, &bad); if (bad) return -1;
        if (nt < 0) q->topics_nil = 1;
        for (int64_t t = 0; t < nt; t++) {
            int32_t o, l; dec_string(&d, &o, &l); add_topic(q, o, l);
            if (d.err) break;
        }
        if (ver >= 4) (void)dec_int(&d, 1);
        break;
    case 8: { /* OffsetCommit */
        int32_t o, l; dec_string(&d, &o, &l);
        if (ver >= 1) { (void)dec_int(&d, 4); dec_string(&d, &o, &l); }
        if (ver >= 2) (void)dec_int(&d, 8);
        nt = dec_arraylen(&d, 0, &bad); if (bad) return -1;
        for (int64_t t = 0; t < nt; t++) {
            dec_string(&d, &o, &l); add_topic(q, o, l);
            np = dec_arraylen(&d, 0, &bad); if (bad) return -1;
            for (int64_t p = 0; p < np; p++) {
                (void)dec_int(&d, 4); (void)dec_int(&d, 8);
                if (ver == 1) (void)dec_int(&d, 8);
                int32_t o2, l2; dec_string(&d, &o2, &l2);
                if (d.err) break;
            }
            if (d.err) break;
        }
        break;
    }
    case 9: { /* OffsetFetch */
        int32_t o, l; dec_string(&d, &o, &l);
        nt = dec_arraylen(&d, 1, &bad); if (bad) return -1;
        if (nt < 0) q->topics_nil = 1;
        for (int64_t t = 0; t < nt; t++) {
            dec_string(&d, &o, &l); add_topic(q, o, l);
            np = dec_arraylen(&d, 0, &bad); if (bad) return -1;
            for (int64_t p = 0; p < np; p++) { (void)dec_int(&d, 4); if (d.err) break; }
            if (d.err) break;
        }
        break;
    }
    case 10: { /* ConsumerMetadata */
        int32_t o, l; dec_string(&d, &o, &l);
        if (ver >= 1) (void)dec_int(&d, 1);
        break;
    }
    default:
        return 0;
    }
    return d.err ? -1 : 0;
}

static int is_topic_api_key(int k) {
    switch (k) {
    case 0: case 1: case 2: case 3: case 4: case 5: case 6: case 8: case 9: case 19: case 20:
    case 21: case 23: case 24: case 27: case 28: case 34: case 35: case 37: return 1;
    }
    return 0;
}

static int rule_matches(const kreq *q, const uint8_t *raw, const ref_kafka_rule *r) {
    if (!r->any_key) {
        if (q->kind < 0 || q->kind > 63 || !((r->keymask >> q->kind) & 1)) return 0;
    }
    if (r->has_version && r->version != q->version) return 0;
    if (r->topiclen == 0 && r->clientlen == 0) return 1;
    switch (q->typed) {
    case 1:
        if (r->clientlen != 0 && (r->clientlen != (size_t)q->client_len || memcmp(r->client, raw + q->client_off, r->clientlen))) return 0;
        return 1;
    case 2: return 1;
    default: return !(r->topiclen != 0 && is_topic_api_key(q->kind));
    }
}

/* MatchesRule over the rule list (pointers to rules); returns 1 allow */
static int matches_rule(const kreq *q, const uint8_t *raw, const ref_kafka_rule **rules, int nr, int32_t *rid) {
    int nt = q->ntopics;
    /* reqTopicsMap: distinct topic names still to be covered */
    int *pending = calloc((size_t)(nt ? nt : 1), sizeof(int));
    int npend = 0;
    for (int i = 0; i < nt; i++) {
        int dup = 0;
        for (int j = 0; j < i; j++)
            if (q->topics[j].len == q->topics[i].len && !memcmp(raw + q->topics[j].off, raw + q->topics[i].off, (size_t)q->topics[i].len)) { dup = 1; break; }
        pending[i] = !dup;
        npend += !dup;
    }
    int res = 0;
    for (int k = 0; k < nr && !res; k++) {
        const ref_kafka_rule *r = rules[k];
        if (r->topiclen == 0 || nt == 0) {
            if (rule_matches(q, raw, r)) { res = 1; *rid = r->id; }
        } else {
            int hit = -1;
            for (int i = 0; i < nt; i++)
                if (pending[i] && (size_t)q->topics[i].len == r->topiclen && !memcmp(raw + q->topics[i].off, r->topic, r->topiclen)) { hit = i; break; }
            if (hit >= 0 && rule_matches(q, raw, r)) {
                pending[hit] = 0; npend--;
                if (npend == 0) { res = 1; *rid = r->id; }
            }
        }
    }
    free(pending);
    return res;
}

void ref_kafka_verdict(const ref_policy *pol, const ref_conn_t *c, const uint8_t *buf, uint32_t len, ref_out_t *o) {
    crc_init();
    o->rule = -1; o->consumed = 0;
    /* proto.ReadReq */
    if (len < 4) { o->verdict = L7_INCOMPLETE; return; }
    int32_t size = (int32_t)be(buf, 4);
    if (size <= 0) { o->verdict = L7_PARSE_ERROR; return; }
    if (len < 6) { o->verdict = L7_INCOMPLETE; return; }
    int16_t kind = (int16_t)be(buf + 4, 2);
    if ((int64_t)size + 4 > MAX_PARSE_BUF) { o->verdict = L7_PARSE_ERROR; return; }
    size_t rawlen = (size_t)size + 4;
    if (rawlen > len) { o->verdict = L7_INCOMPLETE; return; }
    /* the bytes the reference actually sees: the kind is re-written only when
     * it was part of the message (len(b) >= 6); for size < 2 the stream would
     * also be desynchronised, but rawlen < 12 is an error anyway. */
    if (rawlen < 12) { o->verdict = L7_PARSE_ERROR; return; }
    kreq q; memset(&q, 0, sizeof q);
    q.kind = kind;
    q.version = (int16_t)be(buf + 6, 2);
    int e = 0;
    switch (kind) {
    case 0: case 1: case 2: case 3: case 8: case 9: q.typed = 1; e = read_body(&q, buf, rawlen); break;
    case 10: q.typed = 2; e = read_body(&q, buf, rawlen); break;
    default: q.typed = 0; break;
    }
    if (e == -1) { o->verdict = L7_PARSE_ERROR; free(q.topics); return; }
    if (q.typed != 1) q.ntopics = 0; /* GetTopics: nil for ConsumerMetadata / unknown */

    /* canAccess: GetRelevantRules(source identity) */
    o->verdict = L7_DENY;
    if (c->policy < 0 || c->policy >= pol->np) { o->consumed = (uint32_t)rawlen; free(q.topics); return; }
    const ref_netpolicy *np = &pol->p[c->policy];
    const ref_port *ex, *wc;
    ref_port_lookup(np, c->ingress, c->port, &ex, &wc);
    const ref_kafka_rule **rules = NULL; int nr = 0, cap = 0, any = 0;
    static const ref_kafka_rule WILDCARD = {0, 1, 0, 0, NULL, 0, NULL, 0, -1};
    const ref_port *cands[2] = {ex, wc};
    const int px = (c->flags & L7_CONN_PROXYLIB) != 0;
    for (int k = 0; k < 2; k++) {
        const ref_port *pp = cands[k];
        if (!pp) continue;
        if (px) {
            /* the proxylib "kafka" parser: installed entries only; a port without
             * L7 rules or a group with an empty L7 set admits everything; the
             * groups' Kafka rules form one MatchesRule list */
            if (!ref_px_installed(pp)) continue;
            int all_ok = !ref_px_have_l7(pp) || pp->nrules == 0;
            for (int r = 0; r < pp->nrules || all_ok; r++) {
                const ref_pnp_rule *pr = all_ok ? NULL : &pp->rules[r];
                if (pr && !ref_remote_ok(pr, c->src_id)) continue;
                int wild = all_ok || ref_px_nl7(pr) == 0;
                int add = wild ? 1 : (pr->l7type == L7T_KAFKA ? pr->nkafka : 0);
                if (nr + add > cap) { cap = (nr + add) * 2 + 8; rules = realloc(rules, sizeof(*rules) * cap); }
                if (wild) { rules[nr++] = &WILDCARD; any = 1; }
                else if (pr->l7type == L7T_KAFKA) { for (int i = 0; i < pr->nkafka; i++) rules[nr++] = &pr->kafka[i]; any = 1; }
                if (all_ok) break;
            }
            continue;
        }
        for (int r = 0; r < pp->nrules; r++) {
            const ref_pnp_rule *pr = &pp->rules[r];
            if (!ref_remote_ok(pr, c->src_id)) continue;
            int add = pr->l7type == L7T_KAFKA ? pr->nkafka : (pr->l7type == L7T_NONE ? 1 : 0);
            if (nr + add > cap) { cap = (nr + add) * 2 + 8; rules = realloc(rules, sizeof(*rules) * cap); }
            if (pr->l7type == L7T_KAFKA) { for (int i = 0; i < pr->nkafka; i++) rules[nr++] = &pr->kafka[i]; any = 1; }
            else if (pr->l7type == L7T_NONE) { rules[nr++] = &WILDCARD; any = 1; } /* L3-only: L7 wildcard */
        }
    }
    if (any) {
        int32_t rid = -1;
        if (matches_rule(&q, buf, rules, nr, &rid)) { o->verdict = L7_ALLOW; o->rule = rid; }
    }
    o->consumed = (uint32_t)rawlen; /* consumed is reported for ALLOW/DENY only */
    free(rules);
    free(q.topics);
}
