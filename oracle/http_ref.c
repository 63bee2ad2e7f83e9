/*
 * http_ref.c — TEST INFRASTRUCTURE ONLY (parity oracle, see l7ref.h).
 *
 * 1. HTTP/1 request framing: a byte-at-a-time restatement of the request
 *    grammar Envoy's HTTP/1 codec (http_parser, external, envoy/WORKSPACE:10)
 *    applies before the cilium.l7policy filter sees :method/:path/:authority.
 *    The exact contract (shared with the product) is in DESIGN.md §HTTP framing.
 * 2. Policy evaluation: envoy/cilium_network_policy.h
 *      NetworkPolicyMap::Allowed            :223-237
 *      PolicyInstance::Allowed              :198-203
 *      PortNetworkPolicy::Matches           :169-192  (exact port, then port 0,
 *                                                      no entry at all => ALLOW)
 *      PortNetworkPolicyRules::Matches      :128-146  (!have_http_rules => ALLOW,
 *                                                      empty => ALLOW)
 *      PortNetworkPolicyRule::Matches       :90-108   (remote in set, any http rule)
 *      HttpNetworkPolicyRule::Matches       :68-71    (HeaderUtility::matchHeaders, AND)
 *    remote id selection: envoy/cilium_l7policy.cc:144-150 (ingress: source
 *    identity, egress: destination identity).
 */
#include <ctype.h>
#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include "ref_internal.h"

typedef struct { int32_t noff, nlen, voff, vlen; } hdr_t;

static int is_tchar(uint8_t c) {
    if (c >= '0' && c <= '9') return 1;
    if ((c | 0x20) >= 'a' && (c | 0x20) <= 'z') return 1;
    return c && strchr("!#$%&'*+-.^_`|~", c) != NULL;
}

static int name_is(const uint8_t *buf, int32_t off, int32_t len, const char *lc) {
    size_t l = strlen(lc);
    if ((size_t)len != l) return 0;
    for (size_t i = 0; i < l; i++) if (tolower(buf[off + i]) != lc[i]) return 0;
    return 1;
}

typedef struct {
    ref_http_info_t info;
    hdr_t *h; int nh, caph;
} http_msg;

/* Sequential framing.  Returns status; on OK fills msg. */
static int http_frame(const uint8_t *b, uint32_t len, http_msg *m) {
    uint32_t i = 0;
    memset(&m->info, 0, sizeof m->info);
    m->info.method_off = m->info.path_off = m->info.host_off = -1;
    m->nh = 0;
#define NEED(k) do { if (i + (k) > len) return L7_INCOMPLETE; } while (0)
    /* method */
    uint32_t ms = i;
    for (;;) {
        NEED(1);
        uint8_t c = b[i];
        if (c == ' ') break;
        if (!is_tchar(c)) return L7_PARSE_ERROR;
        i++;
    }
    if (i == ms) return L7_PARSE_ERROR;
    m->info.method_off = (int32_t)ms; m->info.method_len = (int32_t)(i - ms);
    i++; /* SP */
    uint32_t ps = i;
    for (;;) {
        NEED(1);
        uint8_t c = b[i];
        if (c == ' ') break;
        if (c <= 0x20 || c == 0x7F) return L7_PARSE_ERROR;
        i++;
    }
    if (i == ps) return L7_PARSE_ERROR;
    m->info.path_off = (int32_t)ps; m->info.path_len = (int32_t)(i - ps);
    i++; /* SP */
    static const char V[] = "HTTP/";
    for (int k = 0; k < 5; k++) { NEED(1); if (b[i] != (uint8_t)V[k]) return L7_PARSE_ERROR; i++; }
    NEED(1); if (b[i] < '0' || b[i] > '9') return L7_PARSE_ERROR; i++;
    NEED(1); if (b[i] != '.') return L7_PARSE_ERROR; i++;
    NEED(1); if (b[i] < '0' || b[i] > '9') return L7_PARSE_ERROR; i++;
    NEED(1); if (b[i] != '\r') return L7_PARSE_ERROR; i++;
    NEED(1); if (b[i] != '\n') return L7_PARSE_ERROR; i++;

    int have_cl = 0, chunked = 0; uint64_t cl = 0;
    for (;;) {
        NEED(1);
        uint8_t c = b[i];
        if (c == '\r') {
            i++; NEED(1); if (b[i] != '\n') return L7_PARSE_ERROR; i++;
            break; /* end of headers */
        }
        if (c == ' ' || c == '\t') return L7_PARSE_ERROR; /* obs-fold */
        uint32_t ns = i;
        for (;;) {
            NEED(1);
            c = b[i];
            if (c == ':') break;
            if (!is_tchar(c)) return L7_PARSE_ERROR;
            i++;
        }
        if (i == ns) return L7_PARSE_ERROR;
        uint32_t ne = i;
        i++; /* ':' */
        for (;;) { NEED(1); if (b[i] == ' ' || b[i] == '\t') i++; else break; }
        uint32_t vs = i, ve = i;
        for (;;) {
            NEED(1);
            c = b[i];
            if (c == '\r') break;
            if ((c < 0x20 && c != '\t') || c == 0x7F) return L7_PARSE_ERROR;
            i++;
            if (c != ' ' && c != '\t') ve = i;
        }
        i++; NEED(1); if (b[i] != '\n') return L7_PARSE_ERROR; i++;
        /* line complete */
        if (name_is(b, (int32_t)ns, (int32_t)(ne - ns), "content-length")) {
            if (have_cl) return L7_PARSE_ERROR;
            have_cl = 1;
            if (ve == vs || ve - vs > 10) return L7_PARSE_ERROR;
            cl = 0;
            for (uint32_t k = vs; k < ve; k++) { if (b[k] < '0' || b[k] > '9') return L7_PARSE_ERROR; cl = cl * 10 + (b[k] - '0'); }
        } else if (name_is(b, (int32_t)ns, (int32_t)(ne - ns), "transfer-encoding")) {
            /* http_parser (Envoy's HTTP/1 codec at the pinned commit) sets
             * F_CHUNKED when a Transfer-Encoding value is "chunked"; any
             * other value leaves the body framed by Content-Length. */
            if (name_is(b, (int32_t)vs, (int32_t)(ve - vs), "chunked")) chunked = 1;
        }
        if (m->nh == m->caph) { m->caph = m->caph ? 2 * m->caph : 16; m->h = realloc(m->h, sizeof(hdr_t) * m->caph); }
        m->h[m->nh++] = (hdr_t){(int32_t)ns, (int32_t)(ne - ns), (int32_t)vs, (int32_t)(ve - vs)};
        if (m->info.host_off < 0 && name_is(b, (int32_t)ns, (int32_t)(ne - ns), "host")) {
            m->info.host_off = (int32_t)vs; m->info.host_len = (int32_t)(ve - vs);
        }
    }
    m->info.nheaders = m->nh;
    if (chunked) {
        /* chunked body: chunk = 1*HEXDIG [";" ext] CRLF data CRLF,
         * last chunk size 0, then trailer lines up to an empty line */
        for (;;) {
            uint32_t st = i;
            uint64_t size = 0;
            for (;;) {
                NEED(1);
                uint8_t c = b[i];
                int d = c >= '0' && c <= '9' ? c - '0' : (c | 0x20) >= 'a' && (c | 0x20) <= 'f' ? (c | 0x20) - 'a' + 10 : -1;
                if (d < 0) break;
                size = size * 16 + (uint64_t)d;
                if (size > 0xFFFFFFFFull) return L7_PARSE_ERROR;
                i++;
            }
            if (i == st) return L7_PARSE_ERROR;
            if (b[i] == ';') {
                i++;
                for (;;) { NEED(1); if (b[i] == '\r' || b[i] == '\n') break; i++; }
            }
            if (b[i] != '\r') return L7_PARSE_ERROR;
            i++; NEED(1); if (b[i] != '\n') return L7_PARSE_ERROR; i++;
            if (size == 0) break;
            if ((uint64_t)i + size > 0xFFFFFFFFull) return L7_PARSE_ERROR;
            if ((uint64_t)i + size > len) return L7_INCOMPLETE;
            i += (uint32_t)size;
            NEED(1); if (b[i] != '\r') return L7_PARSE_ERROR; i++;
            NEED(1); if (b[i] != '\n') return L7_PARSE_ERROR; i++;
        }
        for (;;) {  /* trailer section */
            NEED(1);
            if (b[i] == '\r') { i++; NEED(1); if (b[i] != '\n') return L7_PARSE_ERROR; i++; break; }
            for (;;) { NEED(1); if (b[i] == '\r') break; if (b[i] == '\n') return L7_PARSE_ERROR; i++; }
            i++; NEED(1); if (b[i] != '\n') return L7_PARSE_ERROR; i++;
        }
        m->info.consumed = i;
        return L7_ALLOW; /* "ok" */
    }
    uint64_t total = (uint64_t)i + cl;
    if (total > 0xFFFFFFFFull) return L7_PARSE_ERROR;
    if (total > len) return L7_INCOMPLETE;
    m->info.consumed = (uint32_t)total;
    return L7_ALLOW; /* "ok" */
#undef NEED
}

int ref_http_parse(const uint8_t *buf, uint32_t len, ref_http_info_t *info) {
    http_msg m; memset(&m, 0, sizeof m);
    int st = http_frame(buf, len, &m);
    m.info.status = st;
    *info = m.info;
    free(m.h);
    return st;
}

/* HeaderMap::get(name): pseudo headers, else first regular header with that
 * lower-cased name.  Host is only visible as :authority;
 * x-envoy-original-dst-host is removed by the filter (cilium_l7policy.cc:128). */
static int hdr_get(const uint8_t *b, const http_msg *m, const char *name, size_t nl, int32_t *voff, int32_t *vlen) {
    if (nl == 7 && !memcmp(name, ":method", 7)) { *voff = m->info.method_off; *vlen = m->info.method_len; return 1; }
    if (nl == 5 && !memcmp(name, ":path", 5)) { *voff = m->info.path_off; *vlen = m->info.path_len; return 1; }
    if (nl == 10 && !memcmp(name, ":authority", 10)) {
        if (m->info.host_off < 0) return 0;
        *voff = m->info.host_off; *vlen = m->info.host_len; return 1;
    }
    if (nl == 4 && !memcmp(name, "host", 4)) return 0;
    if (nl == 25 && !memcmp(name, "x-envoy-original-dst-host", 25)) return 0;
    for (int k = 0; k < m->nh; k++) {
        if ((size_t)m->h[k].nlen != nl) continue;
        int eq = 1;
        for (size_t q = 0; q < nl; q++) if (tolower(b[m->h[k].noff + q]) != (unsigned char)name[q]) { eq = 0; break; }
        if (eq) { *voff = m->h[k].voff; *vlen = m->h[k].vlen; return 1; }
    }
    return 0;
}

/* StringUtil::atol (Envoy): strtoll over the whole string, base 10 */
static int env_atol(const uint8_t *s, int32_t n, int64_t *out) {
    if (n <= 0) return 0;
    char tmp[64];
    if (n > 63) return 0;
    memcpy(tmp, s, (size_t)n); tmp[n] = 0;
    if (memchr(tmp, 0, (size_t)n)) return 0;
    char *end; errno = 0;
    long long v = strtoll(tmp, &end, 10);
    if (*end != 0 || errno) return 0;
    *out = v;
    return 1;
}

/* HeaderUtility::matchHeaders(headers, header_data) */
static int hmatch(const uint8_t *b, const http_msg *m, const ref_hmatch *h) {
    int32_t vo, vl;
    if (!hdr_get(b, m, h->name, h->namelen, &vo, &vl)) return 0;
    const uint8_t *v = b + vo;
    int r = 0;
    switch (h->type) {
    case HM_EXACT: r = h->vlen == 0 || ((size_t)vl == h->vlen && !memcmp(v, h->value, h->vlen)); break;
    case HM_REGEX: r = ref_re_match(h->re, v, (size_t)vl, 1); break;
    case HM_PRESENT: r = 1; break;
    case HM_PREFIX: r = (size_t)vl >= h->vlen && !memcmp(v, h->value, h->vlen); break;
    case HM_SUFFIX: r = (size_t)vl >= h->vlen && !memcmp(v + vl - h->vlen, h->value, h->vlen); break;
    case HM_RANGE: { int64_t x; r = env_atol(v, vl, &x) && x >= h->rstart && x < h->rend; break; }
    }
    return r != h->invert;
}

/* PortNetworkPolicyRules::Matches; returns 1 = allow (rule id in *rule), 0 = no */
static int port_rules_match(const ref_port *pp, uint64_t remote, const uint8_t *b, const http_msg *m, int32_t *rule) {
    *rule = -1;
    if (!pp->has_http) return 1;
    if (pp->nrules == 0) return 1;
    for (int r = 0; r < pp->nrules; r++) {
        const ref_pnp_rule *pr = &pp->rules[r];
        if (!ref_remote_ok(pr, remote)) continue;
        if (pr->l7type == L7T_HTTP && pr->nhttp > 0) {
            for (int k = 0; k < pr->nhttp; k++) {
                const ref_http_rule *hr = &pr->http[k];
                int all = 1;
                for (int q = 0; q < hr->n && all; q++) all = hmatch(b, m, &hr->m[q]);
                if (all) { *rule = hr->id; return 1; }
            }
            continue;
        }
        return 1; /* empty set matches any payload */
    }
    return 0;
}

void ref_http_verdict(const ref_policy *pol, const ref_conn_t *c, const uint8_t *buf, uint32_t len, ref_out_t *o) {
    http_msg m; memset(&m, 0, sizeof m);
    int st = http_frame(buf, len, &m);
    o->rule = -1; o->consumed = 0;
    if (st != L7_ALLOW) { o->verdict = (uint8_t)st; free(m.h); return; }
    o->consumed = m.info.consumed;
    if (c->policy < 0 || c->policy >= pol->np) { o->verdict = L7_DENY; free(m.h); return; }
    const ref_netpolicy *np = &pol->p[c->policy];
    if (c->flags & L7_CONN_PROXYLIB) {
        /* the proxylib "http" parser: Instance.PolicyMatches -> PortNetworkPolicies.Matches
         * (proxylib/proxylib/policymap.go:150-236): SrcId is the remote in both
         * directions (connection.go:176-179), installed entries only, no entry => drop */
        const ref_port *ex, *wc;
        ref_port_lookup(np, c->ingress, c->port, &ex, &wc);
        const ref_port *cands[2] = {ex, wc};
        o->verdict = L7_DENY;
        for (int k = 0; k < 2; k++) {
            const ref_port *pp = cands[k];
            if (!pp || !ref_px_installed(pp)) continue;
            if (!ref_px_have_l7(pp) || pp->nrules == 0) { o->verdict = L7_ALLOW; break; }
            int hit = 0;
            for (int r = 0; r < pp->nrules && !hit; r++) {
                const ref_pnp_rule *pr = &pp->rules[r];
                if (!ref_remote_ok(pr, c->src_id)) continue;
                if (ref_px_nl7(pr) == 0) { hit = 1; break; }
                if (pr->l7type != L7T_HTTP) continue;
                for (int q = 0; q < pr->nhttp; q++) {
                    const ref_http_rule *hr = &pr->http[q];
                    int all = 1;
                    for (int j = 0; j < hr->n && all; j++) all = hmatch(buf, &m, &hr->m[j]);
                    if (all) { hit = 1; o->rule = hr->id; break; }
                }
            }
            if (hit) { o->verdict = L7_ALLOW; break; }
        }
        free(m.h);
        return;
    }
    uint64_t remote = c->ingress ? c->src_id : c->dst_id;
    const ref_port *ex, *wc;
    ref_port_lookup(np, c->ingress, c->port, &ex, &wc);
    int found = 0;
    int32_t rule;
    const ref_port *cands[2] = {ex, wc};
    for (int k = 0; k < 2; k++) {
        if (!cands[k]) continue;
        if (port_rules_match(cands[k], remote, buf, &m, &rule)) { o->verdict = L7_ALLOW; o->rule = rule; free(m.h); return; }
        found = 1;
    }
    o->verdict = found ? L7_DENY : L7_ALLOW;
    free(m.h);
}
