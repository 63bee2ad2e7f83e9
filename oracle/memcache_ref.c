/*
 * memcache_ref.c — TEST INFRASTRUCTURE ONLY (parity oracle, see l7ref.h).
 *
 * Request-side memcached verdict for one buffer, restating:
 *   proxylib/memcached/parser.go:186-202   text / binary dispatch on the first byte
 *   proxylib/memcached/text/parser.go:72-198, 275-296   text framing (first CRLF,
 *                                          bytes.Fields tokens, command classes,
 *                                          storage data-block length)
 *   proxylib/memcached/binary/parser.go:58-139, 174-191 24-byte header framing
 *   proxylib/memcached/parser.go:47-110    Rule.Matches (empty / command or opcode /
 *                                          keyExact > keyPrefix > keyRegex, all keys)
 *   proxylib/proxylib/policymap.go:91-236  PortNetworkPolicyRule(s).Matches and
 *                                          PortNetworkPolicies.Matches (exact port,
 *                                          then port 0, none => deny); remote = SrcId
 *                                          (proxylib/proxylib/connection.go:176-179)
 * Batch conventions (shared with the product): PASS/DROP =>
 * ALLOW/DENY with consumed = the frame length proxylib returns (it may exceed
 * the buffer); MORE n => INCOMPLETE with consumed = n (NOP => 0); a Go panic
 * or ERROR, 0 => PARSE_ERROR with consumed 0; the binary parser's ERROR,
 * INVALID_FRAME_TYPE => PARSE_ERROR with consumed 2; frame lengths outside
 * 1..2^32-1 => PARSE_ERROR.  The connection's flags carry the parser chosen
 * by its first byte (0 = not yet: this buffer's first byte decides).
 */
#include <stdlib.h>
#include <string.h>
#include "ref_internal.h"

/* ------------------------------------------------ bytes.Fields (Go 1.10) */
/* Length of a Unicode White_Space rune (unicode.IsSpace) starting at s, or 0.
 * ASCII: \t \n \v \f \r SP; multi-byte: U+0085, U+00A0, U+1680, U+2000-200A,
 * U+2028, U+2029, U+202F, U+205F, U+3000.  These encodings are complete valid
 * sequences whose first byte is a lead byte, so matching them at any position
 * that is not a continuation of a valid rune equals utf8.DecodeRune there. */
static int mc_space_len(const uint8_t *s, size_t n) {
    uint8_t c = s[0];
    if (c == ' ' || (c >= 0x09 && c <= 0x0D)) return 1;
    if (c == 0xC2 && n >= 2 && (s[1] == 0x85 || s[1] == 0xA0)) return 2;
    if (n >= 3) {
        if (c == 0xE1 && s[1] == 0x9A && s[2] == 0x80) return 3;
        if (c == 0xE2 && s[1] == 0x80 && (s[2] <= 0x8A || s[2] == 0xA8 || s[2] == 0xA9 || s[2] == 0xAF) && s[2] >= 0x80) return 3;
        if (c == 0xE2 && s[1] == 0x81 && s[2] == 0x9F) return 3;
        if (c == 0xE3 && s[1] == 0x80 && s[2] == 0x80) return 3;
    }
    return 0;
}

/* Length of the rune utf8.DecodeRune would consume at s (1 for invalid). */
static int mc_rune_len(const uint8_t *s, size_t n) {
    uint8_t c = s[0];
    if (c < 0x80) return 1;
    if (c < 0xC2 || c > 0xF4) return 1;
    if (c < 0xE0) return (n >= 2 && (s[1] & 0xC0) == 0x80) ? 2 : 1;
    if (c < 0xF0) {
        if (n < 3) return 1;
        uint8_t lo = 0x80, hi = 0xBF;
        if (c == 0xE0) lo = 0xA0;
        if (c == 0xED) hi = 0x9F;
        if (s[1] < lo || s[1] > hi || (s[2] & 0xC0) != 0x80) return 1;
        return 3;
    }
    if (n < 4) return 1;
    uint8_t lo = 0x80, hi = 0xBF;
    if (c == 0xF0) lo = 0x90;
    if (c == 0xF4) hi = 0x8F;
    if (s[1] < lo || s[1] > hi || (s[2] & 0xC0) != 0x80 || (s[3] & 0xC0) != 0x80) return 1;
    return 4;
}

typedef struct { uint32_t off, len; } mc_tok;

/* Tokens of line[0..n); returns the count (tokens beyond cap are counted, not stored). */
static int mc_fields(const uint8_t *line, uint32_t n, mc_tok *tok, int cap) {
    int nt = 0;
    uint32_t i = 0;
    int infield = 0;
    uint32_t start = 0;
    while (i < n) {
        int sp = mc_space_len(line + i, n - i);
        if (sp) {
            if (infield) { if (nt < cap) tok[nt] = (mc_tok){start, i - start}; nt++; infield = 0; }
            i += (uint32_t)sp;
        } else {
            if (!infield) { start = i; infield = 1; }
            i += (uint32_t)mc_rune_len(line + i, n - i);
        }
    }
    if (infield) { if (nt < cap) tok[nt] = (mc_tok){start, n - start}; nt++; }
    return nt;
}

/* strconv.Atoi on 64-bit: optional sign, decimal digits, int64 range. */
static int mc_atoi(const uint8_t *s, uint32_t n, int64_t *out) {
    uint32_t i = 0;
    int neg = 0;
    if (n == 0) return 0;
    if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; if (n == 1) return 0; }
    uint64_t v = 0;
    for (; i < n; i++) {
        if (s[i] < '0' || s[i] > '9') return 0;
        uint64_t d = (uint64_t)(s[i] - '0');
        if (v > (UINT64_MAX - d) / 10) return 0;
        v = v * 10 + d;
        if (v > (uint64_t)INT64_MAX + (neg ? 1u : 0u)) return 0;
    }
    *out = neg ? (int64_t)(0 - v) : (int64_t)v;
    return 1;
}

static int tok_is(const uint8_t *line, mc_tok t, const char *s) {
    size_t n = strlen(s);
    return t.len == n && memcmp(line + t.off, s, n) == 0;
}

/* ------------------------------------------------ rule model */
/* MemcacheOpCodeMap (proxylib/memcached/parser.go:214-474): group name ->
 * text command names (space separated) and binary opcodes. */
typedef struct { const char *name; const char *text; int nbin; uint8_t bin[16]; } mc_group;
static const mc_group MC_GROUPS[] = {
    {"add", "add", 2, {2, 18}}, {"set", "set", 2, {1, 17}}, {"replace", "replace", 2, {3, 19}},
    {"append", "append", 2, {14, 25}}, {"prepend", "prepend", 2, {15, 26}}, {"cas", "cas", 0, {0}},
    {"incr", "incr", 2, {5, 21}}, {"decr", "decr", 2, {6, 22}},
    {"storage", "add set replace append prepend cas incr decr", 12, {1, 2, 3, 5, 6, 17, 18, 19, 21, 22, 25, 26}},
    {"get", "get gets", 4, {0, 9, 12, 13}},
    {"delete", "delete", 2, {4, 20}}, {"touch", "touch", 1, {28}}, {"gat", "gat gats", 2, {29, 30}},
    {"writeGroup", "add set replace append prepend cas incr decr delete touch", 15,
     {1, 2, 3, 4, 5, 6, 17, 18, 19, 20, 21, 22, 25, 26, 28}},
    {"slabs", "slabs", 0, {0}}, {"lru", "lru", 0, {0}}, {"lru_crawler", "lru_crawler", 0, {0}},
    {"watch", "watch", 0, {0}}, {"stats", "stats", 1, {16}}, {"flush_all", "flush_all", 2, {8, 24}},
    {"cache_memlimit", "cache_memlimit", 0, {0}}, {"version", "version", 1, {11}},
    {"misbehave", "misbehave", 0, {0}}, {"quit", "quit", 2, {7, 23}},
    {"noop", "", 1, {10}}, {"verbosity", "", 1, {27}}, {"sasl-list-mechs", "", 1, {32}}, {"sasl-auth", "", 1, {33}},
    {"sasl-step", "", 1, {34}}, {"rget", "", 1, {48}}, {"rset", "", 1, {49}}, {"rsetq", "", 1, {50}},
    {"rappend", "", 1, {51}}, {"rappendq", "", 1, {52}}, {"rprepend", "", 1, {53}}, {"rprependq", "", 1, {54}},
    {"rdelete", "", 1, {55}}, {"rdeleteq", "", 1, {56}}, {"rincr", "", 1, {57}}, {"rincrq", "", 1, {58}},
    {"rdecr", "", 1, {59}}, {"rdecrq", "", 1, {60}}, {"set-vbucket", "", 1, {61}}, {"get-vbucket", "", 1, {62}},
    {"del-vbucket", "", 1, {63}}, {"tap-connect", "", 1, {64}}, {"tap-mutation", "", 1, {65}},
    {"tap-delete", "", 1, {66}}, {"tap-flush", "", 1, {67}}, {"tap-opaque", "", 1, {68}},
    {"tap-vbucket-set", "", 1, {69}}, {"tap-checkpoint-start", "", 1, {70}}, {"tap-checkpoint-end", "", 1, {71}},
};

const void *ref_mc_group(const char *name, size_t n) {
    for (size_t g = 0; g < sizeof MC_GROUPS / sizeof MC_GROUPS[0]; g++)
        if (strlen(MC_GROUPS[g].name) == n && !memcmp(MC_GROUPS[g].name, name, n)) return &MC_GROUPS[g];
    return NULL;
}

static int group_has_text(const mc_group *g, const uint8_t *cmd, uint32_t n) {
    const char *p = g->text;
    while (*p) {
        const char *e = strchr(p, ' ');
        size_t l = e ? (size_t)(e - p) : strlen(p);
        if (l == n && !memcmp(p, cmd, n)) return 1;
        if (!e) break;
        p = e + 1;
    }
    return 0;
}

static int group_has_opcode(const mc_group *g, uint8_t op) {
    for (int i = 0; i < g->nbin; i++) if (g->bin[i] == op) return 1;
    return 0;
}

typedef struct {
    int binary;
    uint8_t opcode;
    const uint8_t *cmd; uint32_t cmdlen;
    const uint8_t *base;     /* key token bytes are base + tok[i].off */
    const mc_tok *keys; int nkeys;
} mc_meta;

/* memcache.Rule.Matches (parser.go:47-100) */
static int mc_rule_matches(const ref_mc_rule *r, const mc_meta *m) {
    if (r->empty) return 1;
    const mc_group *g = (const mc_group *)r->group;
    if (m->binary) { if (!g || !group_has_opcode(g, m->opcode)) return 0; }
    else if (!g || !group_has_text(g, m->cmd, m->cmdlen)) return 0;
    if (r->key_exact && r->key_exact_len > 0) {
        for (int k = 0; k < m->nkeys; k++)
            if (m->keys[k].len != r->key_exact_len || memcmp(m->base + m->keys[k].off, r->key_exact, r->key_exact_len)) return 0;
        return 1;
    }
    if (r->key_prefix && r->key_prefix_len > 0) {
        for (int k = 0; k < m->nkeys; k++)
            if (m->keys[k].len < r->key_prefix_len || memcmp(m->base + m->keys[k].off, r->key_prefix, r->key_prefix_len)) return 0;
        return 1;
    }
    if (r->key_re) {
        for (int k = 0; k < m->nkeys; k++)
            if (!ref_re_match(r->key_re, m->base + m->keys[k].off, m->keys[k].len, 0)) return 0;
        return 1;
    }
    return 1;
}

/* PortNetworkPolicyRules.Matches (policymap.go:150-171) */
static int mc_port_rules_match(const ref_port *pp, uint64_t remote, const mc_meta *m, int32_t *rule) {
    *rule = -1;
    if (!ref_px_have_l7(pp)) return 1;
    if (pp->nrules == 0) return 1;
    for (int r = 0; r < pp->nrules; r++) {
        const ref_pnp_rule *pr = &pp->rules[r];
        if (!ref_remote_ok(pr, remote)) continue;
        if (ref_px_nl7(pr) == 0) return 1;  /* empty L7 set matches any payload */
        if (pr->l7type != L7T_L7) continue;  /* HTTP / Kafka rules never match a memcached request */
        for (int k = 0; k < pr->nl7; k++)
            if (mc_rule_matches(&pr->l7[k], m)) { *rule = pr->l7[k].id; return 1; }
    }
    return 0;
}

void ref_memcache_verdict(const ref_policy *pol, const ref_conn_t *c, const uint8_t *b, uint32_t len, ref_out_t *o) {
    o->rule = -1;
    o->consumed = 0;
    mc_meta m;
    memset(&m, 0, sizeof m);
    uint64_t frame = 0;
    mc_tok onekey, toks[256];
    mc_tok *big = NULL;
    int mode = c->flags & 3;
    if (len == 0 && mode == 0) { o->verdict = L7_INCOMPLETE; return; }  /* NOP, 0 (no parser yet) */
    if (mode == 0) mode = b[0] >= 128 ? L7_CONN_MC_BINARY : L7_CONN_MC_TEXT;
    if (mode == L7_CONN_MC_BINARY) {  /* binary (binary/parser.go:58-139) */
        if (len < 24) { o->verdict = L7_INCOMPLETE; o->consumed = 24 - len; return; }  /* MORE headerMissing */
        uint32_t body = (uint32_t)b[8] << 24 | (uint32_t)b[9] << 16 | (uint32_t)b[10] << 8 | b[11];
        uint32_t keylen = (uint32_t)b[2] << 8 | b[3];
        uint32_t extras = b[4];
        if (keylen > 0 && 24 + keylen + extras > len) {  /* MORE keyMissing */
            o->verdict = L7_INCOMPLETE; o->consumed = 24 + keylen + extras - len; return;
        }
        if ((b[0] & 0x80) != 0x80) { o->verdict = L7_PARSE_ERROR; o->consumed = 2; return; }  /* ERROR, INVALID_FRAME_TYPE */
        m.binary = 1;
        m.opcode = b[1];
        onekey = (mc_tok){keylen ? 24 + extras : 0, keylen};
        m.base = b; m.keys = &onekey; m.nkeys = 1;
        frame = (uint32_t)(body + 24u);
    } else {  /* text (text/parser.go:72-198) */
        uint32_t lf = 0;
        int found = 0;
        for (uint32_t i = 0; i + 1 < len; i++) if (b[i] == '\r' && b[i + 1] == '\n') { lf = i; found = 1; break; }
        if (!found) {  /* MORE 1 if the data ends in '\r', else MORE 2 (text/parser.go:87-93) */
            o->verdict = L7_INCOMPLETE; o->consumed = (len > 0 && b[len - 1] == '\r') ? 1 : 2; return;
        }
        int nt = mc_fields(b, lf, toks, 256);
        mc_tok *t = toks;
        if (nt > 256) { big = malloc(sizeof(mc_tok) * (size_t)nt); mc_fields(b, lf, big, nt); t = big; }
        if (nt == 0) { o->verdict = L7_PARSE_ERROR; free(big); return; }  /* tokens[0] panics */
        m.cmd = b + t[0].off; m.cmdlen = t[0].len; m.base = b;
        frame = (uint64_t)lf + 2;
        const uint8_t *cmd = m.cmd; uint32_t cl = m.cmdlen;
        int ok = 1;
        if (cl >= 3 && (!memcmp(cmd, "get", 3) || !memcmp(cmd, "gat", 3))) {
            if (cmd[1] == 'e') { m.keys = t + 1; m.nkeys = nt - 1; }           /* get*: tokens[1:] */
            else if (nt < 2) ok = 0;                                            /* gat*: tokens[2:] */
            else { m.keys = t + 2; m.nkeys = nt - 2; }
        } else if (tok_is(b, t[0], "set") || tok_is(b, t[0], "add") || tok_is(b, t[0], "replace") ||
                   tok_is(b, t[0], "append") || tok_is(b, t[0], "prepend") || tok_is(b, t[0], "cas")) {
            int64_t nbytes;
            if (nt < 2) ok = 0;
            else {
                m.keys = t + 1; m.nkeys = 1;
                if (nt < 5) ok = 0;                                             /* tokens[4] panics */
                else if (!mc_atoi(b + t[4].off, t[4].len, &nbytes)) ok = 0;     /* ERROR, 0 */
                else frame = frame + (uint64_t)nbytes + 2u;  /* Go int arithmetic (wraps) */
            }
        } else if (tok_is(b, t[0], "delete") || tok_is(b, t[0], "incr") || tok_is(b, t[0], "decr") ||
                   tok_is(b, t[0], "touch")) {
            if (nt < 2) ok = 0;
            else { m.keys = t + 1; m.nkeys = 1; }
        } else if (tok_is(b, t[0], "slabs") || tok_is(b, t[0], "lru") || tok_is(b, t[0], "lru_crawler") ||
                   tok_is(b, t[0], "stats") || tok_is(b, t[0], "version") || tok_is(b, t[0], "misbehave") ||
                   tok_is(b, t[0], "flush_all") || tok_is(b, t[0], "cache_memlimit") || tok_is(b, t[0], "quit") ||
                   tok_is(b, t[0], "watch")) {
            m.nkeys = 0;
        } else {
            ok = 0;  /* unknown command: ERROR, 0 */
        }
        if (!ok) { o->verdict = L7_PARSE_ERROR; free(big); return; }
    }
    if ((int64_t)frame <= 0 || frame > 0xFFFFFFFFull) { o->verdict = L7_PARSE_ERROR; free(big); return; }
    o->consumed = (uint32_t)frame;
    /* Instance.PolicyMatches (instance.go:157-165) */
    o->verdict = L7_DENY;
    if (c->policy >= 0 && c->policy < pol->np) {
        const ref_netpolicy *np = &pol->p[c->policy];
        const ref_port *ex, *wc;
        ref_port_lookup(np, c->ingress, c->port, &ex, &wc);
        const ref_port *cands[2] = {ex, wc};
        for (int k = 0; k < 2; k++) {
            int32_t rule;
            if (!cands[k] || !ref_px_installed(cands[k])) continue;
            if (mc_port_rules_match(cands[k], c->src_id, &m, &rule)) { o->verdict = L7_ALLOW; o->rule = rule; break; }
        }
    }
    free(big);
}
