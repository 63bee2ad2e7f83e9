/* r2d2 (proxylib/r2d2/r2d2parser.go) -- oracle restatement (TEST
 * INFRASTRUCTURE: only tests/, smoke() and bench.py's cpu_baseline use it).
 *
 *   OnData (:140-214): no "\r\n" -> MORE 1; the request is the bytes before
 *   the first "\r\n", frame = that + 2; fields = strings.Split(req, " ");
 *   cmd = fields[0]; file = fields[1] when len(fields) == 2, else "".
 *   R2d2Rule.Matches (:42-67): cmdExact unset or equal, file regex unset or
 *   MatchString(file).  Connection.Matches over the proxylib policymap
 *   (policymap.go:150-236): exact port then port 0, installed entries only,
 *   SrcId as the remote; no entry => drop. */
#include <stdlib.h>
#include <string.h>

#include "ref_internal.h"

static int r2_rule_matches(const ref_mc_rule *r, const uint8_t *cmd, size_t clen, const uint8_t *file, size_t flen) {
    if (r->r2_cmd && (r->r2_cmd_len != clen || memcmp(r->r2_cmd, cmd, clen))) return 0;
    if (r->r2_file && !ref_re_match(r->r2_file, file, flen, 0)) return 0;
    return 1;
}

static int r2_port_rules_match(const ref_port *pp, uint64_t remote, const uint8_t *cmd, size_t clen,
                               const uint8_t *file, size_t flen, int32_t *rule) {
    *rule = -1;
    if (!ref_px_have_l7(pp)) return 1;
    if (pp->nrules == 0) return 1;
    for (int r = 0; r < pp->nrules; r++) {
        const ref_pnp_rule *pr = &pp->rules[r];
        if (!ref_remote_ok(pr, remote)) continue;
        if (ref_px_nl7(pr) == 0) return 1;  /* empty L7 set matches any payload */
        if (pr->l7type != L7T_L7 || !pr->l7proto || strcmp(pr->l7proto, "r2d2")) continue;  /* other parsers' rules */
        for (int k = 0; k < pr->nl7; k++)
            if (r2_rule_matches(&pr->l7[k], cmd, clen, file, flen)) { *rule = pr->l7[k].id; return 1; }
    }
    return 0;
}

void ref_r2d2_verdict(const ref_policy *pol, const ref_conn_t *c, const uint8_t *b, uint32_t len, ref_out_t *o) {
    o->rule = -1;
    o->consumed = 0;
    uint32_t lf = 0;
    int found = 0;
    for (uint32_t i = 0; i + 1 < len; i++)
        if (b[i] == '\r' && b[i + 1] == '\n') { lf = i; found = 1; break; }
    if (!found) { o->verdict = L7_INCOMPLETE; o->consumed = 1; return; }  /* MORE, 1 */
    /* strings.Split(msgStr, " ") */
    uint32_t nsp = 0, sp1 = lf;
    for (uint32_t i = 0; i < lf; i++)
        if (b[i] == ' ') { if (nsp == 0) sp1 = i; nsp++; }
    const uint8_t *cmd = b;
    size_t clen = nsp ? sp1 : lf;
    const uint8_t *file = b;
    size_t flen = 0;
    if (nsp == 1) { file = b + sp1 + 1; flen = lf - sp1 - 1; }
    o->consumed = lf + 2;
    o->verdict = L7_DENY;
    if (c->policy < 0 || c->policy >= pol->np) return;
    const ref_port *ex, *wc;
    ref_port_lookup(&pol->p[c->policy], c->ingress, c->port, &ex, &wc);
    const ref_port *cands[2] = {ex, wc};
    for (int k = 0; k < 2; k++) {
        if (!cands[k] || !ref_px_installed(cands[k])) continue;
        int32_t rule;
        if (r2_port_rules_match(cands[k], c->src_id, cmd, clen, file, flen, &rule)) {
            o->verdict = L7_ALLOW;
            o->rule = rule;
            return;
        }
    }
}
