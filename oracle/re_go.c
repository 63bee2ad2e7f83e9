/*
 * re_go.c — TEST INFRASTRUCTURE ONLY (parity oracle, see l7ref.h).
 *
 * CPU restatement of Go 1.10.3's regexp as used by the reference:
 *   - regexp/syntax.Parse(expr, syntax.Perl)   (parse.go: parse, repeat,
 *     parsePerlFlags, parseClass, parseEscape, parseUnicodeClass,
 *     parsePerlClassEscape, parseNamedClass, appendFoldedRange, literal)
 *   - regexp.(*Regexp).Match: leftmost search over runes decoded with
 *     utf8.DecodeRune (invalid byte => U+FFFD, width 1), empty-width
 *     assertions from syntax.EmptyOpContext (exec.go, regexp.go).
 * Reference call sites: pkg/policy/api/http.go:69,76 (validation),
 * proxylib/memcached/parser.go:91,132, proxylib/r2d2/r2d2parser.go:79,103.
 *
 * Matching is a Pike VM over *runes* (Go's own execution model); the product
 * compiles to byte-level DFAs instead, so agreement between the two is a real
 * check, not a tautology.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

#include "l7ref.h"
#include "unicode_tables.h"

#define MAX_RUNE 0x10FFFF
#define RUNE_ERROR 0xFFFD

/* ---- UTF-8 decoding exactly as Go's unicode/utf8.DecodeRune ---- */
static int go_decode(const uint8_t *s, size_t n, int32_t *r) {
    if (n == 0) { *r = RUNE_ERROR; return 0; }
    uint8_t b0 = s[0];
    if (b0 < 0x80) { *r = b0; return 1; }
    int sz; uint8_t lo = 0x80, hi = 0xBF;
    if (b0 >= 0xC2 && b0 <= 0xDF) sz = 2;
    else if (b0 >= 0xE0 && b0 <= 0xEF) { sz = 3; if (b0 == 0xE0) lo = 0xA0; if (b0 == 0xED) hi = 0x9F; }
    else if (b0 >= 0xF0 && b0 <= 0xF4) { sz = 4; if (b0 == 0xF0) lo = 0x90; if (b0 == 0xF4) hi = 0x8F; }
    else { *r = RUNE_ERROR; return 1; }
    if (n < (size_t)sz) { *r = RUNE_ERROR; return 1; }
    uint8_t b1 = s[1];
    if (b1 < lo || b1 > hi) { *r = RUNE_ERROR; return 1; }
    if (sz == 2) { *r = ((int32_t)(b0 & 0x1F) << 6) | (b1 & 0x3F); return 2; }
    uint8_t b2 = s[2];
    if (b2 < 0x80 || b2 > 0xBF) { *r = RUNE_ERROR; return 1; }
    if (sz == 3) { *r = ((int32_t)(b0 & 0x0F) << 12) | ((int32_t)(b1 & 0x3F) << 6) | (b2 & 0x3F); return 3; }
    uint8_t b3 = s[3];
    if (b3 < 0x80 || b3 > 0xBF) { *r = RUNE_ERROR; return 1; }
    *r = ((int32_t)(b0 & 0x07) << 18) | ((int32_t)(b1 & 0x3F) << 12) | ((int32_t)(b2 & 0x3F) << 6) | (b3 & 0x3F);
    return 4;
}

/* ---- unicode.SimpleFold ---- */
static int32_t simple_fold(int32_t r) {
    int lo = 0, hi = UNI_FOLD_NPAIRS;
    while (lo < hi) {
        int m = (lo + hi) / 2;
        if ((int32_t)UNI_FOLD_PAIRS[m][0] < r) lo = m + 1; else hi = m;
    }
    if (lo < UNI_FOLD_NPAIRS && (int32_t)UNI_FOLD_PAIRS[lo][0] == r) return (int32_t)UNI_FOLD_PAIRS[lo][1];
    return r;
}

/* ---------------------------------------------------------------------------
 * Character classes: growable arrays of inclusive [lo,hi] pairs.
 * ------------------------------------------------------------------------- */
typedef struct { int32_t *r; int n, cap; } cls_t; /* n = number of int32 (2 per range) */

static void cls_add(cls_t *c, int32_t lo, int32_t hi) {
    if (c->n + 2 > c->cap) { c->cap = c->cap ? c->cap * 2 : 16; c->r = realloc(c->r, sizeof(int32_t) * c->cap); }
    c->r[c->n++] = lo; c->r[c->n++] = hi;
}
static int cmp_rng(const void *a, const void *b) {
    const int32_t *x = a, *y = b;
    if (x[0] != y[0]) return x[0] < y[0] ? -1 : 1;
    return x[1] < y[1] ? 1 : (x[1] > y[1] ? -1 : 0);
}
static void cls_clean(cls_t *c) { /* syntax.cleanClass */
    if (c->n == 0) return;
    qsort(c->r, c->n / 2, 2 * sizeof(int32_t), cmp_rng);
    int w = 2;
    for (int i = 2; i < c->n; i += 2) {
        int32_t lo = c->r[i], hi = c->r[i + 1];
        if (lo <= c->r[w - 1] + 1) { if (hi > c->r[w - 1]) c->r[w - 1] = hi; continue; }
        c->r[w] = lo; c->r[w + 1] = hi; w += 2;
    }
    c->n = w;
}
static void cls_negate(cls_t *c) { /* syntax.negateClass (on a clean class) */
    cls_t o = {0};
    int32_t next = 0;
    for (int i = 0; i < c->n; i += 2) {
        if (c->r[i] > next) cls_add(&o, next, c->r[i] - 1);
        next = c->r[i + 1] + 1;
    }
    if (next <= MAX_RUNE) cls_add(&o, next, MAX_RUNE);
    free(c->r); *c = o;
}
/* appendFoldedRange: every rune in [lo,hi] plus its whole fold orbit. */
static void cls_add_folded(cls_t *c, int32_t lo, int32_t hi) {
    cls_add(c, lo, hi);
    /* only runes present in the orbit table can add anything */
    int a = 0, b = UNI_FOLD_NPAIRS;
    while (a < b) { int m = (a + b) / 2; if ((int32_t)UNI_FOLD_PAIRS[m][0] < lo) a = m + 1; else b = m; }
    for (int i = a; i < UNI_FOLD_NPAIRS && (int32_t)UNI_FOLD_PAIRS[i][0] <= hi; i++) {
        int32_t r0 = (int32_t)UNI_FOLD_PAIRS[i][0];
        for (int32_t f = simple_fold(r0); f != r0; f = simple_fold(f)) cls_add(c, f, f);
    }
}
static void cls_append_class(cls_t *dst, const cls_t *src, int fold, int negate) {
    cls_t tmp = {0};
    for (int i = 0; i < src->n; i += 2) {
        if (fold) cls_add_folded(&tmp, src->r[i], src->r[i + 1]);
        else cls_add(&tmp, src->r[i], src->r[i + 1]);
    }
    cls_clean(&tmp);
    if (negate) cls_negate(&tmp);
    for (int i = 0; i < tmp.n; i += 2) cls_add(dst, tmp.r[i], tmp.r[i + 1]);
    free(tmp.r);
}

/* ---------------------------------------------------------------------------
 * AST
 * ------------------------------------------------------------------------- */
enum {
    OP_NOMATCH = 1, OP_EMPTY, OP_CLASS, OP_ANYNOTNL, OP_ANY,
    OP_BOL, OP_EOL, OP_BOT, OP_EOT, OP_WB, OP_NWB,
    OP_STAR, OP_PLUS, OP_QUEST, OP_REPEAT, OP_CONCAT, OP_ALT,
    /* pseudo ops on the parse stack */
    OP_LPAREN = 100, OP_VBAR,
};

typedef struct node {
    int op;
    int flags;          /* parser flags at creation (for LPAREN: flags to restore) */
    int min, max;
    struct node **sub; int nsub, capsub;
    cls_t cls;
} node;

#define F_FOLD 1
#define F_DOTNL 2
#define F_ONELINE 4
#define F_NONGREEDY 8
#define F_PERLX 16

static node *mk(int op, int flags) { node *n = calloc(1, sizeof(node)); n->op = op; n->flags = flags; return n; }
static void add_sub(node *n, node *s) {
    if (n->nsub == n->capsub) { n->capsub = n->capsub ? 2 * n->capsub : 4; n->sub = realloc(n->sub, sizeof(node *) * n->capsub); }
    n->sub[n->nsub++] = s;
}
static void free_node(node *n) {
    if (!n) return;
    for (int i = 0; i < n->nsub; i++) free_node(n->sub[i]);
    free(n->sub); free(n->cls.r); free(n);
}

typedef struct {
    node **st; int n, cap;
    int flags;
    const char *whole; size_t wholelen;
    char *err; size_t errlen; int failed;
} parser;

static void push(parser *p, node *x) {
    if (p->n == p->cap) { p->cap = p->cap ? 2 * p->cap : 16; p->st = realloc(p->st, sizeof(node *) * p->cap); }
    p->st[p->n++] = x;
}
static int fail(parser *p, const char *code, const char *expr, size_t exprlen) {
    if (!p->failed) {
        snprintf(p->err, p->errlen, "error parsing regexp: %s: `%.*s`", code, (int)exprlen, expr);
        p->failed = 1;
    }
    return -1;
}

static const char *E_INVALID_CLASS_RANGE = "invalid character class range";
static const char *E_INVALID_ESCAPE = "invalid escape sequence";
static const char *E_INVALID_NAMED_CAPTURE = "invalid named capture";
static const char *E_INVALID_PERL_OP = "invalid or unsupported Perl syntax";
static const char *E_INVALID_REPEAT_OP = "invalid nested repetition operator";
static const char *E_INVALID_REPEAT_SIZE = "invalid repeat count";
static const char *E_INVALID_UTF8 = "invalid UTF-8";
static const char *E_MISSING_BRACKET = "missing closing ]";
static const char *E_MISSING_PAREN = "missing closing )";
static const char *E_MISSING_REPEAT_ARG = "missing argument to repetition operator";
static const char *E_TRAILING_BACKSLASH = "trailing backslash at end of expression";
static const char *E_UNEXPECTED_PAREN = "unexpected )";

/* nextRune: decode one rune of the pattern; invalid UTF-8 is an error. */
static int next_rune(parser *p, const char *s, size_t n, int32_t *r) {
    int w = go_decode((const uint8_t *)s, n, r);
    if (*r == RUNE_ERROR && w == 1) { fail(p, E_INVALID_UTF8, s, n); return -1; }
    return w;
}

/* literal rune => class of its fold orbit under (?i) */
static void push_literal(parser *p, int32_t r) {
    node *x = mk(OP_CLASS, p->flags);
    if (p->flags & F_FOLD) cls_add_folded(&x->cls, r, r);
    else cls_add(&x->cls, r, r);
    cls_clean(&x->cls);
    push(p, x);
}

/* p.concat(): collapse stack entries above the topmost pseudo op into a concat */
static void do_concat(parser *p) {
    int i = p->n;
    while (i > 0 && p->st[i - 1]->op < OP_LPAREN) i--;
    int cnt = p->n - i;
    node *c;
    if (cnt == 0) c = mk(OP_EMPTY, p->flags);
    else if (cnt == 1) c = p->st[i];
    else { c = mk(OP_CONCAT, p->flags); for (int k = i; k < p->n; k++) add_sub(c, p->st[k]); }
    p->n = i;
    push(p, c);
}
/* p.alternate(): collapse entries above the topmost LPAREN (alternatives are
 * separated by VBAR markers in this restatement) into an alternation. */
static void do_alternate(parser *p) {
    /* stack: ... LPAREN? alt1 VBAR alt2 VBAR ... altk  (each alt already a concat) */
    int i = p->n;
    while (i > 0 && p->st[i - 1]->op != OP_LPAREN) i--;
    int cnt = 0;
    for (int k = i; k < p->n; k++) if (p->st[k]->op != OP_VBAR) cnt++;
    node *a;
    if (cnt == 1) {
        a = NULL;
        for (int k = i; k < p->n; k++) { if (p->st[k]->op != OP_VBAR) a = p->st[k]; else free_node(p->st[k]); }
    } else {
        a = mk(OP_ALT, p->flags);
        for (int k = i; k < p->n; k++) { if (p->st[k]->op != OP_VBAR) add_sub(a, p->st[k]); else free_node(p->st[k]); }
    }
    p->n = i;
    push(p, a);
}

static int isalnum_ascii(int32_t c) { return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'); }
static int unhex(int32_t c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

/* parseEscape: s points at '\\'. Returns consumed byte count, -1 on error. */
static int parse_escape(parser *p, const char *s, size_t n, int32_t *out) {
    size_t i = 1;
    if (i >= n) return fail(p, E_TRAILING_BACKSLASH, "", 0);
    int32_t c; int w = next_rune(p, s + i, n - i, &c); if (w < 0) return -1; i += w;
    switch (c) {
    case '1': case '2': case '3': case '4': case '5': case '6': case '7':
        if (i >= n || s[i] < '0' || s[i] > '7') break;
        /* fallthrough */
    case '0': {
        int32_t r = c - '0';
        for (int k = 1; k < 3; k++) {
            if (i >= n || s[i] < '0' || s[i] > '7') break;
            r = r * 8 + (s[i] - '0'); i++;
        }
        *out = r; return (int)i;
    }
    case 'x': {
        if (i >= n) break;
        w = next_rune(p, s + i, n - i, &c); if (w < 0) return -1; i += w;
        if (c == '{') {
            int nhex = 0; int32_t r = 0;
            for (;;) {
                if (i >= n) goto bad;
                w = next_rune(p, s + i, n - i, &c); if (w < 0) return -1; i += w;
                if (c == '}') break;
                int v = unhex(c); if (v < 0) goto bad;
                r = r * 16 + v; if (r > MAX_RUNE) goto bad;
                nhex++;
            }
            if (nhex == 0) goto bad;
            *out = r; return (int)i;
        }
        int x = unhex(c);
        int32_t c2; w = next_rune(p, s + i, n - i, &c2); if (w < 0) return -1; i += w;
        int y = unhex(c2);
        if (x < 0 || y < 0) break;
        *out = x * 16 + y; return (int)i;
    }
    case 'a': *out = 7; return (int)i;
    case 'f': *out = 12; return (int)i;
    case 'n': *out = 10; return (int)i;
    case 'r': *out = 13; return (int)i;
    case 't': *out = 9; return (int)i;
    case 'v': *out = 11; return (int)i;
    default:
        if (c < 0x80 && !isalnum_ascii(c)) { *out = c; return (int)i; }
        break;
    }
bad:
    return fail(p, E_INVALID_ESCAPE, s, i);
}

/* Perl and POSIX ASCII groups (perl_groups.go) */
typedef struct { const char *name; int sign; const int32_t *r; int n; } group_t;
static const int32_t G_DIGIT[] = {'0', '9'};
static const int32_t G_SPACE[] = {'\t', '\n', '\f', '\r', ' ', ' '};
static const int32_t G_WORD[] = {'0', '9', 'A', 'Z', '_', '_', 'a', 'z'};
static const int32_t G_ALNUM[] = {'0', '9', 'A', 'Z', 'a', 'z'};
static const int32_t G_ALPHA[] = {'A', 'Z', 'a', 'z'};
static const int32_t G_ASCII[] = {0, 0x7F};
static const int32_t G_BLANK[] = {'\t', '\t', ' ', ' '};
static const int32_t G_CNTRL[] = {0, 0x1F, 0x7F, 0x7F};
static const int32_t G_GRAPH[] = {'!', '~'};
static const int32_t G_LOWER[] = {'a', 'z'};
static const int32_t G_PRINT[] = {' ', '~'};
static const int32_t G_PUNCT[] = {'!', '/', ':', '@', '[', '`', '{', '~'};
static const int32_t G_PSPACE[] = {'\t', '\r', ' ', ' '};
static const int32_t G_UPPER[] = {'A', 'Z'};
static const int32_t G_XDIGIT[] = {'0', '9', 'A', 'F', 'a', 'f'};
#define G(name, sign, arr) {name, sign, arr, (int)(sizeof(arr) / sizeof(arr[0]))}
static const group_t PERL_GROUPS[] = {
    G("\\d", 1, G_DIGIT), G("\\D", -1, G_DIGIT), G("\\s", 1, G_SPACE), G("\\S", -1, G_SPACE),
    G("\\w", 1, G_WORD), G("\\W", -1, G_WORD),
};
static const group_t POSIX_GROUPS[] = {
    G("[:alnum:]", 1, G_ALNUM), G("[:^alnum:]", -1, G_ALNUM), G("[:alpha:]", 1, G_ALPHA), G("[:^alpha:]", -1, G_ALPHA),
    G("[:ascii:]", 1, G_ASCII), G("[:^ascii:]", -1, G_ASCII), G("[:blank:]", 1, G_BLANK), G("[:^blank:]", -1, G_BLANK),
    G("[:cntrl:]", 1, G_CNTRL), G("[:^cntrl:]", -1, G_CNTRL), G("[:digit:]", 1, G_DIGIT), G("[:^digit:]", -1, G_DIGIT),
    G("[:graph:]", 1, G_GRAPH), G("[:^graph:]", -1, G_GRAPH), G("[:lower:]", 1, G_LOWER), G("[:^lower:]", -1, G_LOWER),
    G("[:print:]", 1, G_PRINT), G("[:^print:]", -1, G_PRINT), G("[:punct:]", 1, G_PUNCT), G("[:^punct:]", -1, G_PUNCT),
    G("[:space:]", 1, G_PSPACE), G("[:^space:]", -1, G_PSPACE), G("[:upper:]", 1, G_UPPER), G("[:^upper:]", -1, G_UPPER),
    G("[:word:]", 1, G_WORD), G("[:^word:]", -1, G_WORD), G("[:xdigit:]", 1, G_XDIGIT), G("[:^xdigit:]", -1, G_XDIGIT),
};

static void append_group(parser *p, cls_t *dst, const group_t *g) { /* p.appendGroup */
    cls_t src = {(int32_t *)g->r, g->n, g->n};
    cls_append_class(dst, &src, (p->flags & F_FOLD) != 0, g->sign < 0);
}

/* parsePerlClassEscape: returns consumed bytes (2) or 0 */
static int parse_perl_class(parser *p, const char *s, size_t n, cls_t *dst) {
    if (n < 2 || s[0] != '\\') return 0;
    for (size_t k = 0; k < sizeof(PERL_GROUPS) / sizeof(PERL_GROUPS[0]); k++)
        if (PERL_GROUPS[k].name[1] == s[1]) { append_group(p, dst, &PERL_GROUPS[k]); return 2; }
    return 0;
}

/* parseNamedClass: s at "[:"; returns consumed, 0 if not a class, -1 error */
static int parse_named_class(parser *p, const char *s, size_t n, cls_t *dst) {
    if (n < 2 || s[0] != '[' || s[1] != ':') return 0;
    const char *e = NULL;
    for (size_t i = 2; i + 1 < n; i++) if (s[i] == ':' && s[i + 1] == ']') { e = s + i; break; }
    if (!e) return 0;
    size_t nl = (size_t)(e - s) + 2;
    for (size_t k = 0; k < sizeof(POSIX_GROUPS) / sizeof(POSIX_GROUPS[0]); k++)
        if (strlen(POSIX_GROUPS[k].name) == nl && memcmp(POSIX_GROUPS[k].name, s, nl) == 0) {
            append_group(p, dst, &POSIX_GROUPS[k]); return (int)nl;
        }
    return fail(p, E_INVALID_CLASS_RANGE, s, nl);
}

/* unicodeTable(name): tables that also carry a Go fold table (FoldCategory / FoldScript) */
static int unicode_fold_name(const char *name, size_t n) {
    static const char *F[] = {"L", "Ll", "Lt", "Lu", "M", "Mn", "Common", "Greek", "Inherited"};
    for (size_t i = 0; i < sizeof(F) / sizeof(F[0]); i++) if (strlen(F[i]) == n && memcmp(F[i], name, n) == 0) return 1;
    return 0;
}
static const uni_table_t *unicode_table(const char *name, size_t n) {
    for (int i = 0; i < UNI_NTABLES; i++)
        if (strlen(UNI_TABLES[i].name) == n && memcmp(UNI_TABLES[i].name, name, n) == 0) return &UNI_TABLES[i];
    return NULL;
}

/* parseUnicodeClass: s at "\p" or "\P"; returns consumed, 0 if not, -1 error */
static int parse_unicode_class(parser *p, const char *s, size_t n, cls_t *dst) {
    if (n < 2 || s[0] != '\\' || (s[1] != 'p' && s[1] != 'P')) return 0;
    int sign = s[1] == 'P' ? -1 : 1;
    size_t i = 2;
    int32_t c; int w = go_decode((const uint8_t *)s + i, n - i, &c);
    if (c == RUNE_ERROR && w == 1) return fail(p, E_INVALID_UTF8, s + i, n - i);
    const char *name; size_t nlen, seqlen;
    if (c != '{') {
        seqlen = i + w; name = s + 2; nlen = (size_t)w;
    } else {
        const char *e = memchr(s, '}', n);
        if (!e) return fail(p, E_INVALID_CLASS_RANGE, s, n);
        seqlen = (size_t)(e - s) + 1; name = s + 3; nlen = (size_t)(e - s) - 3;
    }
    if (nlen > 0 && name[0] == '^') { sign = -sign; name++; nlen--; }
    cls_t tab = {0};
    int fold = 0;
    if (nlen == 3 && memcmp(name, "Any", 3) == 0) {
        cls_add(&tab, 0, MAX_RUNE);
    } else {
        const uni_table_t *t = unicode_table(name, nlen);
        if (!t) { free(tab.r); return fail(p, E_INVALID_CLASS_RANGE, s, seqlen); }
        for (int k = 0; k < t->n; k++) cls_add(&tab, (int32_t)UNI_RANGES[t->off + k][0], (int32_t)UNI_RANGES[t->off + k][1]);
        fold = unicode_fold_name(name, nlen);
    }
    cls_append_class(dst, &tab, (p->flags & F_FOLD) && fold, sign < 0);
    free(tab.r);
    return (int)seqlen;
}

/* parseClass: s at '['. returns consumed or -1 */
static int parse_class(parser *p, const char *s, size_t n) {
    size_t i = 1;
    node *x = mk(OP_CLASS, p->flags);
    int sign = 1;
    if (i < n && s[i] == '^') { sign = -1; i++; }
    /* ClassNL is set in syntax.Perl, so [^a] may match \n: nothing to add. */
    int first = 1;
    while (i >= n || s[i] != ']' || first) {
        first = 0;
        int k;
        if (n - i > 2 && s[i] == '[' && s[i + 1] == ':') {
            k = parse_named_class(p, s + i, n - i, &x->cls);
            if (k < 0) goto err;
            if (k > 0) { i += k; continue; }
        }
        k = parse_unicode_class(p, s + i, n - i, &x->cls);
        if (k < 0) goto err;
        if (k > 0) { i += k; continue; }
        k = parse_perl_class(p, s + i, n - i, &x->cls);
        if (k > 0) { i += k; continue; }
        /* single char or range */
        size_t rstart = i;
        int32_t lo, hi;
        if (i >= n) { fail(p, E_MISSING_BRACKET, s, n); goto err; }
        if (s[i] == '\\') { k = parse_escape(p, s + i, n - i, &lo); if (k < 0) goto err; i += k; }
        else { k = next_rune(p, s + i, n - i, &lo); if (k < 0) goto err; i += k; }
        hi = lo;
        if (n - i >= 2 && s[i] == '-' && s[i + 1] != ']') {
            i++;
            if (i >= n) { fail(p, E_MISSING_BRACKET, s, n); goto err; }
            if (s[i] == '\\') { k = parse_escape(p, s + i, n - i, &hi); if (k < 0) goto err; i += k; }
            else { k = next_rune(p, s + i, n - i, &hi); if (k < 0) goto err; i += k; }
            if (hi < lo) { fail(p, E_INVALID_CLASS_RANGE, s + rstart, i - rstart); goto err; }
        }
        if (p->flags & F_FOLD) cls_add_folded(&x->cls, lo, hi); else cls_add(&x->cls, lo, hi);
    }
    i++; /* ']' */
    cls_clean(&x->cls);
    if (sign < 0) cls_negate(&x->cls);
    push(p, x);
    return (int)i;
err:
    free_node(x);
    return -1;
}

/* syntax.(*parser).repeat */
static int do_repeat(parser *p, int op, int min, int max, const char *before, size_t beforelen,
                     size_t *afterpos, const char *lastrep, size_t lastreplen) {
    /* *afterpos: offset into `before` of the text after the operator */
    size_t after = *afterpos;
    if (after < beforelen && before[after] == '?') after++; /* non-greedy: irrelevant to booleans */
    if (lastrep) {
        /* lastRepeat[:len(lastRepeat)-len(after)] */
        size_t rem = beforelen - after;
        return fail(p, E_INVALID_REPEAT_OP, lastrep, lastreplen - rem);
    }
    if (p->n == 0 || p->st[p->n - 1]->op >= OP_LPAREN)
        return fail(p, E_MISSING_REPEAT_ARG, before, after);
    node *sub = p->st[p->n - 1];
    node *x = mk(op, p->flags);
    x->min = min; x->max = max;
    add_sub(x, sub);
    p->st[p->n - 1] = x;
    *afterpos = after;
    return 0;
}

/* repeatIsValid(re, 1000): nested counted repetitions may not multiply past 1000 */
static int repeat_is_valid(node *re, int n) {
    if (re->op == OP_REPEAT) {
        int m = re->max;
        if (m == 0) return 1;
        if (m < 0) m = re->min;
        if (m > n) return 0;
        if (m > 0) n /= m;
    }
    for (int i = 0; i < re->nsub; i++) if (!repeat_is_valid(re->sub[i], n)) return 0;
    return 1;
}

/* parseRepeat: s at '{' ; returns 1 ok and sets min,max,consumed */
static int parse_int(const char *s, size_t n, size_t *i, int *val) {
    size_t st = *i;
    if (st >= n || s[st] < '0' || s[st] > '9') return 0;
    if (n - st >= 2 && s[st] == '0' && s[st + 1] >= '0' && s[st + 1] <= '9') return 0;
    size_t e = st;
    while (e < n && s[e] >= '0' && s[e] <= '9') e++;
    long v = 0;
    for (size_t k = st; k < e; k++) { if (v >= 100000000) { v = -1; break; } v = v * 10 + (s[k] - '0'); }
    *val = (int)v; *i = e;
    return 1;
}
static int parse_repeat(const char *s, size_t n, int *min, int *max, size_t *consumed) {
    if (n == 0 || s[0] != '{') return 0;
    size_t i = 1;
    if (!parse_int(s, n, &i, min)) return 0;
    if (i >= n) return 0;
    if (s[i] != ',') *max = *min;
    else {
        i++;
        if (i >= n) return 0;
        if (s[i] == '}') *max = -1;
        else {
            if (!parse_int(s, n, &i, max)) return 0;
            if (*max < 0) *min = -1;
        }
    }
    if (i >= n || s[i] != '}') return 0;
    *consumed = i + 1;
    return 1;
}

/* parsePerlFlags: s at "(?" ; returns consumed or -1 */
static int parse_perl_flags(parser *p, const char *s, size_t n) {
    if (n > 4 && s[2] == 'P' && s[3] == '<') {
        const char *e = memchr(s, '>', n);
        if (!e) return fail(p, E_INVALID_NAMED_CAPTURE, s, n);
        size_t end = (size_t)(e - s);
        const char *name = s + 4; size_t nl = end - 4;
        int ok = nl > 0;
        for (size_t k = 0; k < nl; k++) {
            char c = name[k];
            if (!(c == '_' || isalnum_ascii((unsigned char)c))) ok = 0;
        }
        if (!ok) return fail(p, E_INVALID_NAMED_CAPTURE, s, end + 1);
        push(p, mk(OP_LPAREN, p->flags));
        return (int)(end + 1);
    }
    size_t i = 2;
    int flags = p->flags, sign = 1, saw = 0;
    while (i < n) {
        int32_t c; int w = next_rune(p, s + i, n - i, &c); if (w < 0) return -1; i += w;
        switch (c) {
        case 'i': flags |= F_FOLD; saw = 1; break;
        case 'm': flags &= ~F_ONELINE; saw = 1; break;
        case 's': flags |= F_DOTNL; saw = 1; break;
        case 'U': flags |= F_NONGREEDY; saw = 1; break;
        case '-':
            if (sign < 0) goto bad;
            sign = -1; flags = ~flags; saw = 0; break;
        case ':': case ')':
            if (sign < 0) { if (!saw) goto bad; flags = ~flags; }
            if (c == ':') push(p, mk(OP_LPAREN, p->flags));
            p->flags = flags;
            return (int)i;
        default: goto bad;
        }
    }
bad:
    return fail(p, E_INVALID_PERL_OP, s, i);
}

static int parse_right_paren(parser *p) {
    do_concat(p);
    do_alternate(p);
    if (p->n < 2) return fail(p, E_UNEXPECTED_PAREN, p->whole, p->wholelen);
    node *re1 = p->st[p->n - 1], *re2 = p->st[p->n - 2];
    if (re2->op != OP_LPAREN) return fail(p, E_UNEXPECTED_PAREN, p->whole, p->wholelen);
    p->n -= 2;
    p->flags = re2->flags;
    free_node(re2);
    push(p, re1);
    return 0;
}

static node *parse(parser *p, const char *s, size_t n) {
    p->flags = F_ONELINE | F_PERLX; /* syntax.Perl = ClassNL|OneLine|PerlX|UnicodeGroups */
    p->whole = s; p->wholelen = n;
    const char *lastrep = NULL; size_t lastreplen = 0;
    size_t i = 0;
    while (i < n) {
        const char *rep = NULL; size_t replen = 0;
        const char *t = s + i; size_t tn = n - i;
        switch (t[0]) {
        case '(':
            if (tn >= 2 && t[1] == '?') {
                int k = parse_perl_flags(p, t, tn); if (k < 0) goto err; i += k; break;
            }
            push(p, mk(OP_LPAREN, p->flags)); i++;
            break;
        case '|':
            do_concat(p);
            push(p, mk(OP_VBAR, p->flags)); i++;
            break;
        case ')':
            if (parse_right_paren(p) < 0) goto err; i++;
            break;
        case '^':
            push(p, mk((p->flags & F_ONELINE) ? OP_BOT : OP_BOL, p->flags)); i++;
            break;
        case '$':
            push(p, mk((p->flags & F_ONELINE) ? OP_EOT : OP_EOL, p->flags)); i++;
            break;
        case '.':
            push(p, mk((p->flags & F_DOTNL) ? OP_ANY : OP_ANYNOTNL, p->flags)); i++;
            break;
        case '[': {
            int k = parse_class(p, t, tn); if (k < 0) goto err; i += k; break;
        }
        case '*': case '+': case '?': {
            int op = t[0] == '*' ? OP_STAR : (t[0] == '+' ? OP_PLUS : OP_QUEST);
            size_t after = 1;
            if (do_repeat(p, op, 0, 0, t, tn, &after, lastrep, lastreplen) < 0) goto err;
            rep = t; replen = tn;
            i += after;
            break;
        }
        case '{': {
            int min, max; size_t cons;
            if (!parse_repeat(t, tn, &min, &max, &cons)) { push_literal(p, '{'); i++; break; }
            if (min < 0 || min > 1000 || max > 1000 || (max >= 0 && min > max)) {
                fail(p, E_INVALID_REPEAT_SIZE, t, cons); goto err;
            }
            size_t after = cons;
            if (do_repeat(p, OP_REPEAT, min, max, t, tn, &after, lastrep, lastreplen) < 0) goto err;
            node *top = p->st[p->n - 1];
            if ((min >= 2 || max >= 2) && !repeat_is_valid(top, 1000)) { fail(p, E_INVALID_REPEAT_SIZE, t, after); goto err; }
            rep = t; replen = tn;
            i += after;
            break;
        }
        case '\\': {
            if (tn >= 2) {
                char c1 = t[1];
                if (c1 == 'A') { push(p, mk(OP_BOT, p->flags)); i += 2; break; }
                if (c1 == 'b') { push(p, mk(OP_WB, p->flags)); i += 2; break; }
                if (c1 == 'B') { push(p, mk(OP_NWB, p->flags)); i += 2; break; }
                if (c1 == 'C') { fail(p, E_INVALID_ESCAPE, t, 2); goto err; }
                if (c1 == 'z') { push(p, mk(OP_EOT, p->flags)); i += 2; break; }
                if (c1 == 'Q') {
                    const char *lit = t + 2; size_t ln = tn - 2; size_t adv = tn;
                    for (size_t k = 2; k + 1 < tn; k++) if (t[k] == '\\' && t[k + 1] == 'E') { ln = k - 2; adv = k + 2; break; }
                    size_t j = 0;
                    while (j < ln) {
                        int32_t c; int w = next_rune(p, lit + j, ln - j, &c); if (w < 0) goto err;
                        push_literal(p, c); j += w;
                    }
                    i += adv;
                    break;
                }
            }
            node *x = mk(OP_CLASS, p->flags);
            int k = parse_unicode_class(p, t, tn, &x->cls);
            if (k < 0) { free_node(x); goto err; }
            if (k == 0) k = parse_perl_class(p, t, tn, &x->cls);
            if (k > 0) { cls_clean(&x->cls); push(p, x); i += k; break; }
            free_node(x);
            int32_t c;
            k = parse_escape(p, t, tn, &c); if (k < 0) goto err;
            push_literal(p, c); i += k;
            break;
        }
        default: {
            int32_t c; int w = next_rune(p, t, tn, &c); if (w < 0) goto err;
            push_literal(p, c); i += w;
            break;
        }
        }
        lastrep = rep; lastreplen = replen;
    }
    do_concat(p);
    do_alternate(p);
    if (p->n != 1) { fail(p, E_MISSING_PAREN, s, n); goto err; }
    node *r = p->st[0]; p->n = 0;
    return r;
err:
    for (int k = 0; k < p->n; k++) free_node(p->st[k]);
    p->n = 0;
    return NULL;
}

/* ---------------------------------------------------------------------------
 * Program + Pike VM
 * ------------------------------------------------------------------------- */
enum { I_MATCH, I_CLASS, I_ANYNOTNL, I_ANY, I_EMPTY, I_SPLIT, I_NOP, I_FAIL };
#define EW_BOL 1
#define EW_EOL 2
#define EW_BOT 4
#define EW_EOT 8
#define EW_WB 16
#define EW_NWB 32

typedef struct { int op; int x, y; int cond; int cls; } inst_t;

struct ref_re {
    inst_t *prog; int np, capp;
    cls_t *classes; int ncls, capcls;
    int start;
};

static int emit(ref_re *re, int op) {
    if (re->np == re->capp) { re->capp = re->capp ? 2 * re->capp : 64; re->prog = realloc(re->prog, sizeof(inst_t) * re->capp); }
    memset(&re->prog[re->np], 0, sizeof(inst_t));
    re->prog[re->np].op = op;
    return re->np++;
}
static int add_class(ref_re *re, const cls_t *c) {
    if (re->ncls == re->capcls) { re->capcls = re->capcls ? 2 * re->capcls : 16; re->classes = realloc(re->classes, sizeof(cls_t) * re->capcls); }
    cls_t cp = {0};
    for (int i = 0; i < c->n; i += 2) cls_add(&cp, c->r[i], c->r[i + 1]);
    re->classes[re->ncls] = cp;
    return re->ncls++;
}

/* compile node so that it continues at `next`; returns entry pc */
static int compile(ref_re *re, const node *x, int next) {
    switch (x->op) {
    case OP_NOMATCH: return emit(re, I_FAIL);
    case OP_EMPTY: return next;
    case OP_CLASS: {
        if (x->cls.n == 0) return emit(re, I_FAIL);
        int pc = emit(re, I_CLASS); re->prog[pc].cls = add_class(re, &x->cls); re->prog[pc].x = next; return pc;
    }
    case OP_ANYNOTNL: { int pc = emit(re, I_ANYNOTNL); re->prog[pc].x = next; return pc; }
    case OP_ANY: { int pc = emit(re, I_ANY); re->prog[pc].x = next; return pc; }
    case OP_BOL: case OP_EOL: case OP_BOT: case OP_EOT: case OP_WB: case OP_NWB: {
        int pc = emit(re, I_EMPTY);
        re->prog[pc].cond = x->op == OP_BOL ? EW_BOL : x->op == OP_EOL ? EW_EOL : x->op == OP_BOT ? EW_BOT
                          : x->op == OP_EOT ? EW_EOT : x->op == OP_WB ? EW_WB : EW_NWB;
        re->prog[pc].x = next;
        return pc;
    }
    case OP_CONCAT: {
        int pc = next;
        for (int i = x->nsub - 1; i >= 0; i--) pc = compile(re, x->sub[i], pc);
        return pc;
    }
    case OP_ALT: {
        int pc = compile(re, x->sub[x->nsub - 1], next);
        for (int i = x->nsub - 2; i >= 0; i--) {
            int a = compile(re, x->sub[i], next);
            int s = emit(re, I_SPLIT); re->prog[s].x = a; re->prog[s].y = pc; pc = s;
        }
        return pc;
    }
    case OP_STAR: {
        int s = emit(re, I_SPLIT);
        int body = compile(re, x->sub[0], s);
        re->prog[s].x = body; re->prog[s].y = next;
        return s;
    }
    case OP_PLUS: {
        int s = emit(re, I_SPLIT);
        int body = compile(re, x->sub[0], s);
        re->prog[s].x = body; re->prog[s].y = next;
        return body;
    }
    case OP_QUEST: {
        int body = compile(re, x->sub[0], next);
        int s = emit(re, I_SPLIT); re->prog[s].x = body; re->prog[s].y = next;
        return s;
    }
    case OP_REPEAT: { /* syntax.simplify: x{n,m} -> x^n (x(x...)?)? ; x{n,} -> x^n x* */
        int pc = next;
        if (x->max < 0) {
            int s = emit(re, I_SPLIT);
            int body = compile(re, x->sub[0], s);
            re->prog[s].x = body; re->prog[s].y = next;
            pc = s;
        } else {
            for (int k = x->min; k < x->max; k++) {
                int body = compile(re, x->sub[0], pc);
                int s = emit(re, I_SPLIT); re->prog[s].x = body; re->prog[s].y = next;
                pc = s;
            }
        }
        for (int k = 0; k < x->min; k++) pc = compile(re, x->sub[0], pc);
        return pc;
    }
    }
    return emit(re, I_FAIL);
}

ref_re *ref_re_compile(const char *pat, size_t patlen, char *err, size_t errlen) {
    char dummy[8];
    parser p; memset(&p, 0, sizeof p);
    p.err = err ? err : dummy; p.errlen = err ? errlen : sizeof dummy;
    if (p.errlen) p.err[0] = 0;
    node *ast = parse(&p, pat, patlen);
    free(p.st);
    if (!ast) return NULL;
    ref_re *re = calloc(1, sizeof(ref_re));
    int m = emit(re, I_MATCH);
    re->start = compile(re, ast, m);
    free_node(ast);
    return re;
}

void ref_re_free(ref_re *re) {
    if (!re) return;
    for (int i = 0; i < re->ncls; i++) free(re->classes[i].r);
    free(re->classes); free(re->prog); free(re);
}

static int is_word(int32_t r) { return r >= 0 && r < 0x80 && (isalnum_ascii(r) || r == '_'); }
/* syntax.EmptyOpContext(r1, r2) */
static int empty_ctx(int32_t r1, int32_t r2) {
    int op = 0;
    if (r1 < 0) op |= EW_BOT | EW_BOL;
    if (r1 == '\n') op |= EW_BOL;
    if (r2 < 0) op |= EW_EOT | EW_EOL;
    if (r2 == '\n') op |= EW_EOL;
    if (is_word(r1) != is_word(r2)) op |= EW_WB; else op |= EW_NWB;
    return op;
}

static int cls_has(const cls_t *c, int32_t r) {
    int lo = 0, hi = c->n / 2;
    while (lo < hi) {
        int m = (lo + hi) / 2;
        if (r < c->r[2 * m]) hi = m;
        else if (r > c->r[2 * m + 1]) lo = m + 1;
        else return 1;
    }
    return 0;
}

typedef struct { int *dense; int *sparse; int n; } sset;
static int sset_has(sset *s, int pc) { unsigned i = (unsigned)s->sparse[pc]; return i < (unsigned)s->n && s->dense[i] == pc; }
static void sset_add(sset *s, int pc) { s->sparse[pc] = s->n; s->dense[s->n++] = pc; }

/* add pc and its epsilon closure under empty-width context ctx */
static void addthread(const ref_re *re, sset *s, int pc, int ctx, int *stack) {
    int sp = 0;
    stack[sp++] = pc;
    while (sp > 0) {
        pc = stack[--sp];
        if (sset_has(s, pc)) continue;
        sset_add(s, pc);
        const inst_t *in = &re->prog[pc];
        switch (in->op) {
        case I_SPLIT: stack[sp++] = in->y; stack[sp++] = in->x; break;
        case I_EMPTY: if ((in->cond & ~ctx) == 0) stack[sp++] = in->x; break;
        default: break;
        }
    }
}

int ref_re_match(const ref_re *re, const uint8_t *s, size_t n, int anchored) {
    int np = re->np;
    int *buf = malloc(sizeof(int) * ((size_t)np * 7 + 16)); /* 2 sparse sets + closure stack (<= 2*np+1) */
    sset a = {buf, buf + np, 0}, b = {buf + 2 * np, buf + 3 * np, 0};
    int *stack = buf + 4 * np;
    sset *cl = &a, *nl = &b;
    size_t pos = 0;
    int32_t r1 = -1, r2; int w;
    if (n > 0) w = go_decode(s, n, &r2); else { r2 = -1; w = 0; }
    int result = 0;
    for (;;) {
        int ctx = empty_ctx(r1, r2);
        if (!anchored || pos == 0) addthread(re, cl, re->start, ctx, stack);
        if (cl->n == 0 && anchored) break;
        /* next position context */
        int32_t r3 = -1; int w2 = 0;
        if (pos + w < n) w2 = go_decode(s + pos + w, n - pos - w, &r3);
        int nctx = empty_ctx(r2, r3);
        nl->n = 0;
        for (int i = 0; i < cl->n; i++) {
            const inst_t *in = &re->prog[cl->dense[i]];
            switch (in->op) {
            case I_MATCH:
                if (!anchored || pos == n) { result = 1; goto done; }
                break;
            case I_CLASS: if (r2 >= 0 && cls_has(&re->classes[in->cls], r2)) addthread(re, nl, in->x, nctx, stack); break;
            case I_ANYNOTNL: if (r2 >= 0 && r2 != '\n') addthread(re, nl, in->x, nctx, stack); break;
            case I_ANY: if (r2 >= 0) addthread(re, nl, in->x, nctx, stack); break;
            default: break;
            }
        }
        if (pos >= n) break;
        pos += w; r1 = r2; r2 = r3; w = w2;
        sset *t = cl; cl = nl; nl = t;
    }
done:
    free(buf);
    return result;
}
