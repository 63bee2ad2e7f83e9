/* json.c — TEST INFRASTRUCTURE ONLY: minimal JSON reader for policy files. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "ref_internal.h"

typedef struct { const char *s; size_t n, i; char *err; size_t errlen; int failed; } jp;

static void jerr(jp *p, const char *msg) {
    if (!p->failed) { snprintf(p->err, p->errlen, "json: %s at offset %zu", msg, p->i); p->failed = 1; }
}
static void ws(jp *p) { while (p->i < p->n && (p->s[p->i] == ' ' || p->s[p->i] == '\t' || p->s[p->i] == '\n' || p->s[p->i] == '\r')) p->i++; }
static jnode *newn(int t) { jnode *j = calloc(1, sizeof(jnode)); j->type = t; return j; }

static void put_utf8(char **b, size_t *n, size_t *cap, uint32_t c) {
    if (*n + 5 > *cap) { *cap = (*cap + 8) * 2; *b = realloc(*b, *cap); }
    char *o = *b + *n;
    if (c < 0x80) { o[0] = (char)c; *n += 1; }
    else if (c < 0x800) { o[0] = (char)(0xC0 | (c >> 6)); o[1] = (char)(0x80 | (c & 0x3F)); *n += 2; }
    else if (c < 0x10000) { o[0] = (char)(0xE0 | (c >> 12)); o[1] = (char)(0x80 | ((c >> 6) & 0x3F)); o[2] = (char)(0x80 | (c & 0x3F)); *n += 3; }
    else { o[0] = (char)(0xF0 | (c >> 18)); o[1] = (char)(0x80 | ((c >> 12) & 0x3F)); o[2] = (char)(0x80 | ((c >> 6) & 0x3F)); o[3] = (char)(0x80 | (c & 0x3F)); *n += 4; }
}
static int hex4(jp *p, uint32_t *v) {
    if (p->i + 4 > p->n) return -1;
    *v = 0;
    for (int k = 0; k < 4; k++) {
        char c = p->s[p->i + k]; int d;
        if (c >= '0' && c <= '9') d = c - '0'; else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
        else if (c >= 'A' && c <= 'F') d = c - 'A' + 10; else return -1;
        *v = *v * 16 + (uint32_t)d;
    }
    p->i += 4;
    return 0;
}
static char *jstring(jp *p, size_t *outlen) {
    if (p->i >= p->n || p->s[p->i] != '"') { jerr(p, "expected string"); return NULL; }
    p->i++;
    size_t cap = 16, n = 0; char *b = malloc(cap);
    while (p->i < p->n && p->s[p->i] != '"') {
        unsigned char c = (unsigned char)p->s[p->i++];
        if (c == '\\') {
            if (p->i >= p->n) break;
            char e = p->s[p->i++]; uint32_t u;
            switch (e) {
            case '"': case '\\': case '/': put_utf8(&b, &n, &cap, (uint32_t)e); break;
            case 'b': put_utf8(&b, &n, &cap, 8); break;
            case 'f': put_utf8(&b, &n, &cap, 12); break;
            case 'n': put_utf8(&b, &n, &cap, 10); break;
            case 'r': put_utf8(&b, &n, &cap, 13); break;
            case 't': put_utf8(&b, &n, &cap, 9); break;
            case 'u':
                if (hex4(p, &u) < 0) { jerr(p, "bad \\u escape"); free(b); return NULL; }
                if (u >= 0xD800 && u < 0xDC00 && p->i + 6 <= p->n && p->s[p->i] == '\\' && p->s[p->i + 1] == 'u') {
                    uint32_t lo; p->i += 2;
                    if (hex4(p, &lo) == 0 && lo >= 0xDC00 && lo < 0xE000) u = 0x10000 + ((u - 0xD800) << 10) + (lo - 0xDC00);
                    else { jerr(p, "bad surrogate"); free(b); return NULL; }
                }
                put_utf8(&b, &n, &cap, u);
                break;
            default: jerr(p, "bad escape"); free(b); return NULL;
            }
        } else {
            if (n + 2 > cap) { cap *= 2; b = realloc(b, cap); }
            b[n++] = (char)c;
        }
    }
    if (p->i >= p->n) { jerr(p, "unterminated string"); free(b); return NULL; }
    p->i++;
    if (n + 1 > cap) b = realloc(b, n + 1);
    b[n] = 0;
    *outlen = n;
    return b;
}

static jnode *jvalue(jp *p, int depth);
static void add_item(jnode *j, jnode *v, char *k, size_t kl) {
    if (j->n == j->cap) {
        j->cap = j->cap ? 2 * j->cap : 8;
        j->items = realloc(j->items, sizeof(jnode *) * j->cap);
        j->keys = realloc(j->keys, sizeof(char *) * j->cap);
        j->keylens = realloc(j->keylens, sizeof(size_t) * j->cap);
    }
    j->items[j->n] = v; j->keys[j->n] = k; j->keylens[j->n] = kl; j->n++;
}
static jnode *jvalue(jp *p, int depth) {
    if (depth > 64) { jerr(p, "too deep"); return NULL; }
    ws(p);
    if (p->i >= p->n) { jerr(p, "unexpected end"); return NULL; }
    char c = p->s[p->i];
    if (c == '{' || c == '[') {
        int obj = c == '{';
        jnode *j = newn(obj ? JN_OBJ : JN_ARR);
        p->i++; ws(p);
        if (p->i < p->n && p->s[p->i] == (obj ? '}' : ']')) { p->i++; return j; }
        for (;;) {
            char *k = NULL; size_t kl = 0;
            ws(p);
            if (obj) {
                k = jstring(p, &kl); if (!k) { jfree(j); return NULL; }
                ws(p);
                if (p->i >= p->n || p->s[p->i] != ':') { jerr(p, "expected ':'"); free(k); jfree(j); return NULL; }
                p->i++;
            }
            jnode *v = jvalue(p, depth + 1);
            if (!v) { free(k); jfree(j); return NULL; }
            add_item(j, v, k, kl);
            ws(p);
            if (p->i < p->n && p->s[p->i] == ',') { p->i++; continue; }
            if (p->i < p->n && p->s[p->i] == (obj ? '}' : ']')) { p->i++; return j; }
            jerr(p, "expected ',' or close"); jfree(j); return NULL;
        }
    }
    if (c == '"') {
        jnode *j = newn(JN_STR);
        j->str = jstring(p, &j->slen);
        if (!j->str) { free(j); return NULL; }
        return j;
    }
    if (p->n - p->i >= 4 && !memcmp(p->s + p->i, "true", 4)) { p->i += 4; jnode *j = newn(JN_BOOL); j->b = 1; return j; }
    if (p->n - p->i >= 5 && !memcmp(p->s + p->i, "false", 5)) { p->i += 5; return newn(JN_BOOL); }
    if (p->n - p->i >= 4 && !memcmp(p->s + p->i, "null", 4)) { p->i += 4; return newn(JN_NULL); }
    if (c == '-' || (c >= '0' && c <= '9')) {
        size_t st = p->i; int isint = 1;
        if (p->s[p->i] == '-') p->i++;
        while (p->i < p->n) {
            char d = p->s[p->i];
            if (d >= '0' && d <= '9') { p->i++; continue; }
            if (d == '.' || d == 'e' || d == 'E' || d == '+' || d == '-') { isint = 0; p->i++; continue; }
            break;
        }
        char tmp[64]; size_t l = p->i - st; if (l > 63) l = 63;
        memcpy(tmp, p->s + st, l); tmp[l] = 0;
        jnode *j = newn(JN_NUM);
        j->num = strtod(tmp, NULL); j->is_int = isint; j->inum = isint ? strtoll(tmp, NULL, 10) : (int64_t)j->num;
        return j;
    }
    jerr(p, "bad value");
    return NULL;
}

jnode *jparse(const char *s, size_t n, char *err, size_t errlen) {
    char dummy[4];
    jp p = {s, n, 0, err ? err : dummy, err ? errlen : sizeof dummy, 0};
    jnode *j = jvalue(&p, 0);
    if (j) { ws(&p); if (p.i != p.n) { jerr(&p, "trailing data"); jfree(j); return NULL; } }
    return j;
}

void jfree(jnode *j) {
    if (!j) return;
    for (int i = 0; i < j->n; i++) { jfree(j->items[i]); if (j->keys) free(j->keys[i]); }
    free(j->items); free(j->keys); free(j->keylens); free(j->str); free(j);
}

jnode *jget(const jnode *obj, const char *key) {
    if (!obj || obj->type != JN_OBJ) return NULL;
    size_t kl = strlen(key);
    for (int i = 0; i < obj->n; i++) if (obj->keylens[i] == kl && !memcmp(obj->keys[i], key, kl)) return obj->items[i];
    return NULL;
}
