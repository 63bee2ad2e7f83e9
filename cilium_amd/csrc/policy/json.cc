#include "json.h"

#include <cstdlib>
#include <cstring>

namespace l7 {
namespace json {

const Value *Value::get(const char *key) const {
    if (type != Obj) return nullptr;
    for (auto &kv : obj) if (kv.first == key) return &kv.second;
    return nullptr;
}

namespace {
struct P {
    const char *s; size_t n, i = 0; std::string err;
    bool fail(const char *m) { if (err.empty()) err = std::string("json: ") + m + " at offset " + std::to_string(i); return false; }
    void ws() { while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) i++; }
    static void utf8(std::string &o, uint32_t c) {
        if (c < 0x80) o += (char)c;
        else if (c < 0x800) { o += (char)(0xC0 | (c >> 6)); o += (char)(0x80 | (c & 0x3F)); }
        else if (c < 0x10000) { o += (char)(0xE0 | (c >> 12)); o += (char)(0x80 | ((c >> 6) & 0x3F)); o += (char)(0x80 | (c & 0x3F)); }
        else { o += (char)(0xF0 | (c >> 18)); o += (char)(0x80 | ((c >> 12) & 0x3F)); o += (char)(0x80 | ((c >> 6) & 0x3F)); o += (char)(0x80 | (c & 0x3F)); }
    }
    bool hex4(uint32_t *v) {
        if (i + 4 > n) return false;
        *v = 0;
        for (int k = 0; k < 4; k++) {
            char c = s[i + k]; int d;
            if (c >= '0' && c <= '9') d = c - '0'; else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') d = c - 'A' + 10; else return false;
            *v = *v * 16 + d;
        }
        i += 4;
        return true;
    }
    bool str(std::string &o) {
        if (i >= n || s[i] != '"') return fail("expected string");
        i++;
        while (i < n && s[i] != '"') {
            char c = s[i++];
            if (c != '\\') { o += c; continue; }
            if (i >= n) return fail("bad escape");
            char e = s[i++];
            uint32_t u;
            switch (e) {
            case '"': case '\\': case '/': o += e; break;
            case 'b': o += '\b'; break;
            case 'f': o += '\f'; break;
            case 'n': o += '\n'; break;
            case 'r': o += '\r'; break;
            case 't': o += '\t'; break;
            case 'u':
                if (!hex4(&u)) return fail("bad \\u escape");
                if (u >= 0xD800 && u < 0xDC00) {
                    uint32_t lo;
                    if (i + 2 <= n && s[i] == '\\' && s[i + 1] == 'u') { i += 2; if (!hex4(&lo) || lo < 0xDC00 || lo >= 0xE000) return fail("bad surrogate"); u = 0x10000 + ((u - 0xD800) << 10) + (lo - 0xDC00); }
                    else return fail("bad surrogate");
                }
                utf8(o, u);
                break;
            default: return fail("bad escape");
            }
        }
        if (i >= n) return fail("unterminated string");
        i++;
        return true;
    }
    bool value(Value &v, int depth) {
        if (depth > 64) return fail("too deep");
        ws();
        if (i >= n) return fail("unexpected end");
        char c = s[i];
        if (c == '{' || c == '[') {
            bool obj = c == '{';
            v.type = obj ? Value::Obj : Value::Arr;
            i++; ws();
            if (i < n && s[i] == (obj ? '}' : ']')) { i++; return true; }
            for (;;) {
                ws();
                if (obj) {
                    std::string k;
                    if (!str(k)) return false;
                    ws();
                    if (i >= n || s[i] != ':') return fail("expected ':'");
                    i++;
                    v.obj.emplace_back(std::move(k), Value());
                    if (!value(v.obj.back().second, depth + 1)) return false;
                } else {
                    v.arr.emplace_back();
                    if (!value(v.arr.back(), depth + 1)) return false;
                }
                ws();
                if (i < n && s[i] == ',') { i++; continue; }
                if (i < n && s[i] == (obj ? '}' : ']')) { i++; return true; }
                return fail("expected ',' or close");
            }
        }
        if (c == '"') { v.type = Value::Str; return str(v.str); }
        if (n - i >= 4 && !memcmp(s + i, "true", 4)) { i += 4; v.type = Value::Bool; v.b = true; return true; }
        if (n - i >= 5 && !memcmp(s + i, "false", 5)) { i += 5; v.type = Value::Bool; return true; }
        if (n - i >= 4 && !memcmp(s + i, "null", 4)) { i += 4; v.type = Value::Null; return true; }
        if (c == '-' || (c >= '0' && c <= '9')) {
            size_t st = i;
            bool isint = true;
            if (s[i] == '-') i++;
            while (i < n && ((s[i] >= '0' && s[i] <= '9') || s[i] == '.' || s[i] == 'e' || s[i] == 'E' || s[i] == '+' || s[i] == '-')) {
                if (!(s[i] >= '0' && s[i] <= '9')) isint = false;
                i++;
            }
            std::string t(s + st, i - st);
            v.type = Value::Num;
            v.num = strtod(t.c_str(), nullptr);
            v.inum = isint ? strtoll(t.c_str(), nullptr, 10) : (int64_t)v.num;
            return true;
        }
        return fail("bad value");
    }
};
}  // namespace

bool Parse(const char *s, size_t n, Value *out, std::string *err) {
    P p{s, n};
    *out = Value();
    if (!p.value(*out, 0)) { if (err) *err = p.err; return false; }
    p.ws();
    if (p.i != n) { p.fail("trailing data"); if (err) *err = p.err; return false; }
    return true;
}

}  // namespace json
}  // namespace l7
