// proxylib cassandra request parsing (product code), one implementation for
// the gfx950 kernel (kernels/cassandra_classify.hip) and the host shim's
// access-log records (proxylib/shim.cc): proxylib/cassandra/cassandraparser.go.
//
// The Go parser lower-cases the whole query (strings.ToLower), splits it with
// strings.Fields and builds the path "/<opcode>/<action>/<table>" that
// CassandraRule.Matches splits on "/" again.  Here nothing is copied: the
// query is tokenized once on its raw bytes (lower-casing never creates or
// removes a space rune, so the raw and the lowered token boundaries agree),
// keywords are compared rune by rune against their lowered spelling (only
// U+0130 -> 'i' and U+212A -> 'k' lower into ASCII besides 'A'-'Z'), and the
// one string a rule regex sees -- parts[3] of the path -- is produced as a
// stream of lowered bytes from the token spans (cass_seg3) straight into the
// DFA / NFA.
//
// strings.ToLower of Go 1.10 maps runes with strings.Map, which returns its
// input unchanged up to the first rune the mapping changes and re-encodes
// every rune from there: an invalid UTF-8 byte (utf8 RuneError, width 1)
// before that point stays as it is, one after it becomes U+FFFD (EF BF BD).
// `fc` below is that point.  (Not covered by a reference test: unpinned.)
#pragma once
#include <stdint.h>

#include "../device_tables.h"
#include "../regex/nfa_walk.h"

namespace l7 {

// queryActionMap (cassandraparser.go:319-366); the first kCassTableActions
// take a query_table (actionWithTable), the rest do not (actionNoTable).
constexpr int kCassActions = 38;
constexpr int kCassTableActions = 12;
enum : int {
    CA_SELECT = 0, CA_DELETE, CA_INSERT, CA_UPDATE, CA_CREATE_TABLE, CA_DROP_TABLE, CA_ALTER_TABLE, CA_TRUNCATE_TABLE,
    CA_USE, CA_CREATE_KEYSPACE, CA_ALTER_KEYSPACE, CA_DROP_KEYSPACE, CA_DROP_INDEX, CA_CREATE_INDEX,
    CA_CREATE_MVIEW, CA_DROP_MVIEW, CA_CREATE_ROLE, CA_ALTER_ROLE, CA_DROP_ROLE, CA_GRANT_ROLE, CA_REVOKE_ROLE,
    CA_LIST_ROLES, CA_GRANT_PERMISSION, CA_REVOKE_PERMISSION, CA_LIST_PERMISSIONS, CA_CREATE_USER, CA_ALTER_USER,
    CA_DROP_USER, CA_LIST_USERS, CA_CREATE_FUNCTION, CA_DROP_FUNCTION, CA_CREATE_AGGREGATE, CA_DROP_AGGREGATE,
    CA_CREATE_TYPE, CA_ALTER_TYPE, CA_DROP_TYPE, CA_CREATE_TRIGGER, CA_DROP_TRIGGER,
};
// the action string of each id (host: rule parsing, access log)
inline const char *CassActionName(int a) {
    static const char *const k[kCassActions] = {
        "select", "delete", "insert", "update", "create-table", "drop-table", "alter-table", "truncate-table", "use",
        "create-keyspace", "alter-keyspace", "drop-keyspace", "drop-index", "create-index", "create-materialized-view",
        "drop-materialized-view", "create-role", "alter-role", "drop-role", "grant-role", "revoke-role", "list-roles",
        "grant-permission", "revoke-permission", "list-permissions", "create-user", "alter-user", "drop-user",
        "list-users", "create-function", "drop-function", "create-aggregate", "drop-aggregate", "create-type",
        "alter-type", "drop-type", "create-trigger", "drop-trigger"};
    return a >= 0 && a < kCassActions ? k[a] : "";
}

// Words the grammar compares tokens with (lowered spelling).
enum : uint8_t {
    CW_NONE = 0, CW_SELECT, CW_DELETE, CW_INSERT, CW_UPDATE, CW_USE, CW_ALTER, CW_CREATE, CW_DROP, CW_TRUNCATE,
    CW_LIST, CW_FROM, CW_TABLE, CW_KEYSPACE, CW_IF, CW_MATERIALIZED, CW_CUSTOM, CW_INDEX, CW_ROLE, CW_USER,
    CW_FUNCTION, CW_AGGREGATE, CW_TYPE, CW_TRIGGER, CW_ROLES, CW_PERMISSIONS, CW_USERS, CW_NWORDS
};

// unicode.IsSpace
L7_HD inline bool cass_space(uint32_t r) {
    return (r >= 9 && r <= 13) || r == ' ' || r == 0x85 || r == 0xA0 || r == 0x1680 || (r >= 0x2000 && r <= 0x200A) ||
           r == 0x2028 || r == 0x2029 || r == 0x202F || r == 0x205F || r == 0x3000;
}

// unicode.ToLower over the (rune, lower) pairs of the Unicode 10 tables
// (sorted by rune; csrc/regex/unicode_tables.h UNI_LOWER_PAIRS)
L7_HD inline uint32_t cass_lower(uint32_t r, const uint32_t *pairs, uint32_t npairs) {
    if (r < 0x80) return r - 'A' < 26u ? r + 32 : r;
    uint32_t lo = 0, hi = npairs;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (pairs[2 * m] < r) lo = m + 1;
        else hi = m;
    }
    return lo < npairs && pairs[2 * lo] == r ? pairs[2 * lo + 1] : r;
}

// Does the token q[s, e) lower to the ASCII word w (n bytes)?
L7_HD inline bool cass_word_eq(const uint8_t *q, uint32_t s, uint32_t e, const char *w, uint32_t n) {
    uint32_t p = s;
    for (uint32_t k = 0; k < n; k++) {
        if (p >= e) return false;
        uint32_t width;
        const uint32_t r = nfa_decode(q, p, e, &width);
        const uint32_t c = (uint32_t)(uint8_t)w[k];
        const bool ok = r == c || (c - 'a' < 26u && r == c - 32) || (c == 'i' && r == 0x130) || (c == 'k' && r == 0x212A);
        if (!ok) return false;
        p += width;
    }
    return p == e;
}

L7_HD inline uint32_t cass_word(const uint8_t *q, uint32_t s, uint32_t e) {
    // (first-byte filter: each word's first letter, either case; U+0130 / U+212A lead bytes C4 / E2)
    const uint32_t b = q[s] | 0x20u;
    const bool special = q[s] == 0xC4 || q[s] == 0xE2;
#define CW(id, lit)                                                                   \
    if ((special || b == (uint32_t)lit[0]) && cass_word_eq(q, s, e, lit, sizeof(lit) - 1)) return id;
    CW(CW_SELECT, "select") CW(CW_DELETE, "delete") CW(CW_INSERT, "insert") CW(CW_UPDATE, "update")
    CW(CW_USE, "use") CW(CW_ALTER, "alter") CW(CW_CREATE, "create") CW(CW_DROP, "drop") CW(CW_TRUNCATE, "truncate")
    CW(CW_LIST, "list") CW(CW_FROM, "from") CW(CW_TABLE, "table") CW(CW_KEYSPACE, "keyspace") CW(CW_IF, "if")
    CW(CW_MATERIALIZED, "materialized") CW(CW_CUSTOM, "custom") CW(CW_INDEX, "index") CW(CW_ROLE, "role")
    CW(CW_USER, "user") CW(CW_FUNCTION, "function") CW(CW_AGGREGATE, "aggregate") CW(CW_TYPE, "type")
    CW(CW_TRIGGER, "trigger") CW(CW_ROLES, "roles") CW(CW_PERMISSIONS, "permissions") CW(CW_USERS, "users")
#undef CW
    return CW_NONE;
}

// action id of "<kw>-<word>" (the alter / create / drop / truncate / list forms), -1 if not in queryActionMap
L7_HD inline int cass_action2(uint32_t kw, uint32_t w) {
    switch (kw) {
    case CW_ALTER:
        return w == CW_TABLE ? CA_ALTER_TABLE : w == CW_KEYSPACE ? CA_ALTER_KEYSPACE : w == CW_ROLE ? CA_ALTER_ROLE
             : w == CW_USER ? CA_ALTER_USER : w == CW_TYPE ? CA_ALTER_TYPE : -1;
    case CW_CREATE:
        return w == CW_TABLE ? CA_CREATE_TABLE : w == CW_KEYSPACE ? CA_CREATE_KEYSPACE : w == CW_INDEX ? CA_CREATE_INDEX
             : w == CW_ROLE ? CA_CREATE_ROLE : w == CW_USER ? CA_CREATE_USER : w == CW_FUNCTION ? CA_CREATE_FUNCTION
             : w == CW_AGGREGATE ? CA_CREATE_AGGREGATE : w == CW_TYPE ? CA_CREATE_TYPE
             : w == CW_TRIGGER ? CA_CREATE_TRIGGER : -1;
    case CW_DROP:
        return w == CW_TABLE ? CA_DROP_TABLE : w == CW_KEYSPACE ? CA_DROP_KEYSPACE : w == CW_INDEX ? CA_DROP_INDEX
             : w == CW_ROLE ? CA_DROP_ROLE : w == CW_USER ? CA_DROP_USER : w == CW_FUNCTION ? CA_DROP_FUNCTION
             : w == CW_AGGREGATE ? CA_DROP_AGGREGATE : w == CW_TYPE ? CA_DROP_TYPE
             : w == CW_TRIGGER ? CA_DROP_TRIGGER : -1;
    case CW_TRUNCATE: return w == CW_TABLE ? CA_TRUNCATE_TABLE : -1;
    case CW_LIST: return w == CW_ROLES ? CA_LIST_ROLES : w == CW_PERMISSIONS ? CA_LIST_PERMISSIONS
                       : w == CW_USERS ? CA_LIST_USERS : -1;
    default: return -1;
    }
}

enum : uint8_t { CQ_OK = 0, CQ_INVALID = 1, CQ_PANIC = 2 };
// what parts[3] of the path is made of
enum : uint8_t { S3_NONE = 0, S3_F1 = 1, S3_TABLE = 2, S3_KS_TABLE = 3 };

struct CassQuery {
    uint8_t status;     // CQ_*
    uint8_t kw;         // CW_* of fields[0]
    uint8_t seg3;       // S3_*
    uint8_t is_use;     // a USE: the keyspace becomes trim(fields[1])
    int32_t action;     // action id of parts[2] (CA_*), -1 = none of queryActionMap
    uint32_t fc;        // first rune strings.ToLower changes (query-relative), ~0u = none
    uint32_t s1, e1;    // fields[1] (S3_F1: after its first '/')
    uint32_t ts, te;    // the table token (S3_TABLE / S3_KS_TABLE); USE: the trimmed keyspace
    uint32_t ntok;
    uint32_t f1s, f1e;  // fields[1], whole
    uint8_t has_table;  // ts / te hold a table (or, for USE, the keyspace)
};

// parseQuery (cassandraparser.go:368-469) on q[0, n): tokens, comment check,
// action / table grammar.  The keyspace prefix is left to the caller (S3_KS_TABLE).
L7_HD inline CassQuery cass_parse_query(const uint8_t *q, uint32_t n, const uint32_t *lower, uint32_t nlower) {
    CassQuery Q{};
    Q.status = CQ_INVALID;
    Q.action = -1;
    Q.fc = ~0u;
    while (n > 0 && q[n - 1] == ';') n--;  // strings.TrimRight(query, ";")
    uint32_t ts[6], te[6];
    for (int k = 0; k < 6; k++) ts[k] = te[k] = 0;
    uint32_t nt = 0, start = 0;
    int last_from = -1;
    uint32_t fs = 0, fe = 0;  // token after the last "from"
    bool in = false, comment = false;
    for (uint32_t p = 0; p <= n;) {
        uint32_t r = ' ', width = 1;
        if (p < n) r = nfa_decode(q, p, n, &width);
        const bool sp = p == n || cass_space(r);
        if (p < n && Q.fc == ~0u && !(width == 1 && r == 0xFFFD) && cass_lower(r, lower, nlower) != r) Q.fc = p;
        if (sp && in) {  // token [start, p)
            in = false;
            const uint32_t k = nt++;
            if (k < 6) { ts[k] = start; te[k] = p; }
            if (p - start >= 2 && ((q[start] == '-' && q[start + 1] == '-') || (q[start] == '/' && q[start + 1] == '*') ||
                                   (q[start] == '/' && q[start + 1] == '/')))
                comment = true;
            if (k >= 1 && p - start == 4 && cass_word_eq(q, start, p, "from", 4)) {
                last_from = (int)k;
            } else if (last_from >= 0 && k == (uint32_t)last_from + 1) {
                fs = start;
                fe = p;
            }
        } else if (!sp && !in) {
            in = true;
            start = p;
        }
        if (p == n) break;
        p += width;
    }
    Q.ntok = nt;
    if (comment || nt < 2) return Q;
    Q.s1 = Q.f1s = ts[1];
    Q.e1 = Q.f1e = te[1];
    const uint32_t kw = cass_word(q, ts[0], te[0]);
    Q.kw = (uint8_t)kw;
    bool has_table = false;
    switch (kw) {
    case CW_SELECT:
    case CW_DELETE:
        if (last_from < 0) return Q;                                    // no table: invalid
        if ((uint32_t)last_from == nt - 1) { Q.status = CQ_PANIC; return Q; }  // fields[i+1] out of range
        Q.action = kw == CW_SELECT ? CA_SELECT : CA_DELETE;
        Q.ts = fs; Q.te = fe; has_table = true;
        break;
    case CW_INSERT:
        if (nt < 3) return Q;
        Q.action = CA_INSERT;
        Q.ts = ts[2]; Q.te = te[2]; has_table = true;
        break;
    case CW_UPDATE:
        Q.action = CA_UPDATE;
        Q.ts = ts[1]; Q.te = te[1]; has_table = true;
        break;
    case CW_USE: {
        uint32_t a = ts[1], b = te[1];  // strings.Trim(fields[1], "\"\\'")
        while (a < b && (q[a] == '"' || q[a] == '\\' || q[a] == '\'')) a++;
        while (b > a && (q[b - 1] == '"' || q[b - 1] == '\\' || q[b - 1] == '\'')) b--;
        Q.action = CA_USE;
        Q.is_use = 1;
        Q.has_table = 1;
        Q.ts = a; Q.te = b;
        Q.seg3 = a < b ? S3_TABLE : S3_NONE;
        Q.status = CQ_OK;
        return Q;
    }
    case CW_ALTER: case CW_CREATE: case CW_DROP: case CW_TRUNCATE: case CW_LIST: {
        // action = "<kw>-" + fields[1]; parts[2] ends at a '/' in fields[1]
        uint32_t slash = ts[1];
        while (slash < te[1] && q[slash] != '/') slash++;
        const uint32_t w1 = cass_word(q, ts[1], te[1]);
        if (slash < te[1]) {  // parts[2] = "<kw>-" + fields[1][:slash], parts[3] from after it
            Q.action = cass_action2(kw, cass_word(q, ts[1], slash));
            Q.seg3 = S3_F1;
            Q.s1 = slash + 1;
            Q.status = CQ_OK;
            return Q;
        }
        Q.action = cass_action2(kw, w1);
        if (w1 == CW_TABLE || w1 == CW_KEYSPACE) {
            if (nt < 3) return Q;
            Q.ts = ts[2]; Q.te = te[2]; has_table = true;
            if (cass_word(q, ts[2], te[2]) == CW_IF) {
                if (Q.action == CA_CREATE_TABLE) {
                    if (nt < 6) return Q;
                    Q.ts = ts[5]; Q.te = te[5];
                } else if (Q.action == CA_DROP_TABLE || Q.action == CA_DROP_KEYSPACE) {
                    if (nt < 5) return Q;
                    Q.ts = ts[4]; Q.te = te[4];
                }
            }
        } else if (w1 == CW_MATERIALIZED) {
            Q.action = kw == CW_CREATE ? CA_CREATE_MVIEW : kw == CW_DROP ? CA_DROP_MVIEW : -1;
        } else if (w1 == CW_CUSTOM) {
            Q.action = CA_CREATE_INDEX;
        }
        break;
    }
    default:
        return Q;
    }
    Q.status = CQ_OK;
    Q.has_table = has_table;
    if (!has_table) return Q;  // parts[3] = ""
    bool dot = false;
    for (uint32_t p = Q.ts; p < Q.te; p++) dot |= q[p] == '.';
    Q.seg3 = dot ? S3_TABLE : S3_KS_TABLE;
    return Q;
}

// The lowered text of q[s, e) up to (not including) its first '/', rune by
// rune into the sink: sink.raw(b) for an invalid byte kept as it is (a rune
// of width 1 that decodes as U+FFFD), sink.rune(r) for a rune to encode;
// fc = the query's first changed rune.  Returns true if it stopped at a '/'.
template <class Sink>
L7_HD inline bool cass_emit(const uint8_t *q, uint32_t s, uint32_t e, uint32_t fc, const uint32_t *lower,
                            uint32_t nlower, Sink &sink, bool stop_at_slash = true) {
    for (uint32_t p = s; p < e;) {
        if (stop_at_slash && q[p] == '/') return true;
        uint32_t width;
        const uint32_t r = nfa_decode(q, p, e, &width);
        if (width == 1 && r == 0xFFFD) {  // an invalid byte: raw before fc, U+FFFD after
            if (p < fc) sink.raw(q[p]);
            else sink.rune(0xFFFD);
        } else {
            sink.rune(cass_lower(r, lower, nlower));
        }
        p += width;
    }
    return false;
}

// UTF-8 encoding of r into b (utf8.EncodeRune); returns the length
L7_HD inline uint32_t cass_encode(uint32_t r, uint8_t *b) {
    if (r < 0x80) { b[0] = (uint8_t)r; return 1; }
    if (r < 0x800) { b[0] = (uint8_t)(0xC0 | r >> 6); b[1] = (uint8_t)(0x80 | (r & 0x3F)); return 2; }
    if (r < 0x10000) {
        b[0] = (uint8_t)(0xE0 | r >> 12); b[1] = (uint8_t)(0x80 | ((r >> 6) & 0x3F)); b[2] = (uint8_t)(0x80 | (r & 0x3F));
        return 3;
    }
    b[0] = (uint8_t)(0xF0 | r >> 18); b[1] = (uint8_t)(0x80 | ((r >> 12) & 0x3F));
    b[2] = (uint8_t)(0x80 | ((r >> 6) & 0x3F)); b[3] = (uint8_t)(0x80 | (r & 0x3F));
    return 4;
}

// parts[3] of the request's path (the string a query_table regex sees): the
// lowered table, "<keyspace>.<table>" for an undotted one, or the rest of a
// fields[1] holding a '/', each cut at its first '/'.  ks / ks_n / ks_fc: the
// connection's keyspace as the span of a USE query (cass_parse_query's ts / te
// of that query) and that query's fc; ks == nullptr: the empty keyspace.
template <class Sink>
L7_HD inline void cass_seg3(const CassQuery &Q, const uint8_t *q, const uint8_t *ks, uint32_t ks_s, uint32_t ks_e,
                            uint32_t ks_fc, const uint32_t *lower, uint32_t nlower, Sink &sink) {
    if (Q.seg3 == S3_F1) {
        cass_emit(q, Q.s1, Q.e1, Q.fc, lower, nlower, sink);
    } else if (Q.seg3 == S3_TABLE) {
        cass_emit(q, Q.ts, Q.te, Q.fc, lower, nlower, sink);
    } else if (Q.seg3 == S3_KS_TABLE) {
        if (ks && cass_emit(ks, ks_s, ks_e, ks_fc, lower, nlower, sink)) return;  // '/' in the keyspace
        sink.raw('.');
        cass_emit(q, Q.ts, Q.te, Q.fc, lower, nlower, sink);
    }
}

}  // namespace l7
