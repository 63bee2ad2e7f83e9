// proxylib C-ABI over the GPU verdict path (product code, include/proxylib_abi.h).
//
//   OpenModule / CloseModule   proxylib/proxylib.go:124-155, instance.go:85-143
//   OnNewConnection            proxylib/proxylib.go:57-74, connection.go:65-101
//   OnData                     proxylib/proxylib.go:98-108, connection.go:104-174
//   Close                      proxylib/proxylib.go:112-116
// and five parsers (the registry of parserfactory.go:68-71):
//   "memcache"  proxylib/memcached/parser.go:186-202 with text/parser.go:72-330
//               and binary/parser.go:58-205;
//   "http"      HTTP/1 requests with Envoy's cilium.l7policy verdict
//               (envoy/cilium_l7policy.cc:127-182): allowed => PASS, denied =>
//               DROP and a 403 "Access denied" reply injected (:171-177);
//   "kafka"     Kafka requests with the in-agent proxy's verdict
//               (pkg/proxy/kafka.go:117-153, 249-261): allowed => PASS, denied
//               => DROP and the CreateResponse(ErrTopicAuthorizationFailed)
//               reply injected (kafka_response.cc);
//   "cassandra" proxylib/cassandra/cassandraparser.go: the device parses each
//               query and matches the path; the host keeps the parser's
//               state (the frame that set the keyspace, the PREPARE frames by
//               stream id and by prepared id) and replays it to the device as
//               extra requests of the same launch (see CassClassify);
//   "r2d2"      proxylib/r2d2/r2d2parser.go:140-214: one request per line,
//               denied => DROP and "ERROR\r\n" injected.
// HTTP and Kafka connections use proxylib's policymap semantics
// (L7G_CONN_PROXYLIB: no port entry => drop, SrcId as the remote).
//
// The device gives the verdicts.  Each OnData call in the request direction
// first proposes where the frames in its input start (a cheap host scan: the
// Kafka size prefix, the memcached binary header, the HTTP header block and
// Content-Length, the memcached text line and data length) and classifies all
// of them in ONE l7g_classify_host launch; the op loop then takes each frame's
// verdict from that batch.  A proposal the device's consumed length does not
// confirm is simply not used: the frame at the real position is classified on
// its own, so the scan only saves launches, it never decides anything.  The
// host keeps what proxylib keeps per connection -- the memcached parser chosen
// by the first byte, the text reply-intent queue, the binary inject queue and
// request/reply counts -- and drives the op loop and inject buffers exactly as
// connection.go does.
#include <atomic>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <chrono>

#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>
#include <string>
#include <vector>

#include "../../../include/l7gpu.h"
#include "../../../include/proxylib_abi.h"
#include "../capi_internal.h"
#include "../kernels/cass_parse.h"
#include "../regex/unicode_tables.h"

namespace {

constexpr int64_t NOP = 256;  // proxylib-internal op (types.go:34)

// ---------------------------------------------------------------- access log
// proxylib/accesslog/client.go: one "unixpacket" (SOCK_SEQPACKET) connection
// to the agent's access-log socket per instance, dialled lazily and again
// after a failed write; each record is one protobuf-encoded cilium.LogEntry
// (pkg/envoy/cilium/accesslog.pb.go:263-400) per packet.
struct AccessLog {
    std::string path;
    std::mutex mu;
    int fd = -1;
    uint64_t sent = 0, failed = 0;
    ~AccessLog() { if (fd >= 0) close(fd); }
    bool ConnectLocked() {  // net.DialUnix("unixpacket", ...)
        if (fd >= 0) return true;
        sockaddr_un a{};
        a.sun_family = AF_UNIX;
        if (path.empty() || path.size() >= sizeof a.sun_path) return false;
        memcpy(a.sun_path, path.data(), path.size());
        fd = socket(AF_UNIX, SOCK_SEQPACKET | SOCK_CLOEXEC, 0);
        if (fd >= 0 && connect(fd, (const sockaddr *)&a, sizeof a) != 0) { close(fd); fd = -1; }
        return fd >= 0;
    }
    void Connect() {  // NewClient dials once up front (client.go:97-104)
        std::lock_guard<std::mutex> g(mu);
        ConnectLocked();
    }
    void Send(const std::string &msg) {
        if (path.empty()) return;
        std::lock_guard<std::mutex> g(mu);
        if (!ConnectLocked()) { failed++; return; }
        if (send(fd, msg.data(), msg.size(), MSG_NOSIGNAL) != (ssize_t)msg.size()) {
            close(fd);  // marked broken: redialled on the next record
            fd = -1;
            failed++;
            return;
        }
        sent++;
    }
};

// proto3 wire encoding of the LogEntry fields (zero / empty values omitted)
void PbVarint(std::string &o, uint64_t v) {
    while (v >= 0x80) { o.push_back((char)(v | 0x80)); v >>= 7; }
    o.push_back((char)v);
}
void PbU(std::string &o, uint32_t field, uint64_t v) {
    if (!v) return;
    PbVarint(o, (uint64_t)field << 3);
    PbVarint(o, v);
}
void PbS(std::string &o, uint32_t field, const std::string &s, bool keep_empty = false) {
    if (s.empty() && !keep_empty) return;
    PbVarint(o, (uint64_t)field << 3 | 2);
    PbVarint(o, s.size());
    o += s;
}
enum : uint32_t { kEntryRequest = 0, kEntryResponse = 1, kEntryDenied = 2 };  // cilium.EntryType

struct Instance {
    uint64_t id = 0, open = 0;
    std::string node, xds, alog;
    l7g_engine *eng = nullptr;
    std::mutex mu;                 // slot allocation / policy swaps
    std::vector<uint32_t> free_slots;
    uint32_t next_slot = 0;
    AccessLog log;
};

std::mutex g_inst_mu;
std::map<uint64_t, std::shared_ptr<Instance>> g_instances;
uint64_t g_last_instance = 0;

// ---------------------------------------------------------------- bytes.Fields
// Unicode White_Space rune length at s[i] (unicode.IsSpace), 0 if none; a
// multi-byte space starts with a UTF-8 lead byte, which is always a rune
// start, so no decoding context is needed.
size_t SpaceLen(const uint8_t *s, size_t i, size_t n) {
    uint8_t c = s[i];
    if (c == ' ' || (c >= 0x09 && c <= 0x0D)) return 1;
    if (c < 0xC2 || c > 0xE3 || i + 1 >= n) return 0;
    uint8_t c1 = s[i + 1];
    if (c == 0xC2) return (c1 == 0x85 || c1 == 0xA0) ? 2 : 0;
    if (i + 2 >= n) return 0;
    uint8_t c2 = s[i + 2];
    if (c == 0xE1) return (c1 == 0x9A && c2 == 0x80) ? 3 : 0;
    if (c == 0xE2 && c1 == 0x80) return ((c2 >= 0x80 && c2 <= 0x8A) || c2 == 0xA8 || c2 == 0xA9 || c2 == 0xAF) ? 3 : 0;
    if (c == 0xE2 && c1 == 0x81) return c2 == 0x9F ? 3 : 0;
    if (c == 0xE3) return (c1 == 0x80 && c2 == 0x80) ? 3 : 0;
    return 0;
}

std::vector<std::string> Fields(const uint8_t *s, size_t n) {
    std::vector<std::string> out;
    size_t i = 0, start = 0;
    bool in = false;
    while (i < n) {
        size_t sp = SpaceLen(s, i, n);
        if (sp) {
            if (in) out.emplace_back((const char *)s + start, i - start);
            in = false;
            i += sp;
        } else {
            if (!in) { start = i; in = true; }
            i++;
        }
    }
    if (in) out.emplace_back((const char *)s + start, n - start);
    return out;
}

struct Panic {};  // a Go runtime panic inside the parser (recovered => PARSER_ERROR)

long FindCRLF(const std::string &d, size_t from = 0) {
    size_t p = d.find("\r\n", from);
    return p == std::string::npos ? -1 : (long)p;
}

const char kDeniedText[] = "CLIENT_ERROR access denied\r\n";  // text/parser.go:327
// Envoy's local reply for a denied HTTP request: sendLocalReply(Forbidden,
// denied_403_body = "Access denied" + CRLF) (envoy/cilium_l7policy.cc:90-96,171-177)
const char kDenied403[] =
    "HTTP/1.1 403 Forbidden\r\ncontent-length: 15\r\ncontent-type: text/plain\r\n\r\nAccess denied\r\n";
const uint8_t kDeniedBinary[37] = {0x81, 0, 0, 0, 0, 0, 0, 8, 0, 0, 0, 0x0d, 0, 0, 0, 0, 0, 0, 0,
                                   0,    0, 0, 0, 0, 'a', 'c', 'c', 'e', 's', 's', ' ', 'd', 'e', 'n', 'i', 'e', 'd'};

}  // namespace
namespace l7 {
bool KafkaDenyResponse(const uint8_t *req, size_t len, std::string *out);
}
namespace {

enum Kind { K_MEMCACHE, K_HTTP, K_KAFKA, K_R2D2, K_CASSANDRA };

// ---------------------------------------------------------------- cassandra helpers
uint32_t Be32(const std::string &d, size_t o) {
    return (uint32_t)(uint8_t)d[o] << 24 | (uint32_t)(uint8_t)d[o + 1] << 16 | (uint32_t)(uint8_t)d[o + 2] << 8 |
           (uint8_t)d[o + 3];
}
uint32_t Be16(const std::string &d, size_t o) { return (uint32_t)(uint8_t)d[o] << 8 | (uint8_t)d[o + 1]; }

// unicode.ToLower pairs, flattened (the tables the device gets, engine/cass_compile.cc)
const std::vector<uint32_t> &CassLower() {
    static const std::vector<uint32_t> v = [] {
        std::vector<uint32_t> x;
        for (int i = 0; i < UNI_LOWER_NPAIRS; i++) { x.push_back(UNI_LOWER_PAIRS[i][0]); x.push_back(UNI_LOWER_PAIRS[i][1]); }
        return x;
    }();
    return v;
}

struct StrSink {
    std::string s;
    void raw(uint32_t c) { s.push_back((char)c); }
    void rune(uint32_t r) {
        uint8_t e[4];
        s.append((const char *)e, l7::cass_encode(r, e));
    }
};

// The query of a complete QUERY / PREPARE frame (nullptr: none, or its slice
// expressions panic) -- the device decided that already; this is for the
// host's bookkeeping and access-log records only.
const uint8_t *CassQueryOf(const std::string &f, uint32_t *qn) {
    if (f.size() < 13 || (f[4] != 0x07 && f[4] != 0x09)) return nullptr;
    const uint32_t ql = Be32(f, 9);
    if (13u + ql < 13u || 13u + ql > f.size()) return nullptr;
    *qn = ql;
    return (const uint8_t *)f.data() + 13;
}

// The path cassandraParseRequest builds for a QUERY / PREPARE frame
// ("/<opcode>/<action>/<table>", cassandraparser.go:496-515) under the
// keyspace the frame `use` set ("" = none), as the reference's strings: the
// access log splits it on "/".  Empty if the query does not parse.
std::string CassPath(const std::string &f, const std::string &use) {
    uint32_t qn;
    const uint8_t *q = CassQueryOf(f, &qn);
    if (!q) return "";
    const auto &L = CassLower();
    const l7::CassQuery Q = l7::cass_parse_query(q, qn, L.data(), (uint32_t)(L.size() / 2));
    if (Q.status != l7::CQ_OK) return "";
    StrSink a, t;
    switch (Q.kw) {
    case l7::CW_SELECT: a.s = "select"; break;
    case l7::CW_DELETE: a.s = "delete"; break;
    case l7::CW_INSERT: a.s = "insert"; break;
    case l7::CW_UPDATE: a.s = "update"; break;
    case l7::CW_USE: a.s = "use"; break;
    default: {
        static const char *const kw[] = {"alter", "create", "drop", "truncate", "list"};
        a.s = std::string(kw[Q.kw - l7::CW_ALTER]) + "-";
        l7::cass_emit(q, Q.f1s, Q.f1e, Q.fc, L.data(), (uint32_t)(L.size() / 2), a, false);
        const uint32_t w1 = l7::cass_word(q, Q.f1s, Q.f1e);
        if (w1 == l7::CW_MATERIALIZED) a.s += "-view";
        else if (w1 == l7::CW_CUSTOM) a.s = "create-index";
    }
    }
    if (Q.has_table) {
        l7::cass_emit(q, Q.ts, Q.te, Q.fc, L.data(), (uint32_t)(L.size() / 2), t, false);
        if (!Q.is_use && t.s.find('.') == std::string::npos) {
            StrSink k;
            uint32_t kn;
            const uint8_t *kq = use.empty() ? nullptr : CassQueryOf(use, &kn);
            if (kq) {
                const l7::CassQuery K = l7::cass_parse_query(kq, kn, L.data(), (uint32_t)(L.size() / 2));
                l7::cass_emit(kq, K.ts, K.te, K.fc, L.data(), (uint32_t)(L.size() / 2), k, false);
            }
            t.s = k.s + "." + t.s;
        }
    }
    return std::string("/") + (f[4] == 0x09 ? "prepare" : "query") + "/" + a.s + "/" + t.s;
}

bool CassIsUse(const std::string &f) {
    uint32_t qn;
    const uint8_t *q = CassQueryOf(f, &qn);
    if (!q) return false;
    const auto &L = CassLower();
    const l7::CassQuery Q = l7::cass_parse_query(q, qn, L.data(), (uint32_t)(L.size() / 2));
    return Q.status == l7::CQ_OK && Q.is_use;
}

// A QUERY frame "use ''": the empty keyspace, for replays that must not see
// a USE the batch holds before them
std::string CassEmptyUse() {
    const std::string q = "use ''";
    std::string f = {4, 0, 0, 0, 7, 0, 0, 0, (char)(4 + q.size()), 0, 0, 0, (char)q.size()};
    return f + q;
}

const uint8_t kCassUnauth[35] = {0, 0, 0, 0, 0, 0, 0, 0, 0x1a, 0, 0, 0x21, 0, 0, 0x14, 'R', 'e', 'q',
                                 'u', 'e', 's', 't', ' ', 'U', 'n', 'a', 'u', 't', 'h', 'o', 'r', 'i', 'z',
                                 'e', 'd'};  // unauthMsgBase (cassandraparser.go:269-278)
const uint8_t kCassUnprepared[13] = {0, 0, 0, 0, 0, 0, 0, 0, 0x1a, 0, 0, 0x25, 0};  // unpreparedMsgBase (:284-292)

struct Cached {
    uint8_t v;
    int32_t rule;
    uint32_t consumed;
};

// ---------------------------------------------------------------- frame proposals
// Where the next frame would start if the one at p is complete; 0 = unknown.
// Only proposals: the device decides, and a wrong guess costs one extra launch.
size_t NextKafka(const std::string &d, size_t p) {
    if (d.size() - p < 4) return 0;
    const uint8_t *b = (const uint8_t *)d.data() + p;
    const int32_t size = (int32_t)((uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3]);
    if (size <= 0 || (uint64_t)size + 4 > d.size() - p) return 0;
    return p + 4 + (size_t)size;
}
size_t NextMcBinary(const std::string &d, size_t p) {
    if (d.size() - p < 24) return 0;
    const uint8_t *b = (const uint8_t *)d.data() + p;
    const uint64_t body = (uint32_t)b[8] << 24 | (uint32_t)b[9] << 16 | (uint32_t)b[10] << 8 | b[11];
    return body + 24 <= d.size() - p ? p + 24 + (size_t)body : 0;
}
size_t NextMcText(const std::string &d, size_t p) {
    const size_t lf = d.find("\r\n", p);
    if (lf == std::string::npos) return 0;
    auto tok = Fields((const uint8_t *)d.data() + p, lf - p);
    size_t next = lf + 2;
    if (!tok.empty() && (tok[0] == "set" || tok[0] == "add" || tok[0] == "replace" || tok[0] == "append" ||
                         tok[0] == "prepend" || tok[0] == "cas")) {
        if (tok.size() < 5) return 0;
        char *end = nullptr;
        const long long n = strtoll(tok[4].c_str(), &end, 10);
        if (!end || *end || n < 0) return 0;
        next += (size_t)n + 2;
    }
    return next <= d.size() ? next : 0;
}
size_t NextLine(const std::string &d, size_t p) {
    const size_t lf = d.find("\r\n", p);
    return lf == std::string::npos ? 0 : lf + 2;
}
size_t NextHttp(const std::string &d, size_t p) {
    const size_t he = d.find("\r\n\r\n", p);
    if (he == std::string::npos) return 0;
    uint64_t cl = 0;
    for (size_t ls = d.find("\r\n", p) + 2; ls < he; ) {  // header lines
        const size_t le = d.find("\r\n", ls);
        const size_t colon = d.find(':', ls);
        if (colon != std::string::npos && colon < le) {
            std::string name = d.substr(ls, colon - ls);
            for (auto &ch : name) ch = (char)tolower((unsigned char)ch);
            if (name == "transfer-encoding") return 0;  // chunked or not: leave it to the device
            if (name == "content-length") cl = strtoull(d.c_str() + colon + 1, nullptr, 10);
        }
        ls = le + 2;
    }
    const uint64_t next = he + 4 + cl;
    return next <= d.size() ? (size_t)next : 0;
}

// ---------------------------------------------------------------- connection
struct Connection {
    std::shared_ptr<Instance> ins;
    uint64_t id = 0;
    bool ingress = false;
    uint32_t src = 0, dst = 0, port = 0;
    std::string policy, proto;
    GoSlice *orig = nullptr, *reply = nullptr;
    uint32_t slot = 0;
    Kind kind = K_MEMCACHE;
    // verdicts of this OnData call's proposed frames, by offset from the start
    // of the call's input; `base` = input bytes already consumed in this call
    std::map<uint64_t, Cached> batch;
    uint64_t base = 0;
    // memcache parser state
    int mode = 0;  // 0 none yet, L7G_CONN_MC_TEXT, L7G_CONN_MC_BINARY
    struct Intent { std::string command; bool denied; };
    std::deque<Intent> reply_queue;
    bool watching = false;
    struct Queued { uint8_t magic; uint32_t request; };
    std::deque<Queued> inject_queue;
    uint32_t requests = 0, replies = 0;
    // cassandra parser state (cassandraparser.go:146-160), as raw frames the
    // device re-reads: the frame whose query set the keyspace (a USE), and per
    // stream id / prepared id the PREPARE frame with the USE frame then in force
    std::string cass_use;
    std::map<uint16_t, std::pair<std::string, std::string>> cass_by_stream;
    std::map<std::string, std::pair<std::string, std::string>> cass_by_id;
    std::map<uint64_t, std::pair<std::string, std::string>> cass_exec;  // this call's EXECUTE frames resolved

    GoSlice *InjectBuf(bool r) const { return r ? reply : orig; }
    int64_t Inject(bool r, const void *data, size_t n) {  // connection.go:190-203
        GoSlice *b = InjectBuf(r);
        size_t room = (size_t)(b->cap - b->len), k = n < room ? n : room;
        memcpy((uint8_t *)b->data + b->len, data, k);
        b->len += (GoInt)k;
        return (int64_t)k;
    }
    bool InjectFull(bool r) const { const GoSlice *b = InjectBuf(r); return b->len == b->cap; }

    // Connection.Log (connection.go:211-224): the connection's fields + the
    // parser's L7 record (already encoded as LogEntry field 100 or 102).
    void Log(uint32_t type, const std::string &l7) {
        if (ins->alog.empty()) return;
        std::string m;
        PbU(m, 1, (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                      std::chrono::system_clock::now().time_since_epoch()).count());
        PbU(m, 3, type);
        PbS(m, 4, policy);
        PbU(m, 6, src);
        PbS(m, 7, src_addr);
        PbS(m, 8, dst_addr);
        PbU(m, 15, ingress ? 1 : 0);
        PbU(m, 16, dst);
        m += l7;
        ins->log.Send(m);
    }
    // cilium.L7LogEntry{proto, fields} as LogEntry.generic_l7 (field 102); fields sorted by key
    static std::string GenericL7(const std::string &proto, std::map<std::string, std::string> fields) {
        std::string e;
        PbS(e, 1, proto);
        for (auto &kv : fields) {
            std::string ent;
            PbS(ent, 1, kv.first, true);
            PbS(ent, 2, kv.second, true);
            PbS(e, 2, ent, true);
        }
        std::string o;
        PbS(o, 102, e, true);
        return o;
    }
    // cilium.HttpLogEntry as LogEntry.http (field 100): HTTP/1.1, method, path, host (and status for a denial)
    static std::string HttpL7(const std::string &d, uint32_t status) {
        std::string e, method, path, host;
        const size_t sp1 = d.find(' '), le = d.find("\r\n");
        if (sp1 != std::string::npos && le != std::string::npos && sp1 < le) {
            method = d.substr(0, sp1);
            const size_t sp2 = d.find(' ', sp1 + 1);
            if (sp2 != std::string::npos && sp2 < le) path = d.substr(sp1 + 1, sp2 - sp1 - 1);
            const size_t he = d.find("\r\n\r\n");
            for (size_t ls = le + 2; he != std::string::npos && ls < he;) {
                const size_t e2 = d.find("\r\n", ls), colon = d.find(':', ls);
                if (colon != std::string::npos && colon < e2 && colon - ls == 4) {
                    std::string nm = d.substr(ls, 4);
                    for (auto &ch : nm) ch = (char)tolower((unsigned char)ch);
                    if (nm == "host") {
                        size_t v = colon + 1, ve = e2;
                        while (v < ve && (d[v] == ' ' || d[v] == '\t')) v++;
                        while (ve > v && (d[ve - 1] == ' ' || d[ve - 1] == '\t')) ve--;
                        host = d.substr(v, ve - v);
                        break;
                    }
                }
                ls = e2 + 2;
            }
        }
        PbU(e, 1, 1);  // HttpProtocol HTTP11
        PbS(e, 3, host);
        PbS(e, 4, path);
        PbS(e, 5, method);
        PbU(e, 7, status);
        std::string o;
        PbS(o, 100, e, true);
        return o;
    }
    std::string src_addr, dst_addr;

    l7g_conn_t Attrs() const {
        l7g_conn_t a{};
        a.policy = l7g_policy_index(ins->eng, policy.data(), policy.size());
        a.port = port;
        a.ingress = ingress ? 1 : 0;
        a.proto = kind == K_HTTP ? L7G_PROTO_HTTP : kind == K_KAFKA ? L7G_PROTO_KAFKA
                : kind == K_R2D2 ? L7G_PROTO_R2D2 : kind == K_CASSANDRA ? L7G_PROTO_CASSANDRA : L7G_PROTO_MEMCACHE;
        a.flags = kind == K_MEMCACHE ? (uint16_t)mode : (kind == K_R2D2 || kind == K_CASSANDRA) ? (uint16_t)0
                : (uint16_t)L7G_CONN_PROXYLIB;
        a.src_id = src;
        a.dst_id = dst;
        return a;
    }
    // Device verdict for the request at the start of `data`: from this call's
    // batch if it proposed a frame there, else one kernel lane on its own.
    bool Verdict(const std::string &data, uint8_t *v, int32_t *rule, uint32_t *consumed) {
        auto it = batch.find(base);
        if (it != batch.end()) {
            *v = it->second.v;
            *rule = it->second.rule;
            *consumed = it->second.consumed;
            return true;
        }
        uint64_t off = 0;
        uint32_t len = (uint32_t)data.size(), cid = slot;
        return l7g_classify_host(ins->eng, (const uint8_t *)data.data(), data.size(), &off, &len, &cid, 1, v, rule,
                                 consumed) == 0;
    }
    // Propose the frames of a request-direction input and classify them all in
    // one launch (at most `max` frames).
    bool Prefetch(const std::string &d, size_t max) {
        batch.clear();
        if (d.empty() || max == 0) return true;
        if (kind == K_MEMCACHE && mode == 0) return true;  // the parser is chosen by the first byte first
        std::vector<uint64_t> offs;
        std::vector<uint32_t> lens, cids;
        for (size_t p = 0; p < d.size() && offs.size() < max;) {
            offs.push_back(p);
            lens.push_back((uint32_t)(d.size() - p));
            cids.push_back(slot);
            const size_t q = kind == K_KAFKA ? NextKafka(d, p)
                           : kind == K_HTTP ? NextHttp(d, p)
                           : kind == K_R2D2 ? NextLine(d, p)
                           : mode == L7G_CONN_MC_BINARY ? NextMcBinary(d, p) : NextMcText(d, p);
            if (q <= p) break;
            p = q;
        }
        if (offs.size() < 2) return true;  // one frame: classified when it is reached
        const size_t n = offs.size();
        std::vector<uint8_t> v(n);
        std::vector<int32_t> r(n);
        std::vector<uint32_t> c(n);
        if (l7g_classify_host(ins->eng, (const uint8_t *)d.data(), d.size(), offs.data(), lens.data(), cids.data(),
                              (uint32_t)n, v.data(), r.data(), c.data()) != 0)
            return false;
        for (size_t i = 0; i < n; i++) batch[offs[i]] = Cached{v[i], r[i], c[i]};
        return true;
    }

    // ---- "cassandra" (proxylib/cassandra/cassandraparser.go)
    // Classify the frames at offs of d in one launch, as the device sees a
    // connection's frames: [the frame that set the keyspace] + the frames +
    // per resolvable EXECUTE [its USE frame (or "use ''"), its PREPARE frame],
    // the replayed PREPARE's verdict standing for the EXECUTE's.  Results are
    // kept under key + offset (key = where d starts in this call's input).
    bool CassClassify(const std::string &d, const std::vector<uint64_t> &offs, uint64_t key) {
        std::string arena = cass_use;
        std::vector<uint64_t> o;
        std::vector<uint32_t> l;
        if (!cass_use.empty()) { o.push_back(0); l.push_back((uint32_t)cass_use.size()); }
        const size_t first = o.size();
        for (uint64_t p : offs) { o.push_back(arena.size() + p); l.push_back((uint32_t)(d.size() - p)); }
        arena += d;
        std::vector<std::pair<uint64_t, size_t>> replay;  // (frame offset in d, request index of its PREPARE)
        for (uint64_t p : offs) {
            if (d.size() - p < 11 || d[p + 4] != 0x0A || (d[p] & 0x80) || (d[p + 1] & 1)) continue;
            const uint32_t fl = 9 + Be32(d, p + 5);
            const uint32_t il = Be16(d, p + 9);
            if (fl > d.size() - p || 11u + il > d.size() - p) continue;  // (capacity-bounded slices)
            auto it = cass_by_id.find(d.substr(p + 11, il));
            if (it == cass_by_id.end()) continue;
            const std::string u = it->second.first.empty() ? CassEmptyUse() : it->second.first;
            o.push_back(arena.size()); l.push_back((uint32_t)u.size()); arena += u;
            o.push_back(arena.size()); l.push_back((uint32_t)it->second.second.size()); arena += it->second.second;
            replay.emplace_back(p, o.size() - 1);
            cass_exec[key + p] = it->second;
        }
        const size_t n = o.size();
        std::vector<uint32_t> cids(n, slot);
        std::vector<uint8_t> v(n);
        std::vector<int32_t> r(n);
        std::vector<uint32_t> c(n);
        if (l7g_classify_host(ins->eng, (const uint8_t *)arena.data(), arena.size(), o.data(), l.data(), cids.data(),
                              (uint32_t)n, v.data(), r.data(), c.data()) != 0)
            return false;
        for (size_t i = 0; i < offs.size(); i++) batch[key + offs[i]] = Cached{v[first + i], r[first + i], c[first + i]};
        for (auto &rp : replay) {
            const std::string &pf = cass_exec[key + rp.first].second;
            batch[key + rp.first] =
                Cached{v[rp.second], r[rp.second], 9 + Be32(pf, 5) == c[rp.second] ? 9 + Be32(d, rp.first + 5) : 0};
        }
        return true;
    }
    bool CassPrefetch(const std::string &d, size_t max) {
        cass_exec.clear();
        std::vector<uint64_t> offs;
        for (size_t p = 0; p + 9 <= d.size() && offs.size() < max;) {
            offs.push_back(p);
            const uint64_t fl = 9 + (uint64_t)Be32(d, p + 5);
            if (fl > d.size() - p) break;
            p += fl;
        }
        if (offs.empty()) return true;
        return CassClassify(d, offs, 0);
    }
    int64_t CassOnData(bool r, const std::vector<std::string> &in, int64_t *n, bool *err) {
        std::string d;
        for (auto &b : in) d += b;
        if (d.size() < 9) { *n = 9 - (int64_t)d.size(); return FILTEROP_MORE; }
        const uint32_t rl = Be32(d, 5);
        if (rl > 268435456u) { *n = FILTEROP_ERROR_INVALID_FRAME_LENGTH; return FILTEROP_ERROR; }
        const int64_t missing = 9 + (int64_t)rl - (int64_t)d.size();
        if (missing > 0) { *n = missing; return FILTEROP_MORE; }
        const uint32_t fl = 9 + rl;
        const std::string f = d.substr(0, fl);
        if (r) {  // cassandraParseReply (:605-642): RESULT / prepared binds a prepared id
            // (slices of data[0:fl] are bounded by the joined buffer's capacity, d.size())
            if ((f[0] & 0x80) && !(f[1] & 1) && f[4] == 0x08) {
                if (d.size() < 13) throw Panic();
                if (Be32(d, 9) == 4) {
                    if (d.size() < 15) throw Panic();
                    const uint32_t il = Be16(d, 13);
                    if (15u + il > d.size()) throw Panic();
                    auto it = cass_by_stream.find((uint16_t)Be16(f, 2));
                    if (it != cass_by_stream.end()) cass_by_id[d.substr(15, il)] = it->second;
                }
            }
            *n = fl;
            return FILTEROP_PASS;
        }
        if (batch.find(base) == batch.end() && !CassClassify(d, {0}, base)) { *err = true; *n = 0; return FILTEROP_ERROR; }
        const Cached res = batch[base];
        if (res.v == L7G_PARSE_ERROR) {
            if (res.consumed == 0) throw Panic();  // a Go panic in cassandraParseRequest
            if (f[4] == 0x0A && res.consumed == FILTEROP_ERROR_INVALID_FRAME_TYPE) {  // no cached path: sendUnpreparedMsg
                uint8_t m[sizeof kCassUnprepared];
                memcpy(m, kCassUnprepared, sizeof m);
                m[0] = (uint8_t)(0x80 | (f[0] & 0x07));
                m[2] = (uint8_t)f[2];
                m[3] = (uint8_t)f[3];
                Inject(true, m, sizeof m);
                Inject(true, d.data() + 9, 2 + Be16(d, 9));
            }
            *n = res.consumed;
            return FILTEROP_ERROR;
        }
        if (res.v != L7G_ALLOW && res.v != L7G_DENY) { *n = res.consumed ? res.consumed : 1; return FILTEROP_MORE; }
        // the request's path: the parser state's bookkeeping, and the access log
        std::string path;
        if (f[4] == 0x0A) {
            auto it = cass_exec.find(base);
            if (it != cass_exec.end()) {
                path = CassPath(it->second.second, it->second.first);
                const size_t k = path.find("prepare");  // strings.Replace(path, "prepare", "execute", 1)
                if (k != std::string::npos) path.replace(k, 7, "execute");
            }
        } else if (f[4] == 0x07 || f[4] == 0x09) {
            // the bytes the parse read: the frame, or up to the query's end when its
            // slice runs past the frame into the buffer (capacity-bounded, as above);
            // kept whole so that a replay to the device parses the same query
            size_t ext = fl;
            if (d.size() >= 13 && 13u + (uint64_t)Be32(d, 9) <= d.size()) ext = std::max<size_t>(ext, 13u + Be32(d, 9));
            const std::string fx = d.substr(0, ext);
            const std::string use_before = cass_use;
            path = CassPath(fx, use_before);
            if (CassIsUse(fx)) cass_use = fx;
            if (f[4] == 0x09) cass_by_stream[(uint16_t)Be16(f, 2)] = {use_before, fx};
        }
        std::vector<std::string> parts;
        for (size_t a = 0;;) {
            const size_t s = path.find('/', a);
            parts.push_back(path.substr(a, s == std::string::npos ? std::string::npos : s - a));
            if (s == std::string::npos) break;
            a = s + 1;
        }
        const bool ok = res.v == L7G_ALLOW;
        if (parts.size() == 4)
            Log(ok ? kEntryRequest : kEntryDenied, GenericL7("cassandra", {{"query_action", parts[2]}, {"query_table", parts[3]}}));
        *n = fl;
        if (ok) return FILTEROP_PASS;
        uint8_t m[sizeof kCassUnauth];
        memcpy(m, kCassUnauth, sizeof m);
        m[0] = (uint8_t)(0x80 | (f[0] & 0x07));
        m[2] = (uint8_t)f[2];
        m[3] = (uint8_t)f[3];
        Inject(true, m, sizeof m);
        return FILTEROP_DROP;
    }

    // ---- "http": a request's verdict from its headers (cilium_l7policy.cc:127-182)
    int64_t HttpOnData(bool r, const std::vector<std::string> &in, int64_t *n, bool *err) {
        std::string d;
        for (auto &b : in) d += b;
        if (r) {  // responses pass; a denial's 403 was injected when the request was dropped
            if (d.empty()) { *n = 0; return NOP; }
            *n = (int64_t)d.size();
            return FILTEROP_PASS;
        }
        if (d.empty()) { *n = 0; return NOP; }
        uint8_t v;
        int32_t rule;
        uint32_t cons;
        if (!Verdict(d, &v, &rule, &cons)) { *err = true; *n = 0; return FILTEROP_ERROR; }
        if (v == L7G_INCOMPLETE) { *n = 1; return FILTEROP_MORE; }
        if (v != L7G_ALLOW && v != L7G_DENY) { *n = FILTEROP_ERROR_INVALID_FRAME_TYPE; return FILTEROP_ERROR; }
        *n = cons;
        if (v == L7G_ALLOW) {
            Log(kEntryRequest, HttpL7(d.substr(0, cons), 0));
            return FILTEROP_PASS;
        }
        Inject(true, kDenied403, sizeof kDenied403 - 1);
        Log(kEntryDenied, HttpL7(d.substr(0, cons), 403));
        return FILTEROP_DROP;
    }

    // ---- "kafka": proto.ReadReq framing, canAccess verdict, deny response
    int64_t KafkaOnData(bool r, const std::vector<std::string> &in, int64_t *n, bool *err) {
        std::string d;
        for (auto &b : in) d += b;
        if (r) {  // responses pass; a denial's error response was injected with the drop
            if (d.empty()) { *n = 0; return NOP; }
            *n = (int64_t)d.size();
            return FILTEROP_PASS;
        }
        if (d.empty()) { *n = 0; return NOP; }
        uint8_t v;
        int32_t rule;
        uint32_t cons;
        if (!Verdict(d, &v, &rule, &cons)) { *err = true; *n = 0; return FILTEROP_ERROR; }
        if (v == L7G_INCOMPLETE) {  // the size prefix tells how much is missing
            if (d.size() < 4) { *n = 4 - (int64_t)d.size(); return FILTEROP_MORE; }
            const uint8_t *b = (const uint8_t *)d.data();
            const uint64_t size = (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3];
            *n = size + 4 > d.size() ? (int64_t)(size + 4 - d.size()) : 1;
            return FILTEROP_MORE;
        }
        if (v != L7G_ALLOW && v != L7G_DENY) { *n = FILTEROP_ERROR_INVALID_FRAME_TYPE; return FILTEROP_ERROR; }
        *n = cons;
        const uint8_t *kb = (const uint8_t *)d.data();
        const std::string l7 = GenericL7("kafka", {
            {"api_key", std::to_string((int16_t)(kb[4] << 8 | kb[5]))},
            {"api_version", std::to_string((int16_t)(kb[6] << 8 | kb[7]))},
            {"correlation_id", std::to_string((int32_t)((uint32_t)kb[8] << 24 | (uint32_t)kb[9] << 16 | (uint32_t)kb[10] << 8 | kb[11]))}});
        if (v == L7G_ALLOW) {
            Log(kEntryRequest, l7);
            return FILTEROP_PASS;
        }
        Log(kEntryDenied, l7);
        std::string resp;
        if (l7::KafkaDenyResponse((const uint8_t *)d.data(), cons, &resp)) Inject(true, resp.data(), resp.size());
        return FILTEROP_DROP;
    }

    // ---- text parser (text/parser.go:72-262)
    int64_t TextInjectFromQueue() {
        int injected = 0;
        for (auto &r : reply_queue) {
            if (!r.denied) break;
            injected++;
            Inject(true, kDeniedText, sizeof kDeniedText - 1);
        }
        for (int i = 0; i < injected; i++) reply_queue.pop_front();
        return (int64_t)injected * (int64_t)(sizeof kDeniedText - 1);
    }
    static bool IsStorage(const std::string &c) {
        return c == "set" || c == "add" || c == "replace" || c == "append" || c == "prepend" || c == "cas";
    }
    static bool IsRetrieval(const std::string &c) { return c.compare(0, 3, "get") == 0 || c.compare(0, 3, "gat") == 0; }
    int64_t UntilEnd(const std::string &d, int64_t *n) {  // text/parser.go:266-273
        size_t e = d.find("\r\nEND\r\n");
        if (e != std::string::npos && e > 0) { *n = (int64_t)e + 7; return FILTEROP_PASS; }
        *n = 1;
        return FILTEROP_MORE;
    }
    int64_t TextOnData(bool r, const std::vector<std::string> &in, int64_t *n, bool *err) {
        if (r) {
            int64_t inj = TextInjectFromQueue();
            if (inj > 0) { *n = inj; return FILTEROP_INJECT; }
            if (in.empty()) { *n = 0; return NOP; }
        }
        std::string d;
        for (auto &b : in) d += b;
        long lf = FindCRLF(d);
        if (lf < 0) { *n = (!d.empty() && d.back() == '\r') ? 1 : 2; return FILTEROP_MORE; }
        auto tok = Fields((const uint8_t *)d.data(), (size_t)lf);
        if (!r) {
            uint8_t v;
            int32_t rule;
            uint32_t cons;
            if (!Verdict(d, &v, &rule, &cons)) { *err = true; *n = 0; return FILTEROP_ERROR; }
            if (v == L7G_INCOMPLETE) { *n = cons; return FILTEROP_MORE; }  // (not reached: CRLF found)
            if (v != L7G_ALLOW && v != L7G_DENY) { *n = 0; return FILTEROP_ERROR; }  // panic / ERROR, 0
            const std::string &cmd = tok[0];
            const size_t nt = tok.size();
            bool noreply = false;
            if (IsRetrieval(cmd)) noreply = false;
            else if (IsStorage(cmd)) noreply = nt == (cmd[0] == 'c' ? 7u : 6u);
            else if (cmd == "delete") noreply = nt == 3;
            else if (cmd == "incr" || cmd == "decr" || cmd == "touch") noreply = nt == 4;
            else if (cmd == "flush_all" || cmd == "cache_memlimit") noreply = tok.back() == "noreply";
            else if (cmd == "quit") noreply = true;
            else if (cmd == "watch") watching = true;
            *n = cons;
            // text/parser.go:163-171: the command and its keys, joined by ", "
            std::string keys;
            const size_t k0 = IsRetrieval(cmd) ? (cmd.compare(0, 3, "gat") == 0 ? 2 : 1) : (IsStorage(cmd) || cmd == "delete" || cmd == "incr" || cmd == "decr" || cmd == "touch") ? 1 : nt;
            const size_t k1 = IsRetrieval(cmd) ? nt : k0 + 1;
            for (size_t k = k0; k < k1 && k < nt; k++) keys += (keys.empty() ? "" : ", ") + tok[k];
            const std::string l7 = GenericL7("textmemcached", {{"command", cmd}, {"keys", keys}});
            if (v == L7G_ALLOW) {
                if (!noreply) reply_queue.push_back({cmd, false});
                Log(kEntryRequest, l7);
                return FILTEROP_PASS;
            }
            if (!noreply) {
                if (reply_queue.empty()) Inject(true, kDeniedText, sizeof kDeniedText - 1);
                else reply_queue.push_back({cmd, true});
            }
            Log(kEntryDenied, l7);
            return FILTEROP_DROP;
        }
        if (reply_queue.empty()) throw Panic();  // p.replyQueue[0]
        const Intent intent = reply_queue.front();
        if (watching) { *n = lf + 2; return FILTEROP_PASS; }
        if (tok.empty()) throw Panic();  // tokens[0]
        const std::string &c = intent.command, &t0 = tok[0];
        if (t0 == "ERROR" || t0 == "CLIENT_ERROR" || t0 == "SERVER_ERROR" || IsStorage(c) || c == "delete" || c == "incr" ||
            c == "decr" || c == "touch" || c == "slabs" || c == "lru" || c == "flush_all" || c == "cache_memlimit" ||
            c == "version" || c == "misbehave") {
            reply_queue.pop_front();
            *n = lf + 2;
            return FILTEROP_PASS;
        }
        if (IsRetrieval(c) || c == "stats") {
            int64_t op = UntilEnd(d, n);
            if (op == FILTEROP_PASS) reply_queue.pop_front();
            return op;
        }
        if (c == "lru_crawler") {
            if (t0 == "OK" || t0 == "BUSY" || t0 == "BADCLASS") { reply_queue.pop_front(); *n = lf + 2; return FILTEROP_PASS; }
            int64_t op = UntilEnd(d, n);
            if (op == FILTEROP_PASS) reply_queue.pop_front();
            return op;
        }
        *n = 0;
        return FILTEROP_ERROR;
    }

    // ---- binary parser (binary/parser.go:58-205)
    void BinaryInjectDenied(uint8_t magic) {
        uint8_t m[sizeof kDeniedBinary];
        memcpy(m, kDeniedBinary, sizeof m);
        m[0] = magic;
        Inject(true, m, sizeof m);
        replies++;
    }
    int64_t BinaryOnData(bool r, const std::vector<std::string> &in, int64_t *n, bool *err) {
        if (r) {
            if (!inject_queue.empty() && inject_queue.front().request == replies + 1) {
                BinaryInjectDenied(inject_queue.front().magic);
                inject_queue.pop_front();
                *n = sizeof kDeniedBinary;
                return FILTEROP_INJECT;
            }
            if (in.empty()) { *n = 0; return NOP; }
        }
        std::string d;
        for (auto &b : in) d += b;
        if (!r) {
            uint8_t v;
            int32_t rule;
            uint32_t cons;
            if (!Verdict(d, &v, &rule, &cons)) { *err = true; *n = 0; return FILTEROP_ERROR; }
            if (v == L7G_INCOMPLETE) { *n = cons; return FILTEROP_MORE; }
            if (v != L7G_ALLOW && v != L7G_DENY) { *n = cons; return FILTEROP_ERROR; }  // ERROR, INVALID_FRAME_TYPE / 0
            requests++;
            *n = cons;
            const uint8_t *hb = (const uint8_t *)d.data();
            const uint32_t klen = (uint32_t)hb[2] << 8 | hb[3], ext = hb[4];
            const std::string l7 = GenericL7("binarymemcached", {{"opcode", std::to_string(hb[1])},
                                                                 {"key", d.size() >= 24 + ext + klen ? d.substr(24 + ext, klen) : std::string()}});
            if (v == L7G_ALLOW) {
                Log(kEntryRequest, l7);
                return FILTEROP_PASS;
            }
            Log(kEntryDenied, l7);
            const uint8_t magic = (uint8_t)(0x81 | (uint8_t)d[0]);
            if (requests == replies + 1) BinaryInjectDenied(magic);
            else inject_queue.push_back({magic, requests});
            inject_queue.push_back({magic, requests});  // enqueued again (binary/parser.go:129-135)
            return FILTEROP_DROP;
        }
        const uint8_t *b = (const uint8_t *)d.data();
        if (d.size() < 24) { *n = 24 - (int64_t)d.size(); return FILTEROP_MORE; }
        const uint32_t body = (uint32_t)b[8] << 24 | (uint32_t)b[9] << 16 | (uint32_t)b[10] << 8 | b[11];
        const uint32_t keylen = (uint32_t)b[2] << 8 | b[3], extras = b[4];
        if (keylen > 0 && 24 + keylen + extras > d.size()) { *n = 24 + keylen + extras - (int64_t)d.size(); return FILTEROP_MORE; }
        if ((b[0] & 0x80) != 0x80) { *n = FILTEROP_ERROR_INVALID_FRAME_TYPE; return FILTEROP_ERROR; }
        Log(kEntryResponse, GenericL7("binarymemcached", {{"opcode", std::to_string(b[1])},
                                                          {"key", d.size() >= 24 + extras + keylen ? d.substr(24 + extras, keylen) : std::string()}}));
        replies++;
        *n = (int64_t)(uint32_t)(body + 24u);
        return FILTEROP_PASS;
    }

    // ---- "r2d2" (proxylib/r2d2/r2d2parser.go:140-214)
    int64_t R2d2OnData(bool r, const std::vector<std::string> &in, int64_t *n, bool *err) {
        std::string d;
        for (auto &b : in) d += b;
        const size_t lf = d.find("\r\n");
        if (lf == std::string::npos) { *n = 1; return FILTEROP_MORE; }
        const int64_t msg_len = (int64_t)lf + 2;
        if (r) { *n = msg_len; return FILTEROP_PASS; }  // replies are not processed
        uint8_t v;
        int32_t rule;
        uint32_t cons;
        if (!Verdict(d, &v, &rule, &cons)) { *err = true; *n = 0; return FILTEROP_ERROR; }
        if (v != L7G_ALLOW && v != L7G_DENY) { *n = 0; return FILTEROP_ERROR; }
        const std::string line = d.substr(0, lf);
        std::vector<std::string> f;  // strings.Split(msgStr, " ")
        for (size_t a = 0;;) {
            const size_t sp = line.find(' ', a);
            f.push_back(line.substr(a, sp == std::string::npos ? std::string::npos : sp - a));
            if (sp == std::string::npos) break;
            a = sp + 1;
        }
        const std::string l7 = GenericL7("r2d2", {{"cmd", f[0]}, {"file", f.size() == 2 ? f[1] : std::string()}});
        *n = msg_len;
        if (v == L7G_ALLOW) {
            Log(kEntryRequest, l7);
            return FILTEROP_PASS;
        }
        Log(kEntryDenied, l7);
        Inject(true, "ERROR\r\n", 7);
        return FILTEROP_DROP;
    }

    // the connection's parser
    int64_t ParserOnData(bool r, const std::vector<std::string> &in, bool first_nonempty, int64_t *n, bool *err) {
        if (kind == K_HTTP) return HttpOnData(r, in, n, err);
        if (kind == K_R2D2) return R2d2OnData(r, in, n, err);
        if (kind == K_KAFKA) return KafkaOnData(r, in, n, err);
        if (kind == K_CASSANDRA) return CassOnData(r, in, n, err);
        // memcache.Parser.OnData (memcached/parser.go:186-202)
        if (mode == 0) {
            if (!first_nonempty) { *n = 0; return NOP; }
            mode = (uint8_t)in[0][0] >= 128 ? L7G_CONN_MC_BINARY : L7G_CONN_MC_TEXT;
            std::lock_guard<std::mutex> g(ins->mu);
            l7g_conn_t a = Attrs();
            if (l7g_conn_update(ins->eng, slot, &a, nullptr, 0) != 0) { *err = true; *n = 0; return FILTEROP_ERROR; }
        }
        return mode == L7G_CONN_MC_TEXT ? TextOnData(r, in, n, err) : BinaryOnData(r, in, n, err);
    }
};

std::shared_mutex g_conn_mu;
std::map<uint64_t, std::shared_ptr<Connection>> g_conns;

std::string Str(GoString s) { return s.p && s.n > 0 ? std::string(s.p, (size_t)s.n) : std::string(); }

// net.SplitHostPort + strconv.ParseUint(port, 10, 32), port != 0 (connection.go:71-78)
bool DstPort(const std::string &addr, uint32_t *port) {
    std::string p;
    if (!addr.empty() && addr[0] == '[') {
        size_t e = addr.find(']');
        if (e == std::string::npos || e + 1 >= addr.size() || addr[e + 1] != ':') return false;
        if (addr.find_first_of("[]", e + 1) != std::string::npos) return false;
        p = addr.substr(e + 2);
    } else {
        size_t c = addr.rfind(':');
        if (c == std::string::npos) return false;
        if (addr.find(':') != c) return false;  // too many colons
        if (addr.find_first_of("[]") != std::string::npos) return false;
        p = addr.substr(c + 1);
    }
    if (p.empty() || p.size() > 20) return false;
    uint64_t v = 0;
    for (char ch : p) {
        if (ch < '0' || ch > '9') return false;
        v = v * 10 + (uint64_t)(ch - '0');
        if (v > 0xFFFFFFFFull) return false;
    }
    if (v == 0) return false;
    *port = (uint32_t)v;
    return true;
}

std::shared_ptr<Instance> FindInstance(uint64_t id) {
    std::lock_guard<std::mutex> g(g_inst_mu);
    auto it = g_instances.find(id);
    return it == g_instances.end() ? nullptr : it->second;
}

}  // namespace

extern "C" {

uint64_t OpenModule(GoSlice params, uint8_t debug) {
    (void)debug;
    std::string node, xds, alog;
    const GoString *kv = (const GoString *)params.data;
    for (GoInt i = 0; i < params.len; i++) {
        std::string k = Str(kv[2 * i]), v = Str(kv[2 * i + 1]);
        if (k == "access-log-path") alog = v;
        else if (k == "xds-path") xds = v;
        else if (k == "node-id") node = v;
        else return 0;
    }
    std::lock_guard<std::mutex> g(g_inst_mu);
    for (auto &it : g_instances) {  // instance.go:91-105
        Instance &o = *it.second;
        if ((node.empty() || o.node == node) && xds == o.xds && alog == o.alog) {
            o.open++;
            return o.id;
        }
    }
    const char *dev = getenv("L7G_DEVICE");
    int device = dev && *dev ? atoi(dev) : 0;
    char err[256];
    l7g_engine *e = l7g_engine_create(device, err, sizeof err);
    if (!e) return 0;  // no GPU: fail loudly, there is no CPU verdict path
    auto ins = std::make_shared<Instance>();
    ins->id = ++g_last_instance;
    ins->open = 1;
    ins->node = node.empty() ? "host~127.0.0.1~libcilium-" + std::to_string(ins->id) + "~localdomain" : node;
    ins->xds = xds;
    ins->alog = alog;
    ins->log.path = alog;
    ins->log.Connect();
    ins->eng = e;
    g_instances[ins->id] = ins;
    return ins->id;
}

void CloseModule(uint64_t id) {
    std::shared_ptr<Instance> dead;
    {
        std::lock_guard<std::mutex> g(g_inst_mu);
        auto it = g_instances.find(id);
        if (it == g_instances.end()) return;
        if (--it->second->open > 0) return;
        dead = it->second;
        g_instances.erase(it);
    }
    // connections still referencing the instance keep it alive until closed
    std::unique_lock<std::shared_mutex> g(g_conn_mu);
    bool used = false;
    for (auto &c : g_conns) used |= c.second->ins == dead;
    if (!used) { l7g_engine_destroy(dead->eng); dead->eng = nullptr; }
}

FilterResult OnNewConnection(uint64_t instance_id, GoString proto, uint64_t connection_id, uint8_t ingress,
                             uint32_t src_id, uint32_t dst_id, GoString src_addr, GoString dst_addr,
                             GoString policy_name, GoSlice *orig_buf, GoSlice *reply_buf) {
    auto ins = FindInstance(instance_id);
    if (!ins) return FILTER_INVALID_INSTANCE;
    std::string p = Str(proto);
    Kind kind;
    if (p == "memcache") kind = K_MEMCACHE;
    else if (p == "http") kind = K_HTTP;
    else if (p == "kafka") kind = K_KAFKA;
    else if (p == "r2d2") kind = K_R2D2;
    else if (p == "cassandra") kind = K_CASSANDRA;
    else return FILTER_UNKNOWN_PARSER;
    uint32_t port;
    if (!DstPort(Str(dst_addr), &port)) return FILTER_INVALID_ADDRESS;
    auto c = std::make_shared<Connection>();
    c->ins = ins;
    c->id = connection_id;
    c->ingress = ingress != 0;
    c->src = src_id;
    c->dst = dst_id;
    c->port = port;
    c->policy = Str(policy_name);
    c->src_addr = Str(src_addr);
    c->dst_addr = Str(dst_addr);
    c->proto = p;
    c->kind = kind;
    c->orig = orig_buf;
    c->reply = reply_buf;
    {
        std::lock_guard<std::mutex> g(ins->mu);
        if (!ins->free_slots.empty()) { c->slot = ins->free_slots.back(); ins->free_slots.pop_back(); }
        else c->slot = ins->next_slot++;
        l7g_conn_t a = c->Attrs();
        if (l7g_conn_update(ins->eng, c->slot, &a, nullptr, 0) != 0) {
            ins->free_slots.push_back(c->slot);
            return FILTER_UNKNOWN_ERROR;
        }
    }
    std::shared_ptr<Connection> old;
    {
        std::unique_lock<std::shared_mutex> g(g_conn_mu);
        auto &slot = g_conns[connection_id];
        old = slot;
        slot = c;
    }
    if (old) {
        std::lock_guard<std::mutex> g(old->ins->mu);
        old->ins->free_slots.push_back(old->slot);
    }
    return FILTER_OK;
}

FilterResult OnData(uint64_t connection_id, uint8_t reply, uint8_t end_stream, GoSlice *data, GoSlice *ops) {
    (void)end_stream;
    std::shared_ptr<Connection> c;
    {
        std::shared_lock<std::shared_mutex> g(g_conn_mu);
        auto it = g_conns.find(connection_id);
        if (it == g_conns.end()) return FILTER_UNKNOWN_CONNECTION;
        c = it->second;
    }
    // input: copies of the caller's [][]byte (not retained past the call)
    std::vector<std::string> in;
    const GoSlice *bufs = (const GoSlice *)data->data;
    for (GoInt i = 0; i < data->len; i++) in.emplace_back((const char *)bufs[i].data, (size_t)bufs[i].len);
    int64_t *op = (int64_t *)ops->data;
    c->base = 0;
    c->batch.clear();
    if (!reply) {  // the request frames of this call: one device launch
        std::string all;
        for (auto &b : in) all += b;
        const size_t room = (size_t)(ops->cap - ops->len);
        if (!(c->kind == K_CASSANDRA ? c->CassPrefetch(all, room) : c->Prefetch(all, room))) return FILTER_UNKNOWN_ERROR;
    }
    try {
        while (ops->len < ops->cap) {  // connection.go:138-172
            int64_t n = 0;
            bool err = false;
            const bool first_nonempty = !in.empty() && !in[0].empty();
            int64_t o = c->ParserOnData(reply != 0, in, first_nonempty, &n, &err);
            if (err) return FILTER_UNKNOWN_ERROR;  // device failure
            if (o == NOP) break;
            if (n == 0) return FILTER_PARSER_ERROR;
            op[2 * ops->len] = o;
            op[2 * ops->len + 1] = n;
            ops->len++;
            if (o == FILTEROP_MORE) break;
            if (o == FILTEROP_PASS || o == FILTEROP_DROP) {  // advanceInput (connection.go:104-116)
                c->base += (uint64_t)n;
                int64_t k = n;
                while (k > 0 && !in.empty()) {
                    if ((size_t)k < in[0].size()) { in[0].erase(0, (size_t)k); k = 0; }
                    else { k -= (int64_t)in[0].size(); in.erase(in.begin()); }
                }
            }
            if (o == FILTEROP_INJECT && c->InjectFull(reply != 0)) break;
        }
    } catch (const Panic &) {
        c->batch.clear();
        return FILTER_PARSER_ERROR;
    }
    c->batch.clear();
    return FILTER_OK;
}

void Close(uint64_t connection_id) {
    std::shared_ptr<Connection> c;
    {
        std::unique_lock<std::shared_mutex> g(g_conn_mu);
        auto it = g_conns.find(connection_id);
        if (it == g_conns.end()) return;
        c = it->second;
        g_conns.erase(it);
    }
    std::lock_guard<std::mutex> g(c->ins->mu);
    l7g_conn_t none{};
    none.policy = -1;
    if (c->ins->eng) l7g_conn_update(c->ins->eng, c->slot, &none, nullptr, 0);
    c->ins->free_slots.push_back(c->slot);
}

}  // extern "C"

// A policy version for one instance (JSON or NPDS protobuf), then every
// connection of the instance re-resolved: policy names may map to new indices.
template <class Update>
static int InstancePolicyUpdate(uint64_t instance_id, Update update, char *err, size_t errlen) {
    auto ins = FindInstance(instance_id);
    if (!ins) {
        if (err && errlen) snprintf(err, errlen, "unknown instance %llu", (unsigned long long)instance_id);
        return -1;
    }
    std::lock_guard<std::mutex> g(ins->mu);
    if (update(ins->eng) != 0) return -1;
    std::shared_lock<std::shared_mutex> gc(g_conn_mu);
    for (auto &kv : g_conns) {
        Connection &c = *kv.second;
        if (c.ins != ins) continue;
        l7g_conn_t a = c.Attrs();
        if (l7g_conn_update(ins->eng, c.slot, &a, err, errlen) != 0) return -1;
    }
    return 0;
}

extern "C" {

int l7g_proxylib_policy_update(uint64_t instance_id, const char *json, size_t len, char *err, size_t errlen) {
    return InstancePolicyUpdate(
        instance_id,
        [&](l7g_engine *e) { return l7g_policy_update_view(e, (const uint8_t *)json, len, 0, 1, err, errlen); }, err,
        errlen);
}

int l7g_proxylib_policy_update_proto(uint64_t instance_id, const uint8_t *buf, size_t len, char *err, size_t errlen) {
    return InstancePolicyUpdate(
        instance_id, [&](l7g_engine *e) { return l7g_policy_update_view(e, buf, len, 1, 1, err, errlen); }, err,
        errlen);
}

uint64_t l7g_proxylib_connections(void) {
    std::shared_lock<std::shared_mutex> g(g_conn_mu);
    return g_conns.size();
}

}  // extern "C"
