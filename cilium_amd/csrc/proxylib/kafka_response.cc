// Kafka deny response (product code, host side): what the reference's Kafka
// proxy sends back for a request policy denies.
//
//   pkg/proxy/kafka.go:249-261      canAccess fails => req.CreateResponse(
//                                   proto.ErrTopicAuthorizationFailed), enqueued
//                                   to the client; a nil (untyped) request has
//                                   no response (CreateResponse errors)
//   pkg/kafka/request.go:158-182    CreateResponse: one builder per typed kind
//   pkg/kafka/response.go:81-315    the builders: every topic and partition of
//                                   the request echoed with the error set
//   vendor/.../proto/messages.go    the encoders: MetadataResp.Bytes :610,
//                                   FetchResp.Bytes :911, ConsumerMetadataResp
//                                   .Bytes :1117, OffsetCommitResp.Bytes :1342,
//                                   OffsetFetchResp.Bytes :1531, ProduceResp
//                                   .Bytes :1716, OffsetResp.Bytes :1975
//   vendor/.../proto/errors.go:37   ErrTopicAuthorizationFailed = errno 29
//
// The request is decoded here again, on the host (it is only done for denied
// requests, whose verdict the device has already given): the typed decoders
// restated sequentially (messages.go:504-1858, serialization.go), keeping only
// what the response echoes -- correlation id, version, topic names, partition
// ids, and whether a nullable topic array was null.
#include <cstdint>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

namespace l7 {
namespace kresp {

constexpr uint32_t kMaxParseBuf = 6553500;
constexpr int16_t kErrTopicAuthorizationFailed = 29;
// time.Time{}.UnixNano() / int64(time.Millisecond) under Go 1.10's int64
// wrap-around: the ListOffsets v1+ timestamp of a response built from
// OffsetRespPartition{} (messages.go:1996)
constexpr int64_t kZeroTimeMillis = -6795364578871LL;

struct Dec {  // decoder over a bytes.Buffer: short reads leave zeros, errors are sticky
    const uint8_t *b;
    size_t pos, end;
    bool err = false;
    uint64_t Int(int n) {
        if (err) return 0;
        if (end - pos < (size_t)n) { err = true; pos = end; return 0; }
        uint64_t v = 0;
        for (int i = 0; i < n; i++) v = v << 8 | b[pos + i];
        pos += (size_t)n;
        return v;
    }
    std::string Str() {  // DecodeString: i16 length, < 1 => ""
        int16_t n = (int16_t)Int(2);
        if (err || n < 1) return std::string();
        if (end - pos < (size_t)n) { err = true; pos = end; return std::string(); }
        std::string s((const char *)b + pos, (size_t)n);
        pos += (size_t)n;
        return s;
    }
    int64_t ArrLen(bool nullable, bool *bad) {  // DecodeArrayLen
        int32_t l = (int32_t)Int(4);
        *bad = false;
        if (l < 0) {
            if (nullable) return -1;
            *bad = true;
            return 0;
        }
        if ((uint32_t)l > kMaxParseBuf) { *bad = true; return 0; }
        return l;
    }
    void Skip(size_t n) {
        if (err) return;
        if (end - pos < n) { err = true; pos = end; return; }
        pos += n;
    }
    void Bytes() {  // DecodeBytes, dropped
        int32_t n = (int32_t)Int(4);
        if (err || n < 1) return;
        if ((uint32_t)n > kMaxParseBuf) { err = true; return; }
        Skip((size_t)n);
    }
};

struct Topic {
    std::string name;
    std::vector<int32_t> parts;
};
struct Req {
    int16_t kind = 0, version = 0;
    int32_t corr = 0;
    bool topics_null = false;  // Metadata / OffsetFetch: a null topic array
    std::vector<Topic> topics;
    std::vector<std::string> meta_topics;  // Metadata: the raw topic strings
};

uint32_t Crc32(const uint8_t *p, size_t n) {  // hash/crc32.ChecksumIEEE
    static uint32_t tab[256];
    static bool init = [] {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            tab[i] = c;
        }
        return true;
    }();
    (void)init;
    uint32_t c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; i++) c = tab[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return ~c;
}

// readMessageSet (messages.go:363-494) for its effect on the position and on
// errors (a CRC mismatch stops the set without draining it); 0 ok, -1 error.
int SkipMessageSet(Dec &d, int32_t size, int16_t version) {
    if (size < 0) return 0;
    if ((uint32_t)size > kMaxParseBuf) return -1;
    const size_t lim = std::min(d.end, d.pos + (size_t)size);
    Dec s{d.b, d.pos, lim};
    for (;;) {
        (void)s.Int(8);
        if (s.err) break;
        int32_t msize = (int32_t)s.Int(4);
        if (s.err || msize <= 0) break;
        if ((uint32_t)msize > kMaxParseBuf) return -1;
        const size_t at = s.pos;
        s.Skip((size_t)msize);
        if (s.err) break;
        if (msize <= 4) break;
        const uint32_t crc = (uint32_t)d.b[at] << 24 | (uint32_t)d.b[at + 1] << 16 | (uint32_t)d.b[at + 2] << 8 | d.b[at + 3];
        if (crc != Crc32(d.b + at + 4, (size_t)msize - 4)) break;  // stop, no drain
        Dec m{d.b, at + 4, at + (size_t)msize};
        (void)m.Int(1);
        const int8_t attr = (int8_t)m.Int(1);
        if (version >= 1) (void)m.Int(8);
        if ((attr & 3) == 3) break;
        m.Bytes();
        m.Bytes();
        if (m.err) return -1;
        if ((attr & 3) != 0) break;  // compressed: the inner set does not change the echoed fields
    }
    d.pos = s.pos;
    return 0;
}

// kafka.ReadRequest + the typed decoder; false = no response (untyped kind,
// framing or decode error).
bool Decode(const uint8_t *b, size_t len, Req *q) {
    if (len < 12) return false;
    const int32_t size = (int32_t)((uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3]);
    if (size <= 0 || (uint64_t)size + 4 > len || (uint64_t)size + 4 > kMaxParseBuf || size + 4 < 12) return false;
    Dec d{b, 0, (size_t)size + 4};
    (void)d.Int(4);
    q->kind = (int16_t)d.Int(2);
    q->version = (int16_t)d.Int(2);
    q->corr = (int32_t)d.Int(4);
    const int16_t v = q->version;
    (void)d.Str();  // ClientID
    bool bad = false;
    int64_t nt = 0, np = 0;
    switch (q->kind) {
    case 0:  // Produce (messages.go:1591-1647)
        if (v >= 3) (void)d.Str();
        (void)d.Int(2);
        (void)d.Int(4);
        nt = d.ArrLen(false, &bad);
        if (bad) return false;
        for (int64_t t = 0; t < nt; t++) {
            Topic T;
            T.name = d.Str();
            if (d.err) return false;
            np = d.ArrLen(false, &bad);
            if (bad) return false;
            for (int64_t p = 0; p < np; p++) {
                T.parts.push_back((int32_t)d.Int(4));
                const int32_t ss = (int32_t)d.Int(4);
                if (d.err) return false;
                if (SkipMessageSet(d, ss, v) < 0) return false;
            }
            q->topics.push_back(std::move(T));
        }
        break;
    case 1:  // Fetch (messages.go:767-824)
        d.Skip(12);
        if (v >= 3) d.Skip(4);
        if (v >= 4) d.Skip(1);
        nt = d.ArrLen(false, &bad);
        if (bad) return false;
        for (int64_t t = 0; t < nt && !d.err; t++) {
            Topic T;
            T.name = d.Str();
            np = d.ArrLen(false, &bad);
            if (bad) return false;
            for (int64_t p = 0; p < np && !d.err; p++) {
                T.parts.push_back((int32_t)d.Int(4));
                d.Skip(v >= 5 ? 20 : 12);
            }
            q->topics.push_back(std::move(T));
        }
        break;
    case 2:  // ListOffsets (messages.go:1810-1858)
        d.Skip(4);
        if (v >= 2) d.Skip(1);
        nt = d.ArrLen(false, &bad);
        if (bad) return false;
        for (int64_t t = 0; t < nt && !d.err; t++) {
            Topic T;
            T.name = d.Str();
            np = d.ArrLen(false, &bad);
            if (bad) return false;
            for (int64_t p = 0; p < np && !d.err; p++) {
                T.parts.push_back((int32_t)d.Int(4));
                d.Skip(v == 0 ? 12 : 8);
            }
            q->topics.push_back(std::move(T));
        }
        break;
    case 3:  // Metadata (messages.go:504-537)
        nt = d.ArrLen(true, &bad);
        if (bad) return false;
        q->topics_null = nt < 0;
        for (int64_t t = 0; t < nt && !d.err; t++) {
            std::string s = d.Str();
            if (!d.err) q->meta_topics.push_back(std::move(s));
        }
        if (v >= 4) d.Skip(1);
        break;
    case 8:  // OffsetCommit (messages.go:1173-1228)
        (void)d.Str();
        if (v >= 1) { d.Skip(4); (void)d.Str(); }
        if (v >= 2) d.Skip(8);
        nt = d.ArrLen(false, &bad);
        if (bad) return false;
        for (int64_t t = 0; t < nt && !d.err; t++) {
            Topic T;
            T.name = d.Str();
            np = d.ArrLen(false, &bad);
            if (bad) return false;
            for (int64_t p = 0; p < np && !d.err; p++) {
                T.parts.push_back((int32_t)d.Int(4));
                d.Skip(v == 1 ? 16 : 8);
                (void)d.Str();
            }
            q->topics.push_back(std::move(T));
        }
        break;
    case 9:  // OffsetFetch (messages.go:1389-1430)
        (void)d.Str();
        nt = d.ArrLen(true, &bad);
        if (bad) return false;
        q->topics_null = nt < 0;
        for (int64_t t = 0; t < nt && !d.err; t++) {
            Topic T;
            T.name = d.Str();
            np = d.ArrLen(false, &bad);
            if (bad) return false;
            for (int64_t p = 0; p < np && !d.err; p++) T.parts.push_back((int32_t)d.Int(4));
            q->topics.push_back(std::move(T));
        }
        break;
    case 10:  // ConsumerMetadata (messages.go:1033-1054)
        (void)d.Str();
        if (v >= 1) d.Skip(1);
        break;
    default:
        return false;  // request == nil: "unsupported request API key"
    }
    return !d.err;
}

struct Enc {
    std::string out;
    void I8(int8_t v) { out.push_back((char)v); }
    void I16(int16_t v) { out.push_back((char)(v >> 8)); out.push_back((char)v); }
    void I32(int32_t v) { for (int s = 24; s >= 0; s -= 8) out.push_back((char)((uint32_t)v >> s)); }
    void I64(int64_t v) { for (int s = 56; s >= 0; s -= 8) out.push_back((char)((uint64_t)v >> s)); }
    void Str(const std::string &s) { I16((int16_t)(uint16_t)s.size()); out += s; }
    void Arr(int32_t n) { I32(n); }
};

// The *Resp.Bytes encoders for a response built by createXResponse with err.
std::string Encode(const Req &q, int16_t err) {
    Enc e;
    const int16_t v = q.version;
    e.I32(0);  // size placeholder
    e.I32(q.corr);
    switch (q.kind) {
    case 0:  // ProduceResp.Bytes (:1716)
        e.Arr((int32_t)q.topics.size());
        for (auto &t : q.topics) {
            e.Str(t.name);
            e.Arr((int32_t)t.parts.size());
            for (int32_t p : t.parts) {
                e.I32(p);
                e.I16(err);
                e.I64(0);             // Offset
                if (v >= 2) e.I64(0);  // LogAppendTime
            }
        }
        if (v >= 1) e.I32(0);  // ThrottleTime
        break;
    case 1:  // FetchResp.Bytes (:911)
        if (v >= 1) e.I32(0);
        e.Arr((int32_t)q.topics.size());
        for (auto &t : q.topics) {
            e.Str(t.name);
            e.Arr((int32_t)t.parts.size());
            for (int32_t p : t.parts) {
                e.I32(p);
                e.I16(err);
                e.I64(0);  // TipOffset
                if (v >= 4) {
                    e.I64(0);              // LastStableOffset
                    if (v >= 5) e.I64(0);  // LogStartOffset
                    e.Arr(-1);             // AbortedTransactions: nil
                }
                e.I32(0);  // message set size (no messages)
            }
        }
        break;
    case 2:  // OffsetResp.Bytes (:1975)
        if (v >= 2) e.I32(0);
        e.Arr((int32_t)q.topics.size());
        for (auto &t : q.topics) {
            e.Str(t.name);
            e.Arr((int32_t)t.parts.size());
            for (int32_t p : t.parts) {
                e.I32(p);
                e.I16(err);
                if (v >= 1) e.I64(kZeroTimeMillis);
                e.Arr(0);  // Offsets: empty, not nil
            }
        }
        break;
    case 3:  // MetadataResp.Bytes (:610)
        if (v >= 3) e.I32(0);
        e.Arr(0);              // Brokers: empty, not nil
        if (v >= 2) e.Str(""); // ClusterID
        if (v >= 1) e.I32(0);  // ControllerID
        if (q.topics_null) {
            e.Arr(-1);
        } else {
            e.Arr((int32_t)q.meta_topics.size());
            for (auto &t : q.meta_topics) {
                e.I16(err);
                e.Str(t);
                if (v >= 1) e.I8(0);  // IsInternal
                e.Arr(0);             // Partitions: empty, not nil
            }
        }
        break;
    case 8:  // OffsetCommitResp.Bytes (:1342)
        if (v >= 3) e.I32(0);
        e.Arr((int32_t)q.topics.size());
        for (auto &t : q.topics) {
            e.Str(t.name);
            e.Arr((int32_t)t.parts.size());
            for (int32_t p : t.parts) {
                e.I32(p);
                e.I16(err);
            }
        }
        break;
    case 9:  // OffsetFetchResp.Bytes (:1531)
        if (v >= 3) e.I32(0);
        if (q.topics_null) {
            e.Arr(-1);
        } else {
            e.Arr((int32_t)q.topics.size());
            for (auto &t : q.topics) {
                e.Str(t.name);
                e.Arr((int32_t)t.parts.size());
                for (int32_t p : t.parts) {
                    e.I32(p);
                    e.I64(0);   // Offset
                    e.Str("");  // Metadata
                    e.I16(err);
                }
            }
        }
        if (v >= 2) e.I16(0);  // Err: nil
        break;
    default:  // 10: ConsumerMetadataResp.Bytes (:1117)
        if (v >= 1) e.I32(0);
        e.I16(err);
        if (v >= 1) e.Str("");  // ErrMsg
        e.I32(0);               // CoordinatorID
        e.Str("");              // CoordinatorHost
        e.I32(0);               // CoordinatorPort
        break;
    }
    const uint32_t n = (uint32_t)(e.out.size() - 4);
    for (int i = 0; i < 4; i++) e.out[i] = (char)(n >> (24 - 8 * i));
    return std::move(e.out);
}

}  // namespace kresp

// The bytes the reference's Kafka proxy answers a denied request with, or
// false if it answers nothing.
bool KafkaDenyResponse(const uint8_t *req, size_t len, std::string *out) {
    kresp::Req q;
    if (!kresp::Decode(req, len, &q)) return false;
    *out = kresp::Encode(q, kresp::kErrTopicAuthorizationFailed);
    return true;
}

}  // namespace l7

extern "C" int l7g_kafka_deny_response(const uint8_t *req, size_t len, uint8_t *out, size_t cap, size_t *outlen) {
    std::string r;
    if (!l7::KafkaDenyResponse(req, len, &r)) return -1;
    if (outlen) *outlen = r.size();
    if (r.size() > cap) return -2;
    if (!r.empty()) memcpy(out, r.data(), r.size());
    return 0;
}
