// Device-resident rule tables (product code).  Plain POD structs shared by the
// host-side compiler (C++) and the gfx950 kernels (HIP).  Everything is laid
// out in one contiguous "table blob" per policy version; the kernels receive
// typed pointers into it through HttpTables / KafkaTables (kernel arguments).
#pragma once
#include <stdint.h>

namespace l7 {

enum : uint8_t {
    V_DENY = 0, V_ALLOW = 1, V_PARSE_ERROR = 2, V_INCOMPLETE = 3, V_UNSUPPORTED = 4,
};
enum : uint8_t { PROTO_NONE = 0, PROTO_HTTP = 1, PROTO_KAFKA = 2, PROTO_MEMCACHE = 3 };

// Header slots recorded by the HTTP framer.
enum : int { SLOT_METHOD = 0, SLOT_PATH = 1, SLOT_AUTHORITY = 2, SLOT_CUSTOM0 = 3 };
constexpr int kMaxCustomHeaders = 8;
constexpr int kNumSlots = SLOT_CUSTOM0 + kMaxCustomHeaders;

// Per connection (8 B): which compiled rule set applies.  Resolved on the host
// once per connection (proxylib OnNewConnection), never per request.
struct DevConn {
    int32_t ruleset;   // index into HttpTables::rulesets / KafkaTables::rulesets
    uint8_t proto;     // PROTO_*
    uint8_t pad[3];
};

// ---------------- HTTP ----------------
struct DevDfa {            // 16 B
    uint32_t trans_off;    // u16 units into HttpTables::trans ([nstates][ncls])
    uint32_t mask_off;     // u64 units into HttpTables::masks ([nstates], rule-chunk mask at EOF)
    uint32_t cls_off;      // byte offset into HttpTables::cls (256 B byte->class map)
    uint16_t ncls;
    uint16_t start;
};
struct DevField {          // 16 B: one header field of one rule chunk
    uint8_t slot;          // SLOT_*
    uint8_t ndfa;
    uint16_t pad;
    uint32_t dfa_first;
    uint64_t absent_mask;  // rules of the chunk satisfied when the header is absent
};
struct DevChunk {          // 32 B: <= 64 rules evaluated with one u64 mask
    uint64_t all_mask;
    uint32_t field_first;
    uint16_t nfields;
    uint16_t nrules;
    uint32_t rule_id_off;  // int32 global rule ids, in evaluation order
    uint32_t pad[3];
};
struct DevHdrName {        // 12 B: custom header names a rule set looks at
    uint32_t hash;         // FNV-1a of the lower-cased name
    uint16_t len;
    uint16_t pad;
    uint32_t name_off;     // byte offset into HttpTables::names
};
struct DevRuleset {        // 16 B
    uint32_t chunk_first;
    uint16_t nchunks;
    uint8_t nhdr;
    uint8_t terminal;      // verdict when no rule matches (V_ALLOW => rule -1)
    uint32_t hdr_first;
    uint32_t pad;
};

struct HttpTables {
    const DevRuleset *rulesets;
    const DevChunk *chunks;
    const DevField *fields;
    const DevDfa *dfas;
    const uint16_t *trans;
    const uint64_t *masks;
    const uint8_t *cls;
    const int32_t *rule_ids;
    const DevHdrName *hdrs;
    const uint8_t *names;
    uint32_t nrulesets;
    uint32_t pad;
};

// ---------------- Kafka ----------------
// Rule semantics: pkg/kafka/policy.go ruleMatches :144-195 / MatchesRule :200-225.
struct DevKafkaRule {      // 24 B
    uint64_t keymask;      // allowed api keys 0..63 (CheckAPIKeyRole)
    int32_t client;        // interned client id, -1 = no ClientID constraint
    int32_t gid;           // global rule id (-1 for the L3-only wildcard)
    int16_t version;
    uint8_t any_key;       // apiKeyInt empty
    uint8_t has_version;
    uint8_t has_topic;
    uint8_t pad[3];
};
struct DevKafkaRuleset {   // 32 B
    uint32_t rule_first, nrules;     // rules in evaluation order
    uint32_t topicless_off, ntopicless;  // u32 rule positions (Topic == "") in index[]
    uint32_t topics_off, ntopics;    // sorted (topic_id, list_off, list_cnt) triples in index[]
    uint32_t bykey_off;              // 65 (off, cnt) pairs in index[]: key 0..63, 64 = other kinds
    uint8_t any;                     // rules.Kafka != nil (pkg/proxy/kafka.go:139-142)
    uint8_t pad[3];
};
struct DevStrSlot {        // 16 B open-addressing slot (topics, client ids)
    uint32_t hash;         // FNV-1a (case-sensitive)
    uint32_t str_off;
    uint16_t len;
    uint16_t used;
    int32_t id;
};
struct KafkaTables {
    const DevKafkaRuleset *rulesets;
    const DevKafkaRule *rules;
    const uint32_t *index;
    const DevStrSlot *topic_hash;
    const DevStrSlot *client_hash;
    const uint8_t *strings;
    uint32_t nrulesets;
    uint32_t topic_mask, client_mask;  // hash table size - 1
    uint32_t pad;
};

// FNV-1a over lower-cased ASCII (header names are tchar, i.e. ASCII)
static inline uint32_t l7_fnv_step(uint32_t h, uint8_t c) {
    if (c >= 'A' && c <= 'Z') c = (uint8_t)(c + 32);
    return (h ^ c) * 16777619u;
}
constexpr uint32_t kFnvBasis = 2166136261u;

}  // namespace l7
