// Device-resident rule tables (product code).  Plain POD structs shared by the
// host-side compiler (C++) and the gfx950 kernels (HIP).  Everything is laid
// out in one contiguous "table blob" per policy version; the kernels receive
// typed pointers into it through HttpTables / KafkaTables (kernel arguments).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define L7_HD __host__ __device__
#else
#define L7_HD
#endif

namespace l7 {

enum : uint8_t {
    V_DENY = 0, V_ALLOW = 1, V_PARSE_ERROR = 2, V_INCOMPLETE = 3, V_UNSUPPORTED = 4,
};
enum : uint8_t { PROTO_NONE = 0, PROTO_HTTP = 1, PROTO_KAFKA = 2, PROTO_MEMCACHE = 3, PROTO_R2D2 = 4, PROTO_CASSANDRA = 5 };
// a protocol some classifier owns (the others answer its requests UNSUPPORTED)
#define L7_PROTO_OWNED(p) ((p) >= PROTO_HTTP && (p) <= PROTO_CASSANDRA)

// partition_kernel groups Kafka requests into this many kind / length classes
#ifndef L7_KAFKA_CLASSES
#define L7_KAFKA_CLASSES 8
#endif

// Header slots recorded by the HTTP framer.
enum : int { SLOT_METHOD = 0, SLOT_PATH = 1, SLOT_AUTHORITY = 2, SLOT_CUSTOM0 = 3 };
constexpr int kMaxCustomHeaders = 8;
constexpr int kNumSlots = SLOT_CUSTOM0 + kMaxCustomHeaders;

// Per connection (8 B): which compiled rule set applies.  Resolved on the host
// once per connection (proxylib OnNewConnection), never per request.
struct DevConn {
    int32_t ruleset;   // index into HttpTables::rulesets / KafkaTables::rulesets
    uint8_t proto;     // PROTO_*
    uint8_t flags;     // memcached: L7G_CONN_MC_TEXT / _BINARY (0 = by first byte)
    uint16_t skey;     // proxy-statistics key (policy, proto, port, direction); 0xFFFF none
};

// One l7g_classify call as the kernels see it (passed by value): request i is
// arena[offs[i] .. offs[i] + lens[i]) on connection conn_ids[i]; outputs are
// indexed by i.  (The call's counters are histogrammed from verdict / rule
// after the classifiers: kernels/counters.hip.)
struct Batch {
    const uint8_t *arena;
    uint64_t arena_len;
    const uint64_t *offs;
    const uint32_t *lens;
    const uint32_t *conn_ids;
    const DevConn *conns;
    uint8_t *verdict;
    int32_t *rule;
    uint32_t *consumed;
    uint32_t n, nconns;
};

// A request whose bytes leave [arena, arena + arena_len) is out of contract:
// every kernel answers it UNSUPPORTED instead of reading past the arena.
L7_HD inline bool l7_in_arena(uint64_t off, uint32_t len, uint64_t arena_len) {
    return off <= arena_len && (uint64_t)len <= arena_len - off;
}

// ---------------- HTTP ----------------
// Every HTTP rule set is one self-contained, 16-byte aligned "image": a
// header, DFA descriptors, per-chunk masks, rule ids, custom header names,
// and the DFA tables themselves.  All offsets are bytes from the image start,
// so the kernel can stage the image of the hottest rule set in LDS and
// address it with the same offsets it uses for images left in HBM.
//
// A rule set's rules are split into chunks of <= 64 rules (u64 masks, bit b
// of chunk c = rule 64c+b in evaluation order).  The patterns of each header
// slot, over all rules of the rule set, are compiled into one DFA (several if
// the state budget is exceeded); a DFA state carries, per chunk, the mask of
// rules whose matcher on that slot holds if the value ends in that state.
constexpr int kChunksPerPass = 4;       // chunk accumulators the kernel keeps in registers
constexpr int kDfasPerPass = 1;         // DFAs per slot walked in one framing pass
constexpr uint32_t kLdsImageBytes = 32 * 1024;  // LDS budget for the hot rule-set image
// Requests grouped by rule set (kernels/http_group.hip): at most this many HTTP
// rule sets (one LDS histogram bin each), runs cut into segments of at most
// kGroupSegEntries entries, images up to kGroupImageBytes staged (the grouped
// kernel keeps two control words after them).
constexpr uint32_t kMaxGroupRulesets = 4096;
// (a workgroup waits at a barrier between segments while the next image is
// staged: cfg4 5.46 / 5.21 / 5.28 / 5.63 ms at 2048 / 4096 / 8192 / 16384
// entries, 5.66 at 1024; profiles/r5/ab5g_group_segment.log)
constexpr uint32_t kGroupSegEntries = 4096;
constexpr uint32_t kGroupImageBytes = kLdsImageBytes - 16;

// Header-name recognition: every image carries a small DFA over the
// lower-cased name bytes that spells out the names the framer must know
// (host, content-length, transfer-encoding and the rule set's custom header
// names).  State 0 = a non-tchar byte was seen, 1 = valid name that is none
// of them, 2 = start.  name_info[state] = NI_* flags of the name ending there.
enum : uint8_t { NI_CUSTOM = 0x0F /* custom index + 1 */, NI_HOST = 0x10, NI_CL = 0x20, NI_TE = 0x40 };
constexpr uint16_t kNameBad = 0, kNameOther = 1, kNameStart = 2;

struct DevDfa {            // 24 B
    uint32_t cls_off;      // u8[256]: byte -> class
    uint32_t trans_off;    // u16[nstates][ncls]; state 0 = dead
    uint32_t mask_off;     // u64[nstates][nchunks]
    uint16_t ncls;
    uint16_t start;
    uint32_t absorb;       // states >= absorb (and 0) loop back on every HT/SP/VCHAR/obs-text byte
    uint32_t pad;
};
struct DevHdrName {        // 12 B: a custom header name the rule set looks at
    uint32_t hash;         // FNV-1a of the lower-cased name
    uint16_t len;
    uint16_t pad;
    uint32_t name_off;     // lower-cased bytes
};
struct ImgHeader {         // 80 B, at offset 0 of every image
    uint8_t nchunks;
    uint8_t nhdr;
    uint8_t terminal;      // verdict when no rule matches (V_ALLOW => rule -1)
    uint8_t ndfa;
    uint8_t slot_dfa[kNumSlots + 1];  // DFAs of slot s: [slot_dfa[s], slot_dfa[s+1])
    uint8_t max_slot_dfas; // most DFAs on one slot (framing passes = ceil(/kDfasPerPass))
    uint8_t pad0[3];
    uint16_t ref_slots;    // slots some rule constrains
    uint16_t pad1;
    uint32_t dfa_off;      // DevDfa[ndfa]
    uint32_t init_off;     // u64[nchunks]: rules of the chunk (minus those on never-present headers)
    uint32_t absent_off;   // u64[kNumSlots][nchunks]: rules satisfied when the slot is absent
    uint32_t rule_off;     // i32[nchunks * 64]: global rule ids
    uint32_t hdr_off;      // DevHdrName[nhdr]
    uint32_t total_states;
    uint32_t name_cls_off;    // u8[256]: byte -> class (0 = not a tchar; case folded)
    uint32_t name_trans_off;  // u16[name_states][name_ncls]
    uint32_t name_info_off;   // u8[name_states]: NI_* flags
    uint16_t name_ncls;
    uint16_t name_states;
    uint32_t nfa_off;      // DevNfaRef[nnfa]
    uint8_t nnfa;
    uint8_t ntab_bits;     // name table: 2^ntab_bits DevNameEnt (0: none)
    uint8_t pad2[2];
    uint32_t ntab_off;     // DevNameEnt[1 << ntab_bits]
    uint32_t ntab_mul;     // multiplier of l7_name_hash, chosen so the names do not collide
};
static_assert(sizeof(ImgHeader) == 80, "ImgHeader layout");

// Header-name table (the framer's one-probe shortcut for the name DFA): the
// names of the name DFA that are at most 15 bytes of [0-9a-z-], lower-cased
// and zero-padded, each in its own slot (a collision-free multiplier is
// searched at compile time).  A header name of <= 15 bytes of [0-9A-Za-z-]
// has NI_* flags info iff its lower-cased bytes equal the slot's name, else 0:
// exactly name_info of the DFA state the name walks to.
struct DevNameEnt {        // 32 B
    uint32_t w[4];         // lower-cased name bytes, zero past len
    uint8_t len;           // 0: empty slot
    uint8_t info;          // NI_* flags
    uint8_t pad[10];
};
L7_HD inline uint32_t l7_name_hash(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t len, uint32_t mul,
                                   uint32_t bits) {
    uint32_t x = w0 ^ (w1 * 0x85EBCA6Bu) ^ (w2 * 0xC2B2AE35u) ^ (w3 * 0x27D4EB2Fu) ^ len;
    x ^= x >> 15;
    return (x * mul) >> (32 - bits);
}

// Bit-parallel rune NFA (the fallback for a pattern whose DFA alone exceeds
// the state budget; re_dfa.h BitNfa, walked by regex/nfa_walk.h).  One DevNfa
// per distinct pattern, in a pool shared by all rule sets; all offsets are
// bytes from the pool start.  t_off: the follow sets tabulated per condition
// class k, per 8-position chunk j of the state and per value v of that chunk:
// u64[K][8W][256][W] (T[k][j][v] = OR of Follow_k(8j + b) for the bits b of v).
constexpr int kNfaMaxWords = 16;  // dense tables, state in registers: <= 1024 positions
// Past that, sparse rows and the state sets in per-lane global scratch (regex/
// nfa_walk.h): Go 1.10 caps each repeat at 1000 and nested repeats at a
// product of 1000 (regexp/syntax repeatIsValid), so a pattern needs about
// 1000 positions per rune class it writes; this bound is the pattern's size.
constexpr int kNfaMaxPositions = 1 << 20;
// Large NFAs (W > kNfaMaxWords) keep their follow sets as sparse rows
// (re_dfa.h BitNfa): DevNfa::t_off then points at this.
struct DevNfaSparse {      // 32 B
    uint64_t row_of_off;   // u32[K][m]: each position's row
    uint64_t row_ptr_off;  // u32[rows + 1]: each row's first pair
    uint64_t pair_w_off;   // u32[pairs]: word index
    uint64_t pair_m_off;   // u64[pairs]: mask
};
struct DevNfa {            // 128 B
    uint32_t m, W, K, nivl;
    uint64_t t_off;
    uint64_t ivl_off;      // u32[nivl]: first rune of each interval (sorted; [0] = 0)
    uint64_t b_off;        // u64[nivl][W]: positions whose class holds the interval
    uint64_t acc_off;      // u64[K][W]
    uint64_t ascii_off;    // u16[128]: interval of each ASCII rune
    uint8_t condmap[64];   // NC_* condition bits -> class
};
// An HTTP rule set's NFA-evaluated matcher (one per distinct pattern): the
// pre-pass (http_nfa_kernel) runs the NFA over the slot's value and sets bit
// k of the request's u64; the framing kernel then ANDs mask row 0 (rejected)
// or 1 (accepted) into the rule accumulators when the slot is present.
constexpr int kMaxNfaPerRuleset = 64;
struct DevNfaRef {         // 16 B
    uint64_t nfa;          // DevNfa offset in the pool
    uint32_t mask_off;     // u64[2][nchunks] in the image
    uint8_t slot;
    uint8_t pad[3];
};

struct DevRuleset {        // 8 B
    uint32_t image_off;    // into HttpTables::images (16-byte aligned)
    uint32_t image_len;
};

struct HttpTables {
    const DevRuleset *rulesets;
    const uint8_t *images;
    uint32_t nrulesets;
    int32_t hot_ruleset;   // rule set whose image is staged in LDS (-1: none)
    const uint8_t *nfa_pool;   // DevNfa pool (null: no rule set has NFA matchers)
    uint64_t *nfa_bits;        // per request: bit k = NFA matcher k of its rule set accepted
    uint64_t *nfa_scratch;     // large NFAs: nfa_lane_words per lane of the launch (null: none in the pool)
    uint32_t nfa_lane_words;
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
static_assert(sizeof(DevKafkaRule) == 24, "DevKafkaRule layout");
struct DevKafkaTopicEnt {  // 48 B: a rule set's rules of one topic (dense, by interned topic id)
    uint32_t p0;           // position of the list's first rule
    uint32_t off, cnt;     // the list: cnt u32 rule positions at index[off] (cnt 0: no rule)
    uint32_t pad;
    DevKafkaRule r0;       // rules[rule_first + p0]
    uint32_t pad2[2];
};
static_assert(sizeof(DevKafkaTopicEnt) == 48, "DevKafkaTopicEnt layout");
struct DevKafkaRuleset {   // 36 B
    uint32_t rule_first, nrules;     // rules in evaluation order
    uint32_t topicless_off, ntopicless;  // u32 rule positions (Topic == "") in index[]
    uint32_t topics_off, ntopics;    // sorted (topic_id, list_off, list_cnt) triples in index[]
    uint32_t bykey_off;              // 65 (off, cnt) pairs in index[]: key 0..63, 64 = other kinds
    uint32_t tdense_off;             // DevKafkaTopicEnt per interned topic id in index[]; ~0u = use the
                                     // sorted directory (rule set x topic count over the dense budget)
    uint8_t any;                     // rules.Kafka != nil (pkg/proxy/kafka.go:139-142)
    uint8_t pad[3];
};
struct DevStrSlot {        // 32 B open-addressing slot (topics, client ids)
    uint32_t hash;         // l7_whash (case-sensitive)
    uint32_t str_off;
    uint16_t len;
    uint16_t used;
    int32_t id;
    uint32_t pre[4];       // the string's first 16 bytes, zero-padded: a string of <= 16
                           // bytes compares in the slot, without the string table
};
static_assert(sizeof(DevStrSlot) == 32, "DevStrSlot layout");
// Topic / client-id hash of the Kafka string tables (host compiler and
// kernel): the string's 32-bit little-endian words, the last one zero-padded,
// then its length.  Strings sit 4-byte aligned and zero-padded in `strings`,
// so the kernel compares them a word at a time.
constexpr uint32_t kWHashSeed = 0x811C9DC5u;
L7_HD inline uint32_t l7_whash_step(uint32_t h, uint32_t w) {
    h = (h ^ w) * 0x9E3779B1u;
    return h ^ (h >> 15);
}
L7_HD inline uint32_t l7_whash_final(uint32_t h, uint32_t n) {
    h = (h ^ n) * 0x85EBCA6Bu;
    return h ^ (h >> 13);
}

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

// ---------------- memcached ----------------
// One image per rule set (same DevRuleset directory as HTTP).  A rule set is
// the ordered memcache.Rule list the connection's port entries evaluate
// (proxylib/proxylib/policymap.go:91-236) up to the first unconditional allow,
// plus the terminal verdict.  Rules are in chunks of <= 64 (u64 masks).
// Rule r holds for a request iff
//   empty_r  ||  (cmd_r(command or opcode)  &&  for every key: pred_r(key))
// (memcache.Rule.Matches, proxylib/memcached/parser.go:47-100).  pred_r is the
// rule's one effective key predicate (keyExact > keyPrefix > keyRegex, none =
// true); they are compiled into byte DFAs whose states carry the mask of
// rules whose predicate holds if the key ends there (exact / prefix as raw-
// byte anchored patterns, keyRegex unanchored as Go regexp.Match).  The kernel
// walks kMcMaxDfas DFAs per pass over the request, as many passes as needed.
constexpr int kMcTextRows = 32;     // McText ids (engine/mc_groups.h), padded
constexpr int kMcMaxChunks = 4;     // <= 256 rules per rule set
constexpr int kMcMaxDfas = 4;       // key DFAs walked per key byte in one pass over the line
struct McImgHeader {       // 64 B, at offset 0 of every memcache image
    uint8_t nchunks;
    uint8_t terminal;      // verdict when no rule matches (V_ALLOW or V_DENY), rule -1
    uint8_t ndfa;
    uint8_t pad0;
    uint32_t text_off;     // u64[kMcTextRows][nchunks]: rules whose command group admits text id
    uint32_t op_off;       // u64[256][nchunks]: rules whose group admits the binary opcode
    uint32_t empty_off;    // u64[nchunks]: empty rules (match everything)
    uint32_t nopred_off;   // u64[nchunks]: rules without a key predicate (informational)
    uint32_t rule_off;     // i32[nchunks * 64]: global rule ids
    uint32_t dfa_off;      // DevDfa[ndfa] (mask rows: u64[nstates][nchunks])
    uint32_t owned_off;    // u64[ndfa][nchunks]: rules whose key predicate DFA d evaluates
    uint32_t nfa_off;      // DevNfaRef[nnfa] (mask_off: u64[nchunks] rules whose predicate NFA k is)
    uint32_t nnfa;
    uint32_t pad1[6];
};
static_assert(sizeof(McImgHeader) == 64, "McImgHeader layout");
constexpr uint32_t kMcDfaOff = sizeof(McImgHeader);  // DevDfa[ndfa] follow the header

struct McTables {
    const DevRuleset *rulesets;
    const uint8_t *images;
    uint32_t nrulesets;
    uint32_t images_len;       // bytes of all images (staged in LDS when they fit)
    const uint8_t *nfa_pool;   // DevNfa pool (null: no keyRegex on the NFA fallback)
    uint32_t max_chunks;       // most 64-rule chunks of any rule set (1: the one-chunk kernel)
    uint32_t nfa_lane_words;   // large NFAs: scratch words per lane of the launch
    uint64_t *nfa_scratch;     // (null: none in the pool)
};

// ---------------- r2d2 ----------------
// proxylib's r2d2 parser (proxylib/r2d2/r2d2parser.go): one line per request;
// fields split on single spaces; rule r holds iff (cmd_r any or equal) and
// (no file regex or it matches the file field, unanchored).  One image per
// rule set (DevRuleset directory), rules in chunks of <= 64.
constexpr int kR2MaxChunks = 4;     // <= 256 rules per rule set
struct R2ImgHeader {       // 64 B
    uint8_t nchunks;
    uint8_t terminal;      // verdict when no rule matches (V_DENY; V_ALLOW when no L7 rules apply)
    uint8_t ndfa;
    uint8_t nnfa;
    uint32_t cmd_off;      // u64[5][nchunks]: rules whose cmd admits READ, WRITE, HALT, RESET, other
    uint32_t nofile_off;   // u64[nchunks]: rules without a file regex
    uint32_t rule_off;     // i32[nchunks * 64]: global rule ids
    uint32_t dfa_off;      // DevDfa[ndfa] (mask rows u64[nstates][nchunks]: rules whose regex accepts)
    uint32_t nfa_off;      // DevNfaRef[nnfa] (mask_off: u64[nchunks], the rules of that regex)
    uint32_t pad[10];
};
static_assert(sizeof(R2ImgHeader) == 64, "R2ImgHeader layout");
struct R2Tables {
    const DevRuleset *rulesets;
    const uint8_t *images;
    uint32_t nrulesets;
    uint32_t nfa_lane_words;   // large NFAs: scratch words per lane of the launch
    const uint8_t *nfa_pool;
    uint64_t *nfa_scratch;     // (null: none in the pool)
};

// ---------------- cassandra ----------------
// proxylib's cassandra parser (proxylib/cassandra/cassandraparser.go): rule r
// holds for a query-like path iff (query_action any or equal to the path's
// action) and (no query_table regex, an empty table part, or the regex matches
// it, unanchored); for other opcodes every rule holds.  One image per rule
// set, rules in chunks of <= 64.
constexpr int kCassMaxChunks = 4;   // <= 256 rules per rule set
struct CassImgHeader {     // 64 B
    uint8_t nchunks;
    uint8_t terminal;      // verdict when no rule matches (V_DENY; V_ALLOW when no L7 rules apply)
    uint8_t ndfa;
    uint8_t nnfa;
    uint32_t act_off;      // u64[kCassActions + 1][nchunks]: rules admitting action a; row kCassActions:
                           // an action outside queryActionMap (rules without query_action)
    uint32_t notab_off;    // u64[nchunks]: rules without a query_table regex
    uint32_t rule_off;     // i32[nchunks * 64]: global rule ids
    uint32_t dfa_off;      // DevDfa[ndfa] (mask rows u64[nstates][nchunks]: rules whose regex accepts)
    uint32_t nfa_off;      // DevNfaRef[nnfa] (mask_off: u64[nchunks], the rules of that regex)
    uint32_t nrules;
    uint32_t pad[9];
};
static_assert(sizeof(CassImgHeader) == 64, "CassImgHeader layout");
struct CassTables {
    const DevRuleset *rulesets;
    const uint8_t *images;
    uint32_t nrulesets;
    uint32_t nlower;           // (rune, lower) pairs of unicode.ToLower
    const uint8_t *nfa_pool;
    const uint32_t *lower;
    uint64_t *nfa_scratch;     // large NFAs: nfa_lane_words per lane of the launch (null: none in the pool)
    uint32_t nfa_lane_words;
};
#if defined(__HIPCC__)
// A lane's large-NFA scratch (2 W words), by its index in the launch
__device__ __forceinline__ uint64_t *l7_nfa_lane_scratch(uint64_t *base, uint32_t words) {
    return base ? base + (size_t)(blockIdx.x * blockDim.x + threadIdx.x) * words : nullptr;
}
#endif

// FNV-1a over lower-cased ASCII (header names are tchar, i.e. ASCII)
static inline uint32_t l7_fnv_step(uint32_t h, uint8_t c) {
    if (c >= 'A' && c <= 'Z') c = (uint8_t)(c + 32);
    return (h ^ c) * 16777619u;
}
constexpr uint32_t kFnvBasis = 2166136261u;

}  // namespace l7
