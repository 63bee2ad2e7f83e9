// C-ABI implementation (include/l7gpu.h): engine state, policy versions,
// connection table, table upload and kernel dispatch (product code).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <map>
#include <thread>
#include <memory>
#include <tuple>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/l7gpu.h"
#include "capi_internal.h"
#include "device_tables.h"
#include "engine/cass_compile.h"
#include "engine/http_compile.h"
#include "engine/kafka_compile.h"
#include "engine/mc_compile.h"
#include "engine/nfa_pool.h"
#include "engine/r2_compile.h"
#include "kernels/copy_in_types.h"
#include "kernels/service_types.h"
#include "policy/npds_proto.h"
#include "policy/policy.h"
#include "regex/nfa_walk.h"
#include "regex/re_dfa.h"

namespace l7 {
hipError_t LaunchHttpClassify(const Batch &B, const HttpTables &T, const uint32_t *sel, const uint32_t *sel_count,
                              bool any_cold, bool answer_other, uint32_t *tile_ctr, bool latency, const CopyIn *ci,
                              hipStream_t stream);
hipError_t LaunchKafkaClassify(const Batch &B, const KafkaTables &T, const uint32_t *sel, const uint32_t *sel_count,
                               bool answer_other, uint32_t *zlist, uint32_t *zcount, uint32_t *work,
                               hipStream_t stream, int leave_per_cu = 0);
hipError_t LaunchKafkaInflate(const Batch &B, const uint32_t *zlist, const uint32_t *zcount, uint8_t *region,
                              hipStream_t stream);
uint32_t KafkaInflateBlocks();
uint32_t KafkaInflateRegionBytes();
hipError_t LaunchMemcacheClassify(const Batch &B, const McTables &T, const uint32_t *sel, const uint32_t *sel2,
                                  const uint32_t *sel_count, bool answer_other, uint32_t scratch_lanes,
                                  hipStream_t stream, const CopyIn *ci = nullptr);
hipError_t LaunchR2d2Classify(const Batch &B, const R2Tables &T, bool answer_other, uint32_t scratch_lanes,
                              hipStream_t stream);
size_t CassandraScratchBytes(uint32_t n);
hipError_t LaunchCassandraClassify(const Batch &B, const CassTables &T, void *scratch, size_t scratch_bytes,
                                   bool answer_other, uint32_t nfa_lanes, hipStream_t stream);
hipError_t LaunchCounters(const uint8_t *verdict, const int32_t *rule, uint32_t n, uint32_t nrules,
                          uint64_t *counters, uint32_t *scratch, hipStream_t stream);
size_t CountersScratchBytes();
hipError_t LaunchFlowStats(const Batch &B, uint32_t nkeys, uint64_t *acc, hipStream_t stream);
uint32_t FlowStatsMaxKeys();
hipError_t LaunchHttpNfa(const Batch &B, const HttpTables &T, uint32_t scratch_lanes, hipStream_t stream);
hipError_t LaunchPartition(const Batch &B, uint32_t *sel_kafka, uint32_t *sel_mc, uint32_t *sel_http, uint32_t *counts,
                           hipStream_t stream);
hipError_t LaunchFrameStreams(const uint8_t *arena, uint64_t arena_len, const uint64_t *s_off, const uint32_t *s_len,
                              const uint32_t *s_conn, uint32_t n, const DevConn *conns, uint32_t nconns,
                              uint32_t max_frames, uint64_t *frame_off, uint32_t *frame_len, uint32_t *conn_out,
                              uint32_t *nframes, hipStream_t stream);
hipError_t HttpPhaseTimes(uint64_t *out, bool reset);
hipError_t KafkaPhaseTimes(uint64_t *out, bool reset);
hipError_t LaunchCopyIn(const CopyIn &c, hipStream_t stream);
hipError_t FramePhaseTimes(uint64_t *out, bool reset);
hipError_t LaunchHttpGroup(const Batch &B, const HttpTables &T, const uint32_t *sel, const uint32_t *sel_count,
                           uint32_t n, bool answer_other, uint32_t *ctl, uint32_t *hist, uint32_t *cursor,
                           uint32_t *segs, uint32_t *gsel, uint32_t *gbig, hipStream_t stream);
hipError_t LaunchHttpGrouped(const Batch &B, const HttpTables &T, const uint32_t *gsel, const uint32_t *segs,
                             const uint32_t *gbig, uint32_t *ctl, bool any_big, hipStream_t stream);
hipError_t LaunchHttpService(SvcBox *box, const SvcStatic &S, const HttpTables &T, uint32_t seen0, uint64_t idle,
                             hipStream_t stream);
hipError_t LaunchMemcacheService(SvcBox *box, const SvcStatic &S, const McTables &T, uint32_t seen0, uint64_t idle,
                                 hipStream_t stream);
}  // namespace l7

using namespace l7;

// Scratch of the l7g_classify calls on one caller stream: the partition lists,
// the NFA pre-pass bits, the counter histograms, the compressed-Kafka decode
// region, and the completion event of the last call on that stream.  Calls on
// different streams use different scratch and run concurrently; calls on one
// stream are ordered by the stream itself.
struct StreamScratch {
    // protocol split (grow-only): [counts(32) | L7_KAFKA_CLASSES x n Kafka idx | n memcached idx |
    // n HTTP idx | n idx of Kafka requests with compressed messages]
    uint32_t *d_sel = nullptr;
    size_t sel_cap = 0;
    // NFA pre-pass results, u64 per request (grow-only)
    uint64_t *d_nfa = nullptr;
    size_t nfa_cap = 0;
    // counter histogram scratch (kernels/counters.hip), allocated on first use
    uint32_t *d_hist = nullptr;
    // cassandra USE list: [count | n request indices] (grow-only)
    void *d_use = nullptr;  // cassandra: USE keys, sorted keys, sort temp (bytes)
    size_t use_cap = 0;
    // work counters of unpartitioned batches (HTTP tile counters), allocated on first use
    uint32_t *d_work = nullptr;
    // HTTP requests grouped by rule set (kernels/http_group.hip), grow-only:
    // [ctl(8) | hist(R) | cursor(R) | segments(3 x (n / kGroupSegEntries + R + 1)) | grouped list(n) | big-image list(n)]
    uint32_t *d_grp = nullptr;
    size_t grp_cap = 0;
    // large NFAs' state sets: a lane's 2 W words for each lane of a launch (grow-only)
    uint64_t *d_bignfa = nullptr;
    size_t bignfa_bytes = 0;
    // completion of the last call's kernels on this stream
    hipEvent_t done_ev = nullptr;
    bool launched = false;
    uint64_t last_use = 0;
    // the memcached kernel beside the Kafka kernel (large mixed batches)
    hipStream_t side = nullptr;
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
    ~StreamScratch() {
        if (side) hipStreamSynchronize(side);
        if (fork_ev) hipEventDestroy(fork_ev);
        if (join_ev) hipEventDestroy(join_ev);
        if (side) hipStreamDestroy(side);
        if (d_bignfa) hipFree(d_bignfa);
        if (d_grp) hipFree(d_grp);
        if (d_sel) hipFree(d_sel);
        if (d_nfa) hipFree(d_nfa);
        if (d_hist) hipFree(d_hist);
        if (d_use) hipFree(d_use);
        if (d_work) hipFree(d_work);
        if (done_ev) hipEventDestroy(done_ev);
    }
};
constexpr size_t kMaxStreamScratch = 16;   // per-stream scratch sets; beyond: the least recently used one is handed over
constexpr uint32_t kDynTilesMin = 1u << 18;  // unpartitioned HTTP batches from this size take tiles from a counter
// l7g_classify_host calls up to this size run zero-copy (kernels on the pinned staging)
constexpr uint32_t kZeroCopyMaxRequests = 256;
constexpr size_t kZeroCopyMaxBytes = 256 * 1024;
// batches below this size skip the protocol split when one classifier can walk them alone
constexpr uint32_t kPartitionMin = 4096;
constexpr uint32_t kBesideMin = 1u << 20;  // memcached kernel beside Kafka from this batch size
constexpr uint32_t kHostScanMax = 4096;
// at most this many requests: the HTTP requests are framed one per wave, their
// lines side by side (http_latency_kernel), not one per lane
constexpr uint32_t kLatencyMax = 64;
// batches from this size with HTTP requests on more than one rule set take the grouped path
constexpr uint32_t kGroupMin = 1u << 16;
constexpr size_t kNfaScratchBytes = 256ull << 20;  // large NFAs: state-set scratch per stream (lanes in flight)  // host calls up to this size check their connections for cold rule sets

// l7g_classify_host's per-thread staging: its own stream, device arena and
// request arrays (grow-only), so host-buffer calls from different threads
// overlap instead of queueing on one stream.
// Inputs go over as ONE copy from a pinned staging buffer ([off u64 | len u32 |
// conn u32 | arena], packed by the host) and outputs come back as ONE copy
// ([verdict u8 | rule i32 | consumed u32]); a small call is not copied at all
// (the kernels read and write the pinned buffers in place, see HostRun).
struct HostCtx {
    hipStream_t s = nullptr;
    uint8_t *dev = nullptr;        // device: [inputs | outputs]
    uint8_t *pin_in = nullptr;     // pinned host staging of the inputs
    uint8_t *pin_out = nullptr;    // pinned host staging of the outputs
    uint8_t *pin_in_dev = nullptr;   // their device addresses (zero-copy; looked up once)
    uint8_t *pin_out_dev = nullptr;
    uint32_t *pin_done = nullptr;     // pinned word the call's last kernel stores its sequence number to
    uint32_t *pin_done_dev = nullptr;
    uint32_t seq = 0;
    size_t in_cap = 0, out_cap = 0;
    ~HostCtx() {
        if (s) hipStreamSynchronize(s);
        if (dev) hipFree(dev);
        if (pin_in) hipHostFree(pin_in);
        if (pin_out) hipHostFree(pin_out);
        if (pin_done) hipHostFree(pin_done);
        if (s) hipStreamDestroy(s);
    }
};

// ---- resident services (kernels/service.h): the synchronous drop-in calls
// (one Allowed(), one OnData) posted to a polling workgroup instead of launched
constexpr uint32_t kSvcHttpMax = 8;    // HTTP requests per call (one per wave of the workgroup)
constexpr uint32_t kSvcMcMax = 64;     // memcached requests per call (one wave)
constexpr size_t kSvcInBytes = SvcArenaOff(kSvcMcMax) + kZeroCopyMaxBytes + 64;
constexpr size_t kSvcOutBytes = kSvcMcMax * 9 + 64;
// a service leaves after this many shader-clock cycles without a call (~50 ms at 2.4 GHz)
constexpr uint64_t kSvcIdleCycles = 120000000ull;
struct Service {
    std::mutex mu;  // one call at a time, held from its posting to its answers
    hipStream_t s = nullptr;
    SvcBox *box = nullptr, *box_dev = nullptr;  // pinned, coherent
    SvcBox *box_ready = nullptr;  // box, published once the service is allocated (read without mu)
    uint8_t *pin_in = nullptr, *pin_in_dev = nullptr, *pin_out = nullptr, *pin_out_dev = nullptr;
    uint8_t *dev_in = nullptr;
    uint32_t seq = 0;
    bool launched = false;  // a workgroup may be serving (launched, not yet seen leaving)
    // its launch arguments: the tables and connections it serves with
    HttpTables ht{};
    McTables mt{};
    const DevConn *conns = nullptr;
    uint32_t nconns = 0;
    uint64_t calls = 0, launches = 0;
    ~Service() {
        if (s) hipStreamSynchronize(s);
        if (dev_in) hipFree(dev_in);
        if (pin_in) hipHostFree(pin_in);
        if (pin_out) hipHostFree(pin_out);
        if (box) hipHostFree(box);
        if (s) hipStreamDestroy(s);
    }
};

struct l7g_engine {
    int device = 0;
    // [0] HTTP, [1] memcached (l7g_service_enable; L7G_SERVICE=0 turns them off)
    Service svc[2];
    bool svc_on = true;
    std::mutex mu;
    std::unique_ptr<PolicySet> ps;
    std::unique_ptr<HttpCompiler> hc;
    std::unique_ptr<KafkaCompiler> kc;
    std::unique_ptr<McCompiler> mc;
    std::unique_ptr<R2Compiler> r2;
    std::unique_ptr<CassCompiler> cs;
    std::vector<l7g_conn_t> attrs;
    std::vector<DevConn> conns;
    uint8_t *d_blob = nullptr;
    size_t blob_bytes = 0;
    // the policy version's source (l7g_tables_export ships it with the compiled tables)
    std::string policy_src;
    int policy_form = 0, policy_px = 0;
    DevConn *d_conns = nullptr;
    size_t conns_cap = 0;
    HttpTables ht{};
    KafkaTables kt{};
    McTables mt{};
    R2Tables rt{};
    CassTables ct{};
    bool tables_dirty = true, conns_dirty = true;
    bool has_http = false, has_kafka = false, has_mc = false, has_r2 = false, has_cs = false;
    int32_t hot_ruleset = -1;  // HTTP rule set staged in LDS (most connections)
    bool any_big_image = false;  // some HTTP rule set's image exceeds kGroupImageBytes
    // l7g_classify_host contexts, one per calling thread (guarded by hmu)
    std::mutex hmu;
    std::map<std::thread::id, std::unique_ptr<HostCtx>> hctx;
    bool any_cold = false;     // some HTTP connection uses another rule set
    // decode region of kafka_inflate_kernel (one slice per workgroup, 1 GiB),
    // allocated with the first Kafka batch and shared by every stream: each
    // call's inflate launch waits for zreg_ev, the previous one's completion
    uint8_t *d_zreg = nullptr;
    hipEvent_t zreg_ev = nullptr;
    bool zreg_used = false;
    // per-stream scratch of l7g_classify (guarded by mu)
    std::map<hipStream_t, std::unique_ptr<StreamScratch>> scr;
    uint64_t calls = 0;
    // proxy statistics: key (policy, proto, port, ingress) per connection, and
    // the device accumulator u64[keys][4] (l7g_flow_stats_*)
    std::map<std::tuple<int32_t, uint8_t, uint32_t, uint8_t>, uint16_t> skeys;
    std::vector<std::tuple<int32_t, uint8_t, uint32_t, uint8_t>> skey_list;
    bool flow_stats = false;
    uint64_t *d_flow = nullptr;
    size_t flow_cap = 0;  // keys the accumulator holds
    // Every stream's last completion event (StreamScratch::done_ev) is waited
    // on -- never a caller's stream, which may be gone by then -- before the
    // engine rewrites or frees anything a launched kernel reads: the
    // connection table, the table blob, the proxy-statistics accumulator.
    // l7g_profile_*: timing events around each launch of the last call
    bool profile = false;
    hipEvent_t prof_ev[5] = {};
    bool prof_ran[4] = {};
};

// Stops a service's workgroup and waits for it to leave (v.mu held): its
// launch arguments (tables, connections) are about to change, or the engine
// goes away.
static hipError_t ServiceStop(Service &v) {
    if (!v.launched) return hipSuccess;
    __atomic_store_n(&v.box->stop, 1u, __ATOMIC_SEQ_CST);
    v.launched = false;
    return hipStreamSynchronize(v.s);  // (it leaves at its next poll; a fault is reported here)
}
static void StopServices(l7g_engine *e) {
    for (Service &v : e->svc) {
        std::lock_guard<std::mutex> g(v.mu);  // (waits for a call in flight)
        ServiceStop(v);
    }
}
// A launch that wants every CU (a persistent grid) asks the services to leave
// without waiting; the next synchronous call starts them again.
static void ReleaseServiceCUs(l7g_engine *e) {
    for (Service &v : e->svc) {
        SvcBox *b = __atomic_load_n(&v.box_ready, __ATOMIC_ACQUIRE);  // (set once; v.mu not taken here)
        if (b && __atomic_load_n(&b->state, __ATOMIC_ACQUIRE) != kSvcStopped) __atomic_store_n(&b->stop, 1u, __ATOMIC_SEQ_CST);
    }
}

// Waits for the kernels of every stream's last call, and stops the services
// (their launch arguments are what the caller is about to rewrite).  Caller
// holds e->mu.
static hipError_t WaitLastClassify(l7g_engine *e) {
    StopServices(e);
    hipError_t rc = hipSuccess;
    for (auto &kv : e->scr)
        if (kv.second->launched) {
            hipError_t r = hipEventSynchronize(kv.second->done_ev);
            if (r != hipSuccess) rc = r;
        }
    return rc;
}

// The scratch of stream s (created on first use; past kMaxStreamScratch the
// least recently used stream's scratch is handed over once s has been made
// to wait for that stream's last call).  Caller holds e->mu.
static hipError_t GetScratch(l7g_engine *e, hipStream_t s, StreamScratch **out) {
    auto it = e->scr.find(s);
    if (it == e->scr.end()) {
        if (e->scr.size() >= kMaxStreamScratch) {
            auto lru = e->scr.begin();
            for (auto j = e->scr.begin(); j != e->scr.end(); ++j)
                if (j->second->last_use < lru->second->last_use) lru = j;
            std::unique_ptr<StreamScratch> sc = std::move(lru->second);
            e->scr.erase(lru);
            if (sc->launched) {
                hipError_t rc = hipStreamWaitEvent(s, sc->done_ev, 0);
                if (rc != hipSuccess) return rc;
            }
            it = e->scr.emplace(s, std::move(sc)).first;
        } else {
            auto sc = std::make_unique<StreamScratch>();
            hipError_t rc = hipEventCreateWithFlags(&sc->done_ev, hipEventDisableTiming);
            if (rc != hipSuccess) return rc;
            it = e->scr.emplace(s, std::move(sc)).first;
        }
    }
    // (a handle can be reused by a new stream while the old one's work is
    // still pending: order the call after that work whatever the stream;
    // nothing to wait for once it has completed -- the synchronous callers)
    if (it->second->launched && hipEventQuery(it->second->done_ev) != hipSuccess) {
        hipError_t rc = hipStreamWaitEvent(s, it->second->done_ev, 0);
        if (rc != hipSuccess) return rc;
    }
    it->second->last_use = ++e->calls;
    *out = it->second.get();
    return hipSuccess;
}

static void set_err(char *err, size_t errlen, const std::string &m) {
    if (!err || errlen == 0) return;
    size_t n = std::min(errlen - 1, m.size());
    memcpy(err, m.data(), n);
    err[n] = 0;
}

namespace {

template <class T>
size_t Put(std::vector<uint8_t> &blob, const std::vector<T> &v) {
    size_t off = (blob.size() + 255) & ~(size_t)255;
    blob.resize(off + v.size() * sizeof(T) + 16);  // +16: aligned 16-byte reads may run past the end
    if (!v.empty()) memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
    return off;
}

// Resolve connection i to its rule set (once per connection / policy version).
bool ResolveOne(l7g_engine *e, size_t i, std::string *err) {
    const l7g_conn_t &a = e->attrs[i];
    DevConn &c = e->conns[i];
    c = DevConn{-1, PROTO_NONE, 0, 0xFFFF};
    c.proto = a.proto;
    if (L7_PROTO_OWNED(a.proto)) {
        const auto key = std::make_tuple(a.policy, a.proto, a.port, (uint8_t)(a.ingress != 0));
        auto it = e->skeys.find(key);
        if (it == e->skeys.end() && e->skey_list.size() < FlowStatsMaxKeys()) {
            it = e->skeys.emplace(key, (uint16_t)e->skey_list.size()).first;
            e->skey_list.push_back(key);
        }
        if (it != e->skeys.end()) c.skey = it->second;
    }
    c.flags = (uint8_t)(a.flags & 3);
    const bool proxylib = (a.flags & L7G_CONN_PROXYLIB) != 0;
    if (a.proto == PROTO_HTTP) {
        // remote identity: Envoy's HTTP filter uses the source on ingress and the
        // destination on egress (cilium_l7policy.cc:144-150); proxylib matches
        // the connection's SrcId in both directions (connection.go:176-179)
        uint64_t remote = (a.ingress || proxylib) ? a.src_id : a.dst_id;
        c.ruleset = e->hc->RulesetFor(a.policy, a.ingress != 0, a.port, remote, proxylib, err);
        if (c.ruleset < 0) return false;
        e->has_http = true;
    } else if (a.proto == PROTO_KAFKA) {
        // Kafka rules are selected by the source identity in both directions
        // (pkg/proxy/kafka.go:327,357)
        c.ruleset = e->kc->RulesetFor(a.policy, a.ingress != 0, a.port, a.src_id, proxylib, err);
        if (c.ruleset < 0) return false;
        e->has_kafka = true;
    } else if (a.proto == PROTO_MEMCACHE) {
        // proxylib matches on the connection's SrcId in both directions
        // (proxylib/proxylib/connection.go:176-179)
        c.ruleset = e->mc->RulesetFor(a.policy, a.ingress != 0, a.port, a.src_id, err);
        if (c.ruleset < 0) return false;
        e->has_mc = true;
    } else if (a.proto == PROTO_R2D2) {  // proxylib r2d2: SrcId in both directions, as memcached
        c.ruleset = e->r2->RulesetFor(a.policy, a.ingress != 0, a.port, a.src_id, err);
        if (c.ruleset < 0) return false;
        e->has_r2 = true;
    } else if (a.proto == PROTO_CASSANDRA) {  // proxylib cassandra: SrcId in both directions
        c.ruleset = e->cs->RulesetFor(a.policy, a.ingress != 0, a.port, a.src_id, err);
        if (c.ruleset < 0) return false;
        e->has_cs = true;
    }
    return true;
}

// The HTTP rule set serving the most connections has its image staged in LDS
// by every workgroup (if it fits); the others are read from HBM/L2.
void PickHot(l7g_engine *e) {
    std::vector<uint32_t> uses(e->hc->image().rulesets.size(), 0);
    for (size_t i = 0; i < e->attrs.size(); i++)
        if (e->attrs[i].proto == PROTO_HTTP && e->conns[i].ruleset >= 0) uses[e->conns[i].ruleset]++;
    e->hot_ruleset = -1;
    uint32_t best = 0;
    for (size_t r = 0; r < uses.size(); r++)
        if (uses[r] > best && e->hc->image().rulesets[r].image_len <= kLdsImageBytes) { best = uses[r]; e->hot_ruleset = (int32_t)r; }
    e->any_cold = false;
    for (size_t i = 0; i < e->attrs.size(); i++)
        if (e->attrs[i].proto == PROTO_HTTP && e->conns[i].ruleset != e->hot_ruleset) e->any_cold = true;
    e->any_big_image = false;
    for (size_t r = 0; r < uses.size(); r++)
        if (uses[r] && e->hc->image().rulesets[r].image_len > kGroupImageBytes) e->any_big_image = true;
}

size_t TableRulesets(const l7g_engine *e) {
    return e->hc->image().rulesets.size() + e->kc->image().rulesets.size() + e->mc->image().rulesets.size() +
           e->r2->image().rulesets.size() + e->cs->image().rulesets.size();
}

// Resolve every connection (policy update / connection table replaced).
bool ResolveConns(l7g_engine *e, std::string *err) {
    e->conns.assign(e->attrs.size(), DevConn{-1, PROTO_NONE, 0, 0xFFFF});
    e->has_http = e->has_kafka = e->has_mc = e->has_r2 = e->has_cs = false;
    for (size_t i = 0; i < e->attrs.size(); i++)
        if (!ResolveOne(e, i, err)) return false;
    PickHot(e);
    e->tables_dirty = e->conns_dirty = true;
    return true;
}

// The device table blob: every compiler's image, each 256-byte aligned.
struct BlobLayout {
    size_t o_rs, o_img, o_nfa, k_rs, k_r, k_idx, k_th, k_ch, k_s, m_rs, m_img, m_nfa, r_rs, r_img, r_nfa, c_rs, c_img,
        c_nfa, c_low;
};
BlobLayout AssembleBlob(const l7g_engine *e, std::vector<uint8_t> &blob) {
    BlobLayout L;
    const HttpImage &H = e->hc->image();
    L.o_rs = Put(blob, H.rulesets); L.o_img = Put(blob, H.images); L.o_nfa = Put(blob, H.nfa_pool);
    const KafkaImage &K = e->kc->image();
    L.k_rs = Put(blob, K.rulesets); L.k_r = Put(blob, K.rules); L.k_idx = Put(blob, K.index);
    L.k_th = Put(blob, K.topic_hash); L.k_ch = Put(blob, K.client_hash); L.k_s = Put(blob, K.strings);
    const McImage &M = e->mc->image();
    L.m_rs = Put(blob, M.rulesets); L.m_img = Put(blob, M.images); L.m_nfa = Put(blob, M.nfa_pool);
    const R2Image &R = e->r2->image();
    L.r_rs = Put(blob, R.rulesets); L.r_img = Put(blob, R.images); L.r_nfa = Put(blob, R.nfa_pool);
    const CassImage &CI = e->cs->image();
    L.c_rs = Put(blob, CI.rulesets); L.c_img = Put(blob, CI.images); L.c_nfa = Put(blob, CI.nfa_pool);
    L.c_low = Put(blob, CI.lower);
    return L;
}

hipError_t Upload(l7g_engine *e) {
    hipError_t rc;
    if (e->tables_dirty) {
        std::vector<uint8_t> blob;
        const BlobLayout L = AssembleBlob(e, blob);
        const size_t o_rs = L.o_rs, o_img = L.o_img, o_nfa = L.o_nfa, k_rs = L.k_rs, k_r = L.k_r, k_idx = L.k_idx,
                     k_th = L.k_th, k_ch = L.k_ch, k_s = L.k_s, m_rs = L.m_rs, m_img = L.m_img, m_nfa = L.m_nfa,
                     r_rs = L.r_rs, r_img = L.r_img, r_nfa = L.r_nfa, c_rs = L.c_rs, c_img = L.c_img, c_nfa = L.c_nfa,
                     c_low = L.c_low;
        const HttpImage &H = e->hc->image();
        const KafkaImage &K = e->kc->image();
        const McImage &M = e->mc->image();
        const R2Image &R = e->r2->image();
        const CassImage &CI = e->cs->image();
        uint8_t *d = nullptr;
        if ((rc = hipMalloc(&d, blob.size())) != hipSuccess) return rc;
        if ((rc = hipMemcpy(d, blob.data(), blob.size(), hipMemcpyHostToDevice)) != hipSuccess) { hipFree(d); return rc; }
        if (e->d_blob) { WaitLastClassify(e); hipFree(e->d_blob); }
        e->d_blob = d;
        e->blob_bytes = blob.size();
        HttpTables &T = e->ht;
        T.rulesets = (const DevRuleset *)(d + o_rs);
        T.images = d + o_img;
        T.nrulesets = (uint32_t)H.rulesets.size();
        T.hot_ruleset = e->hot_ruleset;
        T.nfa_pool = H.nfa_pool.empty() ? nullptr : d + o_nfa;
        T.nfa_bits = nullptr;
        // large NFAs (W > kNfaMaxWords): 2 W words of scratch per lane, given at launch
        auto lane_words = [](uint32_t w) { return w > (uint32_t)kNfaMaxWords ? 2 * w : 0u; };
        T.nfa_scratch = nullptr;
        T.nfa_lane_words = lane_words(e->hc->nfa_max_words());
        KafkaTables &KT = e->kt;
        KT.rulesets = (const DevKafkaRuleset *)(d + k_rs);
        KT.rules = (const DevKafkaRule *)(d + k_r);
        KT.index = (const uint32_t *)(d + k_idx);
        KT.topic_hash = (const DevStrSlot *)(d + k_th);
        KT.client_hash = (const DevStrSlot *)(d + k_ch);
        KT.strings = (const uint8_t *)(d + k_s);
        KT.nrulesets = (uint32_t)K.rulesets.size();
        KT.topic_mask = K.topic_mask;
        KT.client_mask = K.client_mask;
        McTables &MT = e->mt;
        MT.rulesets = (const DevRuleset *)(d + m_rs);
        MT.images = d + m_img;
        MT.nrulesets = (uint32_t)M.rulesets.size();
        MT.images_len = (uint32_t)M.images.size();
        MT.nfa_pool = M.nfa_pool.empty() ? nullptr : d + m_nfa;
        MT.max_chunks = (uint32_t)M.max_chunks;
        MT.nfa_scratch = nullptr;
        MT.nfa_lane_words = lane_words(e->mc->nfa_max_words());
        R2Tables &RT = e->rt;
        RT.rulesets = (const DevRuleset *)(d + r_rs);
        RT.images = d + r_img;
        RT.nrulesets = (uint32_t)R.rulesets.size();
        RT.nfa_pool = R.nfa_pool.empty() ? nullptr : d + r_nfa;
        RT.nfa_scratch = nullptr;
        RT.nfa_lane_words = lane_words(e->r2->nfa_max_words());
        CassTables &CT = e->ct;
        CT.rulesets = (const DevRuleset *)(d + c_rs);
        CT.images = d + c_img;
        CT.nrulesets = (uint32_t)CI.rulesets.size();
        CT.nfa_pool = CI.nfa_pool.empty() ? nullptr : d + c_nfa;
        CT.lower = (const uint32_t *)(d + c_low);
        CT.nlower = (uint32_t)(CI.lower.size() / 2);
        CT.nfa_scratch = nullptr;
        CT.nfa_lane_words = lane_words(e->cs->nfa_max_words());
        e->tables_dirty = false;
    }
    if (e->conns_dirty) {
        // kernels of the previous batch may still read the table: it is
        // rewritten (or freed) only once they have finished
        if ((rc = WaitLastClassify(e)) != hipSuccess) return rc;
        size_t need = std::max<size_t>(e->conns.size(), 1);
        if (need > e->conns_cap) {
            if (e->d_conns) { hipFree(e->d_conns); e->d_conns = nullptr; }
            if ((rc = hipMalloc(&e->d_conns, need * sizeof(DevConn))) != hipSuccess) return rc;
            e->conns_cap = need;
        }
        if (!e->conns.empty() &&
            (rc = hipMemcpy(e->d_conns, e->conns.data(), e->conns.size() * sizeof(DevConn), hipMemcpyHostToDevice)) != hipSuccess)
            return rc;
        e->conns_dirty = false;
    }
    return hipSuccess;
}

}  // namespace

extern "C" {

l7g_engine *l7g_engine_create(int device, char *err, size_t errlen) {
    if (device == L7G_HOST_ONLY) {  // rule compiler only: no HIP calls, classify unavailable
        auto *e = new l7g_engine();
        e->device = -1;
        e->ps = std::make_unique<PolicySet>();
        e->hc = std::make_unique<HttpCompiler>(e->ps.get());
        e->kc = std::make_unique<KafkaCompiler>(e->ps.get());
        e->mc = std::make_unique<McCompiler>(e->ps.get());
        e->r2 = std::make_unique<R2Compiler>(e->ps.get());
        e->cs = std::make_unique<CassCompiler>(e->ps.get());
        return e;
    }
    int ndev = 0;
    hipError_t rc = hipGetDeviceCount(&ndev);
    if (rc != hipSuccess || device < 0 || device >= ndev) {
        set_err(err, errlen, std::string("no such HIP device: ") + std::to_string(device) + " (" + hipGetErrorString(rc) + ")");
        return nullptr;
    }
    if ((rc = hipSetDevice(device)) != hipSuccess) { set_err(err, errlen, hipGetErrorString(rc)); return nullptr; }
    auto *e = new l7g_engine();
    e->device = device;
    {
        const char *v = getenv("L7G_SERVICE");
        e->svc_on = !(v && v[0] == '0');
    }
    e->ps = std::make_unique<PolicySet>();
    e->hc = std::make_unique<HttpCompiler>(e->ps.get());
    e->kc = std::make_unique<KafkaCompiler>(e->ps.get());
    e->mc = std::make_unique<McCompiler>(e->ps.get());
    e->r2 = std::make_unique<R2Compiler>(e->ps.get());
    e->cs = std::make_unique<CassCompiler>(e->ps.get());
    return e;
}

void l7g_engine_destroy(l7g_engine *e) {
    if (!e) return;
    if (e->device < 0) { delete e; return; }
    hipSetDevice(e->device);
    StopServices(e);
    hipDeviceSynchronize();
    if (e->d_blob) hipFree(e->d_blob);
    if (e->d_conns) hipFree(e->d_conns);
    e->hctx.clear();
    e->scr.clear();
    if (e->d_flow) hipFree(e->d_flow);
    if (e->d_zreg) hipFree(e->d_zreg);
    if (e->zreg_ev) hipEventDestroy(e->zreg_ev);
    for (hipEvent_t ev : e->prof_ev)
        if (ev) hipEventDestroy(ev);
    delete e;
}

static int PolicySwap(l7g_engine *e, std::unique_ptr<PolicySet> ps, char *err, size_t errlen);
static int SwapIn(l7g_engine *e, std::unique_ptr<PolicySet> ps, std::unique_ptr<HttpCompiler> hc,
                  std::unique_ptr<KafkaCompiler> kc, std::unique_ptr<McCompiler> mc, std::unique_ptr<R2Compiler> r2,
                  std::unique_ptr<CassCompiler> cs, char *err, size_t errlen);

int l7g_policy_update(l7g_engine *e, const char *json, size_t len, char *err, size_t errlen) {
    return l7g_policy_update_view(e, (const uint8_t *)json, len, 0, 0, err, errlen);
}

int l7g_policy_update_proto(l7g_engine *e, const uint8_t *buf, size_t len, char *err, size_t errlen) {
    return l7g_policy_update_view(e, buf, len, 1, 0, err, errlen);
}

}  // extern "C"

// capi_internal.h: proto_form 0 = JSON, 1 = NPDS DiscoveryResponse; proxylib
// != 0 = the proxylib instance's update (instance.go:168-219), which also
// NACKs what only proxylib's policymap rejects (PolicySet::px_nack).
int l7g_policy_update_view(l7g_engine *e, const uint8_t *buf, size_t len, int proto_form, int proxylib, char *err,
                           size_t errlen) {
    std::lock_guard<std::mutex> g(e->mu);
    auto ps = std::make_unique<PolicySet>();
    std::string m;
    const bool ok = proto_form ? LoadPolicySetProto(buf, len, ps.get(), &m)
                               : LoadPolicySet((const char *)buf, len, ps.get(), &m);
    if (!ok) { set_err(err, errlen, m); return -1; }
    if (proxylib && !ps->px_nack.empty()) { set_err(err, errlen, ps->px_nack); return -1; }
    const int rc = PolicySwap(e, std::move(ps), err, errlen);
    if (rc == 0) {
        e->policy_src.assign((const char *)buf, len);
        e->policy_form = proto_form;
        e->policy_px = proxylib;
    }
    return rc;
}

extern "C" {

// Swap in a loaded policy version; on a compile failure the previous version
// stays in force (an NPDS NACK).  Caller holds e->mu.
static int PolicySwap(l7g_engine *e, std::unique_ptr<PolicySet> ps, char *err, size_t errlen) {
    auto hc = std::make_unique<HttpCompiler>(ps.get());
    auto kc = std::make_unique<KafkaCompiler>(ps.get());
    auto mc = std::make_unique<McCompiler>(ps.get());
    auto r2 = std::make_unique<R2Compiler>(ps.get());
    auto cs = std::make_unique<CassCompiler>(ps.get());
    return SwapIn(e, std::move(ps), std::move(hc), std::move(kc), std::move(mc), std::move(r2), std::move(cs), err,
                  errlen);
}

// Swap in a policy version with its compilers (fresh, or holding imported
// tables); on a compile failure the previous version stays in force.
static int SwapIn(l7g_engine *e, std::unique_ptr<PolicySet> ps, std::unique_ptr<HttpCompiler> hc,
                  std::unique_ptr<KafkaCompiler> kc, std::unique_ptr<McCompiler> mc, std::unique_ptr<R2Compiler> r2,
                  std::unique_ptr<CassCompiler> cs, char *err, size_t errlen) {
    std::string m;
    std::swap(e->ps, ps);
    std::swap(e->hc, hc);
    std::swap(e->kc, kc);
    std::swap(e->mc, mc);
    std::swap(e->r2, r2);
    std::swap(e->cs, cs);
    if (!ResolveConns(e, &m)) {  // roll back: previous version stays in force
        std::swap(e->ps, ps);
        std::swap(e->hc, hc);
        std::swap(e->kc, kc);
        std::swap(e->mc, mc);
        std::swap(e->r2, r2);
        std::swap(e->cs, cs);
        std::string m2;
        ResolveConns(e, &m2);
        set_err(err, errlen, m);
        return -1;
    }
    return 0;
}

// ---- compiled tables across ranks (engine/serial.h)
constexpr uint64_t kTablesMagic = 0x3154473754L;  // "T7G1"
// format and struct-layout tag: an image from a build with another layout of
// the device records is refused (it would be read at the wrong offsets)
constexpr uint64_t kTablesAbi = 2ull << 56 | (uint64_t)sizeof(DevRuleset) << 48 | (uint64_t)sizeof(DevNfa) << 36 |
                                (uint64_t)sizeof(ImgHeader) << 24 | (uint64_t)sizeof(DevKafkaRuleset) << 12 |
                                (uint64_t)sizeof(McImgHeader);

int l7g_tables_export(l7g_engine *e, uint8_t *buf, size_t cap, size_t *len) {
    std::lock_guard<std::mutex> g(e->mu);
    Ser s;
    s.u64(kTablesMagic);
    s.u64(kTablesAbi);
    s.u64((uint64_t)e->policy_form);
    s.u64((uint64_t)e->policy_px);
    s.str(e->policy_src);
    e->hc->Save(s);
    e->kc->Save(s);
    e->mc->Save(s);
    e->r2->Save(s);
    e->cs->Save(s);
    if (len) *len = s.out.size();
    if (!buf || cap < s.out.size()) return -2;
    memcpy(buf, s.out.data(), s.out.size());
    return 0;
}

int l7g_tables_import(l7g_engine *e, const uint8_t *buf, size_t len, char *err, size_t errlen) {
    std::lock_guard<std::mutex> g(e->mu);
    Des d(buf, len);
    if (d.u64() != kTablesMagic) { set_err(err, errlen, "not an l7g_tables_export image"); return -1; }
    if (d.u64() != kTablesAbi) { set_err(err, errlen, "tables image from a build with another table layout"); return -1; }
    const int form = (int)d.u64(), px = (int)d.u64();
    const std::string src = d.str();
    if (!d.ok) { set_err(err, errlen, "truncated tables image"); return -1; }
    auto ps = std::make_unique<PolicySet>();
    std::string m;
    const bool ok = form ? LoadPolicySetProto((const uint8_t *)src.data(), src.size(), ps.get(), &m)
                         : LoadPolicySet(src.data(), src.size(), ps.get(), &m);
    if (!ok) { set_err(err, errlen, m); return -1; }
    auto hc = std::make_unique<HttpCompiler>(ps.get());
    auto kc = std::make_unique<KafkaCompiler>(ps.get());
    auto mc = std::make_unique<McCompiler>(ps.get());
    auto r2 = std::make_unique<R2Compiler>(ps.get());
    auto cs = std::make_unique<CassCompiler>(ps.get());
    if (!hc->Load(d) || !kc->Load(d) || !mc->Load(d) || !r2->Load(d) || !cs->Load(d) || d.p != d.end) {
        set_err(err, errlen, "corrupt or inconsistent tables image");
        return -1;
    }
    const int rc = SwapIn(e, std::move(ps), std::move(hc), std::move(kc), std::move(mc), std::move(r2), std::move(cs),
                          err, errlen);
    if (rc == 0) {
        e->policy_src = src;
        e->policy_form = form;
        e->policy_px = px;
    }
    return rc;
}

uint64_t l7g_tables_compiled(l7g_engine *e) {
    std::lock_guard<std::mutex> g(e->mu);
    return e->hc->compiled + e->kc->compiled + e->mc->compiled + e->r2->compiled + e->cs->compiled;
}

uint64_t l7g_tables_digest(l7g_engine *e) {
    std::lock_guard<std::mutex> g(e->mu);
    std::vector<uint8_t> blob;
    AssembleBlob(e, blob);
    uint64_t h = 1469598103934665603ull;  // FNV-1a 64
    for (uint8_t b : blob) h = (h ^ b) * 1099511628211ull;
    return h;
}

int32_t l7g_policy_index(l7g_engine *e, const char *name, size_t len) {
    std::lock_guard<std::mutex> g(e->mu);
    auto it = e->ps->by_name.find(std::string(name, len));
    return it == e->ps->by_name.end() ? -1 : it->second;
}

int32_t l7g_policy_nrules(l7g_engine *e) {
    std::lock_guard<std::mutex> g(e->mu);
    return e->ps->nrules;
}

int l7g_conns_set(l7g_engine *e, const l7g_conn_t *conns, uint32_t n, char *err, size_t errlen) {
    std::lock_guard<std::mutex> g(e->mu);
    e->attrs.assign(conns, conns + n);
    std::string m;
    if (!ResolveConns(e, &m)) { set_err(err, errlen, m); return -1; }
    return 0;
}

int l7g_conn_update(l7g_engine *e, uint32_t index, const l7g_conn_t *conn, char *err, size_t errlen) {
    std::lock_guard<std::mutex> g(e->mu);
    if (index >= e->attrs.size()) {
        l7g_conn_t none{};
        none.policy = -1;
        e->attrs.resize((size_t)index + 1, none);
        e->conns.resize((size_t)index + 1, DevConn{-1, PROTO_NONE, 0, 0xFFFF});
    }
    const l7g_conn_t prev = e->attrs[index];
    const size_t nrs = TableRulesets(e);
    e->attrs[index] = *conn;
    std::string m;
    if (!ResolveOne(e, index, &m)) {
        e->attrs[index] = prev;
        ResolveOne(e, index, &m);
        set_err(err, errlen, m);
        return -1;
    }
    if (TableRulesets(e) != nrs) e->tables_dirty = true;
    if (conn->proto == PROTO_HTTP || prev.proto == PROTO_HTTP) {
        const int32_t hot = e->hot_ruleset;
        PickHot(e);
        if (hot != e->hot_ruleset) e->tables_dirty = true;
    }
    e->conns_dirty = true;
    return 0;
}

}  // extern "C"

// l7g_classify; host_conn: the connection indices in host memory as well
// (l7g_classify_host's calls), so that a small call whose requests all use the
// hot HTTP rule set skips the general HTTP kernel's launch
// pre: the call's inputs still to be copied from pinned host memory to where
// arena / off / len / conn point (HostRun); done by the first kernel when the
// call is one workgroup of one classifier, else by copy_in_kernel first.
static int Classify(l7g_engine *e, const uint8_t *arena, uint64_t arena_len, const uint64_t *off, const uint32_t *len,
                    const uint32_t *conn, uint32_t n, uint8_t *verdict, int32_t *rule, uint32_t *consumed,
                    uint64_t *counters, void *stream, const uint32_t *host_conn, const CopyIn *pre = nullptr,
                    bool *signaled = nullptr) {
    std::lock_guard<std::mutex> g(e->mu);
    if (e->device < 0) return (int)hipErrorNoDevice;
    hipError_t rc = hipSetDevice(e->device);
    if (rc == hipSuccess) rc = Upload(e);
    if (rc != hipSuccess) return (int)rc;
    hipStream_t s = (hipStream_t)stream;
    Batch B{};
    B.arena = arena;
    B.arena_len = arena_len;
    B.offs = off;
    B.lens = len;
    B.conn_ids = conn;
    B.conns = e->d_conns;
    B.verdict = verdict;
    B.rule = rule;
    B.consumed = consumed;
    B.n = n;
    B.nconns = (uint32_t)e->conns.size();
    if (n == 0) return 0;
    // The kernels each classify only their own protocol's requests, so a
    // mixed batch needs one launch per protocol present.  When the engine
    // serves more than one protocol, partition_kernel runs first: it writes
    // the Kafka and memcached index lists those two kernels walk, and answers
    // the requests no classifier owns (unknown connection, no parser) itself.
    // A single-protocol HTTP or memcached engine skips it; its one kernel walks the whole batch
    // and answers those requests.
    const int nproto = (int)e->has_http + (int)e->has_kafka + (int)e->has_mc + (int)e->has_r2 + (int)e->has_cs;
    // (a Kafka-only or memcached-only engine partitions too: the kind / length
    // lists keep the Kafka kernel's waves converged, 1.55 -> 0.99 ms on cfg3,
    // and the text / binary lists the memcached kernel's)
    // (a small memcached-only batch gains nothing from converged waves: its one
    // kernel walks the batch itself, one launch fewer on the latency path)
    bool partitioned = nproto > 1 || e->has_kafka || (e->has_mc && n >= kPartitionMin);
    bool any_cold = e->any_cold;
    // which kernels run: a small call whose connections the host can read (the
    // synchronous drop-ins: one Allowed(), one OnData) launches only the kernel
    // of the one protocol its requests use, unpartitioned, where it answers the
    // requests no parser owns too -- no partition pass, no counter memset, no
    // launch of the other protocols' kernels on an empty list
    bool run_http = e->has_http || nproto == 0, run_kafka = e->has_kafka, run_mc = e->has_mc;
    bool run_r2 = e->has_r2, run_cs = e->has_cs;
    if (host_conn && n <= kHostScanMax) {
        any_cold = false;
        uint32_t seen = 0;  // bit per parser
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t ci = host_conn[i];
            if (ci >= e->conns.size()) continue;
            const uint32_t pr = e->attrs[ci].proto;
            if (pr < 32) seen |= 1u << pr;
            any_cold = any_cold || (pr == PROTO_HTTP && e->conns[ci].ruleset != e->hot_ruleset);
        }
        any_cold = any_cold && e->any_cold;
        const uint32_t owned = seen & ((1u << PROTO_HTTP) | (1u << PROTO_KAFKA) | (1u << PROTO_MEMCACHE) |
                                       (1u << PROTO_R2D2) | (1u << PROTO_CASSANDRA));
        if (owned == (1u << PROTO_HTTP) && e->has_http) {
            partitioned = run_kafka = run_mc = run_r2 = run_cs = false;
        } else if (owned == (1u << PROTO_MEMCACHE) && e->has_mc) {
            partitioned = run_http = run_kafka = run_r2 = run_cs = false;
        }
    }
    if (n >= kPartitionMin) ReleaseServiceCUs(e);  // (persistent grids: every CU)
    StreamScratch *S = nullptr;
    if ((rc = GetScratch(e, s, &S)) != hipSuccess) return (int)rc;
    uint32_t *sel_k = nullptr, *sel_m = nullptr, *sel_h = nullptr, *sel_z = nullptr, *cnt = nullptr;
    if (partitioned) {
        const size_t need = 32 + (L7_KAFKA_CLASSES + 3) * (size_t)n;
        if (need > S->sel_cap) {
            if (S->d_sel) {  // the previous call on this stream may still use it
                if (S->launched) rc = hipEventSynchronize(S->done_ev);
                hipFree(S->d_sel);
                S->d_sel = nullptr;
                S->sel_cap = 0;
            }
            if (rc == hipSuccess) rc = hipMalloc(&S->d_sel, need * sizeof(uint32_t));
            if (rc == hipSuccess) S->sel_cap = need;
        }
        if (rc != hipSuccess) return (int)rc;
        // [0, L7_KAFKA_CLASSES) Kafka classes, memcached retrievals, binary, HTTP, other text;
        // [26] Kafka entry counter, [28, 29] HTTP tile counters (hot, general launch); [31] compressed
        // Kafka
        cnt = S->d_sel;
        sel_k = S->d_sel + 32;
        sel_m = sel_k + L7_KAFKA_CLASSES * (size_t)n;
        sel_h = sel_m + (size_t)n;
        sel_z = sel_h + (size_t)n;
        if (rc == hipSuccess) rc = hipMemsetAsync(cnt, 0, 32 * sizeof(uint32_t), s);
        if (rc == hipSuccess && e->has_kafka && !e->d_zreg) {
            rc = hipEventCreateWithFlags(&e->zreg_ev, hipEventDisableTiming);
            if (rc == hipSuccess) rc = hipMalloc(&e->d_zreg, (size_t)KafkaInflateBlocks() * KafkaInflateRegionBytes());
        }
        if (rc != hipSuccess) return (int)rc;
    }
    // rule sets with NFA-fallback matchers: the pre-pass writes one u64 per request
    HttpTables ht = e->ht;
    const bool nfa = e->ht.nfa_pool != nullptr && run_http;
    if (nfa && rc == hipSuccess) {
        if (n > S->nfa_cap) {
            if (S->d_nfa) {
                if (S->launched) rc = hipEventSynchronize(S->done_ev);
                hipFree(S->d_nfa);
                S->d_nfa = nullptr;
                S->nfa_cap = 0;
            }
            if (rc == hipSuccess) rc = hipMalloc(&S->d_nfa, (size_t)n * sizeof(uint64_t));
            if (rc == hipSuccess) S->nfa_cap = n;
        }
        if (rc != hipSuccess) return (int)rc;
        ht.nfa_bits = S->d_nfa;
    }
    // large NFAs: one scratch for the call's launches (they run one after
    // another on this stream), as many lanes as a budget allows; the kernels
    // loop over their requests with that many lanes
    McTables mt = e->mt;
    R2Tables rt = e->rt;
    CassTables ct = e->ct;
    uint32_t big_lanes = 0;
    {
        const uint32_t lw = std::max({ht.nfa_lane_words, mt.nfa_lane_words, rt.nfa_lane_words, ct.nfa_lane_words});
        if (lw && rc == hipSuccess) {
            const size_t lane_bytes = (size_t)lw * 8;
            size_t lanes = std::min<size_t>(((size_t)n + 255) & ~(size_t)255, kNfaScratchBytes / lane_bytes);
            lanes = std::max<size_t>(lanes & ~(size_t)255, 256);
            if (lanes * lane_bytes > S->bignfa_bytes) {
                if (S->d_bignfa) {
                    if (S->launched) rc = hipEventSynchronize(S->done_ev);
                    hipFree(S->d_bignfa);
                    S->d_bignfa = nullptr;
                    S->bignfa_bytes = 0;
                }
                if (rc == hipSuccess) rc = hipMalloc(&S->d_bignfa, lanes * lane_bytes);
                if (rc == hipSuccess) S->bignfa_bytes = lanes * lane_bytes;
            }
            if (rc != hipSuccess) return (int)rc;
            big_lanes = (uint32_t)(S->bignfa_bytes / lane_bytes);
            uint64_t *sc = S->d_bignfa;
            if (ht.nfa_lane_words) { ht.nfa_scratch = sc; ht.nfa_lane_words = lw; }
            if (mt.nfa_lane_words) { mt.nfa_scratch = sc; mt.nfa_lane_words = lw; }
            if (rt.nfa_lane_words) { rt.nfa_scratch = sc; rt.nfa_lane_words = lw; }
            if (ct.nfa_lane_words) { ct.nfa_scratch = sc; ct.nfa_lane_words = lw; }
        }
    }
    // profiling: event k is recorded before stage k (partition, http, kafka, memcache), event 4 after the last
    const bool prof = e->profile;
    auto mark = [&](int k) {
        if (prof && rc == hipSuccess) rc = hipEventRecord(e->prof_ev[k], s);
    };
    // the copy of a small call's inputs: inside the one kernel that reads them
    // when that kernel is one workgroup (HTTP: one request per wave, at most 8;
    // memcached: at most 64 requests, one wave), else a launch of its own
    const bool only_http = run_http && !partitioned && !run_kafka && !run_mc && !run_r2 && !run_cs;
    const bool only_mc = run_mc && !partitioned && !run_http && !run_kafka && !run_r2 && !run_cs;
    const CopyIn *fuse_http = pre && only_http && !nfa && n <= 8 ? pre : nullptr;
    const CopyIn *fuse_mc = pre && only_mc && n <= 64 ? pre : nullptr;
    if (pre && !fuse_http && !fuse_mc && rc == hipSuccess) {
        CopyIn c = *pre;
        c.done = nullptr;  // (the classifiers that follow end the call)
        rc = LaunchCopyIn(c, s);
    }
    // the one-workgroup kernel that ends the call stores the done word (and no
    // counters or proxy statistics follow it)
    const bool signal = (fuse_http || fuse_mc) && pre->done && !counters && !(e->flow_stats && !e->skey_list.empty());
    CopyIn fused_c{};
    if (fuse_http || fuse_mc) {
        fused_c = *pre;
        if (!signal) fused_c.done = nullptr;
    }
    if (fuse_http) fuse_http = &fused_c;
    if (fuse_mc) fuse_mc = &fused_c;
    if (signaled) *signaled = signal;
    const bool run[4] = {partitioned, run_http, run_kafka, run_mc};
    for (int k = 0; k < 4; k++) e->prof_ran[k] = run[k];
    mark(0);
    if (rc == hipSuccess && run[0]) rc = LaunchPartition(B, sel_k, sel_m, sel_h, cnt, s);
    mark(1);
    if (rc == hipSuccess && run[1] && nfa) rc = LaunchHttpNfa(B, ht, big_lanes, s);
    // tile counters: in the partition counts (zeroed above), or, for a large
    // unpartitioned batch, two words zeroed here (a small batch keeps the fixed
    // stride and saves the memset)
    uint32_t *tile_ctr = cnt ? cnt + 28 : nullptr;
    if (rc == hipSuccess && run[1] && !cnt && n >= kDynTilesMin) {
        if (!S->d_work) rc = hipMalloc(&S->d_work, 4 * sizeof(uint32_t));
        if (rc == hipSuccess) rc = hipMemsetAsync(S->d_work, 0, 2 * sizeof(uint32_t), s);
        tile_ctr = S->d_work;
    }
    // many rule sets in use: the HTTP requests sorted by rule set, so that each
    // workgroup stages one image per segment (kernels/http_group.hip)
    const bool grouped = run[1] && any_cold && n >= kGroupMin && ht.nrulesets >= 2 &&
                         ht.nrulesets <= kMaxGroupRulesets;
    if (rc == hipSuccess && grouped) {
        const size_t R = ht.nrulesets, segw = 3 * ((size_t)n / kGroupSegEntries + R + 1);
        const size_t need = 8 + 2 * R + segw + 2 * (size_t)n;
        if (need > S->grp_cap) {
            if (S->d_grp) {
                if (S->launched) rc = hipEventSynchronize(S->done_ev);
                hipFree(S->d_grp);
                S->d_grp = nullptr;
                S->grp_cap = 0;
            }
            if (rc == hipSuccess) rc = hipMalloc(&S->d_grp, need * sizeof(uint32_t));
            if (rc == hipSuccess) S->grp_cap = need;
        }
        uint32_t *ctl = S->d_grp, *hist = ctl + 8, *cursor = hist + R, *segs = cursor + R, *gsel = segs + segw,
                 *gbig = gsel + n;
        if (rc == hipSuccess) rc = hipMemsetAsync(ctl, 0, (8 + R) * sizeof(uint32_t), s);
        if (rc == hipSuccess)
            rc = LaunchHttpGroup(B, ht, sel_h, cnt ? cnt + L7_KAFKA_CLASSES + 2 : nullptr, n, !partitioned, ctl, hist,
                                 cursor, segs, gsel, gbig, s);
        if (rc == hipSuccess) rc = LaunchHttpGrouped(B, ht, gsel, segs, gbig, ctl, e->any_big_image, s);
    } else if (rc == hipSuccess && run[1]) {
        rc = LaunchHttpClassify(B, ht, sel_h, cnt ? cnt + L7_KAFKA_CLASSES + 2 : nullptr, any_cold, !partitioned,
                                tile_ctr, n <= kLatencyMax, fuse_http, s);
    }
    mark(2);
    // a large partitioned batch with both Kafka and memcached requests: the
    // memcached kernel runs on a side stream beside the Kafka kernel, which leaves
    // one workgroup slot per CU for it (cfg5: 37.31 -> 36.44 ms per step,
    // profiles/r6/ab6h_kafka_memcached_beside.txt)
    const bool km = partitioned && run[2] && run[3] && !prof && big_lanes == 0 && n >= kBesideMin && !pre;
    const int kafka_leave = km ? 1 : 0;
    hipStream_t ms = s;
    if (km && rc == hipSuccess) {
        if (!S->side) {
            rc = hipStreamCreateWithFlags(&S->side, hipStreamNonBlocking);
            if (rc == hipSuccess) rc = hipEventCreateWithFlags(&S->fork_ev, hipEventDisableTiming);
            if (rc == hipSuccess) rc = hipEventCreateWithFlags(&S->join_ev, hipEventDisableTiming);
        }
        if (rc == hipSuccess) rc = hipEventRecord(S->fork_ev, s);
        if (rc == hipSuccess) rc = hipStreamWaitEvent(S->side, S->fork_ev, 0);
        if (rc == hipSuccess) ms = S->side;
    }
    uint32_t *zcount = cnt ? cnt + 31 : nullptr;
    if (rc == hipSuccess && run[2])
        rc = LaunchKafkaClassify(B, e->kt, sel_k, cnt, !partitioned, sel_z, zcount, cnt ? cnt + 26 : nullptr, s,
                                 kafka_leave);
    // requests with gzip / snappy messages: decoded, their sets read, failures answered
    if (rc == hipSuccess && run[2] && sel_z) {
        // the engine's one decode region: after the previous inflate launch on any stream
        if (e->zreg_used) rc = hipStreamWaitEvent(s, e->zreg_ev, 0);
        if (rc == hipSuccess) rc = LaunchKafkaInflate(B, sel_z, zcount, e->d_zreg, s);
        if (rc == hipSuccess) rc = hipEventRecord(e->zreg_ev, s);
        if (rc == hipSuccess) e->zreg_used = true;
    }
    mark(3);
    if (rc == hipSuccess && run[3])
        rc = LaunchMemcacheClassify(B, mt, sel_m, sel_h, cnt ? cnt + L7_KAFKA_CLASSES : nullptr, !partitioned, big_lanes,
                                    ms, fuse_mc);
    if (ms != s && rc == hipSuccess) {
        rc = hipEventRecord(S->join_ev, ms);
        if (rc == hipSuccess) rc = hipStreamWaitEvent(s, S->join_ev, 0);
    }
    // r2d2 (proxylib's example line protocol): one lane per request over the whole batch
    if (rc == hipSuccess && run_r2) rc = LaunchR2d2Classify(B, rt, !partitioned, big_lanes, s);
    // cassandra (proxylib): the batch's USE requests, then one lane per request
    if (rc == hipSuccess && run_cs) {
        const size_t need = CassandraScratchBytes(n);
        if (need == 0) rc = hipErrorInvalidValue;
        if (rc == hipSuccess && need > S->use_cap) {
            if (S->d_use) {
                if (S->launched) rc = hipEventSynchronize(S->done_ev);
                hipFree(S->d_use);
                S->d_use = nullptr;
                S->use_cap = 0;
            }
            if (rc == hipSuccess) rc = hipMalloc(&S->d_use, need);
            if (rc == hipSuccess) S->use_cap = need;
        }
        if (rc == hipSuccess) rc = LaunchCassandraClassify(B, ct, S->d_use, S->use_cap, !partitioned, big_lanes, s);
    }
    mark(4);
    // proxy statistics (accumulated on the device until read)
    if (rc == hipSuccess && e->flow_stats && !e->skey_list.empty()) {
        const size_t nk = e->skey_list.size();
        if (nk > e->flow_cap) {  // grow, keeping what was accumulated
            uint64_t *d = nullptr;
            // every stream's earlier flowstats kernels may still add into the old
            // accumulator: they finish before it is copied (e->mu is held, so no
            // new launch can race with the copy)
            if (e->d_flow) rc = WaitLastClassify(e);
            if (rc == hipSuccess) rc = hipMalloc(&d, nk * 4 * sizeof(uint64_t));
            if (rc == hipSuccess) rc = hipMemsetAsync(d, 0, nk * 4 * sizeof(uint64_t), s);
            if (rc == hipSuccess && e->d_flow)
                rc = hipMemcpyAsync(d, e->d_flow, e->flow_cap * 4 * sizeof(uint64_t), hipMemcpyDeviceToDevice, s);
            if (rc == hipSuccess) {
                if (e->d_flow) {
                    hipStreamSynchronize(s);
                    hipFree(e->d_flow);
                }
                e->d_flow = d;
                e->flow_cap = nk;
            }
        }
        if (rc == hipSuccess) rc = LaunchFlowStats(B, (uint32_t)nk, e->d_flow, s);
    }
    // per-rule allow hits and per-verdict totals, from the outputs
    if (rc == hipSuccess && counters) {
        if (!S->d_hist) rc = hipMalloc(&S->d_hist, CountersScratchBytes());
        if (rc == hipSuccess) rc = LaunchCounters(verdict, rule, n, (uint32_t)e->ps->nrules, counters, S->d_hist, s);
    }
    if (rc == hipSuccess) rc = hipEventRecord(S->done_ev, s);
    if (rc == hipSuccess) S->launched = true;
    return (int)rc;
}

extern "C" {

int l7g_classify(l7g_engine *e, const uint8_t *arena, uint64_t arena_len, const uint64_t *off, const uint32_t *len,
                 const uint32_t *conn, uint32_t n, uint8_t *verdict, int32_t *rule, uint32_t *consumed,
                 uint64_t *counters, void *stream) {
    return Classify(e, arena, arena_len, off, len, conn, n, verdict, rule, consumed, counters, stream, nullptr);
}

int l7g_frame_streams(l7g_engine *e, const uint8_t *arena, uint64_t arena_len, const uint64_t *s_off,
                      const uint32_t *s_len, const uint32_t *s_conn, uint32_t n, uint32_t max_frames,
                      uint64_t *frame_off, uint32_t *frame_len, uint32_t *frame_conn, uint32_t *nframes, void *stream) {
    std::lock_guard<std::mutex> g(e->mu);
    if (e->device < 0) return (int)hipErrorNoDevice;
    if (max_frames == 0 || (uint64_t)n * max_frames > 0xFFFFFFFFull) return (int)hipErrorInvalidValue;
    hipError_t rc = hipSetDevice(e->device);
    if (rc == hipSuccess) rc = Upload(e);  // (the connection table the walk reads)
    if (rc == hipSuccess)
        rc = LaunchFrameStreams(arena, arena_len, s_off, s_len, s_conn, n, e->d_conns, (uint32_t)e->conns.size(),
                                max_frames, frame_off, frame_len, frame_conn, nframes, (hipStream_t)stream);
    return (int)rc;
}

int l7g_classify_streams(l7g_engine *e, const uint8_t *arena, uint64_t arena_len, const uint64_t *s_off,
                         const uint32_t *s_len, const uint32_t *s_conn, uint32_t n, uint32_t max_frames,
                         uint64_t *frame_off, uint32_t *frame_len, uint32_t *frame_conn, uint32_t *nframes,
                         uint8_t *verdict, int32_t *rule, uint32_t *consumed, uint64_t *counters, void *stream) {
    int rc = l7g_frame_streams(e, arena, arena_len, s_off, s_len, s_conn, n, max_frames, frame_off, frame_len,
                               frame_conn, nframes, stream);
    if (rc != 0) return rc;
    // every slot, the empty ones on connection ~0 (answered UNSUPPORTED)
    return Classify(e, arena, arena_len, frame_off, frame_len, frame_conn, n * max_frames, verdict, rule, consumed,
                    counters, stream, nullptr);
}

}  // extern "C"

// ---- l7g_classify_host's per-thread path, in three steps (the batcher's
// flushers fill the staging in place and skip the copy)

// this thread's stream and staging (the engine lock is held only while
// l7g_classify enqueues, so threads' copies and kernels overlap)
static hipError_t HostCtxFor(l7g_engine *e, HostCtx **out) {
    std::lock_guard<std::mutex> g(e->hmu);
    auto &slot = e->hctx[std::this_thread::get_id()];
    if (!slot) {
        auto h = std::make_unique<HostCtx>();
        hipError_t rc;
        if ((rc = hipStreamCreateWithFlags(&h->s, hipStreamNonBlocking)) != hipSuccess) return rc;
        slot = std::move(h);
    }
    *out = slot.get();
    return hipSuccess;
}

// grow-only staging: inputs [off | len | conn | arena (+64 B so aligned
// 16-byte reads stay inside)], outputs [verdict | rule | consumed]
static size_t HostArenaOff(uint32_t n) { return ((size_t)std::max<uint32_t>(n, 1) * 16 + 255) & ~(size_t)255; }
static hipError_t HostGrow(HostCtx *H, uint32_t n, uint64_t arena_len) {
    const size_t nn = std::max<uint32_t>(n, 1);
    const size_t need_in = HostArenaOff(n) + arena_len + 64;
    const size_t need_out = nn * 9 + 64;
    if (need_in <= H->in_cap && need_out <= H->out_cap) return hipSuccess;
    // (the previous call of this thread has its answers; its kernels may still be
    // retiring after storing the done word)
    if (H->s) hipStreamSynchronize(H->s);
    if (H->dev) hipFree(H->dev);
    if (H->pin_in) hipHostFree(H->pin_in);
    if (H->pin_out) hipHostFree(H->pin_out);
    H->dev = H->pin_in = H->pin_out = H->pin_in_dev = H->pin_out_dev = nullptr;
    H->in_cap = std::max(need_in + need_in / 4, (size_t)1 << 16);  // (some slack: batches vary)
    H->out_cap = std::max(need_out + need_out / 4, (size_t)1 << 14);
    hipError_t rc;
    if ((rc = hipMalloc(&H->dev, H->in_cap + H->out_cap)) != hipSuccess) { H->in_cap = H->out_cap = 0; return rc; }
    if ((rc = hipHostMalloc(&H->pin_in, H->in_cap, hipHostMallocDefault)) != hipSuccess ||
        (rc = hipHostMalloc(&H->pin_out, H->out_cap, hipHostMallocDefault)) != hipSuccess ||
        (rc = hipHostGetDevicePointer((void **)&H->pin_in_dev, H->pin_in, 0)) != hipSuccess ||
        (rc = hipHostGetDevicePointer((void **)&H->pin_out_dev, H->pin_out, 0)) != hipSuccess) {
        H->in_cap = H->out_cap = 0;
        return rc;
    }
    if (!H->pin_done) {
        if ((rc = hipHostMalloc((void **)&H->pin_done, 64, hipHostMallocDefault)) != hipSuccess) return rc;
        *(volatile uint32_t *)H->pin_done = 0;
        H->seq = 0;
        if ((rc = hipHostGetDevicePointer((void **)&H->pin_done_dev, H->pin_done, 0)) != hipSuccess) return rc;
    }
    return hipSuccess;
}

// where a call's inputs lie in pinned host memory: the thread's staging, or a
// batcher slot filled in place (its three arrays `stride` entries apart, its
// request bytes in one piece per lane)
struct HostIn {
    const uint64_t *off;
    const uint32_t *len, *conn;
    size_t stride;  // > 0: len = (u8 *)off + stride * 8, conn = (u8 *)off + stride * 12
    const l7g_host_seg *seg;
    int nseg;  // the arena is these pieces, concatenated
};

// The service's box, staging and stream (v.mu held), on its first call.
static hipError_t ServiceAlloc(Service &v) {
    if (v.s) return hipSuccess;
    hipError_t rc;
    void *p = nullptr;
    if ((rc = hipHostMalloc(&p, sizeof(SvcBox), hipHostMallocCoherent)) != hipSuccess) return rc;
    v.box = (SvcBox *)p;
    memset(v.box, 0, sizeof(SvcBox));
    if ((rc = hipHostGetDevicePointer((void **)&v.box_dev, v.box, 0)) != hipSuccess ||
        (rc = hipHostMalloc((void **)&v.pin_in, kSvcInBytes, hipHostMallocDefault)) != hipSuccess ||
        (rc = hipHostMalloc((void **)&v.pin_out, kSvcOutBytes, hipHostMallocDefault)) != hipSuccess ||
        (rc = hipHostGetDevicePointer((void **)&v.pin_in_dev, v.pin_in, 0)) != hipSuccess ||
        (rc = hipHostGetDevicePointer((void **)&v.pin_out_dev, v.pin_out, 0)) != hipSuccess ||
        (rc = hipMalloc((void **)&v.dev_in, kSvcInBytes)) != hipSuccess)
        return rc;
    if ((rc = hipStreamCreateWithFlags(&v.s, hipStreamNonBlocking)) != hipSuccess) return rc;  // (v.s: allocated)
    __atomic_store_n(&v.box_ready, v.box, __ATOMIC_RELEASE);
    return hipSuccess;
}

// Posts a call to service v (e->mu and v.mu held; the inputs are in
// v.pin_in): the job's words, then req_seq, then the state read that decides
// whether a workgroup must be launched (a new service, one that has left, or
// one whose launch arguments are stale).
static hipError_t ServicePost(l7g_engine *e, Service &v, int kind, uint32_t n, uint64_t arena_len, uint32_t flags,
                              uint32_t *seq_out) {
    hipError_t rc = hipSuccess;
    const uint32_t nconns = (uint32_t)e->conns.size();
    const bool same = kind == 0 ? memcmp(&v.ht, &e->ht, sizeof v.ht) == 0 : memcmp(&v.mt, &e->mt, sizeof v.mt) == 0;
    if (v.launched && !(same && v.conns == e->d_conns && v.nconns == nconns) && (rc = ServiceStop(v)) != hipSuccess)
        return rc;
    SvcBox *b = v.box;
    __atomic_store_n(&b->n, n, __ATOMIC_RELAXED);  // (the line's other words: stored before req_seq)
    __atomic_store_n(&b->arena_len, (uint32_t)arena_len, __ATOMIC_RELAXED);
    __atomic_store_n(&b->flags, flags, __ATOMIC_RELAXED);
    __atomic_store_n(&b->stop, 0u, __ATOMIC_RELAXED);
    std::atomic_thread_fence(std::memory_order_release);
    uint32_t seq = ++v.seq;
    if (!seq) seq = ++v.seq;  // (never 0: the done word's initial value)
    __atomic_store_n(&b->req_seq, seq, __ATOMIC_SEQ_CST);  // (after the inputs and the job's words)
    // the workgroup's exit handshake writes EXITING, fences, reads req_seq:
    // either it sees this call, or this read sees it leaving
    uint32_t st = __atomic_load_n(&b->state, __ATOMIC_SEQ_CST);
    bool start = !v.launched;
    if (v.launched && st != kSvcRunning) {
        const auto t0 = std::chrono::steady_clock::now();
        while ((st = __atomic_load_n(&b->state, __ATOMIC_SEQ_CST)) == kSvcExiting &&
               std::chrono::steady_clock::now() - t0 < std::chrono::seconds(1))
            __builtin_ia32_pause();
        start = st != kSvcRunning;
        if (start && (rc = hipStreamSynchronize(v.s)) != hipSuccess) return rc;  // (the old workgroup has left)
    }
    if (start) {
        __atomic_store_n(&b->state, (uint32_t)kSvcRunning, __ATOMIC_SEQ_CST);
        const SvcStatic S{v.pin_in_dev, v.dev_in, v.pin_out_dev, e->d_conns, nconns, 0};
        rc = kind == 0 ? LaunchHttpService(v.box_dev, S, e->ht, seq - 1, kSvcIdleCycles, v.s)
                       : LaunchMemcacheService(v.box_dev, S, e->mt, seq - 1, kSvcIdleCycles, v.s);
        if (rc != hipSuccess) return rc;
        v.ht = e->ht;
        v.mt = e->mt;
        v.conns = e->d_conns;
        v.nconns = nconns;
        v.launched = true;
        v.launches++;
    }
    v.calls++;
    *seq_out = seq;
    return hipSuccess;
}

// A synchronous call a service can take: the HTTP (at most kSvcHttpMax) or the
// memcached (at most kSvcMcMax) requests of one small call whose inputs lie in
// one piece of pinned memory, with the selection Classify makes for such a
// call (only that protocol's kernel, unpartitioned, answering the requests no
// parser owns) and nothing else to run (no NFA-fallback matchers, no proxy
// statistics).  Returns false when the call takes the launched path; true
// when it was answered (or failed: *rc_out).
static bool ServiceTry(l7g_engine *e, uint32_t n, uint64_t arena_len, const HostIn &in, uint8_t *verdict,
                       int32_t *rule, uint32_t *consumed, hipError_t *rc_out) {
    if (!e->svc_on || n == 0 || n > kSvcMcMax || arena_len > kZeroCopyMaxBytes) return false;
    if (!(in.nseg == 0 || (in.nseg == 1 && in.seg[0].rows <= 1 && in.seg[0].width == arena_len))) return false;
    if (in.nseg == 0 && arena_len) return false;
    Service *v = nullptr;
    uint32_t seq = 0;
    {
        std::lock_guard<std::mutex> g(e->mu);
        if (e->device < 0 || hipSetDevice(e->device) != hipSuccess || Upload(e) != hipSuccess) return false;
        if (e->flow_stats && !e->skey_list.empty()) return false;
        uint32_t seen = 0;
        bool any_cold = false;
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t ci = in.conn[i];
            if (ci >= e->conns.size()) continue;
            const uint32_t pr = e->attrs[ci].proto;
            if (pr < 32) seen |= 1u << pr;
            any_cold = any_cold || (pr == PROTO_HTTP && e->conns[ci].ruleset != e->hot_ruleset);
        }
        any_cold = any_cold && e->any_cold;
        const uint32_t owned = seen & ((1u << PROTO_HTTP) | (1u << PROTO_KAFKA) | (1u << PROTO_MEMCACHE) |
                                       (1u << PROTO_R2D2) | (1u << PROTO_CASSANDRA));
        int kind = -1;
        uint32_t flags = kSvcAnswerOther;
        if (owned == (1u << PROTO_HTTP) && e->has_http && n <= kSvcHttpMax && !e->ht.nfa_pool) {
            kind = 0;
            const bool hot = e->ht.hot_ruleset >= 0;
            flags |= (hot ? kSvcHttpHot : 0u) | (!hot || any_cold ? kSvcHttpGeneral : 0u);
        } else if (owned == (1u << PROTO_MEMCACHE) && e->has_mc && !e->mt.nfa_pool) {
            kind = 1;
        }
        if (kind < 0) return false;
        v = &e->svc[kind];
        if (!v->mu.try_lock()) return false;  // (another thread's call is in the service: launch this one)
        // the inputs, in the service's layout (service_types.h)
        const uint32_t nn = n;
        const size_t a_off = SvcArenaOff(n);
        hipError_t rc = ServiceAlloc(*v);
        if (rc == hipSuccess) {
            memcpy(v->pin_in, in.off, (size_t)nn * 8);
            memcpy(v->pin_in + (size_t)nn * 8, in.len, (size_t)nn * 4);
            memcpy(v->pin_in + (size_t)nn * 12, in.conn, (size_t)nn * 4);
            if (arena_len) memcpy(v->pin_in + a_off, in.seg[0].p, arena_len);
            rc = ServicePost(e, *v, kind, n, arena_len, flags, &seq);
        }
        if (rc != hipSuccess) {
            v->mu.unlock();
            *rc_out = rc;
            return true;
        }
    }
    // the answers: the done word, then pinned memory (no stream wait: a fault
    // shows as a done word that never comes, and the service's stream reports it)
    hipError_t rc = hipSuccess;
    bool done = false;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 0;; k++) {
        if (__atomic_load_n(&v->box->done, __ATOMIC_ACQUIRE) == seq) {
            done = true;
            break;
        }
        if ((k & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(1000)) break;
        __builtin_ia32_pause();
    }
    if (!done) {  // (v->mu held: the service's own fields only, no engine lock)
        rc = hipStreamQuery(v->s);
        if (rc == hipSuccess || rc == hipErrorNotReady) rc = hipErrorLaunchTimeOut;
        const hipError_t r2 = ServiceStop(*v);
        if (rc == hipErrorLaunchTimeOut && r2 != hipSuccess) rc = r2;
    } else {
        const uint32_t nn = n;
        const uint8_t *po = v->pin_out;
        memcpy(verdict, po, n);
        memcpy(rule, po + ((nn + 3) & ~3u), (size_t)n * 4);
        memcpy(consumed, po + ((nn + 3) & ~3u) + (size_t)nn * 4, (size_t)n * 4);
    }
    v->mu.unlock();
    *rc_out = rc;
    return true;
}

// classify a call whose inputs are in pinned host memory, wait for it, copy
// the answers out
static hipError_t HostRun(l7g_engine *e, HostCtx *H, uint32_t n, uint64_t arena_len, const HostIn &in,
                          uint8_t *verdict, int32_t *rule, uint32_t *consumed, bool try_service = true) {
    hipError_t rc = hipSuccess;
    if (try_service && ServiceTry(e, n, arena_len, in, verdict, rule, consumed, &rc)) return rc;
    const size_t nn = std::max<uint32_t>(n, 1);
    const size_t a_off = HostArenaOff(n);
    // A small call (the Envoy adapter's Allowed(), one OnData, a light batch)
    // is latency, not bandwidth: the kernels read the inputs from and write the
    // verdicts to the pinned memory in place (zero-copy, over PCIe), so the
    // call is one launch and a wait instead of copy, launch, copy, wait.
    static const bool zc_on = [] {
        const char *v = getenv("L7G_SYNC_ZEROCOPY");
        return !(v && v[0] == '0');
    }();
    const bool zc = zc_on && (in.nseg == 0 || (in.nseg == 1 && in.seg[0].rows <= 1)) && n <= kZeroCopyMaxRequests &&
                    a_off + arena_len <= kZeroCopyMaxBytes;
    hipStream_t s = H->s;
    const uint64_t *d_o;
    const uint32_t *d_l, *d_c;
    const uint8_t *d_a;
    uint8_t *d_out = H->dev + H->in_cap;
    CopyIn pre{};  // zero-copy: the inputs' copy into HBM, done by the call's first kernel
    if (zc) {
        // The inputs are copied into HBM (one PCIe round trip per 64 KiB, every
        // load in flight before the first store: by the call's first kernel when
        // it is one workgroup, else by copy_in_kernel) and classified there: read
        // in place, every dependent read of a framer was a PCIe round trip.  The
        // verdicts are still written to the pinned memory in place.
        d_out = H->pin_out_dev;
        uint8_t *d_in = H->dev;
        CopyIn ci{};
        const size_t a_at = in.nseg ? (size_t)((const uint8_t *)in.seg[0].p - H->pin_in) : 0;
        if (in.off == (const uint64_t *)H->pin_in && in.len == (const uint32_t *)(H->pin_in + nn * 8) &&
            in.conn == (const uint32_t *)(H->pin_in + nn * 12) && a_at <= a_off && a_at % 16 == 0) {
            // the thread's staging ([off | len | conn | arena at a_off]): one piece
            ci.p[0] = {H->pin_in_dev, d_in, (uint64_t)(a_off + arena_len)};
            ci.n = 1;
            d_o = (const uint64_t *)d_in;
            d_l = (const uint32_t *)(d_in + nn * 8);
            d_c = (const uint32_t *)(d_in + nn * 12);
            d_a = d_in + a_at;
        } else {
            // a batcher slot: four pieces into [off | len | conn | arena], the arrays
            // nn4 entries long so each starts 16-byte aligned (a_off, a multiple of
            // 256 at least 16 nn, is at least 16 nn4)
            void *dp = nullptr;
            auto dev_ptr = [&](const void *h) -> const uint8_t * {
                if (rc == hipSuccess) rc = hipHostGetDevicePointer(&dp, const_cast<void *>(h), 0);
                return (const uint8_t *)dp;
            };
            const uint8_t *h_o = dev_ptr(in.off), *h_l = dev_ptr(in.len), *h_c = dev_ptr(in.conn);
            const uint8_t *h_a = in.nseg ? dev_ptr(in.seg[0].p) : h_o;
            if (rc != hipSuccess) return rc;
            auto al16 = [](const void *p) { return ((uintptr_t)p & 15) == 0; };
            if (!(al16(h_o) && al16(h_l) && al16(h_c) && al16(h_a))) return hipErrorInvalidValue;  // (slots are)
            const size_t nn4 = (nn + 3) & ~(size_t)3;
            ci.p[0] = {h_o, d_in, (uint64_t)nn * 8};
            ci.p[1] = {h_l, d_in + nn4 * 8, (uint64_t)nn * 4};
            ci.p[2] = {h_c, d_in + nn4 * 12, (uint64_t)nn * 4};
            ci.p[3] = {h_a, d_in + a_off, in.nseg ? arena_len : 0};
            ci.n = 4;
            d_o = (const uint64_t *)d_in;
            d_l = (const uint32_t *)(d_in + nn4 * 8);
            d_c = (const uint32_t *)(d_in + nn4 * 12);
            d_a = in.nseg ? d_in + a_off : d_in;
        }
        pre = ci;
        pre.done = H->pin_done_dev;
        pre.seq = ++H->seq ? H->seq : ++H->seq;  // (never 0, the word's initial value)
    } else {
        uint8_t *d_in = H->dev;
        const bool staging = in.off == (const uint64_t *)H->pin_in;
        const size_t st = staging ? nn : in.stride ? in.stride : nn;
        d_o = (const uint64_t *)d_in;
        d_l = (const uint32_t *)(d_in + st * 8);
        d_c = (const uint32_t *)(d_in + st * 12);
        d_a = d_in + HostArenaOff((uint32_t)st);
        if (staging) {  // the thread's staging: one copy of the whole layout
            rc = hipMemcpyAsync(d_in, H->pin_in, a_off + arena_len, hipMemcpyHostToDevice, s);
        } else {
            if (in.stride) {  // the three arrays in one copy
                rc = hipMemcpyAsync(d_in, in.off, st * 12 + (size_t)n * 4, hipMemcpyHostToDevice, s);
            } else {
                rc = hipMemcpyAsync((void *)d_o, in.off, (size_t)n * 8, hipMemcpyHostToDevice, s);
                if (rc == hipSuccess) rc = hipMemcpyAsync((void *)d_l, in.len, (size_t)n * 4, hipMemcpyHostToDevice, s);
                if (rc == hipSuccess) rc = hipMemcpyAsync((void *)d_c, in.conn, (size_t)n * 4, hipMemcpyHostToDevice, s);
            }
            uint64_t at = 0;
            for (int k = 0; k < in.nseg && rc == hipSuccess; k++) {
                const l7g_host_seg &g = in.seg[k];
                if (!g.width || !g.rows) continue;
                if (g.rows == 1)
                    rc = hipMemcpyAsync((void *)(d_a + at), g.p, g.width, hipMemcpyHostToDevice, s);
                else
                    rc = hipMemcpy2DAsync((void *)(d_a + at), g.width, g.p, g.pitch, g.width, g.rows,
                                          hipMemcpyHostToDevice, s);
                at += g.width * g.rows;
            }
        }
    }
    uint8_t *d_v = d_out;
    int32_t *d_r = (int32_t *)(d_out + ((nn + 3) & ~(size_t)3));
    uint32_t *d_cons = (uint32_t *)(d_out + ((nn + 3) & ~(size_t)3) + nn * 4);
    bool signaled = false;
    if (rc == hipSuccess)
        rc = (hipError_t)Classify(e, d_a, arena_len, d_o, d_l, d_c, n, d_v, d_r, d_cons, nullptr, s, in.conn,
                                  pre.n ? &pre : nullptr, &signaled);
    const size_t out_bytes = ((nn + 3) & ~(size_t)3) + nn * 8;
    if (rc == hipSuccess && n && !zc) rc = hipMemcpyAsync(H->pin_out, d_out, out_bytes, hipMemcpyDeviceToHost, s);
    // One workgroup answered the call: its done word says the answers are in
    // pinned memory (a spin on that word is some microseconds shorter than the
    // stream's completion signal); past 2 ms, or otherwise, wait on the stream,
    // which also reports a kernel's failure.
    bool done = false;
    if (rc == hipSuccess && signaled) {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t k = 0;; k++) {
            if (*(volatile uint32_t *)H->pin_done == pre.seq) {
                done = true;
                break;
            }
            if ((k & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
            __builtin_ia32_pause();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
    }
    if (rc == hipSuccess && !done) rc = hipStreamSynchronize(s);
    if (rc == hipSuccess && n) {
        const uint8_t *po = H->pin_out;
        memcpy(verdict, po, n);
        memcpy(rule, po + ((nn + 3) & ~(size_t)3), (size_t)n * 4);
        memcpy(consumed, po + ((nn + 3) & ~(size_t)3) + nn * 4, (size_t)n * 4);
    }
    return rc;
}

int l7g_host_stage(l7g_engine *e, uint32_t n, uint64_t arena_len, uint8_t **arena, uint64_t **off, uint32_t **len,
                   uint32_t **conn) {
    if (e->device < 0) return (int)hipErrorNoDevice;
    hipError_t rc = hipSetDevice(e->device);
    HostCtx *H = nullptr;
    if (rc == hipSuccess) rc = HostCtxFor(e, &H);
    if (rc == hipSuccess) rc = HostGrow(H, n, arena_len);
    if (rc != hipSuccess) return (int)rc;
    const size_t nn = std::max<uint32_t>(n, 1);
    *off = (uint64_t *)H->pin_in;
    *len = (uint32_t *)(H->pin_in + nn * 8);
    *conn = (uint32_t *)(H->pin_in + nn * 12);
    *arena = H->pin_in + HostArenaOff(n);
    return 0;
}

static int HostRunStaged(l7g_engine *e, uint32_t n, uint64_t arena_len, uint8_t *verdict, int32_t *rule,
                         uint32_t *consumed, bool try_service) {
    if (e->device < 0) return (int)hipErrorNoDevice;
    hipError_t rc = hipSetDevice(e->device);
    HostCtx *H = nullptr;
    if (rc == hipSuccess) rc = HostCtxFor(e, &H);
    if (rc == hipSuccess) {
        const size_t nn = std::max<uint32_t>(n, 1);
        const l7g_host_seg seg{H->pin_in + HostArenaOff(n), arena_len, arena_len, 1};
        const HostIn in{(const uint64_t *)H->pin_in, (const uint32_t *)(H->pin_in + nn * 8),
                        (const uint32_t *)(H->pin_in + nn * 12), nn, &seg, 1};
        rc = HostRun(e, H, n, arena_len, in, verdict, rule, consumed, try_service);
    }
    return (int)rc;
}

int l7g_host_run(l7g_engine *e, uint32_t n, uint64_t arena_len, uint8_t *verdict, int32_t *rule, uint32_t *consumed) {
    return HostRunStaged(e, n, arena_len, verdict, rule, consumed, true);
}
int l7g_host_run_pinned(l7g_engine *e, uint32_t n, const uint64_t *off, size_t stride, const l7g_host_seg *seg,
                        int nseg, uint8_t *verdict, int32_t *rule, uint32_t *consumed) {
    if (e->device < 0) return (int)hipErrorNoDevice;
    hipError_t rc = hipSetDevice(e->device);
    HostCtx *H = nullptr;
    uint64_t arena_len = 0;
    for (int k = 0; k < nseg; k++) arena_len += seg[k].width * seg[k].rows;
    const uint32_t st = (uint32_t)std::max<size_t>(stride, n);
    if (rc == hipSuccess) rc = HostCtxFor(e, &H);
    // device staging for `st` entries' arrays and the arena, pinned outputs for n
    if (rc == hipSuccess) rc = HostGrow(H, st, arena_len);
    if (rc == hipSuccess) {
        const uint8_t *b = (const uint8_t *)off;
        const HostIn in{off, (const uint32_t *)(b + stride * 8), (const uint32_t *)(b + stride * 12), stride, seg, nseg};
        rc = HostRun(e, H, n, arena_len, in, verdict, rule, consumed);
    }
    return (int)rc;
}

int l7g_host_reserve(l7g_engine *e, uint32_t n, uint64_t arena_len) {
    if (e->device < 0) return (int)hipErrorNoDevice;
    hipError_t rc = hipSetDevice(e->device);
    HostCtx *H = nullptr;
    if (rc == hipSuccess) rc = HostCtxFor(e, &H);
    if (rc == hipSuccess) rc = HostGrow(H, n, arena_len);
    return (int)rc;
}

int l7g_engine_has_device(const l7g_engine *e) { return e && e->device >= 0 ? 1 : 0; }

extern "C" {
int l7g_service_enable(l7g_engine *e, int on) {
    if (!e) return 0;
    std::lock_guard<std::mutex> g(e->mu);
    const int was = e->svc_on ? 1 : 0;
    e->svc_on = on != 0;
    if (!e->svc_on && e->device >= 0) StopServices(e);
    return was;
}
void l7g_service_stats(l7g_engine *e, uint64_t out[4]) {
    for (int k = 0; k < 2; k++) {
        std::lock_guard<std::mutex> g(e->svc[k].mu);
        out[2 * k] = e->svc[k].calls;
        out[2 * k + 1] = e->svc[k].launches;
    }
}
}  // extern "C"

void *l7g_pinned_alloc(size_t bytes) {
    void *p = nullptr;
    return hipHostMalloc(&p, bytes, hipHostMallocDefault) == hipSuccess ? p : nullptr;
}
void l7g_pinned_free(void *p) {
    if (p) hipHostFree(p);
}

extern "C" {

int l7g_classify_host(l7g_engine *e, const uint8_t *arena, uint64_t arena_len, const uint64_t *off, const uint32_t *len,
                      const uint32_t *conn, uint32_t n, uint8_t *verdict, int32_t *rule, uint32_t *consumed) {
    {  // a call a service takes goes from the caller's buffers straight into the service's staging
        const l7g_host_seg seg{arena, arena_len, arena_len, 1};
        const HostIn in{off, len, conn, 0, &seg, 1};
        hipError_t rc = hipSuccess;
        if (e->device >= 0 && ServiceTry(e, n, arena_len, in, verdict, rule, consumed, &rc)) return (int)rc;
    }
    uint8_t *pa;
    uint64_t *po;
    uint32_t *pl, *pc;
    int rc = l7g_host_stage(e, n, arena_len, &pa, &po, &pl, &pc);
    if (rc != 0) return rc;
    if (n) {
        memcpy(po, off, (size_t)n * 8);
        memcpy(pl, len, (size_t)n * 4);
        memcpy(pc, conn, (size_t)n * 4);
    }
    if (arena_len) memcpy(pa, arena, arena_len);
    return HostRunStaged(e, n, arena_len, verdict, rule, consumed, false);
}

int l7g_stats(l7g_engine *e, l7g_stats_t *out) {
    std::lock_guard<std::mutex> g(e->mu);
    memset(out, 0, sizeof *out);
    out->policies = (uint32_t)e->ps->policies.size();
    out->rules = (uint32_t)e->ps->nrules;
    const HttpImage &H = e->hc->image();
    out->http_rulesets = (uint32_t)H.rulesets.size();
    out->http_chunks = (uint32_t)H.chunks;
    out->http_dfas = (uint32_t)H.dfas;
    out->http_dfa_states = (uint32_t)H.dfa_states;
    const KafkaImage &K = e->kc->image();
    out->kafka_rulesets = (uint32_t)K.rulesets.size();
    out->kafka_rules = (uint32_t)K.rules.size();
    out->kafka_topics = (uint32_t)K.ntopics;
    out->table_bytes = e->blob_bytes;
    out->http_image_bytes = H.images.size();
    out->hot_ruleset = e->hot_ruleset;
    out->hot_image_bytes = e->hot_ruleset >= 0 ? H.rulesets[e->hot_ruleset].image_len : 0;
    const McImage &M = e->mc->image();
    out->mc_rulesets = (uint32_t)M.rulesets.size();
    out->mc_rules = (uint32_t)M.rules;
    out->mc_dfas = (uint32_t)M.dfas;
    out->mc_dfa_states = (uint32_t)M.dfa_states;
    out->http_nfas = (uint32_t)H.nfas;
    out->mc_nfas = (uint32_t)M.nfas;
    out->nfa_pool_bytes = H.nfa_pool.size() + M.nfa_pool.size() + e->r2->image().nfa_pool.size();
    out->r2d2_rulesets = (uint32_t)e->r2->image().rulesets.size();
    out->r2d2_rules = (uint32_t)e->r2->image().rules;
    return 0;
}

int l7g_flow_stats_enable(l7g_engine *e, int on) {
    std::lock_guard<std::mutex> g(e->mu);
    if (e->device < 0) return (int)hipErrorNoDevice;
    e->flow_stats = on != 0;
    return 0;
}

int l7g_flow_stats(l7g_engine *e, l7g_flow_stat_t *out, uint32_t cap, uint32_t *n, int reset) {
    std::lock_guard<std::mutex> g(e->mu);
    if (n) *n = 0;
    if (e->device < 0) return (int)hipErrorNoDevice;
    hipError_t rc = hipSetDevice(e->device);
    if (rc == hipSuccess) rc = WaitLastClassify(e);
    std::vector<uint64_t> h(e->flow_cap * 4, 0);
    if (rc == hipSuccess && e->flow_cap)
        rc = hipMemcpy(h.data(), e->d_flow, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost);
    if (rc != hipSuccess) return (int)rc;
    uint32_t k = 0;
    for (size_t i = 0; i < e->flow_cap && i < e->skey_list.size(); i++) {
        if (!(h[4 * i] | h[4 * i + 1] | h[4 * i + 2] | h[4 * i + 3])) continue;
        if (k < cap && out) {
            const auto &t = e->skey_list[i];
            out[k] = l7g_flow_stat_t{std::get<0>(t), std::get<1>(t), std::get<3>(t), (uint16_t)std::get<2>(t),
                                     h[4 * i], h[4 * i + 1], h[4 * i + 2], h[4 * i + 3]};
        }
        k++;
    }
    if (n) *n = k;
    // the reset completes before e->mu is released: the next call's flowstats
    // kernel (on a non-blocking stream) cannot overlap it
    if (reset && e->flow_cap) {
        rc = hipMemsetAsync(e->d_flow, 0, e->flow_cap * 4 * sizeof(uint64_t), nullptr);
        if (rc == hipSuccess) rc = hipStreamSynchronize(nullptr);
    }
    return (int)rc;
}

int l7g_profile_enable(l7g_engine *e, int on) {
    std::lock_guard<std::mutex> g(e->mu);
    if (e->device < 0) return (int)hipErrorNoDevice;
    hipError_t rc = hipSetDevice(e->device);
    for (hipEvent_t &ev : e->prof_ev)
        if (rc == hipSuccess && !ev) rc = hipEventCreate(&ev);
    if (rc == hipSuccess) e->profile = on != 0;
    return (int)rc;
}

int l7g_profile_last(l7g_engine *e, float out_ms[4]) {
    std::lock_guard<std::mutex> g(e->mu);
    for (int k = 0; k < 4; k++) out_ms[k] = 0.f;
    bool any = false;
    for (auto &kv : e->scr) any = any || kv.second->launched;
    if (!e->profile || !any) return (int)hipErrorNotReady;
    hipError_t rc = hipEventSynchronize(e->prof_ev[4]);
    for (int k = 0; k < 4 && rc == hipSuccess; k++)
        if (e->prof_ran[k]) rc = hipEventElapsedTime(&out_ms[k], e->prof_ev[k], e->prof_ev[k + 1]);
    return (int)rc;
}

int l7g_debug_phase_times(l7g_engine *e, uint64_t *out16, int reset) {
    if (!e || e->device < 0) return (int)hipErrorNoDevice;
    hipSetDevice(e->device);
    return (int)HttpPhaseTimes(out16, reset != 0);
}

int l7g_debug_frame_phase_times(l7g_engine *e, uint64_t *out8, int reset) {
    if (!e || e->device < 0) return (int)hipErrorNoDevice;
    hipSetDevice(e->device);
    return (int)FramePhaseTimes(out8, reset != 0);
}

int l7g_debug_kafka_phase_times(l7g_engine *e, uint64_t *out8, int reset) {
    if (!e || e->device < 0) return (int)hipErrorNoDevice;
    hipSetDevice(e->device);
    return (int)KafkaPhaseTimes(out8, reset != 0);
}

int l7g_debug_regex(const char *pat, size_t patlen, int anchored, const uint8_t *s, size_t slen, char *err,
                    size_t errlen) {
    std::string m;
    auto ast = re::Parse(std::string(pat, patlen), &m);
    if (!ast) { set_err(err, errlen, m); return -1; }
    re::DFA d;
    std::vector<re::Pattern> ps{{ast.get(), anchored != 0}};
    if (!re::BuildDFA(ps, 1 << 16, &d, &m)) { set_err(err, errlen, m); return -1; }
    auto acc = re::RunDFA(d, s, slen);
    return (int)(acc[0] & 1);
}

int l7g_debug_regex_nfa(const char *pat, size_t patlen, int anchored, const uint8_t *s, size_t slen, char *err,
                        size_t errlen) {
    std::string m;
    auto ast = re::Parse(std::string(pat, patlen), &m);
    if (!ast) { set_err(err, errlen, m); return -1; }
    re::BitNfa n;
    if (!re::BuildBitNfa({ast.get(), anchored != 0}, kNfaMaxPositions, &n, &m, kNfaMaxWords)) {
        set_err(err, errlen, m);
        return -1;
    }
    std::vector<uint8_t> pool;
    const uint64_t off = AppendDevNfa(n, &pool, &m);
    if (off == ~0ull) { set_err(err, errlen, m); return -1; }
    std::vector<uint64_t> scratch(2 * (size_t)n.W);  // (a large NFA's state sets)
    return nfa_run(pool.data(), off, s, (uint32_t)slen, scratch.data()) ? 1 : 0;
}

}  // extern "C"
