#include "kafka_compile.h"

#include <algorithm>
#include <cstring>

namespace l7 {

uint32_t KafkaStrHash(const uint8_t *s, size_t n) {
    uint32_t h = kWHashSeed;
    for (size_t i = 0; i < n; i += 4) {
        uint32_t w = 0;
        for (size_t k = 0; k < 4 && i + k < n; k++) w |= (uint32_t)s[i + k] << (8 * k);
        h = l7_whash_step(h, w);
    }
    return l7_whash_final(h, (uint32_t)n);
}

namespace {
void BuildHash(const std::unordered_map<std::string, int> &ids, std::vector<uint8_t> &strings,
               std::vector<DevStrSlot> &table, uint32_t &mask) {
    size_t cap = 16;
    while (cap < ids.size() * 2 + 2) cap <<= 1;
    table.assign(cap, DevStrSlot{});
    mask = (uint32_t)(cap - 1);
    // deterministic insertion order: by id
    std::vector<const std::string *> byid(ids.size());
    for (auto &kv : ids) byid[kv.second] = &kv.first;
    for (size_t id = 0; id < byid.size(); id++) {
        const std::string &s = *byid[id];
        uint32_t h = KafkaStrHash((const uint8_t *)s.data(), s.size());
        uint32_t slot = h & mask;
        while (table[slot].used) slot = (slot + 1) & mask;
        DevStrSlot &d = table[slot];
        d.hash = h;
        d.len = (uint16_t)s.size();
        d.used = 1;
        d.id = (int32_t)id;
        memcpy(d.pre, s.data(), std::min<size_t>(s.size(), sizeof d.pre));
        strings.resize((strings.size() + 3) & ~(size_t)3, 0);  // 4-byte aligned, zero-padded
        d.str_off = (uint32_t)strings.size();
        strings.insert(strings.end(), s.begin(), s.end());
        strings.resize((strings.size() + 3) & ~(size_t)3, 0);
    }
}
}  // namespace

KafkaCompiler::KafkaCompiler(const PolicySet *ps) : ps_(ps) {
    for (auto &np : ps->policies)
        for (auto *dir : {&np.ingress, &np.egress})
            for (auto &pp : *dir)
                for (auto &r : pp.rules)
                    for (auto &k : r.kafka) {
                        if (!k.topic.empty()) topic_id_.emplace(k.topic, (int)topic_id_.size());
                        if (!k.client.empty()) client_id_.emplace(k.client, (int)client_id_.size());
                    }
    BuildHash(topic_id_, img_.strings, img_.topic_hash, img_.topic_mask);
    BuildHash(client_id_, img_.strings, img_.client_hash, img_.client_mask);
    img_.ntopics = topic_id_.size();
}

int KafkaCompiler::RulesetFor(int policy, bool ingress, uint32_t port, uint64_t src_id, bool proxylib,
                              std::string *err) {
    (void)err;
    std::vector<const KafkaRule *> rules;
    bool any = false;
    static const KafkaRule kWildcard;  // {} matches every request (id -1)
    if (policy >= 0 && policy < (int)ps_->policies.size()) {
        const PortPolicy *ex, *wc;
        ps_->policies[policy].Lookup(ingress, port, &ex, &wc);
        for (const PortPolicy *pp : {ex, wc}) {
            if (!pp) continue;
            if (proxylib) {
                // proxylib "kafka" parser: the installed entries of PortNetworkPolicies
                // (policymap.go:150-236); a port without L7 rules, or a group whose L7
                // set is empty, lets everything through; the groups' Kafka rules
                // are evaluated together as one MatchesRule list (the
                // GetRelevantRules view of pkg/policy/l4.go:118-141)
                if (!pp->px_installed) continue;
                if (!pp->px_have_l7 || pp->rules.empty()) { rules.push_back(&kWildcard); any = true; continue; }
                for (auto &r : pp->rules) {
                    if (!r.RemoteOk(src_id)) continue;
                    if (r.NumL7() == 0) { rules.push_back(&kWildcard); any = true; }
                    else if (r.type == PortRule::Kafka) { for (auto &k : r.kafka) rules.push_back(&k); any = true; }
                }
                continue;
            }
            for (auto &r : pp->rules) {
                if (!r.RemoteOk(src_id)) continue;
                if (r.type == PortRule::Kafka) { for (auto &k : r.kafka) rules.push_back(&k); any = true; }
                else if (r.type == PortRule::None) { rules.push_back(&kWildcard); any = true; }
            }
        }
    }
    std::vector<int> key;
    for (auto *r : rules) key.push_back(r == &kWildcard ? -1 : r->id);
    auto ck = std::make_pair(key, (int)any);
    auto it = cache_.find(ck);
    if (it != cache_.end()) return it->second;
    int id = Compile(rules, any);
    cache_.emplace(ck, id);
    return id;
}

static constexpr size_t kDenseTopicBudget = size_t(64) << 20;  // u32 entries in index[] (256 MiB)

int KafkaCompiler::Compile(const std::vector<const KafkaRule *> &rules, bool any) {
    compiled++;
    KafkaImage &I = img_;
    DevKafkaRuleset rs{};
    rs.any = any ? 1 : 0;
    rs.rule_first = (uint32_t)I.rules.size();
    rs.nrules = (uint32_t)rules.size();
    std::map<int, std::vector<uint32_t>> by_topic;
    std::vector<uint32_t> topicless;
    std::vector<std::vector<uint32_t>> bykey(65);
    for (uint32_t pos = 0; pos < rules.size(); pos++) {
        const KafkaRule &k = *rules[pos];
        DevKafkaRule d{};
        d.keymask = k.keymask;
        d.any_key = k.any_key ? 1 : 0;
        d.has_version = k.has_version ? 1 : 0;
        d.version = k.version;
        d.has_topic = k.topic.empty() ? 0 : 1;
        d.client = k.client.empty() ? -1 : client_id_.at(k.client);
        d.gid = k.id;
        I.rules.push_back(d);
        if (k.topic.empty()) topicless.push_back(pos);
        else by_topic[topic_id_.at(k.topic)].push_back(pos);
        for (int key = 0; key < 64; key++)
            if (k.any_key || ((k.keymask >> key) & 1)) bykey[key].push_back(pos);
        if (k.any_key) bykey[64].push_back(pos);
    }
    rs.topicless_off = (uint32_t)I.index.size();
    rs.ntopicless = (uint32_t)topicless.size();
    I.index.insert(I.index.end(), topicless.begin(), topicless.end());
    // per-topic lists, then the sorted (topic, off, cnt) directory
    std::vector<uint32_t> dir;
    for (auto &kv : by_topic) {
        dir.push_back((uint32_t)kv.first);
        dir.push_back((uint32_t)I.index.size());
        dir.push_back((uint32_t)kv.second.size());
        I.index.insert(I.index.end(), kv.second.begin(), kv.second.end());
    }
    rs.topics_off = (uint32_t)I.index.size();
    rs.ntopics = (uint32_t)by_topic.size();
    I.index.insert(I.index.end(), dir.begin(), dir.end());
    // Dense (off, cnt) per interned topic id: one lookup instead of a binary
    // search per request topic.  Bounded so many rule sets over many topics
    // keep to the sorted directory.
    // Each entry (DevKafkaTopicEnt, 48 B, 16-byte aligned) also carries the
    // list's first rule and its position, so the common case -- the first
    // rule decides -- is one table read after the topic's hash probe.
    rs.tdense_off = ~0u;
    constexpr size_t kEntU32 = sizeof(DevKafkaTopicEnt) / 4;
    if (!by_topic.empty() && I.index.size() + 3 + kEntU32 * I.ntopics <= kDenseTopicBudget) {
        I.index.resize((I.index.size() + 3) & ~(size_t)3, 0);
        rs.tdense_off = (uint32_t)I.index.size();
        I.index.resize(I.index.size() + kEntU32 * I.ntopics, 0);
        for (size_t t = 0; t < dir.size(); t += 3) {
            DevKafkaTopicEnt e{};
            e.off = dir[t + 1];
            e.cnt = dir[t + 2];
            e.p0 = I.index[e.off];
            e.r0 = I.rules[rs.rule_first + e.p0];
            memcpy(&I.index[rs.tdense_off + kEntU32 * dir[t]], &e, sizeof e);
        }
    }
    std::vector<uint32_t> keydir;
    for (auto &l : bykey) {
        keydir.push_back((uint32_t)I.index.size() + 0);  // patched below
        keydir.push_back((uint32_t)l.size());
    }
    for (size_t k = 0; k < bykey.size(); k++) {
        keydir[2 * k] = (uint32_t)I.index.size();
        I.index.insert(I.index.end(), bykey[k].begin(), bykey[k].end());
    }
    rs.bykey_off = (uint32_t)I.index.size();
    I.index.insert(I.index.end(), keydir.begin(), keydir.end());
    I.rulesets.push_back(rs);
    return (int)I.rulesets.size() - 1;
}

}  // namespace l7
