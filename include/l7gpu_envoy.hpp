// l7gpu_envoy.hpp -- C++ adapter with the shape of Envoy's
// NetworkPolicyMap::Allowed (envoy/cilium_network_policy.h:223-237) over the
// batch C-ABI (l7gpu.h).  Header-only; links against libl7gpu.so.
//
// Envoy's cilium.l7policy filter (envoy/cilium_l7policy.cc:127-182) asks, per
// request, Allowed(policy_name, ingress, port, remote_id, headers).  The
// adapter keeps that call and adds the batched form the device wants:
//   * each distinct (policy, direction, port, remote identity) becomes one
//     registered connection of the engine (l7g_conn_update), resolved once;
//   * a request's decoded headers (:method, :path, :authority and the regular
//     headers, as Envoy's HeaderMap holds them) are written back as an
//     HTTP/1.1 request head, which the device frames and classifies -- the
//     same bytes Envoy's codec parsed them from;
//   * AllowedBatch classifies any number of requests in one l7g_classify_host;
//   * AllowedAsync queues one request on an l7g_batcher and calls back with
//     the verdict once the batcher's launch (shared with every other
//     worker's requests) completes: decodeHeaders returns StopIteration and
//     the callback resumes the stream (continueDecoding) or sends the 403.
// Remote identity: the source on ingress, the destination on egress
// (cilium_l7policy.cc:144-150), which the engine applies to the registered
// connection's src_id / dst_id.
#pragma once
#include <cstdint>
#include <functional>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

#include "l7gpu.h"

namespace l7gpu {

using Headers = std::vector<std::pair<std::string, std::string>>;

struct AllowedRequest {
    std::string policy_name;
    bool ingress;
    uint32_t port;
    uint64_t remote_id;
    const Headers *headers;
};

class NetworkPolicyMap {
public:
    explicit NetworkPolicyMap(l7g_engine *e) : e_(e) {}

    // cilium_network_policy.h:223-237
    bool Allowed(const std::string &policy_name, bool ingress, uint32_t port, uint64_t remote_id,
                 const Headers &headers) {
        std::vector<uint8_t> v;
        AllowedRequest r{policy_name, ingress, port, remote_id, &headers};
        AllowedBatch(&r, 1, &v, nullptr);
        return v[0] != 0;
    }

    // verdicts[i] = 1 allowed, 0 denied; rules (may be null) = matched global rule id or -1
    void AllowedBatch(const AllowedRequest *reqs, size_t n, std::vector<uint8_t> *verdicts,
                      std::vector<int32_t> *rules) {
        std::lock_guard<std::mutex> g(mu_);
        std::vector<uint8_t> arena;
        std::vector<uint64_t> off(n);
        std::vector<uint32_t> len(n), conn(n);
        for (size_t i = 0; i < n; i++) {
            conn[i] = Slot(reqs[i]);
            off[i] = arena.size();
            Head(*reqs[i].headers, &arena);
            len[i] = (uint32_t)(arena.size() - off[i]);
        }
        std::vector<uint8_t> v(n);
        std::vector<int32_t> r(n);
        std::vector<uint32_t> c(n);
        if (n && l7g_classify_host(e_, arena.data(), arena.size(), off.data(), len.data(), conn.data(), (uint32_t)n,
                                   v.data(), r.data(), c.data()) != 0)
            throw std::runtime_error("l7g_classify_host failed");
        verdicts->assign(n, 0);
        for (size_t i = 0; i < n; i++) (*verdicts)[i] = v[i] == L7G_ALLOW;
        if (rules) *rules = r;
    }

    // Asynchronous form: done(allowed, rule) runs on the batcher's flusher
    // thread once the request's launch has completed.
    void AllowedAsync(l7g_batcher *b, const std::string &policy_name, bool ingress, uint32_t port,
                      uint64_t remote_id, const Headers &headers, std::function<void(bool, int32_t)> done) {
        std::vector<uint8_t> head;
        Head(headers, &head);
        uint32_t slot;
        {
            std::lock_guard<std::mutex> g(mu_);
            slot = Slot(AllowedRequest{policy_name, ingress, port, remote_id, &headers});
        }
        auto *cb = new std::function<void(bool, int32_t)>(std::move(done));
        if (l7g_batcher_submit(b, head.data(), (uint32_t)head.size(), slot, &Trampoline, cb) != 0) {
            delete cb;
            throw std::runtime_error("l7g_batcher_submit: batcher is shutting down");
        }
    }

    // A policy update may renumber policies: forget the resolved connections.
    void PolicyUpdated() {
        std::lock_guard<std::mutex> g(mu_);
        slots_.clear();
    }

private:
    l7g_engine *e_;
    std::mutex mu_;
    std::map<std::tuple<std::string, bool, uint32_t, uint64_t>, uint32_t> slots_;

    static void Trampoline(void *ctx, uint8_t verdict, int32_t rule, uint32_t) {
        auto *cb = (std::function<void(bool, int32_t)> *)ctx;
        (*cb)(verdict == L7G_ALLOW, verdict == L7G_ALLOW ? rule : -1);
        delete cb;
    }

    uint32_t Slot(const AllowedRequest &q) {
        auto key = std::make_tuple(q.policy_name, q.ingress, q.port, q.remote_id);
        auto it = slots_.find(key);
        if (it != slots_.end()) return it->second;
        l7g_conn_t a{};
        a.policy = l7g_policy_index(e_, q.policy_name.data(), q.policy_name.size());
        a.port = q.port;
        a.ingress = q.ingress ? 1 : 0;
        a.proto = L7G_PROTO_HTTP;
        a.src_id = q.ingress ? (uint32_t)q.remote_id : 0;
        a.dst_id = q.ingress ? 0 : (uint32_t)q.remote_id;
        const uint32_t slot = (uint32_t)slots_.size();
        char err[256];
        if (l7g_conn_update(e_, slot, &a, err, sizeof err) != 0) throw std::runtime_error(err);
        slots_.emplace(key, slot);
        return slot;
    }

    // The request head Envoy's HTTP/1 codec decoded these headers from.
    static void Head(const Headers &h, std::vector<uint8_t> *out) {
        std::string method, path, authority, rest;
        for (auto &kv : h) {
            if (kv.first == ":method") method = kv.second;
            else if (kv.first == ":path") path = kv.second;
            else if (kv.first == ":authority") authority = kv.second;
            else if (!kv.first.empty() && kv.first[0] != ':') rest += kv.first + ": " + kv.second + "\r\n";
        }
        std::string s = method + " " + path + " HTTP/1.1\r\n";
        if (!authority.empty()) s += "Host: " + authority + "\r\n";
        s += rest + "\r\n";
        out->insert(out->end(), s.begin(), s.end());
    }
};

}  // namespace l7gpu
