// Test driver for include/l7gpu_envoy.hpp (run by tests/test_gpu_envoy_adapter.py
// on the GPU box).  stdin: the policy JSON on the first line, then one request
// per line: policy_name \t ingress \t port \t remote_id \t name=value \t ...
// stdout: per request "<allowed> <rule>" (the batch form), then a second pass
// through the single-request Allowed() for the first 8 requests, then every
// request through AllowedAsync on an l7g_batcher (4 submitting threads,
// flush at 8 requests or 200 us), "<allowed> <rule>" in request order.
#include <atomic>
#include <iostream>
#include <sstream>
#include <thread>
#include <string>
#include <vector>

#include "../../include/l7gpu_envoy.hpp"

int main() {
    char err[512];
    l7g_engine *e = l7g_engine_create(0, err, sizeof err);
    if (!e) { std::cerr << err << "\n"; return 2; }
    std::string policy;
    std::getline(std::cin, policy);
    if (l7g_policy_update(e, policy.data(), policy.size(), err, sizeof err) != 0) { std::cerr << err << "\n"; return 3; }
    std::vector<l7gpu::Headers> hs;
    std::vector<l7gpu::AllowedRequest> rq;
    std::vector<std::string> names;
    std::string line;
    while (std::getline(std::cin, line)) {
        std::stringstream ss(line);
        std::string f;
        std::vector<std::string> fs;
        while (std::getline(ss, f, '\t')) fs.push_back(f);
        if (fs.size() < 4) continue;
        l7gpu::Headers h;
        for (size_t k = 4; k < fs.size(); k++) {
            const size_t eq = fs[k].find('=');
            h.emplace_back(fs[k].substr(0, eq), eq == std::string::npos ? "" : fs[k].substr(eq + 1));
        }
        hs.push_back(h);
        names.push_back(fs[0]);
        rq.push_back({fs[0], fs[1] == "1", (uint32_t)std::stoul(fs[2]), std::stoull(fs[3]), nullptr});
    }
    for (size_t i = 0; i < rq.size(); i++) rq[i].headers = &hs[i];
    l7gpu::NetworkPolicyMap m(e);
    std::vector<uint8_t> v;
    std::vector<int32_t> r;
    m.AllowedBatch(rq.data(), rq.size(), &v, &r);
    for (size_t i = 0; i < rq.size(); i++) std::cout << (int)v[i] << " " << r[i] << "\n";
    for (size_t i = 0; i < rq.size() && i < 8; i++)
        std::cout << (int)m.Allowed(rq[i].policy_name, rq[i].ingress, rq[i].port, rq[i].remote_id, hs[i]) << "\n";
    // asynchronous: four "worker threads" submit interleaved requests
    l7g_batcher *b = l7g_batcher_create(e, 8, 200);
    std::vector<int> av(rq.size(), -9), ar(rq.size(), -9);
    std::atomic<size_t> got{0};
    std::vector<std::thread> ws;
    for (int t = 0; t < 4; t++)
        ws.emplace_back([&, t] {
            for (size_t i = (size_t)t; i < rq.size(); i += 4)
                m.AllowedAsync(b, rq[i].policy_name, rq[i].ingress, rq[i].port, rq[i].remote_id, hs[i],
                               [&, i](bool ok, int32_t rule) { av[i] = ok; ar[i] = rule; got++; });
        });
    for (auto &w : ws) w.join();
    l7g_batcher_flush(b);
    uint64_t nreq = 0, nl = 0;
    l7g_batcher_stats(b, &nreq, &nl);
    l7g_batcher_destroy(b);
    if (got != rq.size()) { std::cerr << "async: " << got << " of " << rq.size() << " callbacks\n"; return 4; }
    for (size_t i = 0; i < rq.size(); i++) std::cout << av[i] << " " << ar[i] << "\n";
    std::cerr << "async: " << nreq << " requests in " << nl << " launches\n";
    l7g_engine_destroy(e);
    return 0;
}
