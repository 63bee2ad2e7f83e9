// Latency of the drop-in paths (run by bench.py on the GPU box): the
// per-request cost a caller of the reference's interfaces sees.
//   sync     : one request per l7g_classify_host call (the Envoy adapter's
//              Allowed(), NetworkPolicyMap::Allowed's shape) -- H2D, launch, D2H
//   batcher  : AllowedAsync-style submissions through l7g_batcher from T
//              threads at a fixed offered rate; submit -> callback latency
//   ondata   : proxylib OnData (proxylib/proxylib.go:98-108) for one memcached
//              request per call on a registered connection
// stdin: line 1 the policy JSON; line 2 "<policy index> <port> <ingress>
// <src_id> <dst_id>" of the HTTP connection; then HTTP requests, one per line,
// hex.  Memcached line 2b: "mc <policy name> <port> <src_id>" and the memcached
// requests in hex after a line "--".  stdout: one JSON object.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/l7gpu.h"
#include "../../include/proxylib_abi.h"

using Clock = std::chrono::steady_clock;

static std::string unhex(const std::string &h) {
    std::string o;
    for (size_t i = 0; i + 1 < h.size(); i += 2) o.push_back((char)std::stoi(h.substr(i, 2), nullptr, 16));
    return o;
}

static std::string pct(std::vector<double> v) {
    if (v.empty()) return "null";
    std::sort(v.begin(), v.end());
    auto at = [&](double q) { return v[std::min(v.size() - 1, (size_t)(q * (double)(v.size() - 1) + 0.5))]; };
    std::ostringstream s;
    s << "{\"n\": " << v.size() << ", \"p50_us\": " << at(0.50) << ", \"p90_us\": " << at(0.90)
      << ", \"p99_us\": " << at(0.99) << ", \"max_us\": " << v.back() << "}";
    return s.str();
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    std::string policy, line;
    std::getline(std::cin, policy);
    std::getline(std::cin, line);
    l7g_conn_t hc{};
    {
        std::istringstream ss(line);
        int pol, ing;
        ss >> pol >> hc.port >> ing >> hc.src_id >> hc.dst_id;
        hc.policy = pol;
        hc.ingress = (uint8_t)ing;
        hc.proto = L7G_PROTO_HTTP;
    }
    std::getline(std::cin, line);
    std::string mc_policy_name;
    uint32_t mc_port = 0, mc_src = 0;
    {
        std::istringstream ss(line);
        std::string tag;
        ss >> tag >> mc_policy_name >> mc_port >> mc_src;
    }
    std::vector<std::string> http, mc;
    bool second = false;
    while (std::getline(std::cin, line)) {
        if (line == "--") { second = true; continue; }
        if (!line.empty()) (second ? mc : http).push_back(unhex(line));
    }
    char err[512];
    l7g_engine *e = l7g_engine_create(0, err, sizeof err);
    if (!e) { std::cerr << err << "\n"; return 2; }
    if (l7g_policy_update(e, policy.data(), policy.size(), err, sizeof err) != 0) { std::cerr << err << "\n"; return 3; }
    if (l7g_conns_set(e, &hc, 1, err, sizeof err) != 0) { std::cerr << err << "\n"; return 3; }

    // ---- sync: one request per call
    std::vector<double> sync;
    for (int i = 0; i < iters + 50; i++) {
        const std::string &r = http[(size_t)i % http.size()];
        uint64_t off = 0;
        uint32_t len = (uint32_t)r.size(), conn = 0, cons;
        uint8_t v;
        int32_t rule;
        const auto t0 = Clock::now();
        if (l7g_classify_host(e, (const uint8_t *)r.data(), r.size(), &off, &len, &conn, 1, &v, &rule, &cons) != 0) return 4;
        const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
        if (i >= 50) sync.push_back(us);
    }

    // ---- batcher: T threads submit at a fixed rate, flush at N requests or W us
    std::ostringstream bat;
    bat << "[";
    const struct { int threads; double rate_per_thread; uint32_t n, wait_us; } cfgs[] = {
        {8, 20000.0, 256, 100}, {8, 100000.0, 1024, 200}, {8, 600000.0, 4096, 200}};
    bool firstc = true;
    for (auto &cf : cfgs) {
        l7g_batcher *b = l7g_batcher_create(e, cf.n, cf.wait_us);
        // warm-up: the flusher thread's stream and staging are made on its first launch
        for (int i = 0; i < 64; i++)
            l7g_batcher_submit(b, (const uint8_t *)http[(size_t)i % http.size()].data(),
                               (uint32_t)http[(size_t)i % http.size()].size(), 0,
                               [](void *, uint8_t, int32_t, uint32_t) {}, nullptr);
        l7g_batcher_flush(b);
        uint64_t warm_req = 0, warm_l = 0;
        l7g_batcher_stats(b, &warm_req, &warm_l);
        // a quarter second of offered load per configuration (at least iters * 4 requests)
        const int per = std::max(iters * 4 / cf.threads, (int)(cf.rate_per_thread * 0.25));
        // per-request context and latency slot allocated up front: the callbacks
        // write one double and touch nothing shared (the harness itself must not
        // be the bottleneck: a malloc per request freed on the flusher thread was)
        std::vector<std::vector<double>> lat(cf.threads, std::vector<double>(per, -1.0));
        struct Ctx { Clock::time_point t0; double *out; };
        std::vector<std::vector<Ctx>> ctxs(cf.threads, std::vector<Ctx>(per));
        std::atomic<uint64_t> refused{0}, late_ns{0};
        std::vector<std::thread> ws;
        const auto start = Clock::now();
        for (int t = 0; t < cf.threads; t++)
            ws.emplace_back([&, t] {
                const auto gap = std::chrono::duration<double>(1.0 / cf.rate_per_thread);
                int64_t late = 0;  // how far behind its schedule the thread ended (generator-bound if large)
                uint64_t nref = 0;
                for (int i = 0; i < per; i++) {
                    const auto due = start + std::chrono::duration_cast<Clock::duration>(gap * (double)i);
                    if (Clock::now() < due) std::this_thread::sleep_until(due);
                    if (i == per - 1) late = (Clock::now() - due).count();
                    const std::string &r = http[(size_t)(i * cf.threads + t) % http.size()];
                    Ctx *c = &ctxs[t][i];
                    c->out = &lat[t][i];
                    c->t0 = Clock::now();
                    while (l7g_batcher_submit(b, (const uint8_t *)r.data(), (uint32_t)r.size(), 0,
                                              [](void *p, uint8_t, int32_t, uint32_t) {
                                                  auto *c = (Ctx *)p;
                                                  *c->out = std::chrono::duration<double, std::micro>(Clock::now() - c->t0).count();
                                              },
                                              c) == -2)
                        nref++, std::this_thread::yield();  // backpressure: both flushers busy, open slot full
                }
                late_ns += (uint64_t)std::max<int64_t>(late, 0);
                refused += nref;
            });
        for (auto &w : ws) w.join();
        const double submit_secs = std::chrono::duration<double>(Clock::now() - start).count();
        l7g_batcher_flush(b);
        const double secs = std::chrono::duration<double>(Clock::now() - start).count();
        uint64_t nreq = 0, nl = 0, tm[5];
        l7g_batcher_stats(b, &nreq, &nl);
        l7g_batcher_timing(b, tm);
        l7g_batcher_destroy(b);
        std::vector<double> all;
        for (auto &v : lat) all.insert(all.end(), v.begin(), v.end());
        nreq -= warm_req;
        nl -= warm_l;
        bat << (firstc ? "" : ", ") << "{\"threads\": " << cf.threads << ", \"offered_per_s\": "
            << cf.threads * cf.rate_per_thread << ", \"max_requests\": " << cf.n << ", \"max_wait_us\": " << cf.wait_us
            << ", \"achieved_per_s\": " << (double)nreq / secs << ", \"launches\": " << nl
            << ", \"submit_s\": " << submit_secs << ", \"total_s\": " << secs << ", \"refused_retries\": " << refused.load()
            << ", \"mean_end_lag_us\": " << (double)late_ns.load() / cf.threads / 1e3
            << ", \"flusher_ms\": {\"ready_wait\": " << tm[0] / 1e6 << ", \"device\": " << tm[1] / 1e6
            << ", \"callbacks\": " << tm[2] / 1e6 << ", \"order_wait\": " << tm[3] / 1e6 << ", \"max_batch\": " << tm[4] << "}"
            << ", \"latency\": " << pct(all) << "}";
        firstc = false;
    }
    bat << "]";
    l7g_engine_destroy(e);

    // ---- proxylib OnData, one memcached request per call
    std::vector<double> ond;
    {
        GoString kv[2] = {{"node-id", 7}, {"lat", 3}};
        GoSlice params{kv, 1, 1};
        const uint64_t mid = OpenModule(params, 0);
        if (!mid) return 5;
        std::string pj = policy;
        if (l7g_proxylib_policy_update(mid, pj.data(), pj.size(), err, sizeof err) != 0) { std::cerr << err << "\n"; return 6; }
        static uint8_t ibuf[2][1024];
        GoSlice orig{ibuf[0], 0, 1024}, reply{ibuf[1], 0, 1024};
        const std::string dst = "2.2.2.2:" + std::to_string(mc_port);
        GoString proto{"memcache", 8}, src_a{"1.1.1.1:1", 9}, dst_a{dst.data(), (GoInt)dst.size()},
            pname{mc_policy_name.data(), (GoInt)mc_policy_name.size()};
        if (OnNewConnection(mid, proto, 99, 1, mc_src, 7, src_a, dst_a, pname, &orig, &reply) != FILTER_OK) return 7;
        for (int i = 0; i < iters + 50; i++) {
            const std::string &r = mc[(size_t)i % mc.size()];
            GoSlice buf{(void *)r.data(), (GoInt)r.size(), (GoInt)r.size()};
            GoSlice data{&buf, 1, 1};
            int64_t opsmem[16];
            GoSlice ops{opsmem, 0, 8};
            orig.len = reply.len = 0;
            const auto t0 = Clock::now();
            const FilterResult fr = OnData(99, 0, 0, &data, &ops);
            const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
            if (fr != FILTER_OK) return 8;
            if (i >= 50) ond.push_back(us);
        }
        Close(99);
        CloseModule(mid);
    }
    std::cout << "{\"sync_classify_host\": " << pct(sync) << ", \"batcher\": " << bat.str()
              << ", \"proxylib_ondata_memcached\": " << pct(ond) << "}" << std::endl;
    return 0;
}
