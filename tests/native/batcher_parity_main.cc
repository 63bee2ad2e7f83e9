// Batcher parity on the GPU (run by tests/test_gpu_batcher.py): every request
// submitted through l7g_batcher from T threads gets the verdict, rule and
// consumed count that one synchronous l7g_classify_host call over all of them
// gives.  argv: max_requests max_wait_us threads.  stdin: line 1 the policy
// JSON; line 2 the connection table, hex of l7g_conn_t[]; then one request per
// line, "<connection index> <hex>".  stdout: one JSON object.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/l7gpu.h"

static int nib(char x) { return x <= '9' ? x - '0' : (x | 0x20) - 'a' + 10; }
static std::string unhex(const std::string &h) {
    std::string o(h.size() / 2, '\0');
    for (size_t i = 0; i < o.size(); i++) o[i] = (char)(nib(h[2 * i]) << 4 | nib(h[2 * i + 1]));
    return o;
}

int main(int argc, char **argv) {
    if (argc < 4) return 1;
    const uint32_t max_n = (uint32_t)atoi(argv[1]), wait_us = (uint32_t)atoi(argv[2]);
    const int T = atoi(argv[3]);
    std::string policy, line;
    std::getline(std::cin, policy);
    std::getline(std::cin, line);
    const std::string cb = unhex(line);
    std::vector<l7g_conn_t> conns(cb.size() / sizeof(l7g_conn_t));
    memcpy(conns.data(), cb.data(), conns.size() * sizeof(l7g_conn_t));
    std::vector<std::string> reqs;
    std::vector<uint32_t> cid;
    while (std::getline(std::cin, line)) {
        const size_t sp = line.find(' ');
        if (sp == std::string::npos) continue;
        cid.push_back((uint32_t)std::stoul(line.substr(0, sp)));
        reqs.push_back(unhex(line.substr(sp + 1)));
    }
    const uint32_t n = (uint32_t)reqs.size();
    char err[512];
    l7g_engine *e = l7g_engine_create(0, err, sizeof err);
    if (!e) { std::cerr << err << "\n"; return 2; }
    if (l7g_policy_update(e, policy.data(), policy.size(), err, sizeof err) != 0) { std::cerr << err << "\n"; return 3; }
    if (l7g_conns_set(e, conns.data(), (uint32_t)conns.size(), err, sizeof err) != 0) { std::cerr << err << "\n"; return 3; }
    // the synchronous answer
    std::string arena;
    std::vector<uint64_t> off(n);
    std::vector<uint32_t> len(n);
    for (uint32_t i = 0; i < n; i++) {
        off[i] = arena.size();
        len[i] = (uint32_t)reqs[i].size();
        arena += reqs[i];
    }
    std::vector<uint8_t> v(n);
    std::vector<int32_t> r(n);
    std::vector<uint32_t> c(n);
    if (l7g_classify_host(e, (const uint8_t *)arena.data(), arena.size(), off.data(), len.data(), cid.data(), n, v.data(),
                          r.data(), c.data()) != 0)
        return 4;
    // the batcher's: T threads submit interleaved requests flat out
    struct Out { uint8_t v; int32_t r; uint32_t c; std::atomic<int> calls; };
    std::vector<Out> got(n);
    for (auto &o : got) o.calls = 0;
    l7g_batcher *b = l7g_batcher_create(e, max_n, wait_us);
    if (!b) return 5;
    std::atomic<uint64_t> refused{0};
    std::vector<std::thread> ws;
    for (int t = 0; t < T; t++)
        ws.emplace_back([&, t] {
            for (uint32_t i = (uint32_t)t; i < n; i += (uint32_t)T) {
                while (l7g_batcher_submit(b, (const uint8_t *)reqs[i].data(), (uint32_t)reqs[i].size(), cid[i],
                                          [](void *p, uint8_t vv, int32_t rr, uint32_t cc) {
                                              auto *o = (Out *)p;
                                              o->v = vv;
                                              o->r = rr;
                                              o->c = cc;
                                              o->calls++;
                                          },
                                          &got[i]) == -2)
                    refused++, std::this_thread::yield();
            }
        });
    for (auto &w : ws) w.join();
    l7g_batcher_flush(b);
    uint64_t nreq = 0, nl = 0, tm[5];
    l7g_batcher_stats(b, &nreq, &nl);
    l7g_batcher_timing(b, tm);
    l7g_batcher_destroy(b);
    uint32_t bad = 0, twice = 0;
    long first_bad = -1;
    for (uint32_t i = 0; i < n; i++) {
        if (got[i].calls != 1) twice++;
        if (got[i].v != v[i] || got[i].r != r[i] || got[i].c != c[i]) {
            if (first_bad < 0) first_bad = i;
            bad++;
        }
    }
    uint32_t nallow = 0;
    for (uint32_t i = 0; i < n; i++) nallow += v[i] == L7G_ALLOW;
    printf("{\"n\": %u, \"mismatches\": %u, \"calls_not_once\": %u, \"first_bad\": %ld, \"allowed\": %u, "
           "\"requests\": %llu, \"launches\": %llu, \"max_batch\": %llu, \"refused_retries\": %llu}\n",
           n, bad, twice, first_bad, nallow, (unsigned long long)nreq, (unsigned long long)nl,
           (unsigned long long)tm[4], (unsigned long long)refused.load());
    l7g_engine_destroy(e);
    return 0;
}
