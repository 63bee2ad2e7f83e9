// Where the one-request synchronous call's time goes (GPU box, dev tool; not
// product code).  stdin: latency_main's input.  argv[1]: "spin" to set
// hipDeviceScheduleSpin before anything touches the device.
// Prints p50/p99 in us of:
//   empty     : an empty kernel launch + hipStreamSynchronize
//   empty_q   : the same, waiting by polling hipEventQuery
//   dev       : l7g_classify of one request already in device memory + sync
//   dev_q     : the same, polling an event
//   host      : l7g_classify_host of one request (the product's sync path)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/l7gpu.h"

using Clock = std::chrono::steady_clock;

__global__ void empty_kernel(int *p) {
    if (p && threadIdx.x == 1000000) p[0] = 1;
}

static std::string unhex(const std::string &h) {
    std::string o;
    for (size_t i = 0; i + 1 < h.size(); i += 2) o.push_back((char)std::stoi(h.substr(i, 2), nullptr, 16));
    return o;
}

template <class F>
static void timeit(const char *name, int iters, F f) {
    std::vector<double> t;
    for (int i = 0; i < iters + 50; i++) {
        const auto t0 = Clock::now();
        f();
        const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
        if (i >= 50) t.push_back(us);
    }
    std::sort(t.begin(), t.end());
    printf("%-10s p50 %7.2f  p90 %7.2f  p99 %7.2f us\n", name, t[t.size() / 2], t[t.size() * 9 / 10], t[t.size() * 99 / 100]);
}

int main(int argc, char **argv) {
    if (argc > 1 && !strcmp(argv[1], "spin")) (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
    if (argc > 1 && !strcmp(argv[1], "yield")) (void)hipSetDeviceFlags(hipDeviceScheduleYield);
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
    std::vector<std::string> http;
    while (std::getline(std::cin, line)) {
        if (line == "--") break;
        if (!line.empty()) http.push_back(unhex(line));
    }
    char err[512];
    l7g_engine *e = l7g_engine_create(0, err, sizeof err);
    if (!e) { std::cerr << err << "\n"; return 2; }
    if (l7g_policy_update(e, policy.data(), policy.size(), err, sizeof err) != 0) return 3;
    l7g_conn_t cs[2] = {hc, hc};
    cs[1].policy = -1;  // no policy: answered without a walk
    if (l7g_conns_set(e, cs, 2, err, sizeof err) != 0) return 3;
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t ev;
    (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    const int iters = 2000;
    timeit("empty", iters, [&] {
        empty_kernel<<<1, 64, 0, s>>>(nullptr);
        (void)hipStreamSynchronize(s);
    });
    timeit("empty_q", iters, [&] {
        empty_kernel<<<1, 64, 0, s>>>(nullptr);
        (void)hipEventRecord(ev, s);
        while (hipEventQuery(ev) == hipErrorNotReady) {
        }
    });
    // one request resident on the device
    const std::string &r0 = http[0];
    uint8_t *d;
    (void)hipMalloc(&d, 1 << 20);
    uint64_t *d_off = (uint64_t *)d;
    uint32_t *d_len = (uint32_t *)(d + 8), *d_conn = (uint32_t *)(d + 12);
    uint8_t *d_v = d + 16;
    int32_t *d_r = (int32_t *)(d + 32);
    uint32_t *d_c = (uint32_t *)(d + 48);
    uint8_t *d_a = d + 256;
    uint64_t off = 0;
    uint32_t len = (uint32_t)r0.size(), conn = 0;
    (void)hipMemcpy(d_off, &off, 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_len, &len, 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_conn, &conn, 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_a, r0.data(), r0.size(), hipMemcpyHostToDevice);
    timeit("dev", iters, [&] {
        l7g_classify(e, d_a, len, d_off, d_len, d_conn, 1, d_v, d_r, d_c, nullptr, s);
        (void)hipStreamSynchronize(s);
    });
    {
        const uint32_t one = 1;
        (void)hipMemcpy(d_conn, &one, 4, hipMemcpyHostToDevice);
        timeit("dev_nopol", iters, [&] {
            l7g_classify(e, d_a, len, d_off, d_len, d_conn, 1, d_v, d_r, d_c, nullptr, s);
            (void)hipStreamSynchronize(s);
        });
        (void)hipMemcpy(d_conn, &conn, 4, hipMemcpyHostToDevice);
        const char *shortreq = "GET / HTTP/1.1\r\nHost: a\r\n\r\n";
        const uint32_t sl = (uint32_t)strlen(shortreq);
        (void)hipMemcpy(d_len, &sl, 4, hipMemcpyHostToDevice);
        (void)hipMemcpy(d_a, shortreq, sl, hipMemcpyHostToDevice);
        timeit("dev_short", iters, [&] {
            l7g_classify(e, d_a, sl, d_off, d_len, d_conn, 1, d_v, d_r, d_c, nullptr, s);
            (void)hipStreamSynchronize(s);
        });
        (void)hipMemcpy(d_len, &len, 4, hipMemcpyHostToDevice);
        (void)hipMemcpy(d_a, r0.data(), r0.size(), hipMemcpyHostToDevice);
        printf("request 0: %u bytes\n", len);
    }
    timeit("dev_q", iters, [&] {
        l7g_classify(e, d_a, len, d_off, d_len, d_conn, 1, d_v, d_r, d_c, nullptr, s);
        (void)hipEventRecord(ev, s);
        while (hipEventQuery(ev) == hipErrorNotReady) {
        }
    });
    timeit("host", iters, [&] {
        uint8_t v;
        int32_t rr;
        uint32_t cc;
        l7g_classify_host(e, (const uint8_t *)r0.data(), r0.size(), &off, &len, &conn, 1, &v, &rr, &cc);
    });
    l7g_engine_destroy(e);
    return 0;
}
