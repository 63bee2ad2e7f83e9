// Byte serialization of compiled rule tables (product code).
//
// A policy version's compiled state -- every compiler's device image and the
// cache that maps a connection's rule list to its rule set -- is written by
// the rank that compiled it (rank 0, the NPDS receiver:
// proxylib/proxylib/instance.go:168-219) and installed by the other ranks
// without compiling (l7g_tables_export / l7g_tables_import, cilium_amd/dist.py).
// Plain little-endian records; a reader that runs past the end or meets a
// size it cannot hold fails (ok = false), and the import is then refused.
#pragma once
#include <stdint.h>
#include <string.h>

#include <map>
#include <string>
#include <unordered_map>
#include <vector>

namespace l7 {

struct Ser {
    std::string out;
    void u64(uint64_t v) { out.append((const char *)&v, sizeof v); }
    void bytes(const void *p, size_t n) {
        u64(n);
        out.append((const char *)p, n);
    }
    void str(const std::string &s) { bytes(s.data(), s.size()); }
    template <class T>
    void vec(const std::vector<T> &v) {
        u64(v.size());
        if (!v.empty()) out.append((const char *)v.data(), v.size() * sizeof(T));
    }
    void cache(const std::map<std::pair<std::vector<int>, int>, int> &m) {
        u64(m.size());
        for (auto &kv : m) {
            vec(kv.first.first);
            u64((uint64_t)(int64_t)kv.first.second);
            u64((uint64_t)(int64_t)kv.second);
        }
    }
    void smap(const std::map<std::string, uint64_t> &m) {
        u64(m.size());
        for (auto &kv : m) { str(kv.first); u64(kv.second); }
    }
    void umap(const std::unordered_map<std::string, int> &m) {
        std::map<std::string, int> sorted(m.begin(), m.end());  // a deterministic byte image
        u64(sorted.size());
        for (auto &kv : sorted) { str(kv.first); u64((uint64_t)(int64_t)kv.second); }
    }
};

struct Des {
    const uint8_t *p, *end;
    bool ok = true;
    Des(const uint8_t *b, size_t n) : p(b), end(b + n) {}
    uint64_t u64() {
        uint64_t v = 0;
        if (!ok || (size_t)(end - p) < sizeof v) { ok = false; return 0; }
        memcpy(&v, p, sizeof v);
        p += sizeof v;
        return v;
    }
    std::string str() {
        const uint64_t n = u64();
        if (!ok || n > (uint64_t)(end - p)) { ok = false; return std::string(); }
        std::string s((const char *)p, (size_t)n);
        p += n;
        return s;
    }
    template <class T>
    void vec(std::vector<T> &v) {
        const uint64_t n = u64();
        if (!ok || n > (uint64_t)(end - p) / sizeof(T)) { ok = false; v.clear(); return; }
        v.resize((size_t)n);
        if (n) memcpy(v.data(), p, (size_t)n * sizeof(T));
        p += (size_t)n * sizeof(T);
    }
    void cache(std::map<std::pair<std::vector<int>, int>, int> &m) {
        m.clear();
        const uint64_t n = u64();
        for (uint64_t i = 0; i < n && ok; i++) {
            std::vector<int> k;
            vec(k);
            const int t = (int)(int64_t)u64();
            const int r = (int)(int64_t)u64();
            if (ok) m[{k, t}] = r;
        }
    }
    void smap(std::map<std::string, uint64_t> &m) {
        m.clear();
        const uint64_t n = u64();
        for (uint64_t i = 0; i < n && ok; i++) {
            std::string k = str();
            const uint64_t v = u64();
            if (ok) m[k] = v;
        }
    }
    void umap(std::unordered_map<std::string, int> &m) {
        m.clear();
        const uint64_t n = u64();
        for (uint64_t i = 0; i < n && ok; i++) {
            std::string k = str();
            const int v = (int)(int64_t)u64();
            if (ok) m[k] = v;
        }
    }
};

}  // namespace l7
