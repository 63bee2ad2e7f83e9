// memcached command groups (product code): MemcacheOpCodeMap
// (proxylib/memcached/parser.go:214-474) — a policy "command" names a group,
// and the group admits a set of text command names and binary opcodes.
//
// Text command names are numbered so that the kernel can derive the framing
// class of text/parser.go:101-156 from the id range:
//   [kMcGet, kMcGats]        retrieval ("get*"/"gat*" prefixes; other
//                            get/gat-prefixed tokens frame as retrieval too
//                            but carry id kMcOther)
//   [kMcSet, kMcCas]         storage (tokens[4] = data block length)
//   [kMcDelete, kMcTouch]    one key (tokens[1])
//   [kMcSlabs, kMcWatch]     no key
//   kMcOther                 any other token: no group admits it
#pragma once
#include <cstdint>
#include <string>

namespace l7 {

enum McText : uint8_t {
    kMcGet, kMcGets, kMcGat, kMcGats,
    kMcSet, kMcAdd, kMcReplace, kMcAppend, kMcPrepend, kMcCas,
    kMcDelete, kMcIncr, kMcDecr, kMcTouch,
    kMcSlabs, kMcLru, kMcLruCrawler, kMcStats, kMcVersion, kMcMisbehave, kMcFlushAll, kMcCacheMemlimit, kMcQuit,
    kMcWatch,
    kMcOther,
    kMcTextIds  // 25
};

// Names of the text ids above (index = McText).
inline const char *McTextName(int id) {
    static const char *const kNames[kMcTextIds] = {
        "get", "gets", "gat", "gats", "set", "add", "replace", "append", "prepend", "cas",
        "delete", "incr", "decr", "touch", "slabs", "lru", "lru_crawler", "stats", "version", "misbehave",
        "flush_all", "cache_memlimit", "quit", "watch", ""};
    return kNames[id];
}

struct McGroup {
    const char *name;
    uint32_t text;      // bit i = McText i admitted
    uint8_t nops;
    uint8_t ops[15];    // binary opcodes admitted
};

#define MCB(x) (1u << (x))
inline const McGroup *McGroups(int *n) {
    static const McGroup kGroups[] = {
        {"add", MCB(kMcAdd), 2, {2, 18}},
        {"set", MCB(kMcSet), 2, {1, 17}},
        {"replace", MCB(kMcReplace), 2, {3, 19}},
        {"append", MCB(kMcAppend), 2, {14, 25}},
        {"prepend", MCB(kMcPrepend), 2, {15, 26}},
        {"cas", MCB(kMcCas), 0, {}},
        {"incr", MCB(kMcIncr), 2, {5, 21}},
        {"decr", MCB(kMcDecr), 2, {6, 22}},
        {"storage",
         MCB(kMcAdd) | MCB(kMcSet) | MCB(kMcReplace) | MCB(kMcAppend) | MCB(kMcPrepend) | MCB(kMcCas) | MCB(kMcIncr) |
             MCB(kMcDecr),
         12, {1, 2, 3, 5, 6, 17, 18, 19, 21, 22, 25, 26}},
        {"get", MCB(kMcGet) | MCB(kMcGets), 4, {0, 9, 12, 13}},
        {"delete", MCB(kMcDelete), 2, {4, 20}},
        {"touch", MCB(kMcTouch), 1, {28}},
        {"gat", MCB(kMcGat) | MCB(kMcGats), 2, {29, 30}},
        {"writeGroup",
         MCB(kMcAdd) | MCB(kMcSet) | MCB(kMcReplace) | MCB(kMcAppend) | MCB(kMcPrepend) | MCB(kMcCas) | MCB(kMcIncr) |
             MCB(kMcDecr) | MCB(kMcDelete) | MCB(kMcTouch),
         15, {1, 2, 3, 4, 5, 6, 17, 18, 19, 20, 21, 22, 25, 26, 28}},
        {"slabs", MCB(kMcSlabs), 0, {}},
        {"lru", MCB(kMcLru), 0, {}},
        {"lru_crawler", MCB(kMcLruCrawler), 0, {}},
        {"watch", MCB(kMcWatch), 0, {}},
        {"stats", MCB(kMcStats), 1, {16}},
        {"flush_all", MCB(kMcFlushAll), 2, {8, 24}},
        {"cache_memlimit", MCB(kMcCacheMemlimit), 0, {}},
        {"version", MCB(kMcVersion), 1, {11}},
        {"misbehave", MCB(kMcMisbehave), 0, {}},
        {"quit", MCB(kMcQuit), 2, {7, 23}},
        // binary-only groups
        {"noop", 0, 1, {10}},
        {"verbosity", 0, 1, {27}},
        {"sasl-list-mechs", 0, 1, {32}},
        {"sasl-auth", 0, 1, {33}},
        {"sasl-step", 0, 1, {34}},
        {"rget", 0, 1, {48}},
        {"rset", 0, 1, {49}},
        {"rsetq", 0, 1, {50}},
        {"rappend", 0, 1, {51}},
        {"rappendq", 0, 1, {52}},
        {"rprepend", 0, 1, {53}},
        {"rprependq", 0, 1, {54}},
        {"rdelete", 0, 1, {55}},
        {"rdeleteq", 0, 1, {56}},
        {"rincr", 0, 1, {57}},
        {"rincrq", 0, 1, {58}},
        {"rdecr", 0, 1, {59}},
        {"rdecrq", 0, 1, {60}},
        {"set-vbucket", 0, 1, {61}},
        {"get-vbucket", 0, 1, {62}},
        {"del-vbucket", 0, 1, {63}},
        {"tap-connect", 0, 1, {64}},
        {"tap-mutation", 0, 1, {65}},
        {"tap-delete", 0, 1, {66}},
        {"tap-flush", 0, 1, {67}},
        {"tap-opaque", 0, 1, {68}},
        {"tap-vbucket-set", 0, 1, {69}},
        {"tap-checkpoint-start", 0, 1, {70}},
        {"tap-checkpoint-end", 0, 1, {71}},
    };
    *n = (int)(sizeof kGroups / sizeof kGroups[0]);
    return kGroups;
}
#undef MCB

inline int McGroupIndex(const std::string &name) {
    int n;
    const McGroup *g = McGroups(&n);
    for (int i = 0; i < n; i++)
        if (name == g[i].name) return i;
    return -1;
}

}  // namespace l7
