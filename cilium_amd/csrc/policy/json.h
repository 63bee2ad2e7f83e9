// Minimal JSON DOM used to ingest policies (product code).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace l7 {
namespace json {

struct Value {
    enum Type { Null, Bool, Num, Str, Arr, Obj } type = Null;
    bool b = false;
    double num = 0;
    int64_t inum = 0;
    std::string str;
    std::vector<Value> arr;
    std::vector<std::pair<std::string, Value>> obj;

    const Value *get(const char *key) const;
    bool isStr() const { return type == Str; }
    bool isArr() const { return type == Arr; }
    bool isObj() const { return type == Obj; }
};

bool Parse(const char *s, size_t n, Value *out, std::string *err);

}  // namespace json
}  // namespace l7
