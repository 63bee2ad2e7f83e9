// NPDS protobuf ingestion (product code): see npds_proto.cc.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>

#include "json.h"
#include "policy.h"

namespace l7 {

// A serialized envoy.api.v2.DiscoveryResponse whose resources are
// google.protobuf.Any{type.googleapis.com/cilium.NetworkPolicy} -> the policy
// tree the JSON loader reads ({"policies": [...]}, field names as in
// npds.proto).  false + *err on any wire-format error or foreign resource.
bool NpdsResponseToTree(const uint8_t *buf, size_t len, json::Value *root, std::string *version, std::string *err);
// NpdsResponseToTree + LoadPolicySetTree.
bool LoadPolicySetProto(const uint8_t *buf, size_t len, PolicySet *out, std::string *err);

}  // namespace l7
