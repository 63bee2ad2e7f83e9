// Library-internal entry points shared by the C-ABI (capi.cc) and the
// proxylib shim (proxylib/shim.cc); not part of include/l7gpu.h.
#pragma once
#include <cstddef>
#include <cstdint>

struct l7g_engine;

// One policy version, JSON (proto_form 0) or an NPDS DiscoveryResponse
// (proto_form 1).  proxylib != 0: the proxylib instance's update, which also
// NACKs what only proxylib's policymap rejects -- mismatching L7 types on one
// port (proxylib/proxylib/policymap.go:135-143, recovered as an update error
// in instance.go:168-176); the previous version then stays in force.
int l7g_policy_update_view(l7g_engine *e, const uint8_t *buf, size_t len, int proto_form, int proxylib, char *err,
                           size_t errlen);
