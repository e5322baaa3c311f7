// mraft_router.cpp — host side of the shard router: the
// shard -> replication-group assignment of the reference's shard controller
// (src/shardctrler/common.go:27-132) and key2shard
// (src/shardkv/client.go:22-29). The router reads the GetState words the
// engine exports / all-gathers (mraft_export_group_status) for the group a
// shard maps to. Deterministic, host-only C ABI (include/mraft.h).
#include <algorithm>
#include <map>
#include <vector>

#include "../../include/mraft.h"

namespace {

using G2S = std::map<int32_t, std::vector<int32_t>>;  // ordered: Go sorts the keys (:53-85)

// GetGIDWithMinimumShards, common.go:53-68: smallest gid among the least
// loaded, gid 0 (the invalid group) excluded.
int32_t gid_min(const G2S &g2s, int32_t nshards) {
  int32_t index = -1;
  size_t mn = (size_t)nshards + 1;
  for (const auto &kv : g2s)
    if (kv.first != 0 && kv.second.size() < mn) { index = kv.first; mn = kv.second.size(); }
  return index;
}

// GetGIDWithMaximumShards, common.go:70-85: smallest gid among the most loaded.
int32_t gid_max(const G2S &g2s) {
  int32_t index = -1;
  long long mx = -1;
  for (const auto &kv : g2s)
    if ((long long)kv.second.size() > mx) { index = kv.first; mx = (long long)kv.second.size(); }
  return index;
}

}  // namespace

extern "C" {

int mraft_key2shard(const char *key, int64_t len, int32_t nshards) {
  if (nshards <= 0) return MRAFT_E_INVAL;
  int shard = 0;
  if (key && len > 0) shard = (int)(unsigned char)key[0];  // int(key[0]) of a Go string byte
  return shard % nshards;
}

int mraft_realloc_gid(int32_t *shards, int32_t nshards, const int32_t *gids, int32_t ngroups) {
  if (!shards || nshards <= 0 || ngroups < 0 || (ngroups > 0 && !gids)) return MRAFT_E_INVAL;
  if (ngroups == 0) {                                                  // :88-93
    std::fill(shards, shards + nshards, 0);
    return MRAFT_OK;
  }
  G2S g2s;
  for (int32_t i = 0; i < ngroups; ++i) g2s[gids[i]];                  // :95-98
  for (int32_t s = 0; s < nshards; ++s) {                              // :99-104
    auto it = g2s.find(shards[s]);
    if (shards[s] != 0 && it != g2s.end()) it->second.push_back(s);
  }
  for (int32_t i = 0; i < nshards; ++i) {                              // leave, :106-113
    if (g2s.find(shards[i]) == g2s.end()) {
      const int32_t gid = gid_min(g2s, nshards);
      if (gid < 0) return MRAFT_E_INVAL;  // only gid 0 configured: Go would index g2s[-1]
      shards[i] = gid;
      g2s[gid].push_back(i);
    }
  }
  for (;;) {                                                           // join, :114-122
    const int32_t source = gid_max(g2s), target = gid_min(g2s, nshards);
    if (target < 0) return MRAFT_E_INVAL;
    if (source != 0 && (long long)g2s[source].size() - (long long)g2s[target].size() <= 1) break;
    if (g2s[source].empty()) return MRAFT_E_INVAL;  // gid 0 only, no progress possible
    g2s[target].push_back(g2s[source].front());
    g2s[source].erase(g2s[source].begin());
  }
  for (const auto &kv : g2s)                                           // :124-131
    for (int32_t s : kv.second) shards[s] = kv.first;
  return MRAFT_OK;
}

}  // extern "C"
