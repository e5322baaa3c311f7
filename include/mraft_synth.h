/*
 * mraft_synth.h — seeded synthetic Multi-Raft workloads,
 * libmraft_synth.so (host-only C++, no HIP dependency).
 *
 * Deterministic per group: group g draws from splitmix64(seed, g), so any
 * contiguous group range [g_begin, g_end) reproduces exactly the groups of the
 * full-size state (used to shard one global workload across GPUs). Output
 * arrays are sized for the range: group g is written at local index
 * g - g_begin. All values < 2^31.
 */
#ifndef MRAFT_SYNTH_H
#define MRAFT_SYNTH_H

#include <stdint.h>
#include "mraft.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Default seeds: 0xC0FFEE + config id. */
#define MRAFT_SYNTH_SEED(config_id) (0xC0FFEEull + (uint64_t)(config_id))

/* Item classes of the mixed AppendEntries workload (config #3). */
enum {
  MRAFT_SYN_MATCH = 0,       /* 40%: prev inside the common prefix: merge/append */
  MRAFT_SYN_MISMATCH = 1,    /* 25%: prev inside the divergent tail: conflict scan */
  MRAFT_SYN_BEYOND = 2,      /* 15%: prev > follower lastIndex                    */
  MRAFT_SYN_STALE = 3,       /* 10%: follower currentTerm > leader term           */
  MRAFT_SYN_BELOW_DUMMY = 4, /*  5%: prev < follower dummyIndex (snapshotted)     */
  MRAFT_SYN_HEARTBEAT = 5    /*  5%: follower up to date, nEntries = 0            */
};

/* Replication-tick state (configs #2/#3/#4): leader = peer g % P with a
 * non-decreasing log of geometric runs (mean 16), 75% of groups with the last
 * run in the leader's current term (25% exercise the Figure-8 gate,
 * raft_append_entry.go:98); followers built per item class above. Every array
 * of `st` must be allocated for (g_end-g_begin) groups. leader_peer gets
 * (g_end-g_begin) entries; item_class (optional) gets (g_end-g_begin)*P
 * entries (-1 for the leader's own slot). nthreads <= 1: single thread. */
int mraft_synth_tick_state(uint64_t seed, int32_t G, int32_t P, int32_t L,
                           int32_t g_begin, int32_t g_end, const mraft_soa *st,
                           int32_t *leader_peer, int32_t *item_class,
                           int32_t nthreads);

/* Reply-fold batch (config #2): for each group's leader, P-1 replies in peer
 * order: 70% success (nEntries ~ U[0, last-prev]), 20% failure (ConflictIndex
 * ~ U[1, prev+1]), 10% higher term; 10% carry a stale prev / args term so the
 * gate of raft_append_entry.go:73-74 rejects them. out_items needs
 * G*(P-1) entries, seg_begin G+1. Returns the number of items. */
int64_t mraft_synth_fold_batch(uint64_t seed, int32_t G, int32_t P, int32_t L,
                               const mraft_soa *st, const int32_t *leader_peer,
                               mraft_ae_result *out_items, int64_t *seg_begin);

/* Election storm (config #5): state for groups [g_begin, g_end) plus
 * cand_mask[r*(g_end-g_begin) + g-g_begin] (r < rounds): 1-3 distinct peers
 * per group and round whose election timer fires. L >= 4. */
int mraft_synth_election_state(uint64_t seed, int32_t G, int32_t P, int32_t L,
                               int32_t g_begin, int32_t g_end, const mraft_soa *st,
                               uint8_t *cand_mask, int32_t rounds,
                               int32_t nthreads);

#ifdef __cplusplus
}
#endif
#endif
