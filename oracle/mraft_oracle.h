/*
 * mraft_oracle.h — CPU restatement of the reference's per-group Raft decision
 * logic (yusong-yan/MultiRaft src/raft), operating on the same struct-of-arrays
 * state and batch structs as libmraft_hip.so (include/mraft.h).
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU
 * baseline. The product path (multiraft_amd/) never links or calls it.
 *
 * Pinning: the reference is Go and there is no Go toolchain in this image, so
 * the reference cannot be run to produce outputs. The reference's own tests
 * hold no golden vectors for this path. The oracle is pinned by
 * (1) known-answer tests hand-derived from the cited Go lines (SURVEY.md §8c
 * K1-K14, tests/golden/), (2) a second independent restatement in pure Python
 * (oracle/pyoracle.py) compared on randomized states, and (3) the assertions of
 * the reference's 2B tests replayed through the deterministic simulator
 * (tests/test_sim2b.py). No reference-run outputs exist: parity is pinned by
 * hand-derived vectors and reference test assertions, not by reference runs.
 */
#ifndef MRAFT_ORACLE_H
#define MRAFT_ORACLE_H

#include <stdint.h>
#include "../include/mraft.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int32_t G, P, L;
  mraft_soa s; /* host arrays, owned by the caller */
} ora_engine;

/* Algorithmic word counting. When enabled, the tick marks every
 * state word the minimal exact algorithm must read / write in two bitmaps. */
int ora_count_enable(ora_engine *e);
/* terms_sorted of every replica from its log (what mraft_load_state does). */
void ora_compute_terms_sorted(ora_engine *e);
void ora_count_disable(void);
void ora_count_result(int64_t out_words[2]);
/* Lines of line_words words holding a counted word: {read, written}. */
void ora_count_result_lines(int32_t line_words, int64_t out_lines[2]);
/* The bitmaps (write = 0: read words) and each array's first bit; arrays in
 * the order term, voted, role, commit, applied, dummy, last, votes, log,
 * match, next, terms_sorted; ora_count_base(12) = total bits. */
const uint64_t *ora_count_bits(int32_t write);
int64_t ora_count_base(int32_t a);

int ora_gather_append_args(ora_engine *e, const int32_t *slots,
                           const int32_t *peers, int64_t n,
                           mraft_ae_args *out_args, int32_t *item_err);
int ora_handle_append_entries(ora_engine *e, const mraft_ae_args *args,
                              int64_t n, const int32_t *entry_terms,
                              int64_t n_entry_terms, mraft_ae_reply *replies,
                              int32_t *item_err);
int ora_process_append_replies(ora_engine *e, const mraft_ae_result *items,
                               int64_t n, const int64_t *seg_begin,
                               int64_t n_seg, int32_t *out_flags,
                               int32_t *item_err);
int ora_replicate_tick(ora_engine *e, const int32_t *leader_peer,
                       int32_t *group_flags);
/* Runs the tick on groups [g_begin, g_end) only (threaded CPU baseline). */
int ora_replicate_tick_range(ora_engine *e, const int32_t *leader_peer,
                             int32_t *group_flags, int32_t g_begin,
                             int32_t g_end);
/* Multi-threaded tick: groups split contiguously over nthreads (groups are
 * independent, like separate Raft instances under separate mutexes). */
int ora_replicate_tick_mt(ora_engine *e, const int32_t *leader_peer,
                          int32_t *group_flags, int32_t nthreads);

int ora_start(ora_engine *e, const int32_t *slots, const int32_t *counts,
              int64_t n, int32_t *out_index, int32_t *out_term,
              int32_t *out_is_leader, int32_t *item_err);
int ora_collect_apply(ora_engine *e, int32_t *out_from, int32_t *out_to, int32_t *out_snap_index,
                      int32_t *out_snap_term);

int ora_snapshot(ora_engine *e, const int32_t *slots, const int32_t *index, int64_t n,
                 int32_t *item_err);
int ora_gather_install_snapshot_args(ora_engine *e, const int32_t *slots, const int32_t *peers,
                                     int64_t n, mraft_is_args *out, int32_t *item_err);
int ora_handle_install_snapshot(ora_engine *e, const mraft_is_args *args, int64_t n,
                                mraft_is_reply *replies, int32_t *out_flags, int32_t *item_err);
int ora_process_install_snapshot_replies(ora_engine *e, const mraft_is_result *items, int64_t n,
                                         const int64_t *seg_begin, int64_t n_seg,
                                         int32_t *out_flags, int32_t *item_err);

int ora_start_election(ora_engine *e, const int32_t *slots, int64_t n,
                       mraft_rv_args *out_args, int32_t *item_err);
int ora_handle_request_vote(ora_engine *e, const mraft_rv_args *args,
                            int64_t n, mraft_rv_reply *replies,
                            int32_t *item_err);
int ora_process_vote_replies(ora_engine *e, const mraft_rv_result *items,
                             int64_t n, const int64_t *seg_begin,
                             int64_t n_seg, int32_t *out_flags,
                             int32_t *item_err);
int ora_election_rounds(ora_engine *e, const uint8_t *cand_mask, int32_t R,
                        int32_t *group_flags);
int ora_election_rounds_mt(ora_engine *e, const uint8_t *cand_mask, int32_t R,
                           int32_t *group_flags, int32_t nthreads);
int ora_export_group_status(ora_engine *e, const int32_t *leader_peer,
                            int32_t *commit, int32_t *term_leader);

int ora_collect_persist(ora_engine *e, int32_t *out_bits);
int ora_read_persistent(ora_engine *e, const int32_t *slots, int64_t n, mraft_persistent *out,
                        int32_t *out_terms, int64_t terms_cap);
int ora_restore(ora_engine *e, const mraft_persistent *in, int64_t n, const int32_t *terms,
                int64_t n_terms, int32_t *item_err);

/* Go-shaped restatement of the tick (mraft_goshape.c): int64 Raft structs,
 * 40-byte Entry slices, per-message entry copies. CPU baseline only. */
typedef struct go_cluster go_cluster;
go_cluster *goshape_build(int32_t G, int32_t P, int32_t L, const mraft_soa *s);
void goshape_store(const go_cluster *c, const mraft_soa *s);
void goshape_free(go_cluster *c);
void goshape_reset(go_cluster *c, const mraft_soa *s, int32_t nthreads);
int64_t goshape_tick(go_cluster *c, const int32_t *leader_peer, int32_t nthreads);

#ifdef __cplusplus
}
#endif
#endif
