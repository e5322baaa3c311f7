// mraft_internal.h — launchers shared between the kernel translation units and
// the C-ABI implementation (mraft_abi.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mraft.h"
#include "mraft_device.h"

namespace mraft {

void launch_replicate_tick(const Dev &s, const int32_t *lpeer, int32_t *gflags, int32_t *exp_commit,
                           int32_t *exp_term_leader, hipStream_t st);
// The light tick (MRAFT_TICK_LIGHT, mraft_tick.hip): k_tick_lite settles the
// steady-state groups eight per wave (32 per workgroup) and lists the others,
// per XCD: list region x = [x * lite_cap(G), ...), its count at cnt[32 x]
// (eight counters, one 128-B line each); the fallback launch (grid
// workgroups, grid-stride) runs them through the full tick, zeroes cnt_next
// (the next light tick's counters) and writes the total to the pinned host
// word hint. A list of G groups needs at most lite_list_words(G) words.
inline int lite_blocks(int G) { return (G + 31) / 32; }
inline int lite_cap(int G) { return (lite_blocks(G) + 7) / 8 * 32; }
inline int64_t lite_list_words(int G) { return 8 * (int64_t)lite_cap(G); }
constexpr int kLiteCntWords = 8 * 32;  // one light tick's counters
struct LiteBufs {
  int32_t *list;
  unsigned *cnt, *cnt_next;
  long long *hint;
  int grid;
};
// mraft_start_and_tick: per group, counts[g] entries to Start at replica
// leader_peer[g] (0: none), and Start's outputs per group.
struct StartIO {
  const int32_t *counts;
  int32_t *oi, *ot, *ol, *err;
};
void launch_replicate_tick_light(const Dev &s, const int32_t *lpeer, int32_t *gflags, int32_t *exp_commit,
                                 int32_t *exp_term_leader, const LiteBufs &lb, const StartIO *sio, hipStream_t st);
// Start at every group's leader replica (k_start per group; mraft_start_and_tick
// on the full tick's path).
void launch_start_groups(const Dev &s, const int32_t *lpeer, const StartIO &sio, hipStream_t st);
// The algorithmic count's buffer (mraft_replicate_tick_count): kCountStripes
// stripes of {reads, writes, active groups}, one 128-B line each, by
// workgroup (one counter word per buffer took every wave's atomic in turn:
// 1.8 ms per config-#3 count); the host sums the stripes.
constexpr int kCountStripes = 64;
constexpr int kCountWords = 16;
void launch_replicate_tick_count(const Dev &s, const int32_t *lpeer, unsigned long long *counts,
                                 hipStream_t st);

void launch_init_state(const Dev &s, hipStream_t st);
void launch_terms_sorted(const Dev &s, hipStream_t st);  // terms_sorted recomputed from the logs

// Duplicate-slot claims: item i (slot read at byte offset slot_off of a record
// of `stride` bytes; or, with seg_begin, the slot of segment i's first item)
// wins iff it is the lowest index addressing its slot in this call.
void launch_claim(const void *items, int64_t n, int stride, int slot_off, const int64_t *seg_begin,
                  int64_t gp, int peers, unsigned long long *claim, uint32_t epoch, int32_t *err,
                  hipStream_t st);

void launch_gather_args(const Dev &s, const int32_t *slots, const int32_t *peers, int64_t n,
                        mraft_ae_args *out, int32_t *err, hipStream_t st);
// AppendEntries by reference (mraft_handle_append_entries, entry_terms NULL):
// the claims and the set heads (sethd, one byte per item), then the main and
// the deferred launch, every count on the device (kernels: mraft_kernels.hip).
void launch_claim_ae(const mraft_ae_args *args, int64_t n, int64_t n_log, int L, int64_t gp, int ni,
                     unsigned long long *claim, uint32_t *srcmark, uint32_t epoch, int32_t *err, uint8_t *sethd,
                     unsigned long long *total, hipStream_t st);
// The by-reference handler's counter buffer (u64 words: [2] the published
// deferred count, [3] the fallback's finished workgroups, then per stripe —
// the main launch workgroup's XCD — its deferred items and its staged words,
// one 128-B line each) and its stripes: stripe x lists its deferred items at
// defer[x * n] (the list buffer holds kAeStripes * n) and stages at
// stage[x * capacity / kAeStripes].
#ifndef MRAFT_AE_STRIPES
#define MRAFT_AE_STRIPES 8
#endif
constexpr int kAeStripes = MRAFT_AE_STRIPES;
constexpr int kAeTotalWords = 16 + 2 * kAeStripes * 16;
// The deferred launch's buffers and grid (mraft_kernels.hip "deferred
// launch's fallback"): per item a 16-B record (writer, arrivals, run flag,
// cycle counter) and a reader count, nslot cycle buffers of L words, the last
// workgroup's L-word buffer, the pinned host word with the last deferred
// count, and the grid the host chose from it.
struct AeDeferBufs {
  int4 *fb;
  unsigned long long *kin;
  int32_t *cslot;
  int nslot;
  int32_t *cyc;
  long long *hint;
  int grid;
};
void launch_handle_ae_ref(const Dev &s, const mraft_ae_args *args, int64_t n, int ni, const unsigned long long *claim,
                          const uint32_t *srcmark, uint32_t epoch, int32_t *err, const uint8_t *sethd, int64_t *soff,
                          int64_t *defer, unsigned long long *total, int32_t *stage, int64_t stage_cap,
                          const AeDeferBufs &db, mraft_ae_reply *rep, mraft_ae_result *res, hipStream_t st);
// AppendEntries with the entries in a caller buffer (claims by launch_claim).
void launch_handle_ae_host(const Dev &s, const mraft_ae_args *args, int64_t n, const int32_t *ent, int64_t n_ent,
                           mraft_ae_reply *rep, int32_t *err, mraft_ae_result *res, hipStream_t st);
void launch_fold(const Dev &s, const mraft_ae_result *items, int64_t n, const int64_t *seg_begin,
                 int64_t n_seg, int64_t gp, unsigned long long *claim, uint32_t epoch, int32_t *seg_err,
                 int32_t *flags, int32_t *item_err, void *scan_buf, hipStream_t st);
size_t fold_scan_bytes(int64_t n, int64_t n_seg);  // scratch launch_fold needs (a1 scan list, long segments)
// Start: the slot claims (k_claim) and k_start, which checks them itself.
void launch_start(const Dev &s, const int32_t *slots, const int32_t *counts, int64_t n, int32_t *oi,
                  int32_t *ot, int32_t *ol, int32_t *err, const unsigned long long *claim, uint32_t epoch,
                  hipStream_t st);
void launch_collect_apply(const Dev &s, int32_t *from, int32_t *to, int32_t *snap_index, int32_t *snap_term,
                          hipStream_t st);
void launch_collect_apply_compact(const Dev &s, int32_t *scratch_bcnt, int64_t cap, int32_t *oslot,
                                  int32_t *osnap_index, int32_t *osnap_term, int32_t *ofrom, int32_t *oto,
                                  int64_t *total, hipStream_t st);
void launch_snapshot(const Dev &s, const int32_t *slots, const int32_t *index, int64_t n,
                     int32_t *err, hipStream_t st);
void launch_gather_is(const Dev &s, const int32_t *slots, const int32_t *peers, int64_t n,
                      mraft_is_args *out, int32_t *err, hipStream_t st);
void launch_handle_is(const Dev &s, const mraft_is_args *args, int64_t n, mraft_is_reply *rep,
                      int32_t *flags, int32_t *err, hipStream_t st);
void launch_process_is(const Dev &s, const mraft_is_result *items, int64_t n, const int64_t *seg_begin,
                       int64_t n_seg, int32_t *seg_err, int32_t *flags, int32_t *item_err,
                       hipStream_t st);
void launch_start_election(const Dev &s, const int32_t *slots, int64_t n, mraft_rv_args *out,
                           int32_t *err, hipStream_t st);
void launch_handle_rv(const Dev &s, const mraft_rv_args *args, int64_t n, mraft_rv_reply *rep,
                      int32_t *err, hipStream_t st);
void launch_tally(const Dev &s, const mraft_rv_result *items, int64_t n, const int64_t *seg_begin,
                  int64_t n_seg, int32_t *seg_err, int32_t *flags, int32_t *item_err,
                  hipStream_t st);
void launch_election_rounds(const Dev &s, const uint8_t *cand, int R, int32_t *gflags,
                            hipStream_t st);
void launch_collect_persist(const Dev &s, int32_t *out, hipStream_t st);
void launch_read_persistent_hdr(const Dev &s, const int32_t *slots, int64_t n,
                                mraft_persistent *out, hipStream_t st);
void launch_read_persistent_terms(const Dev &s, const mraft_persistent *hdr, int64_t n,
                                  int32_t *out, hipStream_t st);
void launch_restore(const Dev &s, const mraft_persistent *in, int64_t n, const int32_t *terms,
                    const int32_t *err, hipStream_t st);
void launch_export(const Dev &s, const int32_t *lpeer, int32_t *commit, int32_t *term_leader,
                   hipStream_t st);

}  // namespace mraft
