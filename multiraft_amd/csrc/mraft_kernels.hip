// mraft_kernels.hip — item-level gfx950 kernels behind the C ABI: the
// per-message entry points of include/mraft.h (a node receiving batches of
// AppendEntries / RequestVote / replies from the network), as
// opposed to the fused co-resident tick of mraft_tick.hip.
#include "mraft_device.h"
#include "mraft_internal.h"
#include "mraft_pass.h"

namespace mraft {

namespace {

constexpr int kBlock = 256;
// The main launch's deferred list and stage offsets are counted per stripe
// (the workgroup's XCD, blockIdx % 8), each counter on its own 128-B line of
// the counter buffer (mraft_abi.hip ae_total, kAeTotalWords u64): one
// same-address counter took an atomic round trip per deferred item and per
// staged item, serialised — 1.3 ms of a 2-cycle-heavy batch (r6_l7). Stripe x
// lists its items at defer[x * n ...] and stages at stage[x * cap / 8 ...].
constexpr int kStripes = kAeStripes;
static_assert(16 + 2 * kStripes * 16 == kAeTotalWords, "the counter buffer's layout (mraft_internal.h)");
constexpr int kStripeWords = 16;                            // 128 B
constexpr int kStripeDef = 16;                              // total[16 + 16 x]: deferred items of stripe x
constexpr int kStripeStg = kStripeDef + kStripes * kStripeWords;  // total[144 + 16 x]: its staged words
#ifndef MRAFT_MSG_BLOCK
#define MRAFT_MSG_BLOCK 64  // workgroup size of the message path's lane-per-item kernels (gather, claims; r4_v26: 64 pipelines -3 %)
#endif
// (a smaller workgroup finds a CU with room sooner while another queue's
// handler or tick holds most wave slots: shard pipelines)
constexpr int kMsgBlock = MRAFT_MSG_BLOCK;

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
// A pointer the wave holds in SGPRs where it is used (a per-lane address
// hoisted out of a loop as a VGPR pair is what the register allocator spills).
template <class T>
__device__ __forceinline__ T *uni_ptr(T *p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return (T *)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

inline int blocks_for(int64_t n, int per_block = kBlock) {
  int64_t b = (n + per_block - 1) / per_block;
  return (int)(b < 1 ? 1 : b);
}

// ---------------------------------------------------------------- Make
__global__ void k_init_state(Dev s) {
  const int64_t gp = (int64_t)s.G * s.P;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < gp;
       i += (int64_t)gridDim.x * blockDim.x) {
    // raft.go:53-68,79-80: Follower, term 0, votedFor -1, logs = [dummy{0,0}],
    // commitIndex = lastApplied = dummyIndex.
    s.term[i] = 0; s.voted[i] = -1; s.role[i] = kFollower; s.commit[i] = 0; s.applied[i] = 0;
    s.dummy[i] = 0; s.last[i] = 0; s.votes[i] = 0; s.head[i] = 0; s.hsnap[i] = 0;
    s.srt[i] = 1;  // [dummy] only: nothing after the dummy to be out of order
    if (s.pdirty) s.pdirty[i] = 0;
  }
}

// ---------------------------------------------------------------- claims
__global__ void k_claim(const char *__restrict__ items, int64_t n, int stride, int slot_off,
                        const int64_t *__restrict__ seg_begin, int64_t gp, int peers,
                        unsigned long long *__restrict__ claim, uint32_t epoch,
                        int32_t *__restrict__ err) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t rec = i;
  if (seg_begin) {
    if (seg_begin[i] >= seg_begin[i + 1]) { err[i] = 0; return; }
    rec = seg_begin[i];
  }
  const int32_t slot = *(const int32_t *)(items + rec * stride + slot_off);
  (void)peers;
  if (slot < 0 || slot >= gp) { err[i] = MRAFT_ITEM_BAD_SLOT; return; }
  err[i] = 0;
  atomicMax(&claim[slot], ((unsigned long long)epoch << 32) | (0xFFFFFFFFull - (uint64_t)i));
}

// The reply fold's claim (mraft_process_append_replies): k_claim over the
// segments, and the zeroing of the per-item outputs (items no segment covers
// keep flag 0, error 0) in the same launch; the duplicate check happens in
// k_fold itself (claim[slot] loads with the replica's state).
__global__ void k_claim_zero(const char *__restrict__ items, int64_t n, int stride, int slot_off,
                             const int64_t *__restrict__ seg_begin, int64_t gp,
                             unsigned long long *__restrict__ claim, uint32_t epoch,
                             int32_t *__restrict__ err, int64_t nz, int32_t *__restrict__ z0,
                             int32_t *__restrict__ z1, unsigned *__restrict__ zc, unsigned *__restrict__ zl) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i < nz) {
    z0[i] = 0;
    z1[i] = 0;
  }
  if (i == 0 && zc) *zc = 0;  // no a1 range pending for k_fold_tail's scans yet
  if (i == 0 && zl) *zl = 0;  // no long segment for k_fold_tail yet
  if (i >= n) return;
  int64_t rec = i;
  if (seg_begin) {
    if (seg_begin[i] >= seg_begin[i + 1]) { err[i] = 0; return; }
    rec = seg_begin[i];
  }
  const int32_t slot = *(const int32_t *)(items + rec * stride + slot_off);
  if (slot < 0 || slot >= gp) { err[i] = MRAFT_ITEM_BAD_SLOT; return; }
  err[i] = 0;
  atomicMax(&claim[slot], ((unsigned long long)epoch << 32) | (0xFFFFFFFFull - (uint64_t)i));
}

__global__ void k_claim_check(const char *__restrict__ items, int64_t n, int stride, int slot_off,
                              const int64_t *__restrict__ seg_begin,
                              const unsigned long long *__restrict__ claim, uint32_t epoch,
                              int32_t *__restrict__ err) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n || err[i]) return;
  int64_t rec = i;
  if (seg_begin) {
    if (seg_begin[i] >= seg_begin[i + 1]) return;
    rec = seg_begin[i];
  }
  const int32_t slot = *(const int32_t *)(items + rec * stride + slot_off);
  if (claim[slot] != (((unsigned long long)epoch << 32) | (0xFFFFFFFFull - (uint64_t)i)))
    err[i] = MRAFT_ITEM_DUP_SLOT;
}

// ---------------------------------------------------------------- a3
__global__ void k_gather_args(Dev s, const int32_t *__restrict__ slots,
                              const int32_t *__restrict__ peers, int64_t n,
                              mraft_ae_args *__restrict__ out, int32_t *__restrict__ err) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int P = s.P, L = s.L;
  const int64_t gp = (int64_t)s.G * P;
  mraft_ae_args a = {};
  int e = 0;
  const int slot = slots[i], peer = peers[i];
  if (slot < 0 || slot >= gp || peer < 0 || peer >= P || peer == slot % P) {
    e = MRAFT_ITEM_BAD_SLOT;
  } else {
    // every word that depends only on the slot in one round trip (the role
    // check does not gate the loads: one dependent round trip fewer)
    const int role = s.role[slot], dummy = s.dummy[slot], last = s.last[slot], head = s.head[slot];
    const int nxt = s.next[(int64_t)slot * P + peer], term = s.term[slot], commit = s.commit[slot];
    const int srt = s.srt[slot];
    const int prev = nxt - 1;                                          // :26
    if (role != kLeader) e = MRAFT_ITEM_BAD_STATE;                     // raft_append_entry.go:22-25
    else if (prev < dummy) e = MRAFT_ITEM_NEED_SNAPSHOT;               // :27
    else if (prev > last) e = MRAFT_ITEM_PREV_BEYOND_LAST;             // :41-43
    else {
      a.slot = (slot / P) * P + peer;
      a.leader_id = slot % P;
      a.term = term;
      a.prev_log_index = prev;
      a.prev_log_term = s.log[(int64_t)slot * L + ring(prev - dummy + head, L)];  // :49
      a.n_entries = last - prev;                                       // :50
      // prevLogTerm, entries: non-decreasing when the leader's terms after its
      // dummy are; prevLogTerm at the dummy itself is compared explicitly
      a.flags = (srt && (prev > dummy || prev == last ||
                         a.prev_log_term <= s.log[(int64_t)slot * L + ring(prev + 1 - dummy + head, L)]))
                    ? MRAFT_AE_ENTRIES_SORTED : 0;
      a.leader_commit = commit;                                        // :51
      a.entries_offset = (int64_t)slot * L + (prev + 1 - dummy);       // :54 (by reference: logical)
    }
  }
  out[i] = a;
  err[i] = e;
}

// ---------------------------------------------------------------- a4
// HandleAppendEntries (raft_append_entry.go:108-162, matchLog
// raft_log.go:92-96), message-level, fully on the device: the host enqueues
// three launches and returns (round 5; rounds 2-4 polled a pinned word for
// the batch plan before enqueuing the second half).
//
// Entries by reference into the engine's own log (entry_terms NULL):
// entries_offset = source slot * L + (Index - dummy) of the first entry, a
// logical position in that replica's ring. The reference copies args.Entries
// when it builds the message (appendOneRound, raft_append_entry.go:50-54),
// before any handler runs, so every item must see its source row as it was
// before the call, even when another item of the batch writes that row (two
// leaders of one group). Per item, from the claims of k_claim_ae (the lowest
// item addressed to a slot owns it; srcmark marks every row some item reads):
//   read   its source row is written by an item of this batch (claimed);
//   written  its own slot is some item's source row (srcmark).
// An item that is not `written` runs in the MAIN launch, reading its source in
// place (a row some item reads and another writes belongs to a `written`
// item, which is deferred: the row is pristine throughout the main launch).
// A `written` item is DEFERRED to a second launch,
// after every main item has read what it needs; if it is also `read`, its
// entries are staged (copied by the main launch, whose items never write the
// rows deferred items read) and the deferred launch reads the copy. Deferred
// items are independent given the copies and run in parallel. When the
// staged words exceed the stage capacity (mraft_set_stage_capacity), the
// deferred launch instead orders them itself on one wave: an item that reads a
// row runs before that row's writer (each item has at most one writer ahead of
// it, so the order is a forest of chains feeding cycles), and a cycle is
// broken by copying one member's entries to an L-word buffer first.
//
// Messages that read the same entries (same source row, same ring position of
// Index 0, same last Index: the P-1 messages one leader's gather makes for
// its followers, consecutive in the batch) form a *set*, up to NI messages,
// served by one wave with one streaming pass over the shared entries, as the
// fused tick serves a group (mraft_pass.h). k_claim_ae cuts the sets from the
// keys alone (a message whose run of same-entry predecessors is NI or longer is
// a set of its own) and writes each head's size; the main launch's wave v
// serves the sets whose heads lie in items [v*NI, (v+1)*NI) — one set per
// wave for a gathered batch — masking members that turn out to be
// duplicates, malformed or deferred.
struct AeKey {
  int64_t row;  // source slot (-1: no key, a set of its own)
  int base;     // ring position of the entries, relative: (offset mod L) - (prev + 1)
  int end;      // Index of the last entry
};

__device__ __forceinline__ bool ae_ref_ok(const mraft_ae_args &a, int64_t n_log, int L) {
  return !(a.n_entries < 0 || a.entries_offset < 0 || a.entries_offset + a.n_entries > n_log ||
           a.entries_offset % L + a.n_entries > L);
}

// The Index domain (include/mraft.h): the last entry's Index prev + n must
// leave room for nextIndex = Index + 1 in int32. Outside it the item is
// malformed (MRAFT_ITEM_BAD_SLOT), as in the oracle.
__device__ __forceinline__ bool ae_index_ok(const mraft_ae_args &a) {
  return (int64_t)a.prev_log_index + a.n_entries <= (int64_t)INT32_MAX - 1;
}

__device__ __forceinline__ unsigned long long claim_tag(uint32_t epoch, int64_t i) {
  return ((unsigned long long)epoch << 32) | (0xFFFFFFFFull - (uint64_t)i);
}

__device__ __forceinline__ AeKey ae_key(const mraft_ae_args &a, int64_t gp, int64_t n_log, int L) {
  if (a.slot < 0 || a.slot >= gp || !ae_ref_ok(a, n_log, L) || !ae_index_ok(a)) return AeKey{-1, 0, 0};
  return AeKey{a.entries_offset / L, (int)(a.entries_offset % L) - (a.prev_log_index + 1),
               a.prev_log_index + a.n_entries};
}

__device__ __forceinline__ bool same_key(const AeKey &x, const AeKey &y) {
  return x.row >= 0 && x.row == y.row && x.base == y.base && x.end == y.end;
}

// The claims of AppendEntries by reference and the set heads, one launch
// (rounds 2-4: a claim kernel, then a plan kernel that classified every item
// and compacted set and deferral lists through contended atomics). Per item:
// the slot check and the claim (atomicMax: the lowest item wins), srcmark of
// the row it reads, and sethd[i] = the size of the set item i heads, else 0
// (keys of the neighbours within kAeHalo from LDS, the halo loaded by the
// wave's edge lanes). Its first threads also arm the counters the main launch
// adds into (per stripe: deferred items and staged words, kStripeDef /
// kStripeStg); the previous call's deferred launch has read them (stream
// order).
constexpr int kAeHalo = 7;

__global__ __launch_bounds__(64) void k_claim_ae(const mraft_ae_args *__restrict__ args, int64_t n, int64_t n_log,
                                                 int L, int64_t gp, int ni, unsigned long long *__restrict__ claim,
                                                 uint32_t *__restrict__ srcmark, uint32_t epoch,
                                                 int32_t *__restrict__ err, uint8_t *__restrict__ sethd,
                                                 unsigned long long *__restrict__ total) {
  __shared__ long long kr[64 + 2 * kAeHalo];
  __shared__ int kb[64 + 2 * kAeHalo], ke[64 + 2 * kAeHalo];
  const int t = (int)threadIdx.x;
  const int64_t i = blockIdx.x * (int64_t)64 + t;
  if (i == 0) total[3] = 0;  // workgroups of the deferred launch's fallback done (total[2]: the published count)
  if (i < kStripes) {
    total[kStripeDef + kStripeWords * i] = 0;  // deferred items of stripe i
    total[kStripeDef + kStripeWords * i + 1] = 0;  // the fallback's finished workgroups of stripe i
    total[kStripeStg + kStripeWords * i] = 0;  // staged words of stripe i
  }
  AeKey k{-1, 0, 0};
  if (i < n) {
    const mraft_ae_args a = args[i];
    if (a.slot < 0 || a.slot >= gp) {
      err[i] = MRAFT_ITEM_BAD_SLOT;
    } else {
      err[i] = 0;
      atomicMax(&claim[a.slot], claim_tag(epoch, i));
      k = ae_key(a, gp, n_log, L);
      if (a.n_entries > 0 && k.row >= 0) srcmark[k.row] = epoch;
    }
  }
  kr[kAeHalo + t] = k.row; kb[kAeHalo + t] = k.base; ke[kAeHalo + t] = k.end;
  if (t < kAeHalo || t >= 64 - kAeHalo) {  // the halo: kAeHalo neighbours on either side of the wave
    const int64_t j = t < kAeHalo ? i - kAeHalo : i + kAeHalo;
    AeKey h{-1, 0, 0};
    if (j >= 0 && j < n) h = ae_key(args[j], gp, n_log, L);
    const int slot = t < kAeHalo ? t : t + 2 * kAeHalo;
    kr[slot] = h.row; kb[slot] = h.base; ke[slot] = h.end;
  }
  __syncthreads();
  if (i >= n) return;
  int hd = 0;
  const int c = kAeHalo + t;
  int pos = 0;  // this item's place in its run of same-entry messages (up to ni back)
  if (k.row >= 0)
    for (int d = 1; d <= ni && same_key(k, AeKey{kr[c - d], kb[c - d], ke[c - d]}); ++d) ++pos;
  if (k.row < 0 || pos >= ni) {
    hd = 1;
  } else if (pos == 0) {
    hd = 1;  // the set's size (up to ni forward)
    for (int d = 1; d < ni && same_key(k, AeKey{kr[c + d], kb[c + d], ke[c + d]}); ++d) ++hd;
  }
  sethd[i] = (uint8_t)hd;
}

// a4 for one set of messages per wave: lane q < size takes message first+q's
// prologue (its args, the claims, the receiving follower's scalars,
// log[prev]); conflict scans run wave-wide one message at a time; every
// merging message joins one streaming pass over the shared entries
// (mraft_pass.h).
enum : int { AE_DEFER = -1, AE_NONE = 0, AE_DONE, AE_BAD, AE_STALE, AE_BELOW, AE_MISS, AE_MERGE };
// The three ways handle_one is entered.
enum : int {
  HM_MAIN = 0,   // by reference, the main launch: classify, defer `written` items
  HM_DEFER = 1,  // by reference, a deferred item: entries staged (soff >= 0) or in place (-2)
  HM_HOST = 2,   // entries in a host-supplied buffer: one message per wave, nothing deferred
  HM_ORDER = 3   // by reference, the ordered fallback: entries in place (-2) or the cycle buffer (0)
};

#ifndef MRAFT_AE_MINW
#define MRAFT_AE_MINW 8  // __launch_bounds__ minimum waves per SIMD of the handler
#endif
// The deferred launch's: its register needs do not fit 8 waves per SIMD (the
// compiler reported 7 against a request of 8); asked for 7 its code is the
// allocator's own choice at that occupancy (profiles/r6_d6: deferred-heavy
// batches within noise or faster, the handler tests green)
#ifndef MRAFT_AE_DMINW
#define MRAFT_AE_DMINW 7
#endif

// The handler's persist mark at the end of a set's wave as a non-returning
// atomic OR: the wave does not wait for a load of the bits (a dependent round
// trip at its very end). Same-box A/B: handle call -8 us on average over three
// passes (profiles/r3_v8/message_path_ab.txt, r3w); the same change in the
// fused tick measured +0.7 % there and is not used.
__device__ __forceinline__ void mark_persist_ae(const Dev &s, int64_t slot, int bits) {
  if (s.pdirty && bits) (void)__hip_atomic_fetch_or(&s.pdirty[slot], bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Grids of the launches enqueued blind (their work is counted on the device
// and is usually small: deferred items need two leaders of one group in a
// batch, long segments more replies than a lane group, a1 scans a range the
// top-term probe did not settle). Small grids: a launch that must find free
// wave slots beside another pipeline's handler finds them at once — two
// pipelines 0.366-0.369 -> 0.358 ms per step, three 0.363-0.365 -> 0.354
// (profiles/r5_g1; 512 / 256 / 2,048 workgroups before).
#ifndef MRAFT_FOLD_TAIL_NL
#define MRAFT_FOLD_TAIL_NL 16  // k_fold_tail workgroups for the long segments (grid-stride)
#endif
#ifndef MRAFT_FOLD_TAIL_NS
#define MRAFT_FOLD_TAIL_NS 256 // k_fold_tail workgroups for the pending a1 scans (grid-stride)
#endif

// Every argument of the handler kernels, as their one kernel argument: the
// handler re-reads them from the kernel-argument segment after the streaming
// pass (reload_hs) instead of holding ~16 pointers live across it (at 8 waves
// per SIMD they spilled through VGPR lanes to scratch: 28 B per lane, ~100 MB
// of scratch write-back per config-#3 call).
struct HsArgs {
  Dev s;
  const mraft_ae_args *args;
  int64_t n;
  const int32_t *ent0;  // HM_HOST: the entries buffer
  int64_t n_ent0;
  int32_t *stage;       // staged entries of deferred `read` items (the cycle buffer in the fallback)
  int64_t stage_cap;    // its capacity in words
  int64_t *soff;        // per deferred item: its staged offset, or -2 (in place)
  const uint8_t *sethd; // per item: the size of the set it heads, else 0
  int64_t *defer;       // the deferred items
  unsigned long long *total;  // [0] staged words, [1] deferred items << 32
  const unsigned long long *claim;
  const uint32_t *srcmark;
  uint32_t epoch;
  // The deferred launch's fallback (staged words past the stage capacity),
  // per item, written by the main launch for its deferred items:
  int4 *fb;                  // {claimant of the row it reads (its writer, fb_writer), readers of its
                             // row already run, run flag, short-cycle readiness at the cycle's
                             // smallest item}: one 16-B record, zeroed but the first word
  unsigned long long *kin;   // epoch-tagged count of the deferred items that read this item's row
  int32_t *cslot;            // per-workgroup cycle buffers, nslot x L words
  int nslot;
  int32_t *cyc;              // the last workgroup's cycle buffer (L words)
  long long *hint;           // pinned host words: [0] the last deferred count (the next call's grid),
                             // [1] staged words of the last batch that exceeded the stage
  mraft_ae_reply *rep;
  int32_t *err;
  mraft_ae_result *res;  // optional: each item's reply as its co-resident leader folds it
};

__device__ __forceinline__ HsArgs reload_hs() {
  const __attribute__((address_space(4))) HsArgs *kp =
      (const __attribute__((address_space(4))) HsArgs *)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(kp));
  HsArgs k;
  k.s.term = kp->s.term; k.s.voted = kp->s.voted; k.s.role = kp->s.role; k.s.commit = kp->s.commit;
  k.s.applied = kp->s.applied; k.s.dummy = kp->s.dummy; k.s.last = kp->s.last; k.s.votes = kp->s.votes;
  k.s.log = kp->s.log; k.s.match = kp->s.match; k.s.next = kp->s.next; k.s.pdirty = kp->s.pdirty;
  k.s.head = kp->s.head; k.s.hsnap = kp->s.hsnap; k.s.srt = kp->s.srt; k.s.G = kp->s.G; k.s.P = kp->s.P; k.s.L = kp->s.L;
  k.args = kp->args; k.n = kp->n; k.ent0 = kp->ent0; k.n_ent0 = kp->n_ent0; k.stage = kp->stage;
  k.stage_cap = kp->stage_cap; k.soff = kp->soff; k.sethd = kp->sethd; k.defer = kp->defer; k.total = kp->total;
  k.claim = kp->claim; k.srcmark = kp->srcmark; k.epoch = kp->epoch; k.fb = kp->fb; k.kin = kp->kin;
  k.cslot = kp->cslot; k.nslot = kp->nslot; k.cyc = kp->cyc; k.hint = kp->hint;
  k.rep = kp->rep; k.err = kp->err; k.res = kp->res;
  return k;
}

// The args half of a failed item's reply record (slot = peer = -1), built
// where it is stored: as a plain constant the compiler kept it in four VGPRs
// from the prologue on and spilled them (a 16-B scratch store per lane in
// every wave of the main launch).
__device__ __forceinline__ int4 no_record() {
  int m = -1, z = 0;
  asm volatile("" : "+v"(m), "+v"(z));
  return make_int4(m, m, z, z);
}

// The number of set bits of m below this lane (v_mbcnt: no per-lane mask
// register, which the compiler would hoist and hold across the pass).
__device__ __forceinline__ int lanes_below(unsigned long long m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ int at_load(int32_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void at_store(int32_t *p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// This wave's own global stores complete before its next loads (a copy it
// reads back): workgroup scope, no cache maintenance.
__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_s_waitcnt(0);
}

// Epoch-tagged counters (high 32 bits: the call's epoch; a stale tag reads as
// 0), so no call has to zero them before counting.
__device__ __forceinline__ void tag_inc(unsigned long long *p, uint32_t epoch) {
  unsigned long long old = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    const unsigned long long nv =
        (uint32_t)(old >> 32) == epoch ? old + 1 : (((unsigned long long)epoch << 32) | 1ull);
    if (__hip_atomic_compare_exchange_strong(p, &old, nv, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      return;
  }
}
__device__ __forceinline__ int tag_count(const unsigned long long *p, uint32_t epoch) {
  const unsigned long long v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (uint32_t)(v >> 32) == epoch ? (int)(uint32_t)v : 0;
}

// The main launch's bookkeeping for the `written` lanes of a wave (rare: a
// stale leader both sending and receiving in one batch): their place in the
// deferred list, and for those that also `read`, a staged offset and the copy
// of their entries (the source row is pristine: its writer is deferred too).
__device__ __forceinline__ void defer_lanes(const HsArgs &k0, bool dfr, bool stg, int64_t i, int n, const int32_t *row,
                                            int head, int from, int L, int wraw) {
  const unsigned long long m = __ballot(dfr);
  const int lane = lane_id(), q0 = first_lane(m);
  const int x = (int)(blockIdx.x & (kStripes - 1));  // this workgroup's stripe
  unsigned long long b = 0;
  if (lane == q0) b = atomicAdd(&k0.total[kStripeDef + kStripeWords * x], (unsigned long long)__popcll(m));
  b = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(b >> 32), q0) << 32) |
      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, q0);
  if (dfr) {
    k0.defer[x * k0.n + (int64_t)b + lanes_below(m)] = i;
    int64_t in_place = -2;  // made here (as a hoisted constant pair it was spilled across the pass)
    asm volatile("" : "+v"(in_place));
    if (!stg) k0.soff[i] = in_place;
    // the fallback's graph (used only when the staged words pass the stage
    // capacity): the claimant of the row this item reads (its writer when that
    // claimant is deferred too, which the fallback checks: fb_writer), its
    // count of readers there, and this item's own counters zeroed
    k0.fb[i] = make_int4(wraw, 0, 0, 0);  // one store (four separate arrays spilled the main launch)
    if (wraw >= 0) tag_inc(&k0.kin[wraw], k0.epoch);
  }
  // the staged lanes' offsets: one atomic per wave on the stripe's counter
  // (an exclusive scan of their sizes), the copies one by one on the wave
  const unsigned long long smask = __ballot(stg);
  if (!smask) return;
  const int64_t cap8 = k0.stage_cap / kStripes;  // stripe x stages in [x cap8, (x + 1) cap8)
  int64_t pre = stg ? (int64_t)n : 0;  // inclusive scan of the staged sizes over the lanes
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t v = __shfl_up(pre, o, 64);
    if (lane >= o) pre += v;
  }
  const int64_t tot = __shfl(pre, 63, 64);
  unsigned long long sb = 0;
  if (lane == first_lane(smask)) sb = atomicAdd(&k0.total[kStripeStg + kStripeWords * x], (unsigned long long)tot);
  sb = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(sb >> 32), first_lane(smask)) << 32) |
       (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sb, first_lane(smask));
  const int64_t my = (int64_t)sb + pre - (stg ? (int64_t)n : 0);  // this lane's offset within the stripe
  if (stg) k0.soff[i] = x * cap8 + my;
  for (unsigned long long sm = smask; sm; sm &= sm - 1) {
    const int q = first_lane(sm);
    const int nq = __builtin_amdgcn_readlane(n, q);
    const int64_t oq = ((int64_t)__builtin_amdgcn_readlane((int)((uint64_t)my >> 32), q) << 32) |
                       (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)my, q);
    const long long o = x * cap8 + oq;
    if (oq + nq <= cap8) {  // past the stripe's capacity the deferred launch takes the ordered fallback
      const uint64_t ra = (uint64_t)(uintptr_t)row;
      const int32_t *rq = (const int32_t *)(uintptr_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(ra >> 32), q) << 32) |
                                                      (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ra, q));
      wave_copy_from_ring(rq, 0, __builtin_amdgcn_readlane(head, q), L, __builtin_amdgcn_readlane(from, q),
                          k0.stage + o, nq);
    }
  }
}

template <int NI, int MODE>
__device__ __forceinline__ void handle_one(const HsArgs &k0, int64_t first, int size, int64_t so_force = -2) {
  const Dev &s = k0.s;
  const mraft_ae_args *__restrict__ args = k0.args;
  const int lane = lane_id();
  const bool mine = lane < size;
  int64_t i = first + (mine ? lane : 0);
  // Three round trips before the pass: the item (error word, args[, staged
  // offset]), the claims with the follower's scalars and the source's ring
  // head, then log[prev] (and the first entry, for a sorted-terms claim).
  const int e = mine ? k0.err[i] : 1;
  mraft_ae_args a = args[i];
  const int64_t so0 = MODE == HM_DEFER ? k0.soff[i] : so_force;  // HM_ORDER: the caller's choice
  asm volatile("" ::"v"(a.slot), "v"(a.term), "v"(a.prev_log_index), "v"(a.prev_log_term),
               "v"(a.n_entries), "v"(a.leader_commit), "v"(a.entries_offset), "v"(so0));
  // L re-read per set: the division by it (a reciprocal) is then computed here,
  // not hoisted out of the wave's loop over sets and held across the pass
  int L = s.L;
  asm volatile("" : "+s"(L));
  const int64_t gp = (int64_t)s.G * s.P;
  int f = a.slot;
  const int prev = a.prev_log_index, nn = a.n_entries;
  // every word that depends only on the args, in one round trip (e == 0: the
  // slot is in range; the follower's words are read before the claims decide
  // whether the item runs here: no extra dependent round trip)
  int fterm = 0, fdummy = 0, flast = 0, fc = 0, fhead = 0;
  if (!e) { fterm = s.term[f]; fdummy = s.dummy[f]; flast = s.last[f]; fc = s.commit[f]; fhead = s.head[f]; }
  // Where the entries are: Index x of this lane's message at src.at(x). A
  // flat source (host buffer, staged copy, cycle buffer) is built relative to
  // its first entry (row = that entry's word, base = -(prev + 1)), so at()'s
  // 32-bit lane offset is x - (prev + 1), small whatever the Raft Index
  // (flat_src; an absolute Index above 2^30 wrapped it).
  RingRow src = flat_src(k0.ent0, 0, prev);
  int64_t n_ent = k0.n_ent0;
  bool ok = true, dup = false, dfr = false, stg = false;
  int64_t srow = 0;  // by reference: the source row
  int rhead = 0;
  unsigned long long cr = 0;  // HM_MAIN: the claim word of the source row
  if (MODE == HM_HOST) {
    if (!e) src = flat_src(k0.ent0, a.entries_offset, prev);
  } else if (!e) {
    ok = ae_ref_ok(a, gp * L, L);
    srow = ok ? a.entries_offset / L : 0;
    unsigned long long cs = 0;
    uint32_t sm = 0;
    if (MODE == HM_MAIN) {
      cs = k0.claim[f];
      sm = k0.srcmark[f];
      if (ok && nn > 0) cr = k0.claim[srow];
    }
    if (ok) rhead = s.head[srow];
    if (MODE == HM_MAIN) {
      dup = cs != claim_tag(k0.epoch, i);
      dfr = !dup && ok && sm == k0.epoch;                              // `written`: deferred
      stg = dfr && nn > 0 && (uint32_t)(cr >> 32) == k0.epoch;        // and `read`: staged
    }
    const int64_t so = MODE == HM_MAIN ? -2 : so0;
    if (so >= 0) {  // staged copy (or the fallback's cycle buffer)
      src = flat_src(k0.stage, so, prev);
      n_ent = k0.stage_cap;  // (HM_ORDER: the cycle buffer, capacity L)
      a.entries_offset = so;
    } else {        // in place through the source ring
      src.p = s.log;
      src.row = srow * L;
      src.L = L;
      src.base = rhead + (int)(a.entries_offset % L) - (prev + 1);
      n_ent = INT64_MAX;
    }
  }
  int cls = e ? AE_NONE : AE_DONE;
  if (dup) cls = AE_NONE;
  else if (dfr) cls = AE_DEFER;
  else if (!e && (!ok || nn < 0 || a.entries_offset < 0 || !ae_index_ok(a) ||
                  (nn > 0 && src.L == INT32_MAX && a.entries_offset + nn > n_ent)))
    cls = AE_BAD;
  const bool live = cls == AE_DONE;
  if (dup && mine) k0.err[i] = MRAFT_ITEM_DUP_SLOT;
  if (MODE == HM_MAIN && __ballot(dfr)) {
    // the claimant of the row this item reads (from the claim word loaded above),
    // for an item that reads anything (the writer check is the fallback's)
    const int wraw = (nn > 0 && ae_index_ok(a) && (uint32_t)(cr >> 32) == k0.epoch)
                         ? (int)(0xFFFFFFFFu - (uint32_t)cr) : -1;
    defer_lanes(k0, dfr, stg, i, nn, s.log + srow * L, rhead, (int)(a.entries_offset % L), L, wraw);
  }
  if (k0.res && mine && cls != AE_DEFER) {
    // the args half of the item's reply record for its co-resident leader's
    // fold, stored now (no reload of the args at the wave's end); the reply
    // half follows with the reply. Failed items: slot = peer = -1.
    int PP = s.P;
    asm volatile("" : "+s"(PP));  // (the division's reciprocal made here, not hoisted and spilled)
    int4 *rr = reinterpret_cast<int4 *>(k0.res + i);
    rr[0] = live ? make_int4((f / PP) * PP + a.leader_id, f % PP, a.term, prev) : no_record();
  }
  // MRAFT_AE_ENTRIES_SORTED is the sender's claim (it crosses the network):
  // honoured only where the terms prevLogTerm, entry 0, ... really never
  // decrease. Here the first step (prevLogTerm <= entry 0, in the round trip
  // of the follower's log[prev]); the entries themselves are checked on the
  // pass's loads (DescTrack). Same rule in the oracle (ae_flag_holds).
  const bool claim = live && nn > 0 && (a.flags & MRAFT_AE_ENTRIES_SORTED) != 0;
  const bool claim0 = claim && a.prev_log_term <= *src.at(prev + 1);
  mraft_ae_reply r = {0, 0, 0, 0};
  int ftp = 0;
  if (live) {
    if (a.term < fterm) {                                              // :112-115
      cls = AE_STALE;
      r.term = fterm;
    } else if (prev < fdummy) {                                        // :123-127
      cls = AE_BELOW;
      r.conflict_index = fdummy + 1;
    } else {
      ftp = prev > flast ? 0 : s.log[(int64_t)f * L + ring(prev - fdummy + fhead, L)];
      if (prev > flast || ftp != a.prev_log_term) {                    // matchLog, raft_log.go:92-96
        cls = AE_MISS;
        r.term = a.term;
        if (prev > flast) r.conflict_index = flast + 1;                // :131-133
        else r.conflict_index = prev;                                  // :136-142 below when prev > dummy + 1
      } else {
        cls = AE_MERGE;
      }
    }
  }
  // :136-142, the ConflictIndex scan, wave-wide for one message at a time
  for (unsigned long long m = __ballot(cls == AE_MISS && prev <= flast && prev > fdummy + 1); m; m &= m - 1) {
    const int q = first_lane(m);
    const int qf = __shfl(f, q, 64), qd = __shfl(fdummy, q, 64), qh = __shfl(fhead, q, 64),
              qp = __shfl(prev, q, 64), qa = __shfl(ftp, q, 64);
    const int ci = wave_conflict_scan(s.log + (int64_t)uni(qf) * L, uni(qd), uni(qh), L, uni(qp), uni(qa));
    if (lane == q) r.conflict_index = ci;
  }
  // :146-155 through the streaming pass the tick uses: compare entries with
  // every merging follower's terms, truncate-and-append from the first
  // mismatch. All messages of a set end at the same Index (AeKey).
  int newlast = -1, fcommit_new = -1, srt_new = -1;
  const int merge_m = (int)(__ballot(cls == AE_MERGE) & ((1ull << NI) - 1));
  // terms_sorted after an append from Index k (include/mraft.h): the args'
  // flag when k - 1 is the dummy, cleared without it, else unchanged — the
  // flag as checked (claim0 here, the entries' descents after the pass);
  // shint: -1 no flag, 1 flag and prev is the dummy, 0 flag otherwise
  int shint = claim0 ? (prev == fdummy ? 1 : 0) : -1;
  if (merge_m) {
    Fol<NI, true> fo;
    fo.log = s.log;
    fo.slot0 = 0;
    fo.skip = NI;
    fo.L = L;
    fo.cmp = merge_m;
    fo.copy = 0;
    fo.capok = (int)(__ballot(cls == AE_MERGE && (int64_t)prev + nn - fdummy <= (int64_t)L - 1) & ((1ull << NI) - 1));
    fo.full = 0;
    const int phi = uni(__shfl(prev + nn, first_lane((unsigned long long)merge_m), 64));
    int plo = phi + 1;
#pragma unroll
    for (int q = 0; q < NI; ++q)
      if ((merge_m >> q) & 1) plo = min(plo, uni(__shfl(prev, q, 64)) + 1);
    // The pass runs on Indexes relative to B = plo - kPassBias (pass_bias):
    // every Index it forms stays in [kPassBias - 35, kPassBias + L + 256], so
    // no chunk end (c + 256) overflows int32 near 2^31 and the lane offsets a
    // source's at() forms stay small. Rows see the same words (their bases
    // absorb B).
    const int B = pass_bias(plo);
    const int pl = plo - B, ph = phi - B, nend = ph + 1;
    // the source as the first merging message sees it (the same for every message of a set)
    const int q0 = first_lane((unsigned long long)merge_m);
    RingRow ss;
    {
      const uint64_t pa = (uint64_t)(uintptr_t)src.p;
      const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)pa, q0, 64), hi = (uint32_t)__shfl((int)(pa >> 32), q0, 64);
      ss.p = (const int32_t *)(uintptr_t)(((uint64_t)uni((int)hi) << 32) | (uint32_t)uni((int)lo));
      const uint64_t ra = (uint64_t)src.row;
      const uint32_t rlo = (uint32_t)__shfl((int)(uint32_t)ra, q0, 64), rhi = (uint32_t)__shfl((int)(ra >> 32), q0, 64);
      ss.row = (long long)(((uint64_t)uni((int)rhi) << 32) | (uint32_t)uni((int)rlo));
      ss.base = uni(__shfl(src.base, q0, 64)) + B;
      ss.L = uni(__shfl(src.L, q0, 64));
    }
    bool vec = (L & 3) == 0 && ((uintptr_t)s.log & 15) == 0;
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      fo.slot[q] = uni(__shfl(f, q, 64));
      const int sp = uni(__shfl(prev, q, 64)), sl = uni(__shfl(flast, q, 64));
      fo.base[q] = 0; fo.start[q] = 0; fo.cend[q] = 0;
      fo.cfrom[q] = 0;  // 0: no mismatch (a relative Index is >= kPassBias - 35 > 0)
      if ((merge_m >> q) & 1) {  // (only merging messages are ever addressed)
        fo.base[q] = uni(__shfl(fhead - fdummy, q, 64)) + B;
        fo.start[q] = sp + 1 - B;
        fo.cend[q] = min(phi, sl) + 1 - B;
        // dwordx4 when the entries and this follower's row are 16-B aligned alike
        vec = vec && ((((uintptr_t)ss.at(fo.start[q]) ^ (uintptr_t)fo.at(q, fo.start[q])) & 15) == 0);
      }
    }
    if (ss.L == INT32_MAX) {  // a flat buffer: every dwordx4 read must stay inside it
      // its size as the first merging message sees it: n_ent is per lane (a
      // lane with no item keeps the host-buffer size, 0 by reference), and a
      // per-lane `vec` would split the wave between the two passes
      const uint64_t nb = (uint64_t)n_ent;
      const uint32_t nlo = (uint32_t)__shfl((int)(uint32_t)nb, q0, 64), nhi = (uint32_t)__shfl((int)(nb >> 32), q0, 64);
      const int64_t sn = (int64_t)(((uint64_t)uni((int)nhi) << 32) | (uint32_t)uni((int)nlo));
      vec = vec && (((uintptr_t)ss.at(pl)) & ~(uintptr_t)15) >= (uintptr_t)ss.p &&
            (((uintptr_t)ss.at(ph)) | 15) < (uintptr_t)(ss.p + sn);
    }
    // the pass is wave-wide (ballots, shuffles): one choice for every lane
    vec = __ballot(!vec) == 0;
    int found = -1;
    DescTrack dt{__ballot(cls == AE_MERGE && claim0) != 0, 0, INT32_MIN};
    // This lane's reply inputs wait in LDS during the pass (the pass needs
    // the registers: at 8 waves per SIMD they would spill to scratch).
    // (plain LDS stores and loads across a compiler memory barrier: a
    // volatile generic pointer made them flat accesses with 64-bit addresses
    // the compiler hoisted and spilled)
    __shared__ int stash[12][64];
    stash[0][lane] = cls; stash[1][lane] = f; stash[2][lane] = fterm; stash[3][lane] = flast;
    stash[4][lane] = fc; stash[5][lane] = a.term; stash[6][lane] = a.leader_commit;
    stash[7][lane] = r.conflict_index; stash[8][lane] = r.term;
    stash[9][lane] = (int)(uint32_t)(uint64_t)i; stash[10][lane] = (int)((uint64_t)i >> 32);
    stash[11][lane] = shint;
    asm volatile("" ::: "memory");
    if (vec) {
      int c = pl - (int)(((uintptr_t)ss.at(pl) >> 2) & 31);            // 128-B aligned chunks
      if (c <= ph && fo.cmp) c = pass_pipe<false>(ss, fo, nend, 1, 0, 0, found, c, pl, ph, dt);
      copy_loop<true, false>(ss, fo, c, nend, pl, ph, 1, 0, 0, found, dt);
    } else {
      int c = pl;
      for (; c <= ph && fo.cmp; c += 256) pass_chunk<1, false, false>(ss, fo, nend, 1, 0, 0, found, c, pl, ph, dt);
      copy_loop<false, false>(ss, fo, c, nend, pl, ph, 1, 0, 0, found, dt);
    }
    asm volatile("" ::: "memory");
    cls = stash[0][lane]; f = stash[1][lane]; fterm = stash[2][lane]; flast = stash[3][lane];
    fc = stash[4][lane]; a.term = stash[5][lane]; a.leader_commit = stash[6][lane];
    r.conflict_index = stash[7][lane]; r.term = stash[8][lane];
    i = (int64_t)(((uint64_t)(uint32_t)stash[10][lane] << 32) | (uint32_t)stash[9][lane]);
    shint = stash[11][lane];
    // kernel arguments re-read from the kernarg segment, not held across the pass
    const HsArgs kr = reload_hs();
    int32_t *__restrict__ err = kr.err;
    mraft_ae_reply *__restrict__ rep = kr.rep;
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      if (lane != q || cls != AE_MERGE) continue;
      if ((fo.full >> q) & 1) {
        cls = AE_DONE;                                                 // engine capacity: no state change
        err[i] = MRAFT_ITEM_LOG_FULL;
        rep[i] = r;
      } else {
        int last_after = flast;
        if (fo.cfrom[q] > 0) {                                         // truncated and appended
          newlast = last_after = phi;
          // a descent among this message's entries (Index start+1 .. phi)
          // voids its flag
          if (dt.last > fo.start[q]) shint = -1;
          // appended from the dummy's successor (prev == dummy, first mismatch
          // at start): the entries are the whole log
          srt_new = shint < 0 ? 0 : (shint == 1 && fo.cfrom[q] == fo.start[q] ? 1 : -1);
        }
        if (a.leader_commit > fc) fcommit_new = min(a.leader_commit, last_after);  // :157-160
        r.term = a.term; r.success = 1;                                // :161
      }
    }
  }
  const HsArgs kt = reload_hs();
  const Dev &s2 = kt.s;
  int32_t *__restrict__ err2 = kt.err;
  mraft_ae_reply *__restrict__ rep2 = kt.rep;
  if (cls == AE_NONE) {
    if (mine) rep2[i] = r;
  } else if (cls == AE_BAD) {
    rep2[i] = r;
    err2[i] = MRAFT_ITEM_BAD_SLOT;
  } else if (cls == AE_STALE) {
    rep2[i] = r;
    mark_persist_ae(s2, f, MRAFT_PERSIST_STATE);                       // deferred :111
  } else if (cls >= AE_BELOW) {
    if (a.term > fterm) { s2.term[f] = a.term; s2.voted[f] = -1; }    // :116-118
    s2.role[f] = kFollower;                                            // :120
    if (newlast >= 0) s2.last[f] = newlast;
    if (srt_new >= 0) s2.srt[f] = srt_new;
    if (fcommit_new >= 0) s2.commit[f] = fcommit_new;
    mark_persist_ae(s2, f, MRAFT_PERSIST_STATE);                       // deferred :111
    rep2[i] = r;
  }
  mraft_ae_result *__restrict__ res = kt.res;
  if (res && mine && cls != AE_DEFER) {
    // the reply half of the record (nEntries, reply term, success,
    // ConflictIndex); an item rejected after the prologue (capacity: cls
    // AE_DONE) gets slot = peer = -1 as well
    int4 *rr = reinterpret_cast<int4 *>(res + i);
    if (cls == AE_DONE) rr[0] = no_record();
    rr[1] = cls >= AE_STALE ? make_int4(nn, r.term, r.success, r.conflict_index) : make_int4(0, 0, 0, 0);
  }
}

// The main launch: wave v serves the sets whose heads lie in items
// [v*NI, (v+1)*NI) (one set for a gathered batch), each XCD a contiguous
// range of waves (neighbouring sets share one L2 for the leaders' entries).
// HM_HOST: wave v serves message v.
template <int NI, int MODE>
__global__ __launch_bounds__(64, MRAFT_AE_MINW) void k_handle_set(HsArgs ka) {
  const int64_t nb = MODE == HM_HOST ? ka.n : (ka.n + NI - 1) / NI;
  int64_t v = blockIdx.x;
  {
    const int64_t x = v & 7, per = nb >> 3, rem = nb & 7, j = v >> 3;
    if (j >= per + (x < rem ? 1 : 0)) return;
    v = x * per + min(x, rem) + j;
  }
  if (MODE == HM_HOST) {
    handle_one<NI, HM_HOST>(ka, v, 1);
    return;
  }
  const int lane = lane_id();
  const int64_t c0 = v * NI;
  const int hd = (lane < NI && c0 + lane < ka.n) ? (int)ka.sethd[c0 + lane] : 0;
  for (unsigned long long m = __ballot(hd > 0); m; m &= m - 1) {
    const int q = first_lane(m);
    handle_one<NI, HM_MAIN>(ka, c0 + q, __builtin_amdgcn_readlane(hd, q));
  }
}

// ---- The deferred launch's fallback: the staged words exceed the stage
// capacity, so deferred items that are also `read` have no staged copy and
// must run in an order (round 6; rounds 4-5 ran the whole fallback on one
// wave). Edge x -> wr[x]: x reads the row its writer wr[x] rewrites, so x runs
// first. Each item has one writer at most, so the graph is trees feeding
// chains that end at an item with no writer or at a cycle. Every workgroup
// takes deferred items grid-stride and nothing ever waits:
//  * an item no deferred item reads (kin 0) starts a chain: it runs, then
//    counts itself at its writer (arr); the reader that completes the
//    writer's count (arr == kin) runs the writer next, and so on;
//  * a cycle of at most kCycWalk items (found by walking wr) runs as a unit
//    on one wave, once every tree feeding it has run: its smallest item's
//    entries are copied to the wave's cycle buffer first, then the members
//    run around the cycle from its writer, that item last from the copy.
//    Readiness is one counter at that item (cpend): each member whose other
//    readers have all run adds 1 (the reader whose arrival leaves only the
//    cycle predecessor missing, arr == kin - 1), and the smallest item's own
//    visit adds kBig - F (F: members with such readers): the add that brings
//    it to kBig runs the cycle;
//  * what is left — cycles longer than the walk, or completed on a workgroup
//    with no cycle buffer — the last workgroup to finish runs one cycle at a
//    time through the L-word buffer (every tree has run by then).
// Nothing another item reads is written before that item has read it; items
// of a chain share no row they both read and write, so the hand-offs need no
// fence beyond the counters' atomics (the runs of a cycle are ordered on one
// wave). Same results as the staged path (tests/test_handler_async.py,
// tests/test_deferred_graphs_gpu.py).
constexpr int kCycWalk = 32;
constexpr unsigned kCycBig = 1u << 30;  // > kCycWalk: the count cannot reach it early

__device__ __forceinline__ int32_t &fb_dn(const HsArgs &k, int64_t x) { return reinterpret_cast<int32_t *>(k.fb + x)[2]; }

// One deferred item in the fallback: its entries in place (buf null) or from
// buf (its copy); then marked run.
__device__ __forceinline__ void fb_run(const HsArgs &k, int64_t x, int32_t *buf) {
  HsArgs kx = k;
  kx.stage = buf;
  kx.stage_cap = k.s.L;
  handle_one<1, HM_ORDER>(kx, x, 1, buf ? 0 : -2);
  if (lane_id() == 0) at_store(&fb_dn(k, x), 1);
}

// x's writer: the claimant of the row x reads when that claimant is a
// well-formed reference (then its slot, read by x, made it deferred too).
__device__ __forceinline__ int64_t fb_writer(const HsArgs &k, int64_t x) {
  const int w = __builtin_amdgcn_readfirstlane(reinterpret_cast<const int32_t *>(k.fb + x)[0]);
  if (w < 0 || (int64_t)w >= k.n) return -1;
  const int L = k.s.L;
  return ae_ref_ok(k.args[w], (int64_t)k.s.G * k.s.P * L, L) ? (int64_t)w : -1;
}

// Whether y lies on a cycle of at most kCycWalk items; then its smallest item
// and length.
__device__ __forceinline__ bool fb_short_cycle(const HsArgs &k, int64_t y, int64_t *least, int *len) {
  int64_t z = y, m = y;
  for (int st = 1; st <= kCycWalk; ++st) {
    z = fb_writer(k, z);
    if (z < 0) return false;
    if (z == y) {
      *least = m;
      *len = st;
      return true;
    }
    m = min(m, z);
  }
  return false;
}

// A cycle whose feeding trees have all run, from its smallest item b: b's
// entries (the pristine row of its writer) copied first, then the members
// from b's writer round to b. With no cycle buffer for this workgroup the
// cycle is left to the last workgroup.
__device__ __forceinline__ void fb_run_cycle(const HsArgs &k, int64_t b) {
  if ((int)blockIdx.x >= k.nslot) return;
  int32_t *buf = k.cslot + (int64_t)blockIdx.x * k.s.L;
  const mraft_ae_args a = k.args[b];
  const int L = k.s.L;
  const int64_t row = a.entries_offset / L;
  wave_copy_from_ring(k.s.log + row * L, 0, k.s.head[row], L, (int)(a.entries_offset % L), buf, a.n_entries);
  wave_fence();  // this wave reads the copy back: a workgroup-scope fence (r6_v9: an agent-scope one per cycle, an L2 write-back each, cost 5 ms per 32k cycles)
  int64_t z = fb_writer(k, b);
  for (int st = 0; z >= 0 && z != b && st < kCycWalk; ++st, z = fb_writer(k, z)) fb_run(k, z, nullptr);
  fb_run(k, b, buf);
}

__device__ __forceinline__ void fb_cycle_add(const HsArgs &k, int64_t b, unsigned add) {
  unsigned old = 0;
  if (lane_id() == 0) old = atomicAdd(reinterpret_cast<unsigned *>(k.fb + b) + 3, add);
  old = (unsigned)__builtin_amdgcn_readfirstlane((int)old);
  if (old + add == kCycBig) fb_run_cycle(k, b);
}

// x, then every writer whose readers x's run completes.
__device__ __forceinline__ void fb_chain(const HsArgs &k, int64_t x) {
  x = ((int64_t)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32) | (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
  for (;;) {
    fb_run(k, x, nullptr);
    const int64_t w = fb_writer(k, x);
    if (w < 0) return;
    unsigned a = 0;
    if (lane_id() == 0) a = atomicAdd(reinterpret_cast<unsigned *>(k.fb + w) + 1, 1u) + 1u;
    a = (unsigned)__builtin_amdgcn_readfirstlane((int)a);
    const unsigned kw = (unsigned)tag_count(&k.kin[w], k.epoch);
    if (a == kw) {
      x = w;
      continue;
    }
    int64_t b;
    int len;
    if (a + 1 == kw && fb_short_cycle(k, w, &b, &len)) fb_cycle_add(k, b, 1);
    return;
  }
}

// The deferred items as one sequence j = 0 .. nd - 1 over the stripes' lists
// (stripe x's count d[x], its list at defer[x * n]); wave-uniform counts.
struct DeferSeq {
  int64_t d[kStripes];
  __device__ __forceinline__ int64_t at(const HsArgs &k, int64_t j) const {
    int x = 0;
#pragma unroll
    for (int y = 0; y < kStripes - 1; ++y)
      if (x == y && j >= d[y]) { j -= d[y]; x = y + 1; }
    return k.defer[x * k.n + j];
  }
};

// The last workgroup: every item not yet run lies on a cycle whose feeding
// trees have run; each such cycle runs from one member x through the L-word
// buffer.
__device__ __forceinline__ void fb_leftover(const HsArgs &k, int64_t nd, const DeferSeq &ds) {
  const int lane = lane_id();
  const int L = k.s.L;
  for (int64_t j0 = 0; j0 < nd; j0 += 64) {
    const int64_t j = j0 + lane;
    const int64_t y = j < nd ? ds.at(k, j) : -1;
    for (unsigned long long m = __ballot(y >= 0 && at_load(&fb_dn(k, y)) == 0); m; m &= m - 1) {
      const int q = first_lane(m);
      const int64_t x = ((int64_t)__builtin_amdgcn_readlane((int)(y >> 32), q) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)y, q);
      if (__builtin_amdgcn_readfirstlane(at_load(&fb_dn(k, x)))) continue;  // run with an earlier one's cycle
      const mraft_ae_args a = k.args[x];
      const int64_t row = a.entries_offset / L;
      if (a.n_entries > 0) wave_copy_from_ring(k.s.log + row * L, 0, k.s.head[row], L, (int)(a.entries_offset % L),
                                               k.cyc, a.n_entries);
      wave_fence();
      int64_t z = fb_writer(k, x);
      for (int64_t st = 0; z >= 0 && z != x && st < nd; ++st) {
        fb_run(k, z, nullptr);
        z = fb_writer(k, z);
      }
      fb_run(k, x, k.cyc);
    }
  }
}

__device__ __forceinline__ void defer_fallback(const HsArgs &k, int64_t nd, const DeferSeq &ds) {
  // only workgroups with a cycle buffer take items (any of them may complete
  // a cycle and must run it: r6_v6 ran 28k of 32k 2-cycles on the last
  // workgroup when the grid was 16x the buffers); the others only count out
  const int64_t nb = min((int64_t)gridDim.x, (int64_t)max(k.nslot, 1));
  if ((int64_t)blockIdx.x >= nb) return;  // (not counted below either)
  for (int64_t j = blockIdx.x; j < nd; j += nb) {
    const int64_t x = ds.at(k, j);
    if (tag_count(&k.kin[x], k.epoch) == 0) {
      fb_chain(k, x);  // no deferred item reads x's row: a chain starts here
    } else {
      int64_t b;
      int len;
      if (fb_short_cycle(k, x, &b, &len) && b == x) {
        // x is its short cycle's smallest item: its visit's share of the count
        int F = 0;
        int64_t z = x;
        for (int st = 0; st < len; ++st) {
          F += tag_count(&k.kin[z], k.epoch) > 1 ? 1 : 0;
          z = fb_writer(k, z);
        }
        fb_cycle_add(k, x, kCycBig - (unsigned)F);
      }
    }
  }
  // the last workgroup to finish runs what is left (it sees every other
  // workgroup's runs: release before each count, acquire after it). Counted
  // in two levels, per stripe (blockIdx % 8, its own line) and then the
  // stripes: one counter taking every workgroup's atomic serialised them
  // (the 2-cycle-heavy batch's fallback, r6_d1)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  int last = 0;
  if (lane_id() == 0) {
    const int64_t x = blockIdx.x & (kStripes - 1);
    const unsigned long long in_x = (unsigned long long)((nb - 1 - x) / kStripes + 1);  // workgroups b < nb, b % 8 == x
    if (atomicAdd(&k.total[kStripeDef + kStripeWords * x + 1], 1ull) == in_x - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
      last = atomicAdd(&k.total[3], 1ull) == (unsigned long long)min(nb, (int64_t)kStripes) - 1;
    }
  }
  if (!__builtin_amdgcn_readfirstlane(last)) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  fb_leftover(k, nd, ds);
}

// The deferred launch: every deferred item (a set of one), grid-stride; the
// counts are read on the device (the host enqueues this launch blind: with no
// deferred item, every workgroup exits at once). Its grid is the host's choice
// from the last call's deferred count, which workgroup 0 publishes to a pinned
// host word when it changes (total[2] keeps the published value).
__global__ __launch_bounds__(64, MRAFT_AE_DMINW) void k_handle_deferred(HsArgs ka) {
  DeferSeq ds;
  int64_t nd = 0;
  long long smax = 0;  // the largest stripe's staged words
#pragma unroll
  for (int x = 0; x < kStripes; ++x) {
    ds.d[x] = (int64_t)ka.total[kStripeDef + kStripeWords * x];
    nd += ds.d[x];
    smax = max(smax, (long long)ka.total[kStripeStg + kStripeWords * x]);
  }
  const long long cap8 = ka.stage_cap / kStripes;
  // the need, as a stage whose every stripe holds the largest one's words
  const long long staged = smax > cap8 ? smax * kStripes : 0;
  if (blockIdx.x == 0 && threadIdx.x == 0 && ka.hint && ka.total[2] != (unsigned long long)nd) {
    ka.total[2] = (unsigned long long)nd;
    __hip_atomic_store(ka.hint, (long long)nd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // a batch whose staged words exceed the stage: the need, for the host's
  // next call (the stage grows to it under MRAFT_STAGE_AUTO, mraft_abi.hip)
  if (blockIdx.x == 0 && threadIdx.x == 0 && ka.hint && smax > cap8)
    __hip_atomic_store(ka.hint + 1, staged, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (nd == 0) return;
  if (smax <= cap8) {
    for (int64_t j = blockIdx.x; j < nd; j += gridDim.x) handle_one<1, HM_DEFER>(ka, ds.at(ka, j), 1);
  } else {
    defer_fallback(ka, nd, ds);
  }
}

// ---------------------------------------------------------------- a2 + a1
// A reply record inside the Index domain (include/mraft.h): the acknowledged
// entries end at prevLogIndex + n <= 2^31 - 2 with n >= 0 (matchIndex and
// nextIndex stay int32); else the segment is malformed, as in the oracle
// (reply_index_ok).
__device__ __forceinline__ bool reply_index_ok(int prev, int n) {
  return n >= 0 && (int64_t)prev + n <= (int64_t)INT32_MAX - 1;
}

template <int P>
__device__ __forceinline__ int quorum_rt(const int (&m)[8], int me) {
  constexpr int h = P / 2;
  if (h == 0) return INT32_MAX;
  int best = INT32_MIN;
#pragma unroll
  for (int j = 0; j < P; ++j) {
    if (j == me) continue;
    int c = 0;
#pragma unroll
    for (int q = 0; q < P; ++q) c += (q != me && m[q] >= m[j]) ? 1 : 0;
    if (c >= h && m[j] > best) best = m[j];
  }
  return best;
}

#ifndef MRAFT_FOLD_GRID
#define MRAFT_FOLD_GRID (1 << 30)  // workgroups of the reply fold (segments beyond: grid-stride)
#endif
// The fold's shape (r3-r5 A/B runs, profiles/INDEX.md): eight reply segments
// per wave, 8 lanes each (four per wave measured 10 % slower; one per wave
// slower still), waves of one XCD on a contiguous segment range (r4_v18: fold
// call -8 %, reads 55 -> 46 MB); each segment's a1 ranges probed by their top
// word in k_fold and the open ones scanned in a second launch, k_fold_tail,
// which also folds the segments longer than a lane group on all 64 lanes
// (r4_v21: -4 % against separate launches; the scans back inside k_fold,
// r5_f1: no difference). Earlier variants live in git history.
constexpr int kFoldGroups = 8;              // reply segments per k_fold wave
constexpr int kFoldScanU = 4;               // long-segment a1 scan: dword loads per lane in flight (64·U terms)
constexpr int kFscanU = 8;                  // k_fold_tail scans: dword loads per lane in flight (4: +7 %)
constexpr int kFscanW = 4;                  // pending a1 ranges per k_fold_tail scan wave

// One iteration of the a1 scan: the highest idx in [max(lo, top - 64·U + 1),
// top] with row[idx] == a, or lo - 1 (wave-uniform arguments).
template <int U>
__device__ __forceinline__ int fold_scan_iter(const int32_t *__restrict__ row, int base, int head, int L,
                                              int lo, int top, int a) {
  const int lane = lane_id();
  int v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int idx = top - lane - kWave * u;
    const int w = row[ring(max(idx, lo) - base + head, L)];  // unconditional: the U loads issue back to back
    v[u] = idx >= lo ? w : a + 1;
  }
  // Every ballot of the iteration (no early exit: an exit per vector lets
  // the compiler sink each load behind the previous compare).
  int r = lo - 1;
#pragma unroll
  for (int u = U - 1; u >= 0; --u) {
    const unsigned long long m = __ballot(v[u] == a);
    r = m ? top - kWave * u - first_lane(m) : r;
  }
  return r;
}

// Highest idx in [lo, hi] with row[idx - base] == a, or lo - 1: the a1 scan
// of the reply fold, 64·U terms per round trip.
template <int U>
__device__ __forceinline__ int fold_scan_down_eq(const int32_t *__restrict__ row, int base, int head, int L,
                                                 int lo, int hi, int a) {
  if (hi < lo) return lo - 1;
  int r = fold_scan_iter<U>(row, base, head, L, lo, hi, a);
  for (int top = hi - kWave * U; r < lo && top >= lo; top -= kWave * U)
    r = fold_scan_iter<U>(row, base, head, L, lo, top, a);
  return r;
}

// Appends the lanes' pending a1 ranges (pred) to k_fold_tail's compact list:
// one atomic per wave on the list's counter. Record: {lo, hi, slot,
// currentTerm}, {dummy, ring head, reply index, 0}. Wave-uniform call.
__device__ __forceinline__ void push_pending(int4 *__restrict__ pend, unsigned *__restrict__ pcount, bool pred,
                                             int4 ra, int4 rb) {
  const unsigned long long m = __ballot(pred);
  if (!m) return;
  const int l0 = first_lane(m);
  unsigned base = 0;
  if (lane_id() == l0) base = atomicAdd(pcount, (unsigned)__popcll(m));
  base = (unsigned)__shfl((int)base, l0, 64);
  if (pred) {
    const unsigned k = base + (unsigned)__popcll(m & ((1ull << lane_id()) - 1));
    pend[2 * (int64_t)k] = ra;
    pend[2 * (int64_t)k + 1] = rb;
  }
}

// A long segment (more replies than a lane group: k_fold_tail), one wave.
// Lane k loads reply k of a 64-reply batch, so a segment's replies arrive in
// one round trip; the fold
// (a2, :66-88) then runs over them in array order on wave-uniform values.
// a1 (:89-105) is evaluated after each successful reply exactly as :78 calls
// it, but its log reads are deferred to the end of the batch: the fold never
// reads commitIndex, and while the replica stays leader its term is the
// segment's initial term, so every evaluation is "the highest index in
// (H, top] whose term is currentTerm", with H the largest top evaluated so
// far (an evaluation that scanned (commit, top] leaves no entry of that term
// above the new commit up to top). The ranges of one batch are disjoint and
// ascending: their top words are probed in parallel (one round trip; on a
// log whose last entries carry the current term, every range ends there) and
// only ranges whose top word differs are scanned, wave-cooperatively.
template <int P>
__device__ __forceinline__ void fold_segment(const Dev &s, const mraft_ae_result *__restrict__ items,
                                             const int64_t *__restrict__ seg_begin, int64_t sg,
                                             const int32_t *__restrict__ seg_err,
                                             const unsigned long long *__restrict__ claim, uint32_t epoch,
                                             int32_t *__restrict__ flags, int32_t *__restrict__ item_err) {
  const int lane = lane_id();
  const int64_t b = seg_begin ? seg_begin[sg] : sg, e = seg_begin ? seg_begin[sg + 1] : sg + 1;
  int bad = uni(seg_err[sg]);  // the claim verdict: a bad segment's slot may be out of range
  if (b >= e) return;
  const int64_t cnt = e - b;
  mraft_ae_result it{};
  if (lane < cnt) it = items[b + lane];
  const int slot = __builtin_amdgcn_readfirstlane(it.slot);
  const int me = slot % P;
  const int64_t mrow = (int64_t)slot * P;
  // The replica's state in one round trip: one load per lane, lanes 0..P-1
  // matchIndex, 8..8+P-1 nextIndex, 16..20 the scalars.
  const int32_t *src = nullptr;
  int64_t si = slot;
  if (lane < P) { src = s.match; si = mrow + lane; }
  else if (lane >= 8 && lane < 8 + P) { src = s.next; si = mrow + lane - 8; }
  else if (lane == 16) src = s.term;
  else if (lane == 17) src = s.role;
  else if (lane == 18) src = s.commit;
  else if (lane == 19) src = s.last;
  else if (lane == 20) src = s.dummy;
  else if (lane == 21) src = s.head;
  else if (lane == 22) src = s.srt;
  const int vs = (src && !bad) ? src[si] : 0;
  // items addressed to one replica slot in several segments: the lowest
  // segment wins (k_claim_zero's atomicMax on the inverted index), the others
  // are rejected before any state change — loaded beside the state
  const unsigned long long cw = !bad ? claim[slot] : 0ull;
  if (!bad && __builtin_amdgcn_readfirstlane((int)(uint32_t)cw) != (int)(0xFFFFFFFFull - (uint64_t)sg) ) bad = MRAFT_ITEM_DUP_SLOT;
  if (!bad && (uint32_t)(cw >> 32) != epoch) bad = MRAFT_ITEM_DUP_SLOT;
  int term = __builtin_amdgcn_readlane(vs, 16), role = __builtin_amdgcn_readlane(vs, 17),
      commit = __builtin_amdgcn_readlane(vs, 18);
  const int last = __builtin_amdgcn_readlane(vs, 19), dummy = __builtin_amdgcn_readlane(vs, 20),
            head = __builtin_amdgcn_readlane(vs, 21), srt = __builtin_amdgcn_readlane(vs, 22);
  for (int64_t base = 0; base < cnt; base += 64) {
    const int64_t i = base + lane;
    int sl = it.slot, pr = it.peer;
    if (base > 0 && i < cnt) { sl = items[b + i].slot; pr = items[b + i].peer; }
    // (a segment that does not own its slot stays MRAFT_ITEM_DUP_SLOT: the
    // claim decides first, include/mraft.h)
    bool dok = true;  // the record inside the Index domain (reply_index_ok)
    if (i < cnt) {
      const mraft_ae_result &r = base > 0 ? items[b + i] : it;
      dok = reply_index_ok(r.args_prev_log_index, r.args_n_entries);
    }
    if (__ballot(i < cnt && (sl != slot || pr < 0 || pr >= P || pr == me || !dok)) && !bad) bad = MRAFT_ITEM_BAD_SLOT;
  }
  if (!bad && commit < dummy) bad = MRAFT_ITEM_BAD_STATE;
  if (bad) {
    for (int64_t i = lane; i < cnt; i += 64) { item_err[b + i] = bad; flags[b + i] = 0; }
    return;
  }
  int m[8], nx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    m[j] = j < P ? __builtin_amdgcn_readlane(vs, j) : 0;
    nx[j] = j < P ? __builtin_amdgcn_readlane(vs, 8 + j) : 0;
  }
  const int c0 = commit, t0 = term, r0 = role;
  const int32_t *lrow = s.log + (int64_t)slot * s.L;
  bool touched_mn = false;
  int H = commit;
  for (int64_t base = 0; base < cnt; base += 64) {
    if (base > 0 && base + lane < cnt) it = items[b + base + lane];
    const int nb = (int)min((int64_t)64, cnt - base);
    int myfl = 0, plo = 1, phi = 0;  // this lane's reply: flags and a1 range
    for (int k = 0; k < nb; ++k) {
      const int pr = __builtin_amdgcn_readlane(it.peer, k);
      const int rt = __builtin_amdgcn_readlane(it.reply_term, k);
      const int at = __builtin_amdgcn_readlane(it.args_term, k);
      const int ap = __builtin_amdgcn_readlane(it.args_prev_log_index, k);
      int fl = 0, nxp = 0;
#pragma unroll
      for (int j = 0; j < P; ++j) if (j == pr) nxp = nx[j];
      if (rt > term) {                                                   // :67-72
        term = rt; role = kFollower;
        fl |= MRAFT_F_STEPPED_DOWN;
      } else if (rt == term && role == kLeader && at == term && ap == nxp - 1) {  // :73-74
        fl |= MRAFT_F_APPLIED;
        touched_mn = true;
        if (__builtin_amdgcn_readlane(it.reply_success, k)) {
          const int mv = __builtin_amdgcn_readlane(it.args_n_entries, k) + ap;  // :76
          nxp = mv + 1;                                                  // :77
#pragma unroll
          for (int j = 0; j < P; ++j) if (j == pr) m[j] = mv;
          const int top = min(quorum_rt<P>(m, me), last);                // a1, :78
          if (top > H) {
            if (lane == k) { plo = H + 1; phi = top; }
            H = top;
          }
        } else {
          nxp = __builtin_amdgcn_readlane(it.reply_conflict_index, k);   // :82
        }
#pragma unroll
        for (int j = 0; j < P; ++j) if (j == pr) nx[j] = nxp;
        if (nxp < last + 1) fl |= MRAFT_F_NEED_MORE;                     // :84-86
      }
      if (lane == k) myfl = fl;
    }
    // The batch's a1 ranges: probe every top word at once, scan the rest.
    int x = -1;
    bool settled = false;
    if (plo <= phi) {
      const int pv = lrow[ring(phi - dummy + head, s.L)];
      if (pv == t0) x = phi;                                             // :98
      else settled = srt && pv < t0;
    }
    unsigned long long pend = __ballot(plo < phi && x < 0 && !settled);
    while (pend) {
      const int src = first_lane(pend);
      pend &= pend - 1;
      const int lo = __shfl(plo, src, 64), hi = __shfl(phi, src, 64) - 1;
      const int r = fold_scan_down_eq<kFoldScanU>(lrow, dummy, head, s.L, lo, hi, t0);  // lo - 1 if none
      if (lane == src && r >= lo) x = r;
    }
    if (x >= 0) myfl |= MRAFT_F_COMMITTED;                               // :99-100
    const unsigned long long fm = __ballot(x >= 0);
    if (fm) commit = __shfl(x, 63 - __builtin_clzll(fm), 64);           // the latest range that found one
    if (lane < nb) {
      flags[b + base + lane] = myfl;
      item_err[b + base + lane] = 0;
    }
  }
  if (term != t0 || role != r0) {
    if (lane == 0) {
      s.term[slot] = term; s.role[slot] = role; s.voted[slot] = -1;
      mark_persist(s, slot, MRAFT_PERSIST_STATE);                        // :72
    }
  }
  if (commit != c0 && lane == 0) s.commit[slot] = commit;
  if (touched_mn) {
    int om = 0, on = 0;
#pragma unroll
    for (int j = 0; j < P; ++j) if (lane == j) { om = m[j]; on = nx[j]; }
    if (lane < P) { s.match[mrow + lane] = om; s.next[mrow + lane] = on; }
  }
}

// a1's scans of the reply fold (raft_append_entry.go:89-105; the loop reads
// terms from the top of the range down to the first one equal to currentTerm),
// for the ranges k_fold's probes left open: wave per kFscanW replies, each
// pending range scanned with the whole wave from its top down, stopping at the
// first hit as Go does. Split from k_fold so the scans of every segment stream
// at once instead of behind each segment's chain of dependent loads (bounds ->
// replies -> replica state -> probe). A hit sets MRAFT_F_COMMITTED on its reply
// and raises the replica's commitIndex (atomicMax: several waves may hold
// ranges of one segment).
__device__ __forceinline__ void fold_scan_blocks(const Dev &s, const int4 *__restrict__ pend,
                                                 const unsigned *__restrict__ pcount, int32_t *__restrict__ flags,
                                                 int64_t bid, int64_t nblk) {
  const int lane = lane_id();
  const int64_t cnt = (int64_t)*pcount;  // k_fold's compact list: nothing pending, nothing to do
  const int L = s.L;
  for (int64_t b0 = bid * kFscanW; b0 < cnt; b0 += nblk * kFscanW) {
    const int64_t i = b0 + lane;
    // the record in one round trip: {lo, hi, slot, currentTerm}, {dummy,
    // head, reply index}
    int4 ra = make_int4(0, -1, 0, 0), rb = make_int4(0, 0, 0, 0);
    if (lane < kFscanW && i < cnt) {
      ra = pend[2 * i];
      rb = pend[2 * i + 1];
    }
    const int lo = ra.x, hi = ra.y;
    for (unsigned long long m = __ballot(hi >= lo); m; m &= m - 1) {
      const int k = first_lane(m);
      const int klo = __builtin_amdgcn_readlane(lo, k), khi = __builtin_amdgcn_readlane(hi, k);
      const int kslot = __builtin_amdgcn_readlane(ra.z, k), kt0 = __builtin_amdgcn_readlane(ra.w, k);
      const int kd = __builtin_amdgcn_readlane(rb.x, k), kh = __builtin_amdgcn_readlane(rb.y, k);
      const int x = fold_scan_down_eq<kFscanU>(s.log + (int64_t)kslot * L, kd, kh, L, klo, khi,
                                                                     kt0);  // klo - 1 if none
      if (lane == k && x >= klo) {
        flags[rb.z] |= MRAFT_F_COMMITTED;                                // :99-100
        atomicMax(&s.commit[kslot], x);
      }
    }
  }
}

// Lane groups of GW lanes (the wave as 64 / GW groups).
template <int GW>
__device__ __forceinline__ int gw_base() { return (int)(lane_id() & ~(unsigned)(GW - 1)); }
template <int GW>
__device__ __forceinline__ unsigned gw_mask(bool pred) {  // this lane's group's ballot, bit k = its lane k
  return (unsigned)((__ballot(pred) >> gw_base<GW>()) & ((1ull << GW) - 1));
}
template <int GW>
__device__ __forceinline__ int gw_bcast(int v, int k) { return __shfl(v, gw_base<GW>() + k, 64); }

// fold_segment for 64 / GW segments at once, one per GW-lane group: the same
// statements on per-group (not wave-uniform) values, so the segments' chains
// of dependent loads (bounds -> replies -> replica state -> probes) overlap in
// one wave. Only segments of at most GW replies: a wave whose segments include
// a longer one folds them one by one on all 64 lanes.
template <int P, int GW>
__device__ __forceinline__ void fold_groupw(const Dev &s, const mraft_ae_result *__restrict__ items,
                                            int64_t n_items, const int64_t *__restrict__ seg_begin, int64_t sg0,
                                            int64_t n_seg, const int32_t *__restrict__ seg_err,
                                            const unsigned long long *__restrict__ claim, uint32_t epoch,
                                            int32_t *__restrict__ flags, int32_t *__restrict__ item_err,
                                            int4 *__restrict__ pend, unsigned *__restrict__ pcount,
                                            unsigned *__restrict__ lcount, int64_t *__restrict__ llist) {
  static_assert(GW >= P && GW >= 7, "a group holds the replica's match / next rows and seven scalars");
  const int lane = lane_id(), gl = lane & (GW - 1);
  const int64_t sg = sg0 + lane / GW;
  const bool live = sg < n_seg;
  int64_t b = 0, e = 0;
  int bad = 0;
  if (live) {
    b = seg_begin ? seg_begin[sg] : sg;
    e = seg_begin ? seg_begin[sg + 1] : sg + 1;
    bad = seg_err[sg];  // the claim verdict: a bad segment's slot may be out of range
  }
  int cnt = (int)(e > b ? min(e - b, (int64_t)(GW + 1)) : 0);  // 0: nothing to fold (empty or inverted)
  {
    // a segment longer than a group goes to the long-segment list (the 64-lane
    // path, k_fold_tail: this kernel stays at 8 waves per SIMD); its group
    // folds nothing here
    const unsigned long long lm = __ballot(gl == 0 && cnt > GW);
    if (lm) {
      const int l0 = first_lane(lm);
      unsigned base = 0;
      if (lane == l0) base = atomicAdd(lcount, (unsigned)__popcll(lm));
      base = (unsigned)__shfl((int)base, l0, 64);
      if (gl == 0 && cnt > GW) llist[base + (unsigned)__popcll(lm & ((1ull << lane) - 1))] = sg;
    }
    if (cnt > GW) cnt = 0;
  }
  (void)n_items;
  mraft_ae_result it{};
  if (gl < cnt) {
    // 32-bit lane offset from an SGPR base, formed here (see uni_ptr)
    const int64_t b0 = (int64_t)(((uint64_t)(uint32_t)uni((int)((uint64_t)b >> 32)) << 32) |
                                 (uint32_t)uni((int)(uint32_t)(uint64_t)b));  // lane 0's b
    int64_t off = b - b0 + gl;
    asm volatile("" : "+v"(off));
    it = uni_ptr(items + b0)[off];
  }
  const int slot = gw_bcast<GW>(it.slot, 0);
  const int me = cnt ? slot % P : 0;
  const int64_t mrow = (int64_t)slot * P;
  // The replica's state, three independent loads per lane: lanes 0..P-1 of
  // the group matchIndex and nextIndex, lanes 0..5 the scalars.
  int va = 0, vn = 0, vb = 0;
  if (cnt && !bad) {
    if (gl < P) {
      va = s.match[mrow + gl];
      vn = s.next[mrow + gl];
    }
    const int32_t *src = gl == 0 ? s.term : gl == 1 ? s.role : gl == 2 ? s.commit : gl == 3 ? s.last
                         : gl == 4 ? s.dummy : gl == 5 ? s.head : gl == 6 ? s.srt : nullptr;
    if (src) vb = src[slot];
  }
  // a slot claimed by an earlier segment of the batch: rejected (k_fold's check)
  const unsigned long long cw = (cnt && !bad) ? claim[slot] : 0ull;
  if (cnt && !bad && ((uint32_t)cw != (uint32_t)(0xFFFFFFFFull - (uint64_t)sg) || (uint32_t)(cw >> 32) != epoch))
    bad = MRAFT_ITEM_DUP_SLOT;
  int term = gw_bcast<GW>(vb, 0), role = gw_bcast<GW>(vb, 1), commit = gw_bcast<GW>(vb, 2);
  const int last = gw_bcast<GW>(vb, 3), dummy = gw_bcast<GW>(vb, 4), head = gw_bcast<GW>(vb, 5);
  const int srt = gw_bcast<GW>(vb, 6);
  // (a segment that does not own its slot stays MRAFT_ITEM_DUP_SLOT: the
  // claim decides first, include/mraft.h)
  if (gw_mask<GW>(gl < cnt && (it.slot != slot || it.peer < 0 || it.peer >= P || it.peer == me ||
                               !reply_index_ok(it.args_prev_log_index, it.args_n_entries))) && !bad)
    bad = MRAFT_ITEM_BAD_SLOT;
  if (!bad && commit < dummy) bad = MRAFT_ITEM_BAD_STATE;
  if (bad) {
    if (gl < cnt) { item_err[b + gl] = bad; flags[b + gl] = 0; }
  }
  const bool go = cnt && !bad;
  int m[8], nx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    m[j] = j < P ? gw_bcast<GW>(va, j) : 0;
    nx[j] = j < P ? gw_bcast<GW>(vn, j) : 0;
  }
  const int c0 = commit, t0 = term, r0 = role;
  const int32_t *lrow = s.log + (int64_t)slot * s.L;
  bool touched_mn = false;
  int H = commit;
  int nmax = 0;
  for (int k = 0; k < GW; ++k)
    if (__ballot(go && k < cnt)) nmax = k + 1;
  int myfl = 0, plo = 1, phi = 0;  // this lane's reply: flags and a1 range
  for (int k = 0; k < nmax; ++k) {
    const int pr = gw_bcast<GW>(it.peer, k), rt = gw_bcast<GW>(it.reply_term, k);
    const int at = gw_bcast<GW>(it.args_term, k), ap = gw_bcast<GW>(it.args_prev_log_index, k);
    const int rs = gw_bcast<GW>(it.reply_success, k), rn = gw_bcast<GW>(it.args_n_entries, k);
    const int rci = gw_bcast<GW>(it.reply_conflict_index, k);
    if (go && k < cnt) {
      int fl = 0, nxp = 0;
#pragma unroll
      for (int j = 0; j < P; ++j) if (j == pr) nxp = nx[j];
      if (rt > term) {                                                   // :67-72
        term = rt; role = kFollower;
        fl |= MRAFT_F_STEPPED_DOWN;
      } else if (rt == term && role == kLeader && at == term && ap == nxp - 1) {  // :73-74
        fl |= MRAFT_F_APPLIED;
        touched_mn = true;
        if (rs) {
          const int mv = rn + ap;                                        // :76
          nxp = mv + 1;                                                  // :77
#pragma unroll
          for (int j = 0; j < P; ++j) if (j == pr) m[j] = mv;
          const int top = min(quorum_rt<P>(m, me), last);                // a1, :78
          if (top > H) {
            if (gl == k) { plo = H + 1; phi = top; }
            H = top;
          }
        } else {
          nxp = rci;                                                     // :82
        }
#pragma unroll
        for (int j = 0; j < P; ++j) if (j == pr) nx[j] = nxp;
        if (nxp < last + 1) fl |= MRAFT_F_NEED_MORE;                     // :84-86
      }
      if (gl == k) myfl = fl;
    }
  }
  // a1's ranges of each group: every top word probed at once, the others scanned
  // With sorted terms (include/mraft.h MRAFT_TERMS_SORTED) a top term below
  // currentTerm settles the range: no lower entry carries currentTerm.
  int x = -1;
  bool settled = false;
  if (go && plo <= phi) {
    const int pv = lrow[ring(phi - dummy + head, s.L)];
    if (pv == t0) x = phi;  // :98
    else settled = srt && pv < t0;
  }
  // the ranges whose top word differs are scanned by k_fold_tail, after this
  // launch: it ORs MRAFT_F_COMMITTED into the reply's flags and raises the
  // replica's commitIndex to the highest index it finds (the ranges of a
  // segment are disjoint and ascending, so "the latest range that found one"
  // is the maximum over all of them, probes included)
  push_pending(pend, pcount, go && plo + 1 <= phi && x < 0 && !settled, make_int4(plo, phi - 1, slot, t0),
               make_int4(dummy, head, (int)(b + gl), 0));
  if (go && x >= 0) myfl |= MRAFT_F_COMMITTED;                           // :99-100
  const unsigned fm = gw_mask<GW>(go && x >= 0);
  if (fm) commit = __shfl(x, gw_base<GW>() + 31 - __clz((int)fm), 64);   // the latest range that found one
  if (go && gl < cnt) {
    flags[b + gl] = myfl;
    item_err[b + gl] = 0;
  }
  if (go && gl == 0 && (term != t0 || role != r0)) {
    s.term[slot] = term; s.role[slot] = role; s.voted[slot] = -1;
    mark_persist(s, slot, MRAFT_PERSIST_STATE);                          // :72
  }
  if (go && gl == 0 && commit != c0) s.commit[slot] = commit;
  if (go && touched_mn) {
    int om = 0, on = 0;
#pragma unroll
    for (int j = 0; j < P; ++j) if (gl == j) { om = m[j]; on = nx[j]; }
    if (gl < P) { s.match[mrow + gl] = om; s.next[mrow + gl] = on; }
  }
}

template <int P>
__global__ __launch_bounds__(64, 8) void k_fold(Dev s, const mraft_ae_result *__restrict__ items,
                                                int64_t n_items, const int64_t *__restrict__ seg_begin, int64_t n_seg,
                                                const int32_t *__restrict__ seg_err,
                                                const unsigned long long *__restrict__ claim, uint32_t epoch,
                                                int32_t *__restrict__ flags, int32_t *__restrict__ item_err,
                                                int4 *__restrict__ pend, unsigned *__restrict__ pcount,
                                                unsigned *__restrict__ lcount, int64_t *__restrict__ llist) {
  // lane groups of GW lanes, one segment each (fold_groupw)
  constexpr int NG = kFoldGroups, GW = 64 / NG;
  if ((int64_t)gridDim.x * NG >= n_seg) {
    // each XCD a contiguous range of waves: neighbouring waves' segments
    // share the lines of the replica arrays in one L2
    const int64_t nb = gridDim.x, b = blockIdx.x, x = b & 7, per = nb >> 3, rem = nb & 7;
    const int64_t wb = x * per + min(x, rem) + (b >> 3);
    fold_groupw<P, GW>(s, items, n_items, seg_begin, NG * wb, n_seg, seg_err, claim, epoch, flags, item_err, pend,
                       pcount, lcount, llist);
    return;
  }
  for (int64_t sg0 = NG * (int64_t)blockIdx.x; sg0 < n_seg; sg0 += NG * (int64_t)gridDim.x)
    fold_groupw<P, GW>(s, items, n_items, seg_begin, sg0, n_seg, seg_err, claim, epoch, flags, item_err, pend,
                       pcount, lcount, llist);
}

// The fold's second launch: the first n_long workgroups fold the segments
// k_fold left for the 64-lane path (longer than a lane group), scanning their
// own ranges, the rest scan the ranges k_fold's probes left open. The two
// halves touch different replicas (one segment per replica slot, the
// claim), so they need no order between them: one kernel boundary fewer per
// fold call.
template <int P>
__global__ __launch_bounds__(64, 8) void k_fold_tail(Dev s, const mraft_ae_result *__restrict__ items,
                                                     const int64_t *__restrict__ seg_begin,
                                                     const int32_t *__restrict__ seg_err,
                                                     const unsigned long long *__restrict__ claim, uint32_t epoch,
                                                     int32_t *__restrict__ flags, int32_t *__restrict__ item_err,
                                                     const int4 *__restrict__ pend, const unsigned *__restrict__ pcount,
                                                     const unsigned *__restrict__ lcount,
                                                     const int64_t *__restrict__ llist, int n_long) {
  if ((int)blockIdx.x < n_long) {
    const int64_t cnt = (int64_t)*lcount;
    for (int64_t k = blockIdx.x; k < cnt; k += n_long)
      fold_segment<P>(s, items, seg_begin, llist[k], seg_err, claim, epoch, flags, item_err);
  } else {
    fold_scan_blocks(s, pend, pcount, flags, (int64_t)blockIdx.x - n_long, (int64_t)gridDim.x - n_long);
  }
}

// ---------------------------------------------------------------- Start
// The duplicate-slot check (k_claim_check's) is done here, on the claim word
// k_claim left: one launch fewer per Start call.
__global__ void k_start(Dev s, const int32_t *__restrict__ slots, const int32_t *__restrict__ counts,
                        int64_t n, int32_t *__restrict__ oi, int32_t *__restrict__ ot,
                        int32_t *__restrict__ ol, int32_t *__restrict__ err,
                        const unsigned long long *__restrict__ claim, uint32_t epoch) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  int idx = -1, term = -1, isl = 0;
  if (!err[i]) {
    const int sl = slots[i], k = counts ? counts[i] : 1;
    if (claim[sl] != (((unsigned long long)epoch << 32) | (0xFFFFFFFFull - (uint64_t)i))) {
      err[i] = MRAFT_ITEM_DUP_SLOT;
    } else if (k < 1) {
      err[i] = MRAFT_ITEM_BAD_SLOT;
    } else if (s.role[sl] == kLeader) {                                // raft.go:93-95
      const int last = s.last[sl], dummy = s.dummy[sl], t = s.term[sl], h = s.head[sl];
      if ((int64_t)last + k - dummy > (int64_t)s.L - 1 || (int64_t)last + k > (int64_t)INT32_MAX - 1) {
        err[i] = MRAFT_ITEM_LOG_FULL;
      } else {
        // terms_sorted: k entries of currentTerm after the last one
        if (last > dummy && s.log[(int64_t)sl * s.L + ring(last - dummy + h, s.L)] > t) s.srt[sl] = 0;
        for (int j = 1; j <= k; ++j) s.log[(int64_t)sl * s.L + ring(last + j - dummy + h, s.L)] = t;  // :96-100
        s.last[sl] = last + k;
        mark_persist(s, sl, MRAFT_PERSIST_STATE);                      // :101
        idx = last + 1; term = t; isl = 1;                             // :103
      }
    }
  }
  oi[i] = idx; ot[i] = term; ol[i] = isl;
}

// Start at every group's leader replica (mraft_start_and_tick on the full
// tick's path): slot g * P + leader_peer[g], counts[g] entries (0: none), the
// rules of k_start; a group whose leader_peer is out of range starts nothing
// (MRAFT_ITEM_BAD_SLOT when it asked for entries with leader_peer >= P).
__global__ void k_start_groups(Dev s, const int32_t *__restrict__ lpeer, StartIO sio) {
  const int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (g >= s.G) return;
  const int lp = lpeer[g], k = sio.counts[g];
  int idx = -1, term = -1, isl = 0, e = 0;
  if (lp >= 0 && lp < s.P) {
    const int64_t sl = g * s.P + lp;
    if (k < 0) {
      e = MRAFT_ITEM_BAD_SLOT;
    } else if (k > 0 && s.role[sl] == kLeader) {                        // raft.go:93-95
      const int last = s.last[sl], dummy = s.dummy[sl], t = s.term[sl], h = s.head[sl];
      if ((int64_t)last + k - dummy > (int64_t)s.L - 1 || (int64_t)last + k > (int64_t)INT32_MAX - 1) {
        e = MRAFT_ITEM_LOG_FULL;
      } else {
        if (last > dummy && s.log[sl * s.L + ring(last - dummy + h, s.L)] > t) s.srt[sl] = 0;
        for (int j = 1; j <= k; ++j) s.log[sl * s.L + ring(last + j - dummy + h, s.L)] = t;  // :96-100
        s.last[sl] = last + k;
        mark_persist(s, sl, MRAFT_PERSIST_STATE);                        // :101
        idx = last + 1; term = t; isl = 1;                               // :103
      }
    }
  } else if (lp >= s.P && k != 0) {
    e = MRAFT_ITEM_BAD_SLOT;
  }
  sio.oi[g] = idx; sio.ot[g] = term; sio.ol[g] = isl; sio.err[g] = e;
}

// ---------------------------------------------------------------- applier
__global__ void k_collect_apply(Dev s, int32_t *__restrict__ from, int32_t *__restrict__ to,
                                int32_t *__restrict__ snap_index, int32_t *__restrict__ snap_term) {
  const int64_t gp = (int64_t)s.G * s.P;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < gp;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (snap_index) {                                                  // raft.go:168-177
      const bool hs = s.hsnap[i] != 0;
      snap_index[i] = hs ? s.dummy[i] : -1;
      snap_term[i] = hs ? s.log[i * s.L + s.head[i]] : 0;              // dummyTerm
      if (hs) s.hsnap[i] = 0;
    }
    const int la = s.applied[i], ci = s.commit[i];
    from[i] = la + 1;                                                  // raft.go:179-190
    to[i] = ci;
    if (ci > la) s.applied[i] = ci;                                    // :200
  }
}

// Compacted applier: slots with a message to send, ascending, in three
// launches (per-block counts, one-workgroup exclusive scan, emit). `snaps`:
// the caller takes SnapshotValid messages (hasSnapshot counts and is
// cleared); without, only commitIndex > lastApplied counts and hasSnapshot
// is left for a later call that takes them (as mraft_collect_apply does).
__global__ __launch_bounds__(256) void k_apply_count(Dev s, int32_t *__restrict__ bcnt, int snaps) {
  const int64_t gp = (int64_t)s.G * s.P;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const bool pend = i < gp && ((snaps && s.hsnap[i] != 0) || s.commit[i] > s.applied[i]);
  const unsigned long long m = __ballot(pend);
  __shared__ int wc[4];
  if (lane_id() == 0) wc[threadIdx.x >> 6] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) bcnt[blockIdx.x] = wc[0] + wc[1] + wc[2] + wc[3];
}

__global__ __launch_bounds__(1024) void k_apply_scan(int32_t *__restrict__ bcnt, int64_t nb,
                                                     int64_t *__restrict__ total) {
  __shared__ int64_t part[1024];
  int64_t carry = 0;
  for (int64_t base = 0; base < nb; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const int64_t v = i < nb ? bcnt[i] : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
      const int64_t add = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0;
      __syncthreads();
      part[threadIdx.x] += add;
      __syncthreads();
    }
    if (i < nb) bcnt[i] = (int32_t)(carry + part[threadIdx.x] - v);  // exclusive offset
    const int64_t chunk = part[1023];
    __syncthreads();
    carry += chunk;
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(256) void k_apply_emit(Dev s, const int32_t *__restrict__ boff, int64_t cap,
                                                    int32_t *__restrict__ oslot, int32_t *__restrict__ osi,
                                                    int32_t *__restrict__ ost, int32_t *__restrict__ ofrom,
                                                    int32_t *__restrict__ oto) {
  const int64_t gp = (int64_t)s.G * s.P;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  int la = 0, ci = 0, hs = 0;
  if (i < gp) { la = s.applied[i]; ci = s.commit[i]; hs = osi ? s.hsnap[i] : 0; }
  const bool pend = i < gp && (hs != 0 || ci > la);
  const unsigned long long m = __ballot(pend);
  __shared__ int wc[4];
  if (lane_id() == 0) wc[threadIdx.x >> 6] = __popcll(m);
  __syncthreads();
  const int w = threadIdx.x >> 6;
  int off = boff[blockIdx.x];
  for (int k = 0; k < w; ++k) off += wc[k];
  off += __popcll(m & ((1ull << lane_id()) - 1));
  if (pend && off < cap) {
    oslot[off] = (int32_t)i;
    if (osi) {
      osi[off] = hs ? s.dummy[i] : -1;                                 // raft.go:168-177
      ost[off] = hs ? s.log[i * s.L + s.head[i]] : 0;                  // dummyTerm
      if (hs) s.hsnap[i] = 0;
    }
    ofrom[off] = la + 1;                                               // raft.go:179-190
    oto[off] = ci;
    if (ci > la) s.applied[i] = ci;                                    // :200
  }
}

// ---------------------------------------------------------------- snapshots
// Snapshot (raft_snapshot.go:3-13): wave per item.
// Snapshot: setLogs(sliceFrom(index)) (raft_snapshot.go:10, raft_log.go:18-21,
// 75-77) is an O(1) rebase of the ring — the head moves to the entry at
// `index`, which becomes the dummy with its own term; no term moves.
__global__ __launch_bounds__(256) void k_snapshot(Dev s, const int32_t *__restrict__ slots,
                                                  const int32_t *__restrict__ index, int64_t n,
                                                  int32_t *__restrict__ err) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n || err[i]) return;
  const int sl = slots[i], x = index[i];
  const int d = s.dummy[sl], last = s.last[sl];
  if (x <= d) return;                                                  // :6-9
  if (x > last) {                                                      // sliceFrom panics
    err[i] = MRAFT_ITEM_PREV_BEYOND_LAST;
    return;
  }
  s.head[sl] = ring(s.head[sl] + (x - d), s.L);                        // :10
  s.dummy[sl] = x;
  mark_persist(s, sl, MRAFT_PERSIST_STATE | MRAFT_PERSIST_SNAPSHOT);    // :12
}

// appendOneRound's snapshot branch (raft_append_entry.go:27-34).
__global__ void k_gather_is(Dev s, const int32_t *__restrict__ slots, const int32_t *__restrict__ peers,
                            int64_t n, mraft_is_args *__restrict__ out, int32_t *__restrict__ err) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int P = s.P;
  const int64_t gp = (int64_t)s.G * P;
  mraft_is_args a = {-1, 0, 0, 0, 0};
  int e = 0;
  const int slot = slots[i], peer = peers[i];
  if (slot < 0 || slot >= gp || peer < 0 || peer >= P || peer == slot % P) {
    e = MRAFT_ITEM_BAD_SLOT;
  } else if (s.role[slot] != kLeader) {
    e = MRAFT_ITEM_BAD_STATE;
  } else if (s.next[(int64_t)slot * P + peer] - 1 < s.dummy[slot]) {
    a.slot = (slot / P) * P + peer;
    a.term = s.term[slot];                                             // :29
    a.leader_id = slot % P;                                            // :30
    a.last_included_index = s.dummy[slot];                             // :31
    a.last_included_term = s.log[(int64_t)slot * s.L + s.head[slot]];  // :32 dummyTerm
  }
  out[i] = a;
  err[i] = e;
}

// HandleInstallSnapshot (raft_snapshot.go:15-54): wave per item.
// HandleInstallSnapshot (raft_snapshot.go:15-54), thread per item. Installing
// by sliceFrom(LastIncludedIndex) (:38-40) is an O(1) ring rebase.
__global__ __launch_bounds__(256) void k_handle_is(Dev s, const mraft_is_args *__restrict__ args,
                                                   int64_t n, mraft_is_reply *__restrict__ rep,
                                                   int32_t *__restrict__ flags,
                                                   int32_t *__restrict__ err) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (err[i]) {
    rep[i] = mraft_is_reply{0, 0};
    flags[i] = 0;
    return;
  }
  const mraft_is_args a = args[i];
  if (a.last_included_index > INT32_MAX - 1) {  // past the Index domain (include/mraft.h): malformed
    rep[i] = mraft_is_reply{0, 0};
    flags[i] = 0;
    err[i] = MRAFT_ITEM_BAD_SLOT;
    return;
  }
  const int f = a.slot, fterm = s.term[f];
  int fl = 0;
  if (a.term < fterm) {                                                // :20-22
    rep[i] = mraft_is_reply{fterm, 0};
    flags[i] = 0;
    return;
  }
  const int lii = a.last_included_index;
  const int fcommit = s.commit[f];
  const bool install = lii > fcommit;                                  // :31-33
  const int fd = s.dummy[f], flast = s.last[f], fh = s.head[f];
  if (install && lii <= flast && lii < fd) {                           // sliceFrom panics
    rep[i] = mraft_is_reply{0, 0};
    flags[i] = 0;
    err[i] = MRAFT_ITEM_BELOW_DUMMY;
    return;
  }
  if (a.term > fterm) { s.term[f] = a.term; s.voted[f] = -1; }         // :23-26
  s.role[f] = kFollower;                                               // :28
  if (install) {
    // :35-37 a new log [dummy] keeps its head; :38-40 sliceFrom moves it
    const int nh = lii > flast ? fh : ring(fh + (lii - fd), s.L);
    s.log[(int64_t)f * s.L + nh] = a.last_included_term;               // :44-45
    if (lii > flast) { s.last[f] = lii; s.srt[f] = 1; }                // [dummy] only
    else s.head[f] = nh;                                               // a suffix: terms_sorted unchanged
    s.hsnap[f] = 1;                                                    // :52 hasSnapshot
    s.dummy[f] = lii;
    s.commit[f] = lii;                                                 // :42
    s.applied[f] = lii;                                                // :43
    fl = MRAFT_F_SNAPSHOT_INSTALLED;
  }
  mark_persist(s, f, (a.term > fterm ? MRAFT_PERSIST_STATE : 0) |     // :26
                         (install ? MRAFT_PERSIST_STATE | MRAFT_PERSIST_SNAPSHOT : 0));  // :47
  rep[i] = mraft_is_reply{a.term, 0};                                  // deferred reply.Term
  flags[i] = fl;
}

// processInstallSnapshotReply (raft_snapshot.go:56-69): lane per segment.
__global__ void k_process_is(Dev s, const mraft_is_result *__restrict__ items, int64_t n,
                             const int64_t *__restrict__ seg_begin, int64_t n_seg,
                             const int32_t *__restrict__ seg_err, int32_t *__restrict__ flags,
                             int32_t *__restrict__ item_err) {
  const int64_t sg = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (sg >= n_seg) return;
  const int64_t b = seg_begin ? seg_begin[sg] : sg, e = seg_begin ? seg_begin[sg + 1] : sg + 1;
  if (b >= e) return;
  const int P = s.P;
  const int slot = items[b].slot;
  int bad = seg_err[sg];
  if (!bad)
    for (int64_t i = b; i < e; ++i) {
      const mraft_is_result it = items[i];
      if (it.slot != slot || it.peer < 0 || it.peer >= P || it.peer == slot % P ||
          it.args_last_included_index > INT32_MAX - 1)  // (past the Index domain, include/mraft.h)
        bad = MRAFT_ITEM_BAD_SLOT;
    }
  if (bad) {
    for (int64_t i = b; i < e; ++i) { item_err[i] = bad; flags[i] = 0; }
    return;
  }
  int term = s.term[slot], role = s.role[slot];
  const int t0 = term;
  for (int64_t i = b; i < e; ++i) {
    const mraft_is_result it = items[i];
    int fl = 0;
    if (it.reply_term > term) {                                        // :59-64
      term = it.reply_term;
      role = kFollower;
      fl = MRAFT_F_STEPPED_DOWN;
    } else if (role == kLeader && it.args_term == term) {              // :65-68
      s.match[(int64_t)slot * P + it.peer] = it.args_last_included_index;
      s.next[(int64_t)slot * P + it.peer] = it.args_last_included_index + 1;
      fl = MRAFT_F_APPLIED;
    }
    flags[i] = fl;
    item_err[i] = 0;
  }
  if (term != t0) {
    s.term[slot] = term; s.role[slot] = role; s.voted[slot] = -1;
    mark_persist(s, slot, MRAFT_PERSIST_STATE);                        // :64
  }
}

// ---------------------------------------------------------------- a6 part 1
__global__ void k_start_election(Dev s, const int32_t *__restrict__ slots, int64_t n,
                                 mraft_rv_args *__restrict__ out, int32_t *__restrict__ err) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  mraft_rv_args a = {};
  if (!err[i]) {
    const int sl = slots[i];
    const int t = s.term[sl] + 1;                                      // raft_election.go:7
    const int last = s.last[sl];
    s.role[sl] = kCandidate;                                           // :6
    s.term[sl] = t;
    s.voted[sl] = sl % s.P;                                            // :14
    s.votes[sl] = 1;                                                   // :17
    mark_persist(s, sl, MRAFT_PERSIST_STATE);                          // :15
    a.slot = sl;
    a.term = t;
    a.candidate_id = sl % s.P;
    a.last_log_index = last;                                           // :12
    a.last_log_term = term_at(s, sl, s.dummy[sl], s.head[sl], last);  // :13
  }
  out[i] = a;
}

// ---------------------------------------------------------------- a5
__global__ void k_handle_rv(Dev s, const mraft_rv_args *__restrict__ args, int64_t n,
                            mraft_rv_reply *__restrict__ rep, int32_t *__restrict__ err) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  mraft_rv_reply r = {0, 0};
  if (!err[i]) {
    const mraft_rv_args a = args[i];
    const int v = a.slot;
    int term = s.term[v], voted = s.voted[v], role = s.role[v];
    const int t0 = term, v0 = voted, r0 = role;
    mark_persist(s, v, MRAFT_PERSIST_STATE);                           // deferred :57
    if (a.term < term) {                                               // raft_election.go:59-62
      r.term = term;
    } else {
      if (a.term > term) { role = kFollower; term = a.term; voted = -1; }  // :63-66
      r.term = term;                                                   // :67
      const int mylast = s.last[v];
      const int mylt = term_at(s, v, s.dummy[v], s.head[v], mylast);
      const bool up = a.last_log_term > mylt ||                        // raft_log.go:99-104
                      (mylt == a.last_log_term && a.last_log_index >= mylast);
      if ((voted == -1 || voted == a.candidate_id) && up) {            // :69-74
        voted = a.candidate_id;
        r.vote_granted = 1;
      }
      if (term != t0) s.term[v] = term;
      if (voted != v0) s.voted[v] = voted;
      if (role != r0) s.role[v] = role;
    }
  }
  rep[i] = r;
}

// ---------------------------------------------------------------- a6 part 2
__global__ void k_tally(Dev s, const mraft_rv_result *__restrict__ items, int64_t n,
                        const int64_t *__restrict__ seg_begin, int64_t n_seg,
                        const int32_t *__restrict__ seg_err, int32_t *__restrict__ flags,
                        int32_t *__restrict__ item_err) {
  const int64_t sg = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (sg >= n_seg) return;
  const int64_t b = seg_begin ? seg_begin[sg] : sg, e = seg_begin ? seg_begin[sg + 1] : sg + 1;
  if (b >= e) return;
  const int P = s.P;
  const int c = items[b].slot;
  int bad = seg_err[sg];
  if (!bad) {
    for (int64_t i = b; i < e; ++i) {
      const mraft_rv_result it = items[i];
      if (it.slot != c || it.peer < 0 || it.peer >= P || it.peer == c % P) bad = MRAFT_ITEM_BAD_SLOT;
    }
  }
  if (bad) {
    for (int64_t i = b; i < e; ++i) { item_err[i] = bad; flags[i] = 0; }
    return;
  }
  int term = s.term[c], role = s.role[c], votes = s.votes[c], voted = s.voted[c];
  const int t0 = term, r0 = role, vs0 = votes, vd0 = voted;
  bool lead = false, stepped = false;
  for (int64_t i = b; i < e; ++i) {
    const mraft_rv_result it = items[i];
    int fl = 0;
    if (term == it.args_term && role == kCandidate) {                  // raft_election.go:29
      if (it.vote_granted) {                                           // :30
        votes += 1;                                                    // :31
        if (votes > P / 2) {                                           // :32
          role = kLeader;                                              // :33
          lead = true;
          fl |= MRAFT_F_BECAME_LEADER;
        }
      } else if (it.reply_term > term) {                               // :42-45
        role = kFollower; term = it.reply_term; voted = -1;
        fl |= MRAFT_F_STEPPED_DOWN;
        stepped = true;
      }
    }
    flags[i] = fl;
    item_err[i] = 0;
  }
  if (term != t0) s.term[c] = term;
  if (role != r0) s.role[c] = role;
  if (votes != vs0) s.votes[c] = votes;
  if (voted != vd0) s.voted[c] = voted;
  if (stepped) mark_persist(s, c, MRAFT_PERSIST_STATE);                // :45
  if (lead) {                                                          // :34-38
    const int nx = s.last[c] + 1;
    for (int j = 0; j < P; ++j) { s.match[(int64_t)c * P + j] = 0; s.next[(int64_t)c * P + j] = nx; }
  }
}

// ---------------------------------------------------------------- persistence
// persist_dirty read-out (copy + clear): the slots the host must save.
__global__ void k_collect_persist(Dev s, int32_t *__restrict__ out) {
  const int64_t gp = (int64_t)s.G * s.P;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < gp;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int v = s.pdirty[i];
    out[i] = v;
    if (v) s.pdirty[i] = 0;
  }
}

// SaveState (raft.go:209-216), scalar part: lane per slot.
__global__ void k_read_persistent_hdr(Dev s, const int32_t *__restrict__ slots, int64_t n,
                                      mraft_persistent *__restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int sl = slots[i];
  mraft_persistent r = {};
  r.slot = sl;
  r.current_term = s.term[sl];
  r.voted_for = s.voted[sl];
  r.dummy_index = s.dummy[sl];
  r.last_index = s.last[sl];
  out[i] = r;
}

// SaveState, log part: wave per slot streams terms[0 .. last-dummy] of its row.
__global__ __launch_bounds__(256) void k_read_persistent_terms(Dev s,
                                                               const mraft_persistent *__restrict__ hdr,
                                                               int64_t n, int32_t *__restrict__ out) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  if (i >= n) return;
  const mraft_persistent r = hdr[i];
  wave_copy_from_ring(s.log + (int64_t)r.slot * s.L, r.dummy_index, s.head[r.slot], s.L, r.dummy_index,
                      out + r.terms_offset, r.last_index - r.dummy_index + 1);
}

// Make (raft.go:51-87) + readPersist (:217-235): wave per (validated) item.
__global__ __launch_bounds__(256) void k_restore(Dev s, const mraft_persistent *__restrict__ in,
                                                 int64_t n, const int32_t *__restrict__ terms,
                                                 const int32_t *__restrict__ err) {
  const int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  if (i >= n || err[i]) return;
  const mraft_persistent r = in[i];
  const int64_t sl = r.slot;
  wave_copy(terms + r.terms_offset, s.log + sl * s.L, r.last_index - r.dummy_index + 1);  // :233
  const bool srt = wave_terms_sorted(terms + r.terms_offset, 0, 0, INT32_MAX, 1, r.last_index - r.dummy_index);
  if (lane_id() == 0) {
    s.srt[sl] = srt ? 1 : 0;
    s.term[sl] = r.current_term;                                       // :231
    s.voted[sl] = r.voted_for;                                         // :232
    s.role[sl] = kFollower;                                            // :58
    s.dummy[sl] = r.dummy_index;
    s.head[sl] = 0;                                                    // a fresh raftLog
    s.hsnap[sl] = 0;                                                   // Make: no snapshot pending
    s.last[sl] = r.last_index;
    s.commit[sl] = r.dummy_index;                                      // :79
    s.applied[sl] = r.dummy_index;                                     // :80
    s.votes[sl] = 0;
    if (s.pdirty) s.pdirty[sl] = 0;
  }
  for (int j = lane_id(); j < s.P; j += 64) {                          // :64-65 make([]int, P)
    s.match[sl * s.P + j] = 0;
    s.next[sl * s.P + j] = 0;
  }
}

// terms_sorted of every replica from its log (mraft_load_state): wave per slot.
__global__ __launch_bounds__(256) void k_terms_sorted(Dev s) {
  const int64_t gp = (int64_t)s.G * s.P;
  for (int64_t sl = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; sl < gp;
       sl += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int d = s.dummy[sl], last = s.last[sl], h = s.head[sl];
    const bool ok = last - d < s.L && wave_terms_sorted(s.log + sl * s.L, d, h, s.L, d + 1, last);
    if (lane_id() == 0) s.srt[sl] = ok ? 1 : 0;
  }
}

// ---------------------------------------------------------------- GetState
__global__ void k_export(Dev s, const int32_t *__restrict__ lpeer, int32_t *__restrict__ commit,
                         int32_t *__restrict__ term_leader) {
  const int g = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (g >= s.G) return;
  int p = lpeer ? lpeer[g] : 0;
  if (p < 0 || p >= s.P) p = 0;
  const int64_t sl = (int64_t)g * s.P + p;
  commit[g] = s.commit[sl];
  term_leader[g] = (int32_t)(((uint32_t)s.term[sl] << 1) | (s.role[sl] == kLeader ? 1u : 0u));  // raft.go:237-246
}

}  // namespace

void launch_terms_sorted(const Dev &s, hipStream_t st) {
  const int64_t gp = (int64_t)s.G * s.P;
  int blocks = blocks_for(gp * 64);
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(k_terms_sorted, dim3(blocks), dim3(kBlock), 0, st, s);
}

void launch_init_state(const Dev &s, hipStream_t st) {
  const int64_t gp = (int64_t)s.G * s.P;
  int blocks = blocks_for(gp);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_init_state, dim3(blocks), dim3(kBlock), 0, st, s);
}

void launch_claim(const void *items, int64_t n, int stride, int slot_off, const int64_t *seg_begin,
                  int64_t gp, int peers, unsigned long long *claim, uint32_t epoch, int32_t *err,
                  hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_claim, dim3(blocks_for(n)), dim3(kBlock), 0, st, (const char *)items, n,
                     stride, slot_off, seg_begin, gp, peers, claim, epoch, err);
  hipLaunchKernelGGL(k_claim_check, dim3(blocks_for(n)), dim3(kBlock), 0, st, (const char *)items,
                     n, stride, slot_off, seg_begin, claim, epoch, err);
}

void launch_gather_args(const Dev &s, const int32_t *slots, const int32_t *peers, int64_t n,
                        mraft_ae_args *out, int32_t *err, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather_args, dim3(blocks_for(n, kMsgBlock)), dim3(kMsgBlock), 0, st, s, slots, peers, n,
                     out, err);
}

void launch_claim_ae(const mraft_ae_args *args, int64_t n, int64_t n_log, int L, int64_t gp, int ni,
                     unsigned long long *claim, uint32_t *srcmark, uint32_t epoch, int32_t *err, uint8_t *sethd,
                     unsigned long long *total, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_claim_ae, dim3(blocks_for(n, 64)), dim3(64), 0, st, args, n, n_log, L, gp,
                     ni < 1 ? 1 : ni > kAeHalo ? kAeHalo : ni, claim, srcmark, epoch, err, sethd, total);
}

// grid for k_handle_set: nb waves, each XCD a contiguous range (k_handle_set)
template <int NI, int MODE>
static void launch_set(const HsArgs &ka, int64_t nb, hipStream_t st) {
  hipLaunchKernelGGL((k_handle_set<NI, MODE>), dim3((unsigned)nb), dim3(64), 0, st, ka);
}

template <int NI>
static void launch_ref(const HsArgs &ka, int grid, hipStream_t st) {
  launch_set<NI, HM_MAIN>(ka, (ka.n + NI - 1) / NI, st);
  // the deferred launch, enqueued blind (its counts are on the device), on the
  // host's grid (from the last call's deferred count) that grid-strides over
  // the deferred items
  const int64_t g = max((int64_t)1, min(ka.n, (int64_t)grid));
  hipLaunchKernelGGL(k_handle_deferred, dim3((unsigned)g), dim3(64), 0, st, ka);
}

void launch_handle_ae_ref(const Dev &s, const mraft_ae_args *args, int64_t n, int ni, const unsigned long long *claim,
                          const uint32_t *srcmark, uint32_t epoch, int32_t *err, const uint8_t *sethd, int64_t *soff,
                          int64_t *defer, unsigned long long *total, int32_t *stage, int64_t stage_cap,
                          const AeDeferBufs &db, mraft_ae_reply *rep, mraft_ae_result *res, hipStream_t st) {
  if (n <= 0) return;
  HsArgs ka{};
  ka.s = s; ka.args = args; ka.n = n; ka.ent0 = nullptr; ka.n_ent0 = 0; ka.stage = stage; ka.stage_cap = stage_cap;
  ka.soff = soff; ka.sethd = sethd; ka.defer = defer; ka.total = total; ka.claim = claim; ka.srcmark = srcmark;
  ka.epoch = epoch; ka.fb = db.fb; ka.kin = db.kin;
  ka.cslot = db.cslot; ka.nslot = db.nslot; ka.cyc = db.cyc; ka.hint = db.hint; ka.rep = rep; ka.err = err;
  ka.res = res;
  switch (ni) {
    case 1: launch_ref<1>(ka, db.grid, st); break;
    case 2: launch_ref<2>(ka, db.grid, st); break;
    case 3: launch_ref<3>(ka, db.grid, st); break;
    case 4: launch_ref<4>(ka, db.grid, st); break;
    case 5: launch_ref<5>(ka, db.grid, st); break;
    case 6: launch_ref<6>(ka, db.grid, st); break;
    default: launch_ref<7>(ka, db.grid, st);
  }
}

void launch_handle_ae_host(const Dev &s, const mraft_ae_args *args, int64_t n, const int32_t *ent, int64_t n_ent,
                           mraft_ae_reply *rep, int32_t *err, mraft_ae_result *res, hipStream_t st) {
  if (n <= 0) return;
  HsArgs ka{};
  ka.s = s; ka.args = args; ka.n = n; ka.ent0 = ent; ka.n_ent0 = n_ent; ka.rep = rep; ka.err = err; ka.res = res;
  launch_set<1, HM_HOST>(ka, n, st);
}

void launch_fold(const Dev &s, const mraft_ae_result *items, int64_t n, const int64_t *seg_begin,
                 int64_t n_seg, int64_t gp, unsigned long long *claim, uint32_t epoch, int32_t *seg_err,
                 int32_t *flags, int32_t *item_err, void *scan_buf, hipStream_t st) {
  // one launch for the claims and the zeroed outputs, one for the fold, one
  // for the long segments and the a1 scans the fold's probes left open
  // (scan_buf: fold_scan_bytes(n, n_seg) of scratch)
  const int64_t nt = max(n_seg, n);
  if (nt <= 0 || !scan_buf) return;
  // scan_buf: pend [2 int4 per reply] | pcount | lcount | llist [n_seg int64]
  int4 *pend = (int4 *)scan_buf;                                      // 2 int4 per pending reply
  unsigned *pcount = (unsigned *)(pend + 2 * n);                      // the a1 list's length
  unsigned *lcount = pcount + 1;                                      // the long-segment list's length
  int64_t *llist = (int64_t *)(pend + 2 * n + 1);
  hipLaunchKernelGGL(k_claim_zero, dim3(blocks_for(nt, kMsgBlock)), dim3(kMsgBlock), 0, st, (const char *)items, n_seg,
                     (int)sizeof(mraft_ae_result), (int)offsetof(mraft_ae_result, slot), seg_begin, gp, claim,
                     epoch, seg_err, n, flags, item_err, pcount, lcount);
  if (n_seg <= 0) return;
  const int64_t waves = (n_seg + kFoldGroups - 1) / kFoldGroups;
  const dim3 gr((unsigned)min(waves, (int64_t)MRAFT_FOLD_GRID)), bl(64);
  // the tail's grids: both halves grid-stride over lists whose lengths are
  // read on the device
  const int nl = (int)min(n_seg, (int64_t)MRAFT_FOLD_TAIL_NL);
  const int64_t ns = min((n + kFscanW - 1) / kFscanW, (int64_t)MRAFT_FOLD_TAIL_NS);
  switch (s.P) {
#define MRAFT_FOLD_CASE(PP)                                                                              \
  case PP:                                                                                               \
    hipLaunchKernelGGL(k_fold<PP>, gr, bl, 0, st, s, items, n, seg_begin, n_seg, seg_err, claim, epoch, flags, \
                       item_err, pend, pcount, lcount, llist);                                           \
    hipLaunchKernelGGL(k_fold_tail<PP>, dim3((unsigned)(nl + ns)), bl, 0, st, s, items, seg_begin, seg_err, claim, \
                       epoch, flags, item_err, pend, pcount, lcount, llist, nl);                         \
    break;
    MRAFT_FOLD_CASE(1) MRAFT_FOLD_CASE(2) MRAFT_FOLD_CASE(3) MRAFT_FOLD_CASE(4)
    MRAFT_FOLD_CASE(5) MRAFT_FOLD_CASE(6) MRAFT_FOLD_CASE(7) MRAFT_FOLD_CASE(8)
#undef MRAFT_FOLD_CASE
    default: return;
  }
}

size_t fold_scan_bytes(int64_t n, int64_t n_seg) {
  // pend records, two counters, the long-segment list
  return 2 * sizeof(int4) * (size_t)(n > 0 ? n : 0) + sizeof(int4) + sizeof(int64_t) * (size_t)(n_seg > 0 ? n_seg : 1);
}

void launch_start(const Dev &s, const int32_t *slots, const int32_t *counts, int64_t n, int32_t *oi,
                  int32_t *ot, int32_t *ol, int32_t *err, const unsigned long long *claim, uint32_t epoch,
                  hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_claim, dim3(blocks_for(n)), dim3(kBlock), 0, st, (const char *)slots, n, (int)sizeof(int32_t),
                     0, (const int64_t *)nullptr, (int64_t)s.G * s.P, s.P, const_cast<unsigned long long *>(claim),
                     epoch, err);
  hipLaunchKernelGGL(k_start, dim3(blocks_for(n)), dim3(kBlock), 0, st, s, slots, counts, n, oi, ot,
                     ol, err, claim, epoch);
}

void launch_start_groups(const Dev &s, const int32_t *lpeer, const StartIO &sio, hipStream_t st) {
  if (s.G <= 0) return;
  hipLaunchKernelGGL(k_start_groups, dim3(blocks_for(s.G)), dim3(kBlock), 0, st, s, lpeer, sio);
}

void launch_collect_apply(const Dev &s, int32_t *from, int32_t *to, int32_t *snap_index, int32_t *snap_term,
                          hipStream_t st) {
  int blocks = blocks_for((int64_t)s.G * s.P);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_collect_apply, dim3(blocks), dim3(kBlock), 0, st, s, from, to, snap_index, snap_term);
}

void launch_collect_apply_compact(const Dev &s, int32_t *scratch_bcnt, int64_t cap, int32_t *oslot,
                                  int32_t *osnap_index, int32_t *osnap_term, int32_t *ofrom, int32_t *oto,
                                  int64_t *total, hipStream_t st) {
  const int64_t gp = (int64_t)s.G * s.P;
  const int64_t nb = (gp + 255) / 256;
  hipLaunchKernelGGL(k_apply_count, dim3((unsigned)nb), dim3(256), 0, st, s, scratch_bcnt,
                     osnap_index ? 1 : 0);
  hipLaunchKernelGGL(k_apply_scan, dim3(1), dim3(1024), 0, st, scratch_bcnt, nb, total);
  hipLaunchKernelGGL(k_apply_emit, dim3((unsigned)nb), dim3(256), 0, st, s, scratch_bcnt, cap, oslot,
                     osnap_index, osnap_term, ofrom, oto);
}

void launch_snapshot(const Dev &s, const int32_t *slots, const int32_t *index, int64_t n,
                     int32_t *err, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_snapshot, dim3(blocks_for(n)), dim3(kBlock), 0, st, s, slots, index, n, err);
}

void launch_gather_is(const Dev &s, const int32_t *slots, const int32_t *peers, int64_t n,
                      mraft_is_args *out, int32_t *err, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather_is, dim3(blocks_for(n)), dim3(kBlock), 0, st, s, slots, peers, n, out, err);
}

void launch_handle_is(const Dev &s, const mraft_is_args *args, int64_t n, mraft_is_reply *rep,
                      int32_t *flags, int32_t *err, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_handle_is, dim3(blocks_for(n)), dim3(kBlock), 0, st, s, args, n, rep,
                     flags, err);
}

void launch_process_is(const Dev &s, const mraft_is_result *items, int64_t n, const int64_t *seg_begin,
                       int64_t n_seg, int32_t *seg_err, int32_t *flags, int32_t *item_err,
                       hipStream_t st) {
  (void)n;
  if (n_seg <= 0) return;
  hipLaunchKernelGGL(k_process_is, dim3(blocks_for(n_seg, 64)), dim3(64), 0, st, s, items, n,
                     seg_begin, n_seg, seg_err, flags, item_err);
}

void launch_start_election(const Dev &s, const int32_t *slots, int64_t n, mraft_rv_args *out,
                           int32_t *err, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_start_election, dim3(blocks_for(n)), dim3(kBlock), 0, st, s, slots, n, out,
                     err);
}

void launch_handle_rv(const Dev &s, const mraft_rv_args *args, int64_t n, mraft_rv_reply *rep,
                      int32_t *err, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_handle_rv, dim3(blocks_for(n)), dim3(kBlock), 0, st, s, args, n, rep, err);
}

void launch_tally(const Dev &s, const mraft_rv_result *items, int64_t n, const int64_t *seg_begin,
                  int64_t n_seg, int32_t *seg_err, int32_t *flags, int32_t *item_err,
                  hipStream_t st) {
  (void)n;
  if (n_seg <= 0) return;
  hipLaunchKernelGGL(k_tally, dim3(blocks_for(n_seg, 64)), dim3(64), 0, st, s, items, n, seg_begin,
                     n_seg, seg_err, flags, item_err);
}

void launch_collect_persist(const Dev &s, int32_t *out, hipStream_t st) {
  int blocks = blocks_for((int64_t)s.G * s.P);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_collect_persist, dim3(blocks), dim3(kBlock), 0, st, s, out);
}

void launch_read_persistent_hdr(const Dev &s, const int32_t *slots, int64_t n,
                                mraft_persistent *out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_read_persistent_hdr, dim3(blocks_for(n)), dim3(kBlock), 0, st, s, slots, n, out);
}

void launch_read_persistent_terms(const Dev &s, const mraft_persistent *hdr, int64_t n,
                                  int32_t *out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_read_persistent_terms, dim3(blocks_for(n * 64)), dim3(kBlock), 0, st, s, hdr,
                     n, out);
}

void launch_restore(const Dev &s, const mraft_persistent *in, int64_t n, const int32_t *terms,
                    const int32_t *err, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_restore, dim3(blocks_for(n * 64)), dim3(kBlock), 0, st, s, in, n, terms, err);
}

void launch_export(const Dev &s, const int32_t *lpeer, int32_t *commit, int32_t *term_leader,
                   hipStream_t st) {
  hipLaunchKernelGGL(k_export, dim3(blocks_for(s.G)), dim3(kBlock), 0, st, s, lpeer, commit,
                     term_leader);
}

}  // namespace mraft

MRAFT_BOUNDS_READER(mraft_debug_bounds_kernels)
