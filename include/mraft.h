/*
 * mraft.h — C ABI of libmraft_hip.so, the MI355X-native batched Multi-Raft
 * decision engine.
 *
 * The reference (yusong-yan/MultiRaft, Go) has no FFI: its hot path sits behind
 * the Go package API of `raft` (src/raft/raft.go:51-104,237-246) and the RPC
 * handlers dispatched by labrpc reflection (`Raft.HandleAppendEntries`,
 * `Raft.HandleRequestVote`; src/labrpc/labrpc.go:457-506). Every entry point
 * below names the reference function it replaces (file:line, relative to the
 * reference's root). A cgo binding for a Go host is shown in INTEGRATION.md.
 *
 * Conventions:
 *  - Plain C types only; no exceptions cross the boundary. Every function
 *    returns an int status (MRAFT_OK = 0, negative = API error) and sets a
 *    thread-local message readable with mraft_last_error_string().
 *  - Where Go would panic (raft_append_entry.go:41-43, raft_log.go:56-58) the
 *    engine does not abort: the affected item/group is flagged in a per-item
 *    (or per-group) error/flag array and left unmodified; the CPU oracle flags
 *    the same items.
 *  - All integers are int32 on the device. Go's `int` is 64-bit; values must be
 *    in [-1, 2^31) and the engine rejects nothing silently. Raft Indexes
 *    (dummy, last, commit, matchIndex, an AppendEntries' last entry
 *    prevLogIndex + len(Entries)) are at most 2^31 - 2, so that nextIndex =
 *    Index + 1 is an int32: an AppendEntries past that is malformed
 *    (MRAFT_ITEM_BAD_SLOT) and a Start past it MRAFT_ITEM_LOG_FULL. Every
 *    Index up to that bound is handled exactly (the streaming
 *    pass runs on Indexes relative to its first one).
 *  - The engine owns its device state (hipMalloc) unless created with
 *    MRAFT_CREATE_NO_ALLOC and bound to caller-owned device buffers with
 *    mraft_bind_state(). Batch buffers belong to the caller and are read/written
 *    only for the duration of the call. `where` says whether batch pointers are
 *    host (MRAFT_HOST) or device (MRAFT_DEVICE) memory. With MRAFT_DEVICE the
 *    call is asynchronous on the engine's stream; with MRAFT_HOST it is
 *    synchronous (results are in the caller's buffers on return).
 *  - Concurrency: calls on one handle must be serialized by the caller (one
 *    handle per GPU, one stream per handle — plus, optionally, the engine's
 *    own tick-shard queues, mraft_set_tick_shards). Within a call, items addressed to
 *    the same replica slot are NOT allowed (the reference serializes them under
 *    rf.mu, raft.go:17): all but the lowest-indexed such item are rejected with
 *    MRAFT_ITEM_DUP_SLOT in item_err and the rest are processed. Host-side
 *    wrappers split batches into rounds of unique slots.
 *
 * Data model: G groups x P peers = G*P replica slots,
 * slot = group*P + peer ("me" of a slot is its peer index). Per slot the Raft
 * struct fields of raft.go:16-40 are stored struct-of-arrays; the log is a
 * ring of L terms per slot whose dummy entry (logs[0], raft_log.go:3-12) sits
 * at log_head: entry with Index i lives at
 *   log[slot*L + (log_head + i - dummy) mod L],   dummy <= i <= last,
 * so Snapshot / InstallSnapshot's sliceFrom (raft_snapshot.go:10,40;
 * raft_log.go:18-21,75-77) are O(1) rebases of log_head and dummyIndex, and a
 * replica holds at most L live entries (last - dummy + 1 <= L).
 * Commands never cross the boundary; they stay index-aligned on the host.
 */
#ifndef MRAFT_H
#define MRAFT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MRAFT_ABI_VERSION 6

/* Largest log capacity L (entries per replica ring): ring offsets are formed
 * as 32-bit byte offsets (4 * (position + 32) < 2^32). */
#define MRAFT_MAX_LOG_CAPACITY ((1 << 30) - 64)

/* Node states, raft_rpc.go:8-12 (values preserved). */
enum { MRAFT_LEADER = 1, MRAFT_CANDIDATE = 2, MRAFT_FOLLOWER = 3 };

/* Where batch pointers live. */
enum { MRAFT_HOST = 0, MRAFT_DEVICE = 1 };

/* mraft_create flags */
enum {
  MRAFT_CREATE_NO_ALLOC = 1,
  /* The engine's own stream is created on a hardware queue of its own
   * (hipExtStreamCreateWithCUMask with every CU) instead of taken from the HIP
   * runtime's pool, where it may share a queue with another stream and its
   * launches would then run after that stream's. Owned and destroyed by
   * mraft_destroy. */
  MRAFT_CREATE_DEDICATED_QUEUE = 2
};

/* Return status codes. */
enum {
  MRAFT_OK = 0,
  MRAFT_E_INVAL = -1,   /* bad argument (null pointer, out-of-range dims)       */
  MRAFT_E_NOMEM = -2,   /* device allocation failed                             */
  MRAFT_E_HIP = -3,     /* HIP runtime error                                    */
  MRAFT_E_NOSTATE = -4  /* engine has no state bound                            */
};

/* Per-item error codes (int32 item_err[]). Items with a non-zero code leave
 * the state they would have touched unmodified and produce no reply. */
enum {
  MRAFT_ITEM_OK = 0,
  MRAFT_ITEM_PREV_BEYOND_LAST = 1, /* a3 panic, raft_append_entry.go:41-43          */
  MRAFT_ITEM_BELOW_DUMMY = 2,      /* convertIndex panic, raft_log.go:56-58         */
  MRAFT_ITEM_LOG_FULL = 3,         /* append would exceed capacity L (engine limit) */
  MRAFT_ITEM_NEED_SNAPSHOT = 4,    /* prev < dummy: InstallSnapshot path,
                                      raft_append_entry.go:27-39 (not an AE)        */
  MRAFT_ITEM_DUP_SLOT = 5,         /* second item for the same slot in one call    */
  MRAFT_ITEM_BAD_SLOT = 6,         /* slot/peer out of range                        */
  MRAFT_ITEM_BAD_STATE = 7         /* commitIndex < dummyIndex (outside the
                                      reference's reachable states, raft.go:79)    */
};

/* Per-reply flags written by the fold (int32 out_flags[]). */
enum {
  MRAFT_F_NEED_MORE = 1,     /* tryAppendCond[peer].Signal(), raft_append_entry.go:84-86 */
  MRAFT_F_COMMITTED = 2,     /* applyCond.Signal(): commitIndex advanced, :99-100        */
  MRAFT_F_STEPPED_DOWN = 4,  /* adopted a higher term and became follower, :67-72        */
  MRAFT_F_BECAME_LEADER = 8, /* vote tally reached a majority, raft_election.go:32-38   */
  MRAFT_F_APPLIED = 16,      /* the reply passed the term/state/prev gate, :73-74       */
  MRAFT_F_SNAPSHOT_INSTALLED = 32 /* HandleInstallSnapshot replaced the log: hasSnapshot,
                                     raft_snapshot.go:38-52 (deliver the bytes)          */
};

/* Per-group flags written by mraft_replicate_tick (int32 group_flags[G]). */
enum {
  MRAFT_G_ACTIVE = 1,        /* the leader replica was a leader and sent AEs          */
  MRAFT_G_COMMITTED = 2,     /* leader commitIndex advanced                            */
  MRAFT_G_STEPPED_DOWN = 4,  /* leader stepped down on a higher reply term             */
  MRAFT_G_NEED_SNAPSHOT = 8, /* some peer had prev < dummy: InstallSnapshot sent        */
  MRAFT_G_ERROR = 16,        /* a3 would panic / bad state / log full: group skipped   */
  MRAFT_G_FOLLOWER_COMMIT = 32, /* some follower advanced its commitIndex              */
  MRAFT_G_LOG_FULL = 64,     /* a follower rejected its AE with MRAFT_ITEM_LOG_FULL    */
  MRAFT_G_ELECTED = 128,     /* mraft_election_rounds: some replica became leader     */
  MRAFT_G_SNAPSHOT_INSTALLED = 256, /* a follower installed the leader's snapshot       */
  MRAFT_G_FOLLOWER_PANIC = 512 /* a follower's handler would panic (InstallSnapshot below
                                  its own dummy, raft_log.go:56-58): message dropped    */
};

/* Per-slot state, struct-of-arrays (raft.go:16-40). Arrays of G*P int32 unless
 * noted. Any pointer may be NULL in mraft_store_state to skip that array. */
typedef struct {
  int32_t *current_term;  /* currentTerm                                    */
  int32_t *voted_for;     /* votedFor (-1 = none)                           */
  int32_t *state;         /* MRAFT_LEADER / CANDIDATE / FOLLOWER            */
  int32_t *commit_index;  /* commitIndex                                    */
  int32_t *last_applied;  /* lastApplied                                    */
  int32_t *dummy_index;   /* logs[0].Index (snapshot base), raft_log.go:33  */
  int32_t *last_index;    /* logs[len-1].Index, raft_log.go:44-46           */
  int32_t *granted_votes; /* StartElection's grantedVotes closure counter   */
  int32_t *log_term;      /* [G*P*L] ring: log[slot*L + (log_head + Index -
                             dummy) mod L] = Term                           */
  int32_t *match_index;   /* [G*P*P] matchIndex[slot*P + peer]              */
  int32_t *next_index;    /* [G*P*P] nextIndex[slot*P + peer]               */
  int32_t *persist_dirty; /* MRAFT_PERSIST_* bits: persist() call sites run
                             since the last mraft_collect_persist (below)  */
  int32_t *log_head;      /* ring position of the dummy entry, in [0, L)    */
  int32_t *has_snapshot;  /* hasSnapshot (raft.go:36,157,168-177): set by an
                             installing HandleInstallSnapshot
                             (raft_snapshot.go:49), consumed by the applier */
  int32_t *terms_sorted;  /* 1: the terms of the entries after the dummy,
                             Index dummy+1 .. last, are non-decreasing (a
                             proof the engine keeps, MRAFT_TERMS_SORTED
                             below); 0: not known */
} mraft_soa;

/* terms_sorted (engine bookkeeping, not a Raft field). The leader's commit
 * rule (advanceCommitIndexForLeader, raft_append_entry.go:89-105) looks for the
 * highest Index i <= min(M*, last) above commitIndex with term(i) ==
 * currentTerm, M* being the matchIndex order statistic. When the log's terms
 * never decrease, term(min(M*, last)) < currentTerm settles it — no lower entry
 * can carry currentTerm — so the engine reads that one term instead of Go's
 * downward loop (the decision is identical). Every Raft log the reference can
 * reach is sorted this way; the engine does not assume it, it keeps a proof
 * per replica:
 *   Make (mraft_create), InstallSnapshot installing a new log: 1;
 *   mraft_load_state, mraft_restore: computed from the terms;
 *   Start (raft.go:96-100): cleared when term(last) > currentTerm;
 *   HandleAppendEntries appending from Index k (truncate + append,
 *   raft_append_entry.go:149-155): set to the args' MRAFT_AE_ENTRIES_SORTED
 *   flag when k - 1 is the dummy (the new entries are the whole log), else
 *   cleared unless that flag is set;
 *   Snapshot / InstallSnapshot's sliceFrom (a suffix of a sorted log is
 *   sorted): unchanged.
 * mraft_bind_state takes the caller's array as it is: 1 must only be set
 * where the terms are non-decreasing (0 everywhere is always correct). */
enum { MRAFT_TERMS_SORTED = 1 };

/* Persistence (SURVEY.md §5 "Checkpoint / resume", §8f #4). The reference
 * persists currentTerm, votedFor and the log (raft.go:205-216) at fixed call
 * sites; the engine ORs one of these bits into persist_dirty[slot] wherever
 * the reference would have called:
 *   persist()              -> MRAFT_PERSIST_STATE:
 *       Start (raft.go:101, leader only), processAppendEntriesReply step-down
 *       (raft_append_entry.go:72), HandleAppendEntries on every handled call
 *       (deferred, :111 — the stale-term reply included), StartElection
 *       (raft_election.go:15), the tally's step-down (:45), HandleRequestVote
 *       on every handled call (deferred, :57), HandleInstallSnapshot's term
 *       adoption (raft_snapshot.go:26), processInstallSnapshotReply's
 *       step-down (:64);
 *   SaveStateAndSnapshot() -> MRAFT_PERSIST_STATE | MRAFT_PERSIST_SNAPSHOT:
 *       Snapshot above dummyIndex (raft_snapshot.go:12, the service's bytes),
 *       HandleInstallSnapshot installing (:47, the leader's bytes).
 * Items the engine rejects (item_err != 0) mark nothing. */
enum { MRAFT_PERSIST_STATE = 1, MRAFT_PERSIST_SNAPSHOT = 2 };

/* The persistent part of one replica (SaveState, raft.go:209-216): the terms
 * of its log entries dummyIndex..lastIndex (the dummy entry first) are
 * terms[terms_offset .. terms_offset + last_index - dummy_index]. Commands
 * stay on the host, index-aligned. */
typedef struct {
  int32_t slot;
  int32_t current_term;
  int32_t voted_for;
  int32_t dummy_index;
  int32_t last_index;
  int32_t _pad;
  int64_t terms_offset;
} mraft_persistent;

/* AppendEntriesArgs, raft_rpc.go:55-62. Entries are passed by reference:
 * entry k (0 <= k < n_entries) has Index prev_log_index+1+k (as built by
 * appendOneRound, raft_append_entry.go:50-54) and Term
 * entry_terms[entries_offset + k]. `slot` is the receiving replica.
 * `flags` (not a Go field): MRAFT_AE_ENTRIES_SORTED when the terms
 * prev_log_term, entry 0, ..., entry n_entries-1 are non-decreasing, set by
 * mraft_gather_append_args from the leader's terms_sorted; 0 is always
 * correct. A host that ships args over the network forwards it unchanged. */
typedef struct {
  int32_t slot;
  int32_t term;
  int32_t leader_id;
  int32_t prev_log_index;
  int32_t prev_log_term;
  int32_t leader_commit;
  int32_t n_entries;
  int32_t flags;
  int64_t entries_offset;
} mraft_ae_args;

enum { MRAFT_AE_ENTRIES_SORTED = 1 };

/* AppendEntriesReply, raft_rpc.go:64-69 (`Conflict` is never set by the
 * reference and is always 0 here). */
typedef struct {
  int32_t term;
  int32_t success;
  int32_t conflict_index;
  int32_t conflict;
} mraft_ae_reply;

/* One AppendEntries reply delivered back to a leader replica, together with
 * the fields of the args it answers that processAppendEntriesReply reads
 * (raft_append_entry.go:66-88). */
typedef struct {
  int32_t slot;          /* leader replica                           */
  int32_t peer;          /* replying follower (0..P-1)               */
  int32_t args_term;
  int32_t args_prev_log_index;
  int32_t args_n_entries;
  int32_t reply_term;
  int32_t reply_success;
  int32_t reply_conflict_index;
} mraft_ae_result;

/* RequestVoteArgs, raft_rpc.go:71-76; `slot` is the receiving voter. */
typedef struct {
  int32_t slot;
  int32_t candidate_id;
  int32_t term;
  int32_t last_log_index;
  int32_t last_log_term;
} mraft_rv_args;

/* RequestVoteReply, raft_rpc.go:78-82 (`State` is never written: omitted). */
typedef struct {
  int32_t term;
  int32_t vote_granted;
} mraft_rv_reply;

/* One RequestVote reply delivered back to a candidate replica with the args
 * term it answers (raft_election.go:22-47). */
typedef struct {
  int32_t slot;       /* candidate replica */
  int32_t peer;       /* voter             */
  int32_t args_term;
  int32_t reply_term;
  int32_t vote_granted;
} mraft_rv_result;

/* InstallSnapshotArgs, raft_rpc.go:84-90 (the snapshot bytes stay on the
 * host); `slot` is the receiving replica. */
typedef struct {
  int32_t slot;
  int32_t term;
  int32_t leader_id;
  int32_t last_included_index;
  int32_t last_included_term;
} mraft_is_args;

/* InstallSnapshotReply, raft_rpc.go:92-95 (`Success` is never set by the
 * reference: always 0). */
typedef struct {
  int32_t term;
  int32_t success;
} mraft_is_reply;

/* One InstallSnapshot reply delivered back to a leader replica with the args
 * fields processInstallSnapshotReply reads (raft_snapshot.go:56-69). */
typedef struct {
  int32_t slot;
  int32_t peer;
  int32_t args_term;
  int32_t args_last_included_index;
  int32_t reply_term;
} mraft_is_result;

typedef struct mraft_engine mraft_engine;

/* ---- lifetime ---------------------------------------------------------- */

/* Replaces Make (raft.go:51-87) for G groups x P peers at once: allocates the
 * device SoA (unless MRAFT_CREATE_NO_ALLOC) and initialises every slot as Make
 * does: Follower, term 0, votedFor -1, dummy entry {0,0}, commit = lastApplied
 * = dummyIndex. peers in [1, 8]; log_capacity in [1, MRAFT_MAX_LOG_CAPACITY]. */
int mraft_create(int32_t groups, int32_t peers, int32_t log_capacity,
                 int32_t device, uint32_t flags, mraft_engine **out);
/* Replaces Kill (utility.go:9-19): waits for the engine's queues, frees device
 * state and every stream / queue the engine created. */
int mraft_destroy(mraft_engine *h);
/* Use a caller-provided hipStream_t (NULL = the engine's own stream); tick
 * shard launches still outstanding and the work already on the old stream are
 * ordered before the new stream's work (device-side waits). */
int mraft_set_stream(mraft_engine *h, void *hip_stream);
/* The engine stream. With tick shards (mraft_set_tick_shards) a tick's
 * launches run on the shard queues; this call first orders the engine stream
 * after every outstanding shard launch (a device-side wait, no host wait), so
 * work the caller enqueues on the returned stream — a copy of group_flags or
 * of the export words, an event — sees the tick's outputs. NULL when the
 * handle is null or that ordering fails (mraft_last_error_string). */
void *mraft_get_stream(mraft_engine *h);
/* Host wait for all work of the handle (engine stream and tick shards). */
int mraft_synchronize(mraft_engine *h);
int mraft_dims(const mraft_engine *h, int32_t *groups, int32_t *peers,
               int32_t *log_capacity);
const char *mraft_last_error_string(void);
int mraft_abi_version(void);

/* ---- state transfer (readPersist / SaveState analogues, raft.go:205-235) --- */

/* Copy a full state image into / out of the engine. All arrays required for
 * load (terms_sorted is recomputed from the logs on load, whatever the source
 * holds); NULL entries are skipped on store. */
int mraft_load_state(mraft_engine *h, const mraft_soa *src, int32_t where);
int mraft_store_state(mraft_engine *h, const mraft_soa *dst, int32_t where);
/* Device pointers of the state the engine currently works on (zero-copy). */
int mraft_state_view(mraft_engine *h, mraft_soa *out_device_ptrs);
/* Bind caller-owned device buffers (all required) as the working state
 * (terms_sorted as the caller holds it: see MRAFT_TERMS_SORTED). */
int mraft_bind_state(mraft_engine *h, const mraft_soa *device_ptrs);

/* ---- hot path: replication & commit ----------- */

/* a3, appendOneRound's args gather (raft_append_entry.go:20-54) for n
 * (slot, peer) pairs: fills args (entries by reference into the leader's own
 * log: entries_offset = leader slot * L + (prev + 1 - dummyIndex), the
 * logical position of the first entry in that replica's ring) and item_err (NEED_SNAPSHOT, PREV_BEYOND_LAST, or
 * MRAFT_ITEM_BAD_STATE when the slot is not a leader — appendOneRound returns
 * without sending, :22-25). */
int mraft_gather_append_args(mraft_engine *h, const int32_t *slots,
                             const int32_t *peers, int64_t n,
                             mraft_ae_args *out_args, int32_t *item_err,
                             int32_t where);

/* a4, HandleAppendEntries (raft_append_entry.go:108-162 with matchLog,
 * raft_log.go:92-96) for n items at distinct slots. entry_terms holds the
 * entries' terms (n_entry_terms >= 0 words; pass NULL to read entries by reference
 * from the engine's own log, as produced by mraft_gather_append_args: every
 * item then sees the log as it was before the call, like the reference's copy
 * of args.Entries at gather time, raft_append_entry.go:50-54). By reference,
 * consecutive items reading the same entries (one leader's messages to its
 * followers, as the gather lays them out) are served together, reading the
 * entries once; an item whose own row another item of the call reads runs
 * after the others (deferred), from a staged copy of its entries when its
 * source row is written in this call too. Every count this takes stays on the
 * device: with MRAFT_DEVICE the call enqueues its launches and returns without
 * waiting (calls may be enqueued back to back with no host synchronisation;
 * a batch larger than any before grows the engine's buffers in stream order,
 * without waiting either). n <= 2^31 - 1.
 * Staged entries use the engine's stage (mraft_set_stage_capacity); a batch
 * that needs more runs its deferred items in an order that needs no stage
 * (slower), with the same results. */
int mraft_handle_append_entries(mraft_engine *h, const mraft_ae_args *args,
                                int64_t n, const int32_t *entry_terms,
                                int64_t n_entry_terms, mraft_ae_reply *replies,
                                int32_t *item_err, int32_t where);

/* mraft_handle_append_entries that also writes, per item, the reply record
 * its co-resident leader folds (results, n records, optional): slot = the
 * follower's group's replica args.leader_id, peer = the follower's peer
 * index, the args' term / prevLogIndex / entry count and the reply's term /
 * success / ConflictIndex — what mraft_process_append_replies takes, with no
 * host-side assembly when every replica of a group lives in this engine (a
 * Go host receiving replies over the network builds its own). Items with
 * item_err != 0 get slot = peer = -1 and must be left out of the fold's
 * segments. */
int mraft_handle_append_entries_ex(mraft_engine *h, const mraft_ae_args *args,
                                   int64_t n, const int32_t *entry_terms,
                                   int64_t n_entry_terms, mraft_ae_reply *replies,
                                   mraft_ae_result *results, int32_t *item_err,
                                   int32_t where);

/* Capacity, in entry words, of the device stage mraft_handle_append_entries
 * copies the entries of deferred by-reference items into (allocated on first
 * use), in eight equal stripes that the batch's deferred items fill by the
 * XCD their set ran on. A batch whose stripe needs more is still handled
 * exactly, in the ordered fallback (as is every batch when the stage cannot
 * be allocated).
 * words in [0, 2^31): that fixed capacity. MRAFT_STAGE_AUTO (the default,
 * from 4 Mi words = 16 MiB; ABI 6): after a batch that needed more, the calls
 * after it get a stage of 5/4 of that need — eight times its fullest
 * stripe's words — (stream-ordered growth, the device
 * publishes the need to a pinned word: no host wait), up to 2^31 - 1 words;
 * growth stops at the first allocation that fails. Returns MRAFT_OK;
 * mraft_get_stage_capacity returns the current capacity (-1: null handle). */
enum { MRAFT_STAGE_AUTO = -1 };
int mraft_set_stage_capacity(mraft_engine *h, int64_t words);
int64_t mraft_get_stage_capacity(const mraft_engine *h);

/* a2 + a1, processAppendEntriesReply + advanceCommitIndexForLeader
 * (raft_append_entry.go:66-105). Items are folded per segment in array order;
 * segment s = items [seg_begin[s], seg_begin[s+1]) all with the same leader
 * slot (distinct across segments). seg_begin == NULL means one item per
 * segment. out_flags[i] gets MRAFT_F_* bits for item i. A segment is rejected,
 * every item_err of it set, in this order: its first record's slot out of
 * range (MRAFT_ITEM_BAD_SLOT); an earlier non-empty segment names the same
 * slot (MRAFT_ITEM_DUP_SLOT, whatever that segment's own outcome); a record
 * of another slot or a bad peer, or one whose args_n_entries is negative or
 * ends past the Index domain, args_prev_log_index + args_n_entries >
 * 2^31 - 2 (MRAFT_ITEM_BAD_SLOT); commitIndex below
 * dummyIndex (MRAFT_ITEM_BAD_STATE). The same rule holds for
 * mraft_process_install_snapshot_replies and mraft_process_vote_replies
 * (without the last). */
int mraft_process_append_replies(mraft_engine *h, const mraft_ae_result *items,
                                 int64_t n, const int64_t *seg_begin,
                                 int64_t n_seg, int32_t *out_flags,
                                 int32_t *item_err, int32_t where);

/* Fused co-resident tick: for every group g with leader_peer[g] >= 0, the
 * leader replica runs appendOneRound for every other peer (a3): an
 * AppendEntries (entries read in place from the leader's log) or, when
 * nextIndex-1 < dummyIndex, an InstallSnapshot; each follower replica handles
 * its message (a4 / HandleInstallSnapshot) and the leader folds the replies
 * in peer order (a2 + a1 / processInstallSnapshotReply). Equivalent to the
 * sequence gather -> handle -> process on the same state.
 * group_flags (optional, [G]) gets MRAFT_G_* bits. */
int mraft_replicate_tick(mraft_engine *h, const int32_t *leader_peer,
                         int32_t *group_flags, int32_t where);

/* Tick group shards (one handle standing for many Raft instances, `Make`
 * raft.go:51-87, whose groups share nothing: raft.go:16-40). With shards >= 2
 * the engine creates that many hardware queues of its own (CU-masked streams:
 * every CU, or every CU the fan-in has not reserved, mraft_fanin_reserve_cus),
 * owned and destroyed by mraft_destroy, and every mraft_replicate_tick[_export]
 * splits the groups into `shards` contiguous ranges (shard s = groups
 * [G*s/S, G*(s+1)/S)), launching shard s on queue s. Each queue first waits for
 * the work already on the engine stream (the tick's inputs), but NOT for the
 * other shards: shard s's tick i+1 follows only its own tick i, so one shard's
 * last waves run beside another shard's steady state instead of the device
 * idling through a launch's ramp-down. Every other call (including a
 * host-buffer tick's copy-back, mraft_synchronize and a non-overlapped fan-in)
 * first orders the engine stream after the outstanding shard launches (a
 * device-side wait, no host wait); an overlapped fan-in waits for them on the
 * fan-in stream only. Decisions are identical to one launch (the groups are
 * independent). shards = 1 (the default) restores one launch on the engine
 * stream. Waits for all outstanding work first. shards in [1, 8], <= G. */
int mraft_set_tick_shards(mraft_engine *h, int32_t shards);
int32_t mraft_get_tick_shards(const mraft_engine *h);
/* The hipStream_t of tick shard `shard` (the engine stream when shards == 1;
 * NULL when out of range): for events that time or order against a shard. */
void *mraft_shard_stream(mraft_engine *h, int32_t shard);

/* Tick path (ABI 6). MRAFT_TICK_FULL: one wave per group, the streaming pass
 * of the fused tick. MRAFT_TICK_LIGHT: for a running
 * deployment's ticks (heartbeats and a few appended entries per leader): a
 * first launch settles, eight groups per wave, every group whose followers all
 * reply success without a compare (prevLogTerm matches; a heartbeat, or an
 * append at the follower's last Index of at most 64 entries that fits the
 * ring) and whose commitIndex settles at log[last]; a second launch runs every
 * other group through the full tick. Outputs and state are identical to
 * MRAFT_TICK_FULL for every state (the groups are independent). Applies to
 * mraft_replicate_tick[_export] with and without shards (each shard its own
 * pair of launches); mraft_replicate_tick_count always counts the full tick.
 * The second launch's grid follows the previous light tick's count (a pinned
 * word the device writes): a jump from few to many non-settling groups costs
 * one slow tick, never a wrong one. MRAFT_TICK_AUTO: per shard, the light
 * tick while the last completed light tick sent at most a quarter of the
 * groups to the full tick (or before any has completed), otherwise the full
 * tick with a light tick every 32nd to measure again (the counts reach the
 * host asynchronously: a choice may follow a count a few ticks old).
 * MRAFT_TICK_AUTO is the default. */
enum { MRAFT_TICK_FULL = 0, MRAFT_TICK_LIGHT = 1, MRAFT_TICK_AUTO = 2 };
int mraft_set_tick_mode(mraft_engine *h, int32_t mode);
int32_t mraft_get_tick_mode(const mraft_engine *h);  /* -1: null handle */
/* Groups the most recent completed MRAFT_TICK_LIGHT tick sent to the full
 * tick, summed over its shards (exact after mraft_synchronize); -1 before the
 * first light tick or for a null handle. */
int64_t mraft_tick_light_fallbacks(mraft_engine *h);

/* Start (raft.go:90-104) at every group's leader replica, then the tick, in
 * one call (ABI 6): for each group g with leader_peer[g] in [0, P),
 * counts[g] >= 1 entries are appended at replica g*P + leader_peer[g]
 * exactly as mraft_start would append them (counts[g] == 0: no Start;
 * counts[g] < 0: MRAFT_ITEM_BAD_SLOT), then mraft_replicate_tick runs on the
 * result. out_index / out_term / out_is_leader / item_err are per group (G
 * each), mraft_start's per-item outputs; a group whose leader_peer is out of
 * range starts nothing (-1, -1, 0; MRAFT_ITEM_BAD_SLOT when leader_peer >= P
 * and counts[g] != 0). Equivalent to mraft_start over those slots followed by
 * mraft_replicate_tick; when the light tick runs (MRAFT_TICK_LIGHT, or AUTO
 * choosing it) Start is done inside its first launch, otherwise as its own
 * launch before the full tick. group_flags optional. */
int mraft_start_and_tick(mraft_engine *h, const int32_t *leader_peer,
                         const int32_t *counts, int32_t *out_index,
                         int32_t *out_term, int32_t *out_is_leader,
                         int32_t *item_err, int32_t *group_flags,
                         int32_t where);

/* mraft_replicate_tick followed by mraft_export_group_status for the same
 * leader_peer, fused into the one launch (the words the shard router
 * all-gathers come out of the tick itself): commit[g] / term_leader[g] are
 * the post-tick GetState words of replica leader_peer[g] (replica 0 when
 * leader_peer[g] is out of range). */
int mraft_replicate_tick_export(mraft_engine *h, const int32_t *leader_peer,
                                int32_t *group_flags, int32_t *commit,
                                int32_t *term_leader, int32_t where);

/* Algorithmic word count of one mraft_replicate_tick on the current state
 * (DESIGN.md §4 definition; does not modify state): out_words[0] = words
 * read, out_words[1] = words written, out_words[2] = active groups. */
int mraft_replicate_tick_count(mraft_engine *h, const int32_t *leader_peer,
                               int64_t out_words[3], int32_t where);

/* Start (raft.go:90-104) for n items: if slots[i] is a leader, append
 * counts[i] >= 1 entries {Index: last+1.., Term: currentTerm} (Go appends one
 * per call; k consecutive calls give consecutive indices) and return the
 * first appended index, the term and is_leader = 1; otherwise -1, -1, 0
 * (:93-95). Capacity overflow: MRAFT_ITEM_LOG_FULL, nothing appended.
 * Commands stay on the host, index-aligned with the returned indices. */
int mraft_start(mraft_engine *h, const int32_t *slots, const int32_t *counts,
                int64_t n, int32_t *out_index, int32_t *out_term,
                int32_t *out_is_leader, int32_t *item_err, int32_t where);

/* Applier (raft.go:153-203): for every slot, in the order the reference
 * sends them on applyCh,
 *   1. when hasSnapshot is set (an InstallSnapshot installed since the last
 *      call, raft_snapshot.go:49): the SnapshotValid message (:168-177),
 *      out_snap_index = SnapshotIndex = dummyIndex, out_snap_term =
 *      SnapshotTerm = dummyTerm, and hasSnapshot is cleared; otherwise
 *      out_snap_index = -1 (the host delivers the snapshot bytes it saved);
 *   2. the CommandValid messages of the index range (lastApplied, commitIndex]
 *      = [out_from, out_to] (out_from > out_to when empty, :179-190), then
 *      lastApplied = max(lastApplied, commitIndex) (:200).
 * Arrays of G*P. out_snap_index / out_snap_term may both be NULL: no
 * snapshot messages, hasSnapshot untouched. The entries' terms are in
 * log_term; the host maps indices to its commands. */
int mraft_collect_apply(mraft_engine *h, int32_t *out_from, int32_t *out_to,
                        int32_t *out_snap_index, int32_t *out_snap_term,
                        int32_t where);

/* Applier, compacted: only the slots with a message to
 * send — hasSnapshot set or commitIndex > lastApplied — in ascending slot
 * order: out_slots[k]; the SnapshotValid message first when there is one
 * (out_snap_index[k] = dummyIndex, out_snap_term[k] = dummyTerm, else -1 / 0;
 * raft.go:168-177), then the entry range (out_from[k] - 1, out_to[k]] =
 * (lastApplied, commitIndex] (:179-190). *out_n = the number of such slots;
 * the first min(*out_n, cap) are written and only those clear hasSnapshot and
 * advance lastApplied to commitIndex (:200), so a caller with a small buffer
 * calls again for the rest. out_snap_index / out_snap_term may both be NULL:
 * then, as in mraft_collect_apply, no SnapshotValid message is taken —
 * only slots with commitIndex > lastApplied count and hasSnapshot stays set
 * for a later call that passes them. */
int mraft_collect_apply_compact(mraft_engine *h, int32_t *out_slots,
                                int32_t *out_snap_index, int32_t *out_snap_term,
                                int32_t *out_from, int32_t *out_to,
                                int64_t cap, int64_t *out_n, int32_t where);

/* ---- snapshots --------------------------------------- */

/* Snapshot (raft_snapshot.go:3-13) for n items: if index[i] > dummyIndex, the
 * log keeps [index, last] with the entry at `index` as the new dummy (the log
 * prefix is dropped; the service keeps the snapshot bytes). index > lastIndex
 * is a Go panic: MRAFT_ITEM_PREV_BEYOND_LAST. */
int mraft_snapshot(mraft_engine *h, const int32_t *slots, const int32_t *index,
                   int64_t n, int32_t *item_err, int32_t where);

/* a3's snapshot branch (raft_append_entry.go:27-34): for leader slots whose
 * nextIndex[peer]-1 < dummyIndex, the InstallSnapshot args
 * {currentTerm, me, dummyIndex, dummyTerm}; other items get
 * MRAFT_ITEM_BAD_STATE (not a leader, :22-25) or MRAFT_ITEM_OK with
 * args.slot = -1 (an AppendEntries is due instead). */
int mraft_gather_install_snapshot_args(mraft_engine *h, const int32_t *slots,
                                       const int32_t *peers, int64_t n,
                                       mraft_is_args *out_args,
                                       int32_t *item_err, int32_t where);

/* HandleInstallSnapshot (raft_snapshot.go:15-54) for n items at distinct
 * slots; out_flags[i] gets MRAFT_F_SNAPSHOT_INSTALLED when the log was
 * replaced (the host then delivers the snapshot to the service, raft.go:168-177).
 * A LastIncludedIndex in (commitIndex, lastIndex] but below the follower's own
 * dummyIndex makes Go's sliceFrom panic: MRAFT_ITEM_BELOW_DUMMY, no change.
 * A LastIncludedIndex past the Index domain (> 2^31 - 2) is malformed:
 * MRAFT_ITEM_BAD_SLOT (also in mraft_process_install_snapshot_replies). */
int mraft_handle_install_snapshot(mraft_engine *h, const mraft_is_args *args,
                                  int64_t n, mraft_is_reply *replies,
                                  int32_t *out_flags, int32_t *item_err,
                                  int32_t where);

/* processInstallSnapshotReply (raft_snapshot.go:56-69), segments as in
 * mraft_process_append_replies. */
int mraft_process_install_snapshot_replies(mraft_engine *h,
                                           const mraft_is_result *items,
                                           int64_t n, const int64_t *seg_begin,
                                           int64_t n_seg, int32_t *out_flags,
                                           int32_t *item_err, int32_t where);

/* ---- elections ------------------------------- */

/* StartElection (raft_election.go:4-15): state=Candidate, term++,
 * votedFor=me, grantedVotes=1, args from lastEntry (raft_log.go:50-53). */
int mraft_start_election(mraft_engine *h, const int32_t *slots, int64_t n,
                         mraft_rv_args *out_args, int32_t *item_err,
                         int32_t where);

/* HandleRequestVote (raft_election.go:54-77 with isLogUpToDate,
 * raft_log.go:99-104) for n items at distinct voter slots. */
int mraft_handle_request_vote(mraft_engine *h, const mraft_rv_args *args,
                              int64_t n, mraft_rv_reply *replies,
                              int32_t *item_err, int32_t where);

/* Vote tally closure (raft_election.go:22-47), segments as in
 * mraft_process_append_replies. On majority: Leader, matchIndex[*]=0,
 * nextIndex[*]=lastIndex+1 (:30-38). */
int mraft_process_vote_replies(mraft_engine *h, const mraft_rv_result *items,
                               int64_t n, const int64_t *seg_begin,
                               int64_t n_seg, int32_t *out_flags,
                               int32_t *item_err, int32_t where);

/* Election storm: R rounds in one launch. In round
 * r, every replica p of group g with bit p of cand_mask[r*G + g] set that is
 * not a leader times out (raft.go:109-114) and runs StartElection
 * (raft_election.go:4-15), in ascending peer order; then every RequestVote is
 * delivered (HandleRequestVote, :54-77), voter by voter in candidate order;
 * then every candidate tallies its replies in voter order (:22-47; on a
 * majority: Leader, matchIndex[*]=0, nextIndex[*]=lastIndex+1). No message
 * is lost. group_flags (optional, [G]) gets MRAFT_G_ELECTED /
 * MRAFT_G_STEPPED_DOWN. P <= 8 (one mask byte per group and round). */
int mraft_election_rounds(mraft_engine *h, const uint8_t *cand_mask,
                          int32_t rounds, int32_t *group_flags, int32_t where);

/* ---- persistence (raft.go:205-235, persister.go) ------------------------- */

/* out_bits[slot] = persist_dirty[slot] for all G*P slots, then clears them:
 * the slots whose raft state (and snapshot) the host must save now. */
int mraft_collect_persist(mraft_engine *h, int32_t *out_bits, int32_t where);

/* SaveState (raft.go:209-216) for n slots, host buffers, synchronous:
 * out[i] gets slot i's currentTerm, votedFor, dummyIndex, lastIndex and a
 * terms_offset into out_terms, where its last-dummy+1 log terms are packed in
 * slot order. If terms_cap is too small, out[] is still filled (so the caller
 * can size the buffer), nothing is copied and MRAFT_E_INVAL is returned. */
int mraft_read_persistent(mraft_engine *h, const int32_t *slots, int64_t n,
                          mraft_persistent *out, int32_t *out_terms,
                          int64_t terms_cap);

/* Crash + restart of n replicas: Make (raft.go:51-87) followed by
 * readPersist (:217-235) of the given persistent state (host buffers,
 * synchronous). Per slot: currentTerm, votedFor and the log from `in`;
 * state Follower; commitIndex = lastApplied = dummyIndex (:79-80);
 * matchIndex = nextIndex = 0; grantedVotes 0; persist_dirty 0. item_err:
 * MRAFT_ITEM_BAD_SLOT (slot out of range or last < dummy),
 * MRAFT_ITEM_LOG_FULL (more than L entries), MRAFT_ITEM_DUP_SLOT. */
int mraft_restore(mraft_engine *h, const mraft_persistent *in, int64_t n,
                  const int32_t *terms, int64_t n_terms, int32_t *item_err);

/* Host-only codec of one replica's persistent state (the bytes a Persister
 * holds, persister.go:39-64). Not gob (labgob.go): little-endian
 * "MRPS" | u32 version 1 | i64 currentTerm | i64 votedFor | i64 dummyIndex |
 * u32 count | count x i64 term (count = lastIndex - dummyIndex + 1; Go's int
 * is 64-bit on the wire). encode returns the byte size (or the size needed,
 * writing nothing, when cap is too small); decode returns MRAFT_OK, or
 * MRAFT_E_INVAL on a malformed buffer or terms_cap < count (terms_offset of
 * `out` is set to 0 and out->slot is left to the caller). */
int64_t mraft_encode_persistent(const mraft_persistent *in, const int32_t *terms,
                                uint8_t *out, int64_t cap);
int mraft_decode_persistent(const uint8_t *buf, int64_t len, mraft_persistent *out,
                            int32_t *terms, int64_t terms_cap);

/* ---- shard router (host-only) ---------------------------- */

/* key2shard (src/shardkv/client.go:22-29): first byte of the key modulo
 * nshards (0 for an empty key). Returns the shard, or MRAFT_E_INVAL. */
int mraft_key2shard(const char *key, int64_t len, int32_t nshards);

/* Config.ReAllocGID (src/shardctrler/common.go:87-132) in place: shards[s] is
 * the gid serving shard s, gids the configured groups (Config.Groups keys).
 * Shards of departed groups go to the least-loaded group, then shards move
 * from the most- to the least-loaded group until the loads differ by at most
 * one; ties break to the smallest gid (the reference sorts the keys), gid 0
 * is the invalid group. Deterministic. */
int mraft_realloc_gid(int32_t *shards, int32_t nshards, const int32_t *gids, int32_t ngroups);

/* ---- read-out (GetState, raft.go:237-246) -------------------------------- */

/* For each group g and its replica leader_peer[g] (or, with leader_peer NULL,
 * replica 0): commit[g] = commitIndex, term_leader[g] = currentTerm<<1 |
 * (state == Leader). These are the words the multi-GPU path all-gathers. */
int mraft_export_group_status(mraft_engine *h, const int32_t *leader_peer,
                              int32_t *commit, int32_t *term_leader,
                              int32_t where);

/* ---- multi-GPU fan-in: RCCL over xGMI ---------------------
 * Groups partition over the GPUs of a node (one engine handle and one process
 * per GPU); no decision reads another group. The only exchange is the shard
 * router's view of every group's GetState words, which replaces the host
 * polling of GetState()/commit progress by the services
 * (src/kvraft/server.go:114, src/shardctrler/server.go:154,
 * src/shardkv/client.go:68-100): once per tick every rank all-gathers its
 * [2*G] status block (commitIndex[0:G], currentTerm<<1|isLeader[G:2G], as
 * written by mraft_replicate_tick_export / mraft_export_group_status into the
 * two halves of one buffer) into a [nranks*2*G] rank-major buffer.
 *
 * The communicator is a plain RCCL ncclComm_t passed as void*: the host may
 * bring its own, or make one with mraft_comm_unique_id (on one rank) +
 * distribution of the 128 id bytes over its own control plane +
 * mraft_comm_init (on every rank). */
#define MRAFT_COMM_ID_BYTES 128

/* ncclGetUniqueId: the bootstrap id of a new communicator (one rank calls it
 * and ships the bytes to the others). */
int mraft_comm_unique_id(uint8_t out[MRAFT_COMM_ID_BYTES]);
/* ncclCommInitRank on the engine's device: *out_comm is an ncclComm_t. Every
 * rank must call it (collectively) with the same id. */
int mraft_comm_init(mraft_engine *h, int32_t nranks, int32_t rank,
                    const uint8_t id[MRAFT_COMM_ID_BYTES], void **out_comm);
int mraft_comm_destroy(void *comm);

/* mraft_allgather_status flags */
enum {
  /* Enqueue on the engine's fan-in stream behind everything already enqueued
   * on its stream (an event, no host wait): later work on the engine stream
   * (the next tick) does not wait for the gather. The caller must not reuse
   * `local`/`gathered` before mraft_fanin_synchronize or a later gather. */
  MRAFT_FANIN_OVERLAP = 1,
  /* As OVERLAP, but the caller has already ordered the fan-in stream
   * (mraft_fanin_stream) after the work that produces `local`, e.g. with
   * hipStreamWaitEvent on an event of its own: the call records no event on
   * the engine stream, so a host that already marks every tick (timing) adds
   * no second marker packet per tick. */
  MRAFT_FANIN_ORDERED = 2
};

/* All-gather of the [2*G] status words of every rank over `comm` (ncclAllGather,
 * int32): gathered[r*2*G + k] = rank r's local[k]. Device buffers
 * (MRAFT_DEVICE, asynchronous) or host buffers (MRAFT_HOST, staged,
 * synchronous; OVERLAP ignored). */
int mraft_allgather_status(mraft_engine *h, void *comm, const int32_t *local,
                           int32_t *gathered, int32_t where, uint32_t flags);
/* Wait for the fan-in stream. */
int mraft_fanin_synchronize(mraft_engine *h);
/* The fan-in stream (a hipStream_t), e.g. for events. */
void *mraft_fanin_stream(mraft_engine *h);
/* Reserve n_cus compute units for the fan-in: the engine's own stream (with
 * tick shards: every shard queue instead) becomes a stream whose kernels (the
 * tick) may use every CU but those, and the fan-in stream one limited to those,
 * so an overlapped gather does not queue for CU slots behind a tick that fills
 * the device. n_cus = 0 restores the unmasked streams. Replaces a stream set
 * with mraft_set_stream (one shard). Hardware queues the engine then owns: the
 * fan-in's, and the tick's (one, or one per shard). */
int mraft_fanin_reserve_cus(mraft_engine *h, int32_t n_cus);

#ifdef __cplusplus
}
#endif

#endif /* MRAFT_H */
