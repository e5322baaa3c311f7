/*
 * mraft_oracle.c — CPU restatement of yusong-yan/MultiRaft's Raft decision
 * logic (src/raft/ Go files), TEST INFRASTRUCTURE ONLY (see mraft_oracle.h).
 *
 * Every function follows the control flow of the Go function it cites,
 * statement by statement, including the reference's quirks (ConflictIndex
 * off-by-one, reply.Term = 0 on prev < dummy, follower commit against the whole
 * log's lastIndex, no ConflictTerm, matchIndex assigned not max-ed, a1's
 * downward O((last-commit)*P) loop). Where Go panics, the item is flagged in
 * item_err and the state it would touch is left unmodified.
 *
 * Go `int` is 64-bit; the state here is int32 like the device layout. Inputs
 * are restricted to [-1, 2^31) so results are identical in that range.
 */
#include "mraft_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Algorithmic word counting.                                 */
/* ------------------------------------------------------------------------ */

enum { A_TERM, A_VOTED, A_ROLE, A_COMMIT, A_APPLIED, A_DUMMY, A_LAST, A_VOTES,
       A_LOG, A_MATCH, A_NEXT, A_SORTED, A_COUNT };

static struct {
  int on;
  int64_t base[A_COUNT + 1];
  uint64_t *rd, *wr;
} cnt;

int ora_count_enable(ora_engine *e) {
  int64_t gp = (int64_t)e->G * e->P;
  int64_t sizes[A_COUNT] = {gp, gp, gp, gp, gp, gp, gp, gp,
                            gp * e->L, gp * e->P, gp * e->P, gp};
  int64_t b = 0;
  for (int a = 0; a < A_COUNT; ++a) { cnt.base[a] = b; b += sizes[a]; }
  cnt.base[A_COUNT] = b;
  free(cnt.rd); free(cnt.wr);
  int64_t nw = (b + 63) / 64;
  cnt.rd = (uint64_t *)calloc((size_t)nw, 8);
  cnt.wr = (uint64_t *)calloc((size_t)nw, 8);
  if (!cnt.rd || !cnt.wr) return MRAFT_E_NOMEM;
  cnt.on = 1;
  return MRAFT_OK;
}

void ora_count_disable(void) {
  cnt.on = 0;
  free(cnt.rd); free(cnt.wr);
  cnt.rd = cnt.wr = NULL;
}

void ora_count_result(int64_t out[2]) {
  out[0] = out[1] = 0;
  if (!cnt.rd) return;
  int64_t nw = (cnt.base[A_COUNT] + 63) / 64;
  for (int64_t i = 0; i < nw; ++i) {
    out[0] += __builtin_popcountll(cnt.rd[i]);
    out[1] += __builtin_popcountll(cnt.wr[i]);
  }
}

/* The same counts at a memory-line granularity: the lines (line_words int32
 * words each, counted from the start of every array — the device allocates
 * each array line-aligned and each log row is a whole number of lines) that
 * hold at least one counted word. out = {read lines, written lines} in
 * lines. Used to split measured HBM traffic into line granularity and
 * re-reads (tools/line_bound.py). */
void ora_count_result_lines(int32_t line_words, int64_t out[2]) {
  out[0] = out[1] = 0;
  if (!cnt.rd || line_words <= 0) return;
  for (int a = 0; a < A_COUNT; ++a) {
    for (int64_t l = cnt.base[a]; l < cnt.base[a + 1]; l += line_words) {
      int64_t e = l + line_words < cnt.base[a + 1] ? l + line_words : cnt.base[a + 1];
      int r = 0, w = 0;
      for (int64_t i = l; i < e && !(r && w); ++i) {
        r |= (int)((cnt.rd[i >> 6] >> (i & 63)) & 1);
        w |= (int)((cnt.wr[i >> 6] >> (i & 63)) & 1);
      }
      out[0] += r;
      out[1] += w;
    }
  }
}

/* The bitmaps themselves (read: write = 0, written: write = 1), bit i of
 * array a at ora_count_base(a) + i; ora_count_base(A_COUNT) = total words. */
const uint64_t *ora_count_bits(int32_t write) { return write ? cnt.wr : cnt.rd; }
int64_t ora_count_base(int32_t a) { return (a >= 0 && a <= A_COUNT) ? cnt.base[a] : -1; }

static inline void CR(int a, int64_t i) {
  if (cnt.on) { int64_t w = cnt.base[a] + i; cnt.rd[w >> 6] |= 1ull << (w & 63); }
}
static inline void CW(int a, int64_t i) {
  if (cnt.on) { int64_t w = cnt.base[a] + i; cnt.wr[w >> 6] |= 1ull << (w & 63); }
}

/* ------------------------------------------------------------------------ */
/* raftLog helpers, src/raft/raft_log.go                                     */
/* ------------------------------------------------------------------------ */

#define S (e->s)

/* A persist() (bits = MRAFT_PERSIST_STATE) or SaveStateAndSnapshot()
 * (| MRAFT_PERSIST_SNAPSHOT) call site of the reference ran for replica s
 * (raft.go:205-216; include/mraft.h lists the sites). Not an algorithmic
 * state word: never counted. */
static inline void persist(ora_engine *e, int64_t s, int32_t bits) {
  if (S.persist_dirty) S.persist_dirty[s] |= bits;
}

/* Position of the entry with Index `index` in the log array: the replica's
 * row is a ring of L terms whose dummy entry (logs[0], raft_log.go:3-12) sits
 * at log_head; convertIndex (raft_log.go:55-60) is index - dummyIndex, taken
 * modulo L from the head. The caller guarantees dummy <= index < dummy + L. */
static inline int64_t lpos(const ora_engine *e, int64_t slot, int32_t index) {
  int64_t k = (int64_t)index - S.dummy_index[slot] + S.log_head[slot];
  if (k >= e->L) k -= e->L;
  return slot * e->L + k;
}

/* getEntry(index).Term, raft_log.go:40-42 + convertIndex :55-60 (caller
 * guarantees index >= dummyIndex; the panic is handled by callers). */
static inline int32_t term_at(const ora_engine *e, int64_t slot, int32_t index) {
  return S.log_term[lpos(e, slot, index)];
}

/* n terms of slot's log from Index `index` on, in order (a ring may wrap). */
static void copy_terms(const ora_engine *e, int64_t slot, int32_t index, int32_t n, int32_t *out) {
  for (int32_t k = 0; k < n; ++k) out[k] = term_at(e, slot, index + k);
}

static inline int32_t imin(int32_t a, int32_t b) { return a < b ? a : b; } /* utility.go:41-46 */

/* terms_sorted (include/mraft.h MRAFT_TERMS_SORTED; engine bookkeeping, not a
 * Go field): whether the terms of Index dummy+1 .. last never decrease. The
 * oracle keeps it with the engine's rules (Make 1, load / restore computed,
 * Start, the AppendEntries append, InstallSnapshot's new log) so the states
 * compare equal; its own a1 (advance_commit) is Go's loop and never reads it. */
static int32_t sorted_after_dummy(const ora_engine *e, int64_t slot) {
  const int32_t d = S.dummy_index[slot], last = S.last_index[slot];
  for (int32_t i = d + 1; i < last; ++i)
    if (term_at(e, slot, i) > term_at(e, slot, i + 1)) return 0;
  return 1;
}

void ora_compute_terms_sorted(ora_engine *e) {
  const int64_t gp = (int64_t)e->G * e->P;
  for (int64_t s = 0; s < gp; ++s)
    S.terms_sorted[s] = (S.last_index[s] - S.dummy_index[s] < e->L) ? sorted_after_dummy(e, s) : 0;
}

/* Duplicate-slot claim: lowest item index wins (include/mraft.h). */
static int32_t *claim_slots(ora_engine *e, const int32_t *slot_of, int64_t n,
                            size_t stride_bytes, int32_t *item_err) {
  int64_t gp = (int64_t)e->G * e->P;
  int32_t *first = (int32_t *)malloc(sizeof(int32_t) * (size_t)(gp ? gp : 1));
  for (int64_t i = 0; i < gp; ++i) first[i] = -1;
  for (int64_t i = 0; i < n; ++i) {
    int32_t slot = *(const int32_t *)((const char *)slot_of + i * stride_bytes);
    if (slot < 0 || slot >= gp) { item_err[i] = MRAFT_ITEM_BAD_SLOT; continue; }
    if (first[slot] >= 0) { item_err[i] = MRAFT_ITEM_DUP_SLOT; continue; }
    first[slot] = (int32_t)i;
    item_err[i] = MRAFT_ITEM_OK;
  }
  return first;
}

/* The owner of every replica slot among a batch of reply segments: the lowest
 * non-empty segment whose first record names that slot (in range). Segments
 * are meant to name distinct slots (one per leader / candidate replica); a
 * later segment naming an owned slot is rejected with MRAFT_ITEM_DUP_SLOT
 * whatever the owner's own outcome (the engine claims slots before it checks
 * records). `slot_of` = the slot field of record 0, records `stride` bytes. */
static int64_t *segment_owners(ora_engine *e, const void *slot_of, size_t stride, int64_t n,
                               const int64_t *seg_begin, int64_t ns) {
  int64_t gp = (int64_t)e->G * e->P;
  int64_t *owner = (int64_t *)malloc(sizeof(int64_t) * (size_t)(gp ? gp : 1));
  for (int64_t i = 0; i < gp; ++i) owner[i] = -1;
  for (int64_t s = 0; s < ns; ++s) {
    int64_t b = seg_begin ? seg_begin[s] : s, en = seg_begin ? seg_begin[s + 1] : s + 1;
    if (b >= en || b < 0 || b >= n) continue;
    int32_t slot = *(const int32_t *)((const char *)slot_of + b * stride);
    if (slot >= 0 && slot < gp && owner[slot] < 0) owner[slot] = s;
  }
  return owner;
}

/* ------------------------------------------------------------------------ */
/* a3: appendOneRound args gather, raft_append_entry.go:20-54                 */
/* ------------------------------------------------------------------------ */

static int32_t gather_one(ora_engine *e, int32_t slot, int32_t peer,
                          mraft_ae_args *a) {
  int32_t P = e->P;
  if (peer < 0 || peer >= P || peer == slot % P) return MRAFT_ITEM_BAD_SLOT;
  if (S.state[slot] != MRAFT_LEADER) return MRAFT_ITEM_BAD_STATE;      /* :22-25 */
  int32_t prev = S.next_index[(int64_t)slot * P + peer] - 1;           /* :26 */
  if (prev < S.dummy_index[slot]) return MRAFT_ITEM_NEED_SNAPSHOT;     /* :27 */
  if (prev > S.last_index[slot]) return MRAFT_ITEM_PREV_BEYOND_LAST;   /* :41-43 */
  a->slot = (slot / P) * P + peer;
  a->leader_id = slot % P;                                             /* :46 */
  a->term = S.current_term[slot];                                      /* :47 */
  a->prev_log_index = prev;                                            /* :48 */
  a->prev_log_term = term_at(e, slot, prev);                           /* :49 */
  a->n_entries = S.last_index[slot] - prev;                            /* :50 */
  a->leader_commit = S.commit_index[slot];                             /* :51 */
  /* flags: prevLogTerm, entries non-decreasing (the leader's terms_sorted,
   * the dummy's own term compared explicitly) */
  a->flags = (S.terms_sorted[slot] && (prev > S.dummy_index[slot] || prev == S.last_index[slot] ||
                                       a->prev_log_term <= term_at(e, slot, prev + 1)))
                 ? MRAFT_AE_ENTRIES_SORTED : 0;
  a->entries_offset = (int64_t)slot * e->L + (prev + 1 - S.dummy_index[slot]); /* :54 */
  return MRAFT_ITEM_OK;
}

int ora_gather_append_args(ora_engine *e, const int32_t *slots,
                           const int32_t *peers, int64_t n,
                           mraft_ae_args *out, int32_t *item_err) {
  int64_t gp = (int64_t)e->G * e->P;
  for (int64_t i = 0; i < n; ++i) {
    memset(&out[i], 0, sizeof(out[i]));
    if (slots[i] < 0 || slots[i] >= gp) { item_err[i] = MRAFT_ITEM_BAD_SLOT; continue; }
    item_err[i] = gather_one(e, slots[i], peers[i], &out[i]);
  }
  return MRAFT_OK;
}

/* ------------------------------------------------------------------------ */
/* a4: HandleAppendEntries, raft_append_entry.go:108-162                      */
/* ------------------------------------------------------------------------ */

/* Whether an AppendEntries' MRAFT_AE_ENTRIES_SORTED claim holds: the terms
 * prevLogTerm, entry 0, ..., entry n-1 never decrease. The flag crosses the
 * network, so the engine honours it only where it holds (include/mraft.h
 * mraft_ae_args); a false claim counts as no flag. Engine bookkeeping for
 * terms_sorted, not a Go rule: the reference keeps no such proof. */
static int ae_flag_holds(const mraft_ae_args *a, const int32_t *ent) {
  if (!(a->flags & MRAFT_AE_ENTRIES_SORTED)) return 0;
  int32_t prev_t = a->prev_log_term;
  for (int32_t k = 0; k < a->n_entries; ++k) {
    if (ent[k] < prev_t) return 0;
    prev_t = ent[k];
  }
  return 1;
}

/* The Index domain (engine limit, include/mraft.h; Go's int has none): the
 * last entry's Index prev + n must leave room for nextIndex = Index + 1 in
 * int32, else the item is malformed (MRAFT_ITEM_BAD_SLOT). */
static int ae_index_ok(const mraft_ae_args *a) {
  return (int64_t)a->prev_log_index + a->n_entries <= (int64_t)INT32_MAX - 1;
}

/* ent = entries' terms (entry k has Index prev+1+k); cnt_src = the leader
 * replica whose log the entries were copied from (for counting its words), or
 * -1. */
static int32_t handle_ae_one(ora_engine *e, int32_t f, const mraft_ae_args *a,
                             const int32_t *ent, int64_t cnt_src,
                             mraft_ae_reply *r, int *follower_committed) {
  const int32_t L = e->L;
  const int32_t prev = a->prev_log_index, n = a->n_entries;
  memset(r, 0, sizeof(*r)); /* reply := new(AppendEntriesReply) */
  *follower_committed = 0;

  /* Capacity pre-check (engine limit, not a Go condition): would this item
   * reach the merge, find a mismatch and grow the log past L slots? Then it is
   * rejected before any mutation. Reads only. */
  if (a->term >= S.current_term[f] && prev >= S.dummy_index[f] &&
      prev <= S.last_index[f] && term_at(e, f, prev) == a->prev_log_term) {
    int32_t dummy = S.dummy_index[f], last = S.last_index[f];
    for (int32_t k = 0; k < n; ++k) {
      int32_t idx = prev + 1 + k;
      if (idx > last || term_at(e, f, idx) != ent[k]) {
        if ((int64_t)prev + n - dummy > (int64_t)L - 1) return MRAFT_ITEM_LOG_FULL;
        break;
      }
    }
  }

  persist(e, f, MRAFT_PERSIST_STATE);                                 /* defer rf.persist(), :111 */
  CR(A_TERM, f);
  if (a->term < S.current_term[f]) {                                  /* :112-115 */
    r->term = S.current_term[f]; r->success = 0;
    return MRAFT_ITEM_OK;
  }
  if (a->term > S.current_term[f]) {                                  /* :116-118 */
    S.current_term[f] = a->term; S.voted_for[f] = -1;
    CW(A_TERM, f); CW(A_VOTED, f);
  }
  S.state[f] = MRAFT_FOLLOWER;                                        /* :120 */
  CW(A_ROLE, f);

  CR(A_DUMMY, f);
  int32_t dummy = S.dummy_index[f];
  if (prev < dummy) {                                                 /* :123-127 */
    r->term = 0; r->success = 0; r->conflict_index = dummy + 1;
    return MRAFT_ITEM_OK;
  }
  /* matchLog, raft_log.go:92-96: Index <= lastIndex && Term == getEntry(Index).Term */
  CR(A_LAST, f);
  int32_t last = S.last_index[f];
  int match = 0;
  if (prev <= last) {
    CR(A_LOG, lpos(e, f, prev));
    match = (a->prev_log_term == term_at(e, f, prev));
  }
  if (!match) {                                                       /* :128-145 */
    r->term = S.current_term[f]; r->success = 0;
    if (prev > last) {
      r->conflict_index = last + 1;                                   /* :131-133 */
    } else {
      int32_t abandoned = term_at(e, f, prev);                        /* :137 */
      int32_t index = prev;                                           /* :138 */
      while (index > dummy + 1) {                                     /* :139-141 */
        CR(A_LOG, lpos(e, f, index));
        if (term_at(e, f, index) != abandoned) break;
        index--;
      }
      r->conflict_index = index;                                      /* :142 */
    }
    return MRAFT_ITEM_OK;
  }
  /* :149-155 — merge without blind truncation (non-FIFO guard). */
  for (int32_t k = 0; k < n; ++k) {
    int32_t index = prev + 1 + k;                                     /* entry.Index */
    int diff;
    if (index - dummy >= last - dummy + 1) {                          /* convertIndex >= len */
      diff = 1;
    } else {
      CR(A_LOG, lpos(e, f, index));
      if (cnt_src >= 0) CR(A_LOG, lpos(e, cnt_src, index));
      diff = (term_at(e, f, index) != ent[k]);
    }
    if (diff) {
      /* trunc(entry.Index) then append(args.Entries[k:]...), raft_log.go:62-75 */
      for (int32_t j = k; j < n; ++j) {
        int32_t idx = prev + 1 + j;
        if (cnt_src >= 0) CR(A_LOG, lpos(e, cnt_src, idx));
        S.log_term[lpos(e, f, idx)] = ent[j];
        CW(A_LOG, lpos(e, f, idx));
      }
      S.last_index[f] = prev + n;
      CW(A_LAST, f);
      /* terms_sorted: the args' flag; the new entries are the whole log when
       * the first appended Index is the dummy's successor */
      if (!ae_flag_holds(a, ent)) { S.terms_sorted[f] = 0; CW(A_SORTED, f); }
      else if (index == dummy + 1) { S.terms_sorted[f] = 1; CW(A_SORTED, f); }
      break;
    }
  }
  CR(A_COMMIT, f);
  if (a->leader_commit > S.commit_index[f]) {                         /* :157-160 */
    S.commit_index[f] = imin(a->leader_commit, S.last_index[f]);
    CW(A_COMMIT, f);
    *follower_committed = 1;
  }
  r->term = S.current_term[f]; r->success = 1;                        /* :161 */
  return MRAFT_ITEM_OK;
}

int ora_handle_append_entries(ora_engine *e, const mraft_ae_args *args,
                              int64_t n, const int32_t *entry_terms,
                              int64_t n_entry_terms, mraft_ae_reply *replies,
                              int32_t *item_err) {
  int32_t *first = claim_slots(e, &args[0].slot, n, sizeof(mraft_ae_args), item_err);
  const int32_t *src = entry_terms ? entry_terms : S.log_term;
  int64_t src_n = entry_terms ? n_entry_terms : (int64_t)e->G * e->P * e->L;
  /* Entries by reference into the engine's own log (entry_terms NULL, the
   * view mraft_gather_append_args hands out): the reference copies
   * args.Entries when it builds the message (appendOneRound,
   * raft_append_entry.go:50-54), before any handler runs, so every item reads
   * the log as it was before the batch — even when another item of the same
   * batch rewrites its source row (two leaders of one group). Stage them.
   * entries_offset is then slot * L + (Index - dummyIndex) of the first entry
   * in the source replica's log (mraft_gather_append_args), read through its
   * ring. */
  int32_t *staged = NULL;
  int64_t *soff = NULL;
  if (!entry_terms && n > 0) {
    soff = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    int64_t tot = 0;
    for (int64_t i = 0; i < n; ++i) {
      const mraft_ae_args *a = &args[i];
      soff[i] = -1;
      if (item_err[i] || a->n_entries < 0 || a->entries_offset < 0 || !ae_index_ok(a) ||
          (a->n_entries > 0 && a->entries_offset + a->n_entries > src_n) ||
          a->entries_offset % e->L + a->n_entries > e->L)
        continue;
      soff[i] = tot;
      tot += a->n_entries;
    }
    staged = (int32_t *)malloc(sizeof(int32_t) * (size_t)(tot > 0 ? tot : 1));
    for (int64_t i = 0; i < n; ++i)
      if (soff[i] >= 0 && args[i].n_entries > 0) {
        const int64_t ss = args[i].entries_offset / e->L;
        const int32_t k0 = (int32_t)(args[i].entries_offset % e->L);
        copy_terms(e, ss, S.dummy_index[ss] + k0, args[i].n_entries, staged + soff[i]);
      }
  }
  for (int64_t i = 0; i < n; ++i) {
    memset(&replies[i], 0, sizeof(replies[i]));
    if (item_err[i]) continue;
    const mraft_ae_args *a = &args[i];
    if (a->n_entries < 0 || a->entries_offset < 0 || !ae_index_ok(a) ||
        (a->n_entries > 0 && a->entries_offset + a->n_entries > src_n) ||
        (!entry_terms && a->entries_offset % e->L + a->n_entries > e->L)) {
      item_err[i] = MRAFT_ITEM_BAD_SLOT;
      continue;
    }
    int fc;
    item_err[i] = handle_ae_one(e, a->slot, a, staged ? staged + soff[i] : src + a->entries_offset, -1,
                                &replies[i], &fc);
  }
  free(staged);
  free(soff);
  free(first);
  return MRAFT_OK;
}

/* ------------------------------------------------------------------------ */
/* a1: advanceCommitIndexForLeader, raft_append_entry.go:89-105               */
/* ------------------------------------------------------------------------ */

static int advance_commit(ora_engine *e, int32_t slot) {
  const int32_t P = e->P, me = slot % P;
  const int32_t *match = &S.match_index[(int64_t)slot * P];
  for (int32_t i = S.last_index[slot]; i > S.commit_index[slot]; i--) {
    int32_t num = 0;
    for (int32_t j = 0; j < P; ++j)
      if (j != me && match[j] >= i) num++;
    /* Go evaluates getEntry(i) only when the count holds (&& short-circuit);
     * commit >= dummy is enforced by callers so i >= dummy here. */
    if (num + 1 > P / 2 && term_at(e, slot, i) == S.current_term[slot]) {
      S.commit_index[slot] = i;                                       /* :99 */
      return 1;                                                       /* applyCond.Signal */
    }
  }
  return 0;
}

/* h-th largest (h = P/2) of matchIndex[j != me]: the largest i whose count in
 * a1 reaches the quorum (used only for counting). */
static int32_t quorum_match(const ora_engine *e, int32_t slot) {
  const int32_t P = e->P, me = slot % P, h = P / 2;
  const int32_t *match = &S.match_index[(int64_t)slot * P];
  if (h == 0) return INT32_MAX;
  int32_t best = INT32_MIN;
  for (int32_t j = 0; j < P; ++j) {
    if (j == me) continue;
    int32_t c = 0;
    for (int32_t k = 0; k < P; ++k)
      if (k != me && match[k] >= match[j]) c++;
    if (c >= h && match[j] > best) best = match[j];
  }
  return best;
}

/* ------------------------------------------------------------------------ */
/* a2: processAppendEntriesReply, raft_append_entry.go:66-88                  */
/* ------------------------------------------------------------------------ */

static int32_t process_reply_one(ora_engine *e, int32_t slot, int32_t peer,
                                 int32_t args_term, int32_t args_prev,
                                 int32_t args_n, int32_t reply_term,
                                 int32_t reply_success, int32_t reply_ci,
                                 int32_t *mstar) {
  const int32_t P = e->P;
  int32_t flags = 0;
  int64_t pi = (int64_t)slot * P + peer;
  if (reply_term > S.current_term[slot]) {                            /* :67-72 */
    S.current_term[slot] = reply_term;
    S.voted_for[slot] = -1;
    S.state[slot] = MRAFT_FOLLOWER;
    CW(A_TERM, slot); CW(A_VOTED, slot); CW(A_ROLE, slot);
    persist(e, slot, MRAFT_PERSIST_STATE);                            /* :72 */
    flags |= MRAFT_F_STEPPED_DOWN;
  } else if (reply_term == S.current_term[slot] &&                    /* :73-74 */
             S.state[slot] == MRAFT_LEADER &&
             args_term == S.current_term[slot] &&
             args_prev == S.next_index[pi] - 1) {
    flags |= MRAFT_F_APPLIED;
    if (reply_success) {
      S.match_index[pi] = args_n + args_prev;                         /* :76 */
      S.next_index[pi] = S.match_index[pi] + 1;                       /* :77 */
      CW(A_MATCH, pi); CW(A_NEXT, pi);
      if (mstar) {
        int32_t m = quorum_match(e, slot);
        if (m > *mstar) *mstar = m;
      }
      if (advance_commit(e, slot)) flags |= MRAFT_F_COMMITTED;        /* :78 */
    } else {
      S.next_index[pi] = reply_ci;                                    /* :82 */
      CW(A_NEXT, pi);
    }
    if (S.next_index[pi] < S.last_index[slot] + 1)                    /* :84-86 */
      flags |= MRAFT_F_NEED_MORE;
  }
  return flags;
}

/* A reply record inside the Index domain (engine limit, include/mraft.h): the
 * entries it acknowledges end at args_prev_log_index + args_n_entries <=
 * 2^31 - 2 (matchIndex, and nextIndex = matchIndex + 1, stay int32), with a
 * non-negative count; else the record is malformed (MRAFT_ITEM_BAD_SLOT, the
 * segment rejected like one with a bad peer). */
static int reply_index_ok(const mraft_ae_result *it) {
  return it->args_n_entries >= 0 &&
         (int64_t)it->args_prev_log_index + it->args_n_entries <= (int64_t)INT32_MAX - 1;
}

int ora_process_append_replies(ora_engine *e, const mraft_ae_result *items,
                               int64_t n, const int64_t *seg_begin,
                               int64_t n_seg, int32_t *out_flags,
                               int32_t *item_err) {
  const int32_t P = e->P;
  int64_t gp = (int64_t)e->G * P;
  int64_t ns = seg_begin ? n_seg : n;
  int64_t *owner = segment_owners(e, &items[0].slot, sizeof(mraft_ae_result), n, seg_begin, ns);
  for (int64_t i = 0; i < n; ++i) { out_flags[i] = 0; item_err[i] = 0; }
  for (int64_t s = 0; s < ns; ++s) {
    int64_t b = seg_begin ? seg_begin[s] : s, en = seg_begin ? seg_begin[s + 1] : s + 1;
    if (b >= en) continue;
    int32_t slot = items[b].slot;
    int32_t bad = 0;
    if (slot < 0 || slot >= gp) bad = MRAFT_ITEM_BAD_SLOT;
    else if (owner[slot] != s) bad = MRAFT_ITEM_DUP_SLOT;
    else {
      for (int64_t i = b; i < en; ++i)
        if (items[i].slot != slot || items[i].peer < 0 || items[i].peer >= P ||
            items[i].peer == slot % P || !reply_index_ok(&items[i])) bad = MRAFT_ITEM_BAD_SLOT;
    }
    if (!bad && S.commit_index[slot] < S.dummy_index[slot]) bad = MRAFT_ITEM_BAD_STATE;
    if (bad) {
      for (int64_t i = b; i < en; ++i) item_err[i] = bad;
      continue;
    }
    for (int64_t i = b; i < en; ++i) {
      const mraft_ae_result *it = &items[i];
      out_flags[i] = process_reply_one(e, slot, it->peer, it->args_term,
                                       it->args_prev_log_index, it->args_n_entries,
                                       it->reply_term, it->reply_success,
                                       it->reply_conflict_index, NULL);
    }
  }
  free(owner);
  return MRAFT_OK;
}

/* ------------------------------------------------------------------------ */
/* Snapshots, src/raft/raft_snapshot.go                                      */
/* ------------------------------------------------------------------------ */

/* raftLog.setLogs(sliceFrom(index)) (raft_log.go:18-21,75-77): keep [index,
 * last], the entry at index becomes the dummy (logs[0]). On the ring this is
 * an index rebase: the head moves to the entry at `index`; no term moves. */
static void slice_from(ora_engine *e, int32_t s, int32_t index) {
  S.log_head[s] = (int32_t)(lpos(e, s, index) - (int64_t)s * e->L);
  S.dummy_index[s] = index;
}

/* Snapshot(index, snapshot), raft_snapshot.go:3-13 */
static int32_t snapshot_one(ora_engine *e, int32_t s, int32_t index) {
  if (index <= S.dummy_index[s]) return MRAFT_ITEM_OK;                /* :6-9 */
  if (index > S.last_index[s]) return MRAFT_ITEM_PREV_BEYOND_LAST;    /* sliceFrom panics */
  slice_from(e, s, index);                                            /* :10-11 */
  persist(e, s, MRAFT_PERSIST_STATE | MRAFT_PERSIST_SNAPSHOT);        /* :12 */
  return MRAFT_ITEM_OK;
}

int ora_snapshot(ora_engine *e, const int32_t *slots, const int32_t *index, int64_t n,
                 int32_t *item_err) {
  int32_t *first = claim_slots(e, slots, n, sizeof(int32_t), item_err);
  for (int64_t i = 0; i < n; ++i)
    if (!item_err[i]) item_err[i] = snapshot_one(e, slots[i], index[i]);
  free(first);
  return MRAFT_OK;
}

/* appendOneRound's snapshot branch, raft_append_entry.go:27-34 */
static int32_t gather_is_one(ora_engine *e, int32_t slot, int32_t peer, mraft_is_args *a) {
  const int32_t P = e->P;
  a->slot = -1;
  if (peer < 0 || peer >= P || peer == slot % P) return MRAFT_ITEM_BAD_SLOT;
  if (S.state[slot] != MRAFT_LEADER) return MRAFT_ITEM_BAD_STATE;
  const int32_t prev = S.next_index[(int64_t)slot * P + peer] - 1;
  if (prev >= S.dummy_index[slot]) return MRAFT_ITEM_OK;            /* an AppendEntries is due */
  a->slot = (slot / P) * P + peer;
  a->term = S.current_term[slot];                                     /* :29 */
  a->leader_id = slot % P;                                            /* :30 */
  a->last_included_index = S.dummy_index[slot];                       /* :31 */
  a->last_included_term = term_at(e, slot, S.dummy_index[slot]);      /* :32 dummyTerm */
  return MRAFT_ITEM_OK;
}

int ora_gather_install_snapshot_args(ora_engine *e, const int32_t *slots, const int32_t *peers,
                                     int64_t n, mraft_is_args *out, int32_t *item_err) {
  int64_t gp = (int64_t)e->G * e->P;
  for (int64_t i = 0; i < n; ++i) {
    memset(&out[i], 0, sizeof(out[i]));
    out[i].slot = -1;
    if (slots[i] < 0 || slots[i] >= gp) { item_err[i] = MRAFT_ITEM_BAD_SLOT; continue; }
    item_err[i] = gather_is_one(e, slots[i], peers[i], &out[i]);
  }
  return MRAFT_OK;
}

/* HandleInstallSnapshot, raft_snapshot.go:15-54 */
static int32_t handle_is_one(ora_engine *e, int32_t f, const mraft_is_args *a, mraft_is_reply *r,
                             int *installed) {
  *installed = 0;
  r->success = 0;
  r->term = 0;
  /* sliceFrom(LastIncludedIndex) below the follower's own dummy panics in Go
   * (raft_log.go:56-58): rejected before any mutation. */
  if (a->term >= S.current_term[f] && a->last_included_index > S.commit_index[f] &&
      a->last_included_index <= S.last_index[f] && a->last_included_index < S.dummy_index[f])
    return MRAFT_ITEM_BELOW_DUMMY;
  CR(A_TERM, f);
  if (a->term < S.current_term[f]) {                                  /* :20-22 */
    r->term = S.current_term[f];                                      /* deferred :17-19 */
    return MRAFT_ITEM_OK;
  }
  if (a->term > S.current_term[f]) {                                  /* :23-26 */
    S.current_term[f] = a->term; S.voted_for[f] = -1;
    CW(A_TERM, f); CW(A_VOTED, f);
    persist(e, f, MRAFT_PERSIST_STATE);                               /* :26 */
  }
  S.state[f] = MRAFT_FOLLOWER;                                        /* :28 */
  CW(A_ROLE, f);
  r->term = S.current_term[f];
  CR(A_COMMIT, f);
  const int32_t lii = a->last_included_index;
  if (lii <= S.commit_index[f]) return MRAFT_ITEM_OK;                 /* :31-33 outdated */
  CR(A_LAST, f);
  if (lii > S.last_index[f]) {                                        /* :35-37 */
    const int64_t at = (int64_t)f * e->L + S.log_head[f];             /* logs = [dummy] */
    S.log_term[at] = a->last_included_term;
    S.last_index[f] = lii;
    S.dummy_index[f] = lii;
    S.terms_sorted[f] = 1;                                            /* [dummy] only */
    CW(A_LOG, at); CW(A_LAST, f); CW(A_SORTED, f);
  } else {                                                            /* :38-40 */
    CR(A_DUMMY, f);
    slice_from(e, f, lii);                                            /* O(1) ring rebase */
    const int64_t at = lpos(e, f, lii);
    S.log_term[at] = a->last_included_term;                           /* :45 setDummyTerm */
    CW(A_LOG, at);
  }
  S.commit_index[f] = lii;                                            /* :42 */
  S.last_applied[f] = lii;                                            /* :43 */
  CW(A_DUMMY, f); CW(A_COMMIT, f); CW(A_APPLIED, f);
  persist(e, f, MRAFT_PERSIST_STATE | MRAFT_PERSIST_SNAPSHOT);        /* :47 */
  S.has_snapshot[f] = 1;                                              /* :52 hasSnapshot */
  *installed = 1;
  return MRAFT_ITEM_OK;
}

int ora_handle_install_snapshot(ora_engine *e, const mraft_is_args *args, int64_t n,
                                mraft_is_reply *replies, int32_t *out_flags, int32_t *item_err) {
  int32_t *first = claim_slots(e, &args[0].slot, n, sizeof(mraft_is_args), item_err);
  for (int64_t i = 0; i < n; ++i) {
    memset(&replies[i], 0, sizeof(replies[i]));
    out_flags[i] = 0;
    if (item_err[i]) continue;
    /* LastIncludedIndex past the Index domain (engine limit, include/mraft.h): malformed */
    if (args[i].last_included_index > INT32_MAX - 1) { item_err[i] = MRAFT_ITEM_BAD_SLOT; continue; }
    int inst = 0;
    item_err[i] = handle_is_one(e, args[i].slot, &args[i], &replies[i], &inst);
    if (inst) out_flags[i] = MRAFT_F_SNAPSHOT_INSTALLED;
  }
  free(first);
  return MRAFT_OK;
}

/* processInstallSnapshotReply, raft_snapshot.go:56-69 */
static int32_t process_is_reply_one(ora_engine *e, int32_t slot, int32_t peer, int32_t args_term,
                                    int32_t lii, int32_t reply_term) {
  const int64_t pi = (int64_t)slot * e->P + peer;
  int32_t fl = 0;
  if (reply_term > S.current_term[slot]) {                            /* :59-64 */
    S.current_term[slot] = reply_term;
    S.voted_for[slot] = -1;
    S.state[slot] = MRAFT_FOLLOWER;
    CW(A_TERM, slot); CW(A_VOTED, slot); CW(A_ROLE, slot);
    persist(e, slot, MRAFT_PERSIST_STATE);                            /* :64 */
    fl |= MRAFT_F_STEPPED_DOWN;
  } else if (S.state[slot] == MRAFT_LEADER && args_term == S.current_term[slot]) {  /* :65 */
    S.match_index[pi] = lii;                                          /* :66 */
    S.next_index[pi] = lii + 1;                                       /* :67 */
    CW(A_MATCH, pi); CW(A_NEXT, pi);
    fl |= MRAFT_F_APPLIED;
  }
  return fl;
}

int ora_process_install_snapshot_replies(ora_engine *e, const mraft_is_result *items, int64_t n,
                                         const int64_t *seg_begin, int64_t n_seg,
                                         int32_t *out_flags, int32_t *item_err) {
  const int32_t P = e->P;
  int64_t gp = (int64_t)e->G * P;
  int64_t ns = seg_begin ? n_seg : n;
  int64_t *owner = segment_owners(e, &items[0].slot, sizeof(mraft_is_result), n, seg_begin, ns);
  for (int64_t i = 0; i < n; ++i) { out_flags[i] = 0; item_err[i] = 0; }
  for (int64_t sg = 0; sg < ns; ++sg) {
    int64_t b = seg_begin ? seg_begin[sg] : sg, en = seg_begin ? seg_begin[sg + 1] : sg + 1;
    if (b >= en) continue;
    int32_t slot = items[b].slot, bad = 0;
    if (slot < 0 || slot >= gp) bad = MRAFT_ITEM_BAD_SLOT;
    else if (owner[slot] != sg) bad = MRAFT_ITEM_DUP_SLOT;
    else
      for (int64_t i = b; i < en; ++i)
        if (items[i].slot != slot || items[i].peer < 0 || items[i].peer >= P ||
            items[i].peer == slot % P || items[i].args_last_included_index > INT32_MAX - 1)
          bad = MRAFT_ITEM_BAD_SLOT;  /* (the last: past the Index domain, include/mraft.h) */
    if (bad) { for (int64_t i = b; i < en; ++i) item_err[i] = bad; continue; }
    for (int64_t i = b; i < en; ++i)
      out_flags[i] = process_is_reply_one(e, slot, items[i].peer, items[i].args_term,
                                          items[i].args_last_included_index, items[i].reply_term);
  }
  free(owner);
  return MRAFT_OK;
}

/* ------------------------------------------------------------------------ */
/* Fused tick = for each group: a3 for every peer, a4 at every follower, a2   */
/* (+a1) at the leader in peer order.                                         */
/* ------------------------------------------------------------------------ */

static void tick_group(ora_engine *e, const int32_t *leader_peer,
                       int32_t *group_flags, int32_t g, int32_t *scratch) {
  const int32_t P = e->P;
  int32_t flags = 0;
  int32_t lp = leader_peer[g];
  if (lp < 0) { if (group_flags) group_flags[g] = 0; return; }
  if (lp >= P) { if (group_flags) group_flags[g] = MRAFT_G_ERROR; return; }
  const int32_t ld = g * P + lp;
  CR(A_ROLE, ld);
  if (S.state[ld] != MRAFT_LEADER) { if (group_flags) group_flags[g] = 0; return; }
  CR(A_TERM, ld); CR(A_COMMIT, ld); CR(A_LAST, ld); CR(A_DUMMY, ld);
  if (S.commit_index[ld] < S.dummy_index[ld]) {
    if (group_flags) group_flags[g] = MRAFT_G_ERROR;
    return;
  }
  CR(A_SORTED, ld);
  int32_t ok[8] = {0};  /* 1: AppendEntries, 2: InstallSnapshot */
  for (int32_t p = 0; p < P; ++p) {
    if (p == lp) continue;
    CR(A_NEXT, (int64_t)ld * P + p);
    int32_t prev = S.next_index[(int64_t)ld * P + p] - 1;
    if (prev < S.dummy_index[ld]) { flags |= MRAFT_G_NEED_SNAPSHOT; ok[p] = 2; }
    else if (prev > S.last_index[ld]) flags |= MRAFT_G_ERROR;
    else ok[p] = 1;
  }
  if (flags & MRAFT_G_ERROR) {
    if (group_flags) group_flags[g] = MRAFT_G_ERROR | (flags & MRAFT_G_NEED_SNAPSHOT);
    return;
  }
  flags |= MRAFT_G_ACTIVE;

  mraft_ae_args args[8];
  mraft_ae_reply rep[8];
  mraft_is_args isa[8];
  mraft_is_reply isr[8];
  int32_t have[8] = {0};
  for (int32_t p = 0; p < P; ++p) {
    if (ok[p] == 2) {                                                 /* InstallSnapshot */
      gather_is_one(e, ld, p, &isa[p]);
      CR(A_LOG, lpos(e, ld, S.dummy_index[ld]));                      /* dummyTerm */
      int inst = 0;
      if (handle_is_one(e, g * P + p, &isa[p], &isr[p], &inst)) {
        flags |= MRAFT_G_FOLLOWER_PANIC;                              /* message dropped */
        continue;
      }
      if (inst) flags |= MRAFT_G_SNAPSHOT_INSTALLED;
      have[p] = 2;
      continue;
    }
    if (!ok[p]) continue;
    gather_one(e, ld, p, &args[p]);                                   /* a3 */
    int32_t prev = args[p].prev_log_index;
    CR(A_LOG, lpos(e, ld, prev));                                     /* PrevLogTerm */
    /* Go copies the entries into the args (raft_append_entry.go:50-54). */
    copy_terms(e, ld, prev + 1, args[p].n_entries, scratch);
    int fc = 0;
    int32_t err = handle_ae_one(e, g * P + p, &args[p], scratch,      /* a4 */
                                ld, &rep[p], &fc);
    if (err) { flags |= MRAFT_G_LOG_FULL; continue; }
    have[p] = 1;
    if (fc) flags |= MRAFT_G_FOLLOWER_COMMIT;
  }
  int32_t commit0 = S.commit_index[ld];
  int32_t term0 = S.current_term[ld];
  int32_t mstar = INT32_MIN;
  int any_eval = 0;
  for (int32_t p = 0; p < P; ++p) {                                   /* fold, peer order */
    if (!have[p]) continue;
    int32_t fl;
    if (have[p] == 2) {
      fl = process_is_reply_one(e, ld, p, isa[p].term, isa[p].last_included_index, isr[p].term);
    } else {
      int32_t ms = INT32_MIN;
      fl = process_reply_one(e, ld, p, args[p].term, args[p].prev_log_index,
                             args[p].n_entries, rep[p].term, rep[p].success,
                             rep[p].conflict_index, cnt.on ? &ms : NULL);
      if ((fl & MRAFT_F_APPLIED) && rep[p].success) {
        any_eval = 1;
        if (ms > mstar) mstar = ms;
      }
    }
    if (fl & MRAFT_F_STEPPED_DOWN) flags |= MRAFT_G_STEPPED_DOWN;
  }
  if (S.commit_index[ld] != commit0) {
    flags |= MRAFT_G_COMMITTED;
    CW(A_COMMIT, ld);
  }
  if (cnt.on && any_eval) {
    /* Minimal exact commit scan: matchIndex of the followers,
     * then log terms from min(M*, last) down to the first term == currentTerm
     * or commit0+1. */
    for (int32_t j = 0; j < P; ++j)
      if (j != lp) CR(A_MATCH, (int64_t)ld * P + j);
    int32_t top = imin(mstar, S.last_index[ld]);
    for (int32_t i = top; i > commit0; --i) {
      CR(A_LOG, lpos(e, ld, i));
      if (term_at(e, ld, i) == term0) break;
      /* sorted terms: a top term below currentTerm settles it */
      if (i == top && S.terms_sorted[ld] && term_at(e, ld, i) < term0) break;
    }
  }
  if (group_flags) group_flags[g] = flags;
}

int ora_replicate_tick_range(ora_engine *e, const int32_t *leader_peer,
                             int32_t *group_flags, int32_t g_begin,
                             int32_t g_end) {
  int32_t *scratch = (int32_t *)malloc(sizeof(int32_t) * (size_t)e->L);
  if (!scratch) return MRAFT_E_NOMEM;
  for (int32_t g = g_begin; g < g_end; ++g)
    tick_group(e, leader_peer, group_flags, g, scratch);
  free(scratch);
  return MRAFT_OK;
}

int ora_replicate_tick(ora_engine *e, const int32_t *leader_peer,
                       int32_t *group_flags) {
  if (e->P > 8) return MRAFT_E_INVAL;
  return ora_replicate_tick_range(e, leader_peer, group_flags, 0, e->G);
}

typedef struct {
  ora_engine *e;
  const int32_t *lp;
  int32_t *gf;
  int32_t b, en;
} tick_job;

static void *tick_worker(void *arg) {
  tick_job *j = (tick_job *)arg;
  ora_replicate_tick_range(j->e, j->lp, j->gf, j->b, j->en);
  return NULL;
}

int ora_replicate_tick_mt(ora_engine *e, const int32_t *leader_peer,
                          int32_t *group_flags, int32_t nthreads) {
  if (cnt.on || nthreads <= 1) return ora_replicate_tick(e, leader_peer, group_flags);
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  tick_job jobs[256];
  int32_t G = e->G;
  for (int32_t t = 0; t < nthreads; ++t) {
    jobs[t].e = e; jobs[t].lp = leader_peer; jobs[t].gf = group_flags;
    jobs[t].b = (int32_t)((int64_t)G * t / nthreads);
    jobs[t].en = (int32_t)((int64_t)G * (t + 1) / nthreads);
    pthread_create(&th[t], NULL, tick_worker, &jobs[t]);
  }
  for (int32_t t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  return MRAFT_OK;
}

/* ------------------------------------------------------------------------ */
/* Start, raft.go:90-104, and the applier, raft.go:153-203                   */
/* ------------------------------------------------------------------------ */

int ora_start(ora_engine *e, const int32_t *slots, const int32_t *counts,
              int64_t n, int32_t *out_index, int32_t *out_term,
              int32_t *out_is_leader, int32_t *item_err) {
  int32_t *first = claim_slots(e, slots, n, sizeof(int32_t), item_err);
  for (int64_t i = 0; i < n; ++i) {
    out_index[i] = -1; out_term[i] = -1; out_is_leader[i] = 0;
    if (item_err[i]) continue;
    int32_t s = slots[i], k = counts ? counts[i] : 1;
    if (k < 1) { item_err[i] = MRAFT_ITEM_BAD_SLOT; continue; }
    if (S.state[s] != MRAFT_LEADER) continue;                         /* :93-95 */
    int32_t last = S.last_index[s], dummy = S.dummy_index[s];
    if ((int64_t)last + k - dummy > (int64_t)e->L - 1 ||   /* capacity, or the Index domain (engine limits) */
        (int64_t)last + k > (int64_t)INT32_MAX - 1) { item_err[i] = MRAFT_ITEM_LOG_FULL; continue; }
    if (last > dummy && term_at(e, s, last) > S.current_term[s]) S.terms_sorted[s] = 0;
    for (int32_t j = 1; j <= k; ++j)                                  /* :96-100 */
      S.log_term[lpos(e, s, last + j)] = S.current_term[s];
    S.last_index[s] = last + k;
    persist(e, s, MRAFT_PERSIST_STATE);                               /* :101 */
    out_index[i] = last + 1; out_term[i] = S.current_term[s]; out_is_leader[i] = 1;  /* :103 */
  }
  free(first);
  return MRAFT_OK;
}

int ora_collect_apply(ora_engine *e, int32_t *out_from, int32_t *out_to, int32_t *out_snap_index,
                      int32_t *out_snap_term) {
  int64_t gp = (int64_t)e->G * e->P;
  for (int64_t s = 0; s < gp; ++s) {
    if (out_snap_index) {                                             /* :168-177 SnapshotValid first */
      const int hs = S.has_snapshot[s] != 0;
      out_snap_index[s] = hs ? S.dummy_index[s] : -1;                 /* SnapshotIndex = dummyIndex */
      out_snap_term[s] = hs ? term_at(e, s, S.dummy_index[s]) : 0;    /* SnapshotTerm = dummyTerm */
      S.has_snapshot[s] = 0;                                          /* rf.hasSnapshot = false */
    }
    int32_t la = S.last_applied[s], ci = S.commit_index[s];
    out_from[s] = la + 1;                                             /* :179-190 */
    out_to[s] = ci;
    if (ci > la) S.last_applied[s] = ci;                              /* :200 Max */
  }
  return MRAFT_OK;
}

/* ------------------------------------------------------------------------ */
/* a6 part 1: StartElection, raft_election.go:4-15                            */
/* ------------------------------------------------------------------------ */

static void start_election_one(ora_engine *e, int32_t s, mraft_rv_args *a) {
  S.state[s] = MRAFT_CANDIDATE;                                       /* :6 */
  S.current_term[s] += 1;                                             /* :7 */
  int32_t last = S.last_index[s];                                     /* lastEntry, raft_log.go:50-53 */
  a->slot = s;
  a->term = S.current_term[s];                                        /* :10 */
  a->candidate_id = s % e->P;                                         /* :11 */
  a->last_log_index = last;                                           /* :12 */
  a->last_log_term = term_at(e, s, last);                             /* :13 */
  S.voted_for[s] = s % e->P;                                          /* :14 */
  persist(e, s, MRAFT_PERSIST_STATE);                                 /* :15 */
  S.granted_votes[s] = 1;                                             /* :17 */
}

int ora_start_election(ora_engine *e, const int32_t *slots, int64_t n,
                       mraft_rv_args *out, int32_t *item_err) {
  int32_t *first = claim_slots(e, slots, n, sizeof(int32_t), item_err);
  for (int64_t i = 0; i < n; ++i) {
    memset(&out[i], 0, sizeof(out[i]));
    if (item_err[i]) continue;
    start_election_one(e, slots[i], &out[i]);
  }
  free(first);
  return MRAFT_OK;
}

/* ------------------------------------------------------------------------ */
/* a5: HandleRequestVote, raft_election.go:54-77 + isLogUpToDate              */
/* ------------------------------------------------------------------------ */

static void handle_rv_one(ora_engine *e, int32_t v, const mraft_rv_args *a, mraft_rv_reply *r) {
  r->term = 0; r->vote_granted = 0;
  persist(e, v, MRAFT_PERSIST_STATE);                                 /* defer rf.persist(), :57 */
  if (a->term < S.current_term[v]) {                                  /* :59-62 */
    r->term = S.current_term[v];
    return;
  }
  if (a->term > S.current_term[v]) {                                  /* :63-66 */
    S.state[v] = MRAFT_FOLLOWER;
    S.current_term[v] = a->term; S.voted_for[v] = -1;
  }
  r->term = S.current_term[v];                                        /* :67 */
  int32_t my_last = S.last_index[v];
  int32_t my_last_term = term_at(e, v, my_last);
  int up_to_date = a->last_log_term > my_last_term ||                 /* raft_log.go:99-104 */
                   (my_last_term == a->last_log_term && a->last_log_index >= my_last);
  if ((S.voted_for[v] == -1 || S.voted_for[v] == a->candidate_id) && up_to_date) {
    S.voted_for[v] = a->candidate_id;                                 /* :71 */
    r->vote_granted = 1;
  }                                                                   /* else :76 */
}

int ora_handle_request_vote(ora_engine *e, const mraft_rv_args *args,
                            int64_t n, mraft_rv_reply *replies,
                            int32_t *item_err) {
  int32_t *first = claim_slots(e, &args[0].slot, n, sizeof(mraft_rv_args), item_err);
  for (int64_t i = 0; i < n; ++i) {
    memset(&replies[i], 0, sizeof(replies[i]));
    if (item_err[i]) continue;
    handle_rv_one(e, args[i].slot, &args[i], &replies[i]);
  }
  free(first);
  return MRAFT_OK;
}

/* ------------------------------------------------------------------------ */
/* a6 part 2: vote tally closure, raft_election.go:22-47 (guard :29)          */
/* ------------------------------------------------------------------------ */

static int32_t tally_one(ora_engine *e, int32_t c, int32_t args_term, int32_t reply_term,
                         int32_t granted) {
  const int32_t P = e->P;
  int32_t fl = 0;
  if (S.current_term[c] == args_term && S.state[c] == MRAFT_CANDIDATE) { /* :29 */
    if (granted) {                                                    /* :30 */
      S.granted_votes[c] += 1;                                        /* :31 */
      if (S.granted_votes[c] > P / 2) {                               /* :32 */
        S.state[c] = MRAFT_LEADER;                                    /* :33 */
        for (int32_t j = 0; j < P; ++j) {                             /* :34-38 */
          S.match_index[(int64_t)c * P + j] = 0;
          S.next_index[(int64_t)c * P + j] = S.last_index[c] + 1;
        }
        fl |= MRAFT_F_BECAME_LEADER;
      }
    } else if (reply_term > S.current_term[c]) {                      /* :42-45 */
      S.state[c] = MRAFT_FOLLOWER;
      S.current_term[c] = reply_term; S.voted_for[c] = -1;
      persist(e, c, MRAFT_PERSIST_STATE);                             /* :45 */
      fl |= MRAFT_F_STEPPED_DOWN;
    }
  }
  return fl;
}

int ora_process_vote_replies(ora_engine *e, const mraft_rv_result *items,
                             int64_t n, const int64_t *seg_begin,
                             int64_t n_seg, int32_t *out_flags,
                             int32_t *item_err) {
  const int32_t P = e->P;
  int64_t gp = (int64_t)e->G * P;
  int64_t ns = seg_begin ? n_seg : n;
  int64_t *owner = segment_owners(e, &items[0].slot, sizeof(mraft_rv_result), n, seg_begin, ns);
  for (int64_t i = 0; i < n; ++i) { out_flags[i] = 0; item_err[i] = 0; }
  for (int64_t s = 0; s < ns; ++s) {
    int64_t b = seg_begin ? seg_begin[s] : s, en = seg_begin ? seg_begin[s + 1] : s + 1;
    if (b >= en) continue;
    int32_t c = items[b].slot;
    int32_t bad = 0;
    if (c < 0 || c >= gp) bad = MRAFT_ITEM_BAD_SLOT;
    else if (owner[c] != s) bad = MRAFT_ITEM_DUP_SLOT;
    else {
      for (int64_t i = b; i < en; ++i)
        if (items[i].slot != c || items[i].peer < 0 || items[i].peer >= P ||
            items[i].peer == c % P) bad = MRAFT_ITEM_BAD_SLOT;
    }
    if (bad) { for (int64_t i = b; i < en; ++i) item_err[i] = bad; continue; }
    for (int64_t i = b; i < en; ++i)
      out_flags[i] = tally_one(e, c, items[i].args_term, items[i].reply_term, items[i].vote_granted);
  }
  free(owner);
  return MRAFT_OK;
}

/* ------------------------------------------------------------------------ */
/* Fused election storm (config #5): R rounds; in round r the peers set in   */
/* cand_mask[r*G + g] that are not leaders time out (raft.go:109-114) and    */
/* StartElection in ascending peer order; every RequestVote is delivered,    */
/* voter by voter in candidate order; every candidate tallies its replies in */
/* voter order.                                                              */
/* ------------------------------------------------------------------------ */

static int election_rounds_range(ora_engine *e, const uint8_t *cand_mask, int32_t R,
                                 int32_t *group_flags, int32_t g_begin, int32_t g_end) {
  const int32_t P = e->P, G = e->G;
  if (P > 8) return MRAFT_E_INVAL;
  for (int32_t g = g_begin; g < g_end; ++g) {
    int32_t fl = 0;
    for (int32_t r = 0; r < R; ++r) {
      const uint8_t m = cand_mask[(int64_t)r * G + g];
      mraft_rv_args args[8];
      mraft_rv_reply rep[8][8];
      int32_t cand[8], nc = 0;
      for (int32_t p = 0; p < P; ++p) {
        int32_t s = g * P + p;
        if (((m >> p) & 1) && S.state[s] != MRAFT_LEADER) {
          start_election_one(e, s, &args[nc]);
          cand[nc++] = p;
        }
      }
      for (int32_t v = 0; v < P; ++v)                                 /* RequestVote deliveries */
        for (int32_t k = 0; k < nc; ++k)
          if (cand[k] != v) handle_rv_one(e, g * P + v, &args[k], &rep[k][v]);
      for (int32_t k = 0; k < nc; ++k)                                /* tallies */
        for (int32_t v = 0; v < P; ++v)
          if (cand[k] != v) {
            int32_t f2 = tally_one(e, g * P + cand[k], args[k].term, rep[k][v].term,
                                   rep[k][v].vote_granted);
            if (f2 & MRAFT_F_BECAME_LEADER) fl |= MRAFT_G_ELECTED;
            if (f2 & MRAFT_F_STEPPED_DOWN) fl |= MRAFT_G_STEPPED_DOWN;
          }
    }
    if (group_flags) group_flags[g] = fl;
  }
  return MRAFT_OK;
}

int ora_election_rounds(ora_engine *e, const uint8_t *cand_mask, int32_t R,
                        int32_t *group_flags) {
  return election_rounds_range(e, cand_mask, R, group_flags, 0, e->G);
}

typedef struct {
  ora_engine *e;
  const uint8_t *m;
  int32_t R, b, en;
  int32_t *gf;
} el_job;

static void *el_worker(void *arg) {
  el_job *j = (el_job *)arg;
  election_rounds_range(j->e, j->m, j->R, j->gf, j->b, j->en);
  return NULL;
}

/* Groups split contiguously over nthreads (CPU baseline of config #5). */
int ora_election_rounds_mt(ora_engine *e, const uint8_t *cand_mask, int32_t R,
                           int32_t *group_flags, int32_t nthreads) {
  if (nthreads <= 1) return ora_election_rounds(e, cand_mask, R, group_flags);
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  el_job jobs[256];
  for (int32_t t = 0; t < nthreads; ++t) {
    jobs[t].e = e; jobs[t].m = cand_mask; jobs[t].R = R; jobs[t].gf = group_flags;
    jobs[t].b = (int32_t)((int64_t)e->G * t / nthreads);
    jobs[t].en = (int32_t)((int64_t)e->G * (t + 1) / nthreads);
    pthread_create(&th[t], NULL, el_worker, &jobs[t]);
  }
  for (int32_t t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  return MRAFT_OK;
}

/* GetState, raft.go:237-246, per group. */
int ora_export_group_status(ora_engine *e, const int32_t *leader_peer,
                            int32_t *commit, int32_t *term_leader) {
  for (int32_t g = 0; g < e->G; ++g) {
    int32_t p = leader_peer ? leader_peer[g] : 0;
    if (p < 0 || p >= e->P) p = 0;
    int64_t s = (int64_t)g * e->P + p;
    commit[g] = S.commit_index[s];
    term_leader[g] = (int32_t)(((uint32_t)S.current_term[s] << 1) | (S.state[s] == MRAFT_LEADER));
  }
  return MRAFT_OK;
}

/* ------------------------------------------------------------------------ */
/* Persistence: the dirty set, SaveState and Make + readPersist               */
/* ------------------------------------------------------------------------ */

int ora_collect_persist(ora_engine *e, int32_t *out_bits) {
  const int64_t gp = (int64_t)e->G * e->P;
  for (int64_t s = 0; s < gp; ++s) {
    out_bits[s] = S.persist_dirty ? S.persist_dirty[s] : 0;
    if (S.persist_dirty) S.persist_dirty[s] = 0;
  }
  return MRAFT_OK;
}

/* SaveState, raft.go:209-216: currentTerm, votedFor, logs (terms here). */
int ora_read_persistent(ora_engine *e, const int32_t *slots, int64_t n, mraft_persistent *out,
                        int32_t *out_terms, int64_t terms_cap) {
  int64_t off = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t s = slots[i];
    memset(&out[i], 0, sizeof(out[i]));
    out[i].slot = s;
    out[i].current_term = S.current_term[s];
    out[i].voted_for = S.voted_for[s];
    out[i].dummy_index = S.dummy_index[s];
    out[i].last_index = S.last_index[s];
    out[i].terms_offset = off;
    off += (int64_t)S.last_index[s] - S.dummy_index[s] + 1;
  }
  if (!out_terms || terms_cap < off) return MRAFT_E_INVAL;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t cnt = (int64_t)out[i].last_index - out[i].dummy_index + 1;
    copy_terms(e, out[i].slot, out[i].dummy_index, (int32_t)cnt, out_terms + out[i].terms_offset);
  }
  return MRAFT_OK;
}

/* Make (raft.go:51-87) + readPersist (:217-235). */
int ora_restore(ora_engine *e, const mraft_persistent *in, int64_t n, const int32_t *terms,
                int64_t n_terms, int32_t *item_err) {
  const int32_t P = e->P;
  const int64_t gp = (int64_t)e->G * P;
  char *seen = (char *)calloc((size_t)(gp ? gp : 1), 1);
  for (int64_t i = 0; i < n; ++i) {
    const mraft_persistent *r = &in[i];
    const int64_t cnt = (int64_t)r->last_index - r->dummy_index + 1;
    if (r->slot < 0 || r->slot >= gp || cnt < 1 || r->dummy_index < 0 || r->terms_offset < 0 ||
        r->terms_offset + cnt > n_terms) { item_err[i] = MRAFT_ITEM_BAD_SLOT; continue; }
    if (cnt > e->L) { item_err[i] = MRAFT_ITEM_LOG_FULL; continue; }
    if (seen[r->slot]) { item_err[i] = MRAFT_ITEM_DUP_SLOT; continue; }
    seen[r->slot] = 1;
    item_err[i] = MRAFT_ITEM_OK;
    const int64_t s = r->slot;
    S.state[s] = MRAFT_FOLLOWER;                                      /* :58 */
    S.current_term[s] = r->current_term;                              /* :231 */
    S.voted_for[s] = r->voted_for;                                    /* :232 */
    memcpy(S.log_term + s * e->L, terms + r->terms_offset, sizeof(int32_t) * (size_t)cnt);  /* :233 */
    S.log_head[s] = 0;                                                /* a fresh raftLog */
    S.has_snapshot[s] = 0;                                            /* Make: no snapshot pending */
    S.dummy_index[s] = r->dummy_index;
    S.last_index[s] = r->last_index;
    S.terms_sorted[s] = sorted_after_dummy(e, s);
    S.commit_index[s] = r->dummy_index;                               /* :79 */
    S.last_applied[s] = r->dummy_index;                               /* :80 */
    S.granted_votes[s] = 0;
    for (int32_t j = 0; j < P; ++j) {                                 /* :64-65 */
      S.match_index[s * P + j] = 0;
      S.next_index[s * P + j] = 0;
    }
    if (S.persist_dirty) S.persist_dirty[s] = 0;
  }
  free(seen);
  return MRAFT_OK;
}
