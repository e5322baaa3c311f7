/*
 * mraft_goshape.c — the replication tick restated on the reference's own data
 * shapes, for the CPU baseline (SURVEY.md §8d "go-shaped" variant).
 * TEST INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg and tests/ use it;
 * the product never does.
 *
 * Where mraft_oracle.c works on the engine's struct-of-arrays int32 layout,
 * this file keeps what the Go code actually touches: one Raft struct per
 * replica with int64 fields (src/raft/raft.go:16-40), its log as a slice of
 * 40-byte Entry{Index, Command interface{}, Term, Id} (raft_rpc.go:39-44,
 * raft_log.go:3-12), an AppendEntriesArgs whose Entries slice is a fresh copy
 * of the leader's tail for every message (raft_append_entry.go:50-54),
 * trunc + append on the follower's slice (raft_log.go:62-75), and
 * advanceCommitIndexForLeader's downward O((last - commit) * P) count
 * (:89-105). Excluded, as in the SoA oracle: the gob persist() and labrpc
 * encoding the reference pays per handler, locks, goroutines.
 *
 * Supported: groups whose followers all take the AppendEntries path (no
 * InstallSnapshot, no Go panic, no engine capacity limit) — the config-#3
 * workload. goshape_tick returns the number of groups it could not run.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "mraft_oracle.h"

typedef struct {            /* raft_rpc.go:39-44 */
  int64_t Index;
  void *Command[2];         /* interface{}: (type, data) words */
  int64_t Term;
  int64_t Id;
} go_entry;

typedef struct {            /* raft.go:16-40, decision fields */
  int64_t currentTerm, votedFor, state, commitIndex, lastApplied;
  go_entry *logs;           /* raftLog.logs []Entry, logs[0] = dummy */
  int64_t nlogs, caplogs;
  int64_t *nextIndex, *matchIndex;
} go_raft;

typedef struct {            /* raft_rpc.go:55-62 */
  int64_t Term, LeaderId;
  go_entry *Entries;
  int64_t nEntries;
  int64_t PrevLogIndex, PrevLogTerm, LeaderCommit;
} go_ae_args;

typedef struct {            /* raft_rpc.go:64-69 */
  int64_t Conflict, ConflictIndex, Term, Success;
} go_ae_reply;

struct go_cluster {
  int32_t G, P, L;
  go_raft *r;
};
typedef struct go_cluster go_cluster;

static inline int64_t dummy_index(const go_raft *r) { return r->logs[0].Index; }
static inline int64_t last_index(const go_raft *r) { return r->logs[r->nlogs - 1].Index; }
static inline go_entry *get_entry(go_raft *r, int64_t i) { return &r->logs[i - dummy_index(r)]; }

static void append_entries(go_raft *r, const go_entry *e, int64_t n) {  /* append(logs, e...) */
  if (r->nlogs + n > r->caplogs) {
    int64_t c = r->caplogs ? r->caplogs : 1;
    while (c < r->nlogs + n) c *= 2;
    r->logs = (go_entry *)realloc(r->logs, sizeof(go_entry) * (size_t)c);
    r->caplogs = c;
  }
  memcpy(r->logs + r->nlogs, e, sizeof(go_entry) * (size_t)n);
  r->nlogs += n;
}

go_cluster *goshape_build(int32_t G, int32_t P, int32_t L, const mraft_soa *s) {
  go_cluster *c = (go_cluster *)calloc(1, sizeof(go_cluster));
  c->G = G; c->P = P; c->L = L;
  c->r = (go_raft *)calloc((size_t)G * P, sizeof(go_raft));
  for (int64_t i = 0; i < (int64_t)G * P; ++i) {
    go_raft *r = &c->r[i];
    r->currentTerm = s->current_term[i]; r->votedFor = s->voted_for[i]; r->state = s->state[i];
    r->commitIndex = s->commit_index[i]; r->lastApplied = s->last_applied[i];
    const int64_t d = s->dummy_index[i], n = (int64_t)s->last_index[i] - d + 1;
    /* capacity L, like a slice that has already grown: the timed tick then
     * copies entries but never reallocates (a realloc of a large block is an
     * mremap syscall that serialises threads on the address-space lock, a
     * cost Go's heap does not have) */
    r->caplogs = n > L ? n : L; r->nlogs = n;
    r->logs = (go_entry *)malloc(sizeof(go_entry) * (size_t)r->caplogs);
    memset(r->logs, 0, sizeof(go_entry) * (size_t)r->caplogs);  /* pre-fault (Go's heap is warm) */
    const int64_t h = s->log_head ? s->log_head[i] : 0;  /* the engine's ring, include/mraft.h */
    for (int64_t k = 0; k < n; ++k) {
      r->logs[k].Index = d + k;
      r->logs[k].Term = s->log_term[i * L + (h + k) % L];
    }
    r->nextIndex = (int64_t *)malloc(sizeof(int64_t) * (size_t)P);
    r->matchIndex = (int64_t *)malloc(sizeof(int64_t) * (size_t)P);
    for (int32_t j = 0; j < P; ++j) {
      r->nextIndex[j] = s->next_index[i * P + j];
      r->matchIndex[j] = s->match_index[i * P + j];
    }
  }
  return c;
}

/* Back to the SoA image (for the tests). */
void goshape_store(const go_cluster *c, const mraft_soa *s) {
  const int32_t P = c->P, L = c->L;
  for (int64_t i = 0; i < (int64_t)c->G * P; ++i) {
    const go_raft *r = &c->r[i];
    s->current_term[i] = (int32_t)r->currentTerm; s->voted_for[i] = (int32_t)r->votedFor;
    s->state[i] = (int32_t)r->state; s->commit_index[i] = (int32_t)r->commitIndex;
    s->last_applied[i] = (int32_t)r->lastApplied;
    s->dummy_index[i] = (int32_t)r->logs[0].Index;
    s->last_index[i] = (int32_t)r->logs[r->nlogs - 1].Index;
    const int64_t h = s->log_head ? s->log_head[i] : 0;
    for (int64_t k = 0; k < r->nlogs && k < L; ++k) s->log_term[i * L + (h + k) % L] = (int32_t)r->logs[k].Term;
    for (int32_t j = 0; j < P; ++j) {
      s->next_index[i * P + j] = (int32_t)r->nextIndex[j];
      s->match_index[i * P + j] = (int32_t)r->matchIndex[j];
    }
  }
}

void goshape_free(go_cluster *c) {
  if (!c) return;
  for (int64_t i = 0; i < (int64_t)c->G * c->P; ++i) {
    free(c->r[i].logs); free(c->r[i].nextIndex); free(c->r[i].matchIndex);
  }
  free(c->r);
  free(c);
}

/* appendOneRound's args (raft_append_entry.go:26-54): the entries are copied
 * (into a per-thread arena standing in for Go's heap allocator: the copy is
 * kept, a malloc/mmap syscall per message is not). */
static void gather(go_raft *ld, int32_t me, int32_t peer, go_ae_args *a, go_entry *arena) {
  const int64_t prev = ld->nextIndex[peer] - 1;
  a->LeaderId = me;
  a->Term = ld->currentTerm;
  a->PrevLogIndex = prev;
  a->PrevLogTerm = get_entry(ld, prev)->Term;
  a->nEntries = last_index(ld) - prev;
  a->Entries = arena;
  memcpy(a->Entries, get_entry(ld, prev + 1), sizeof(go_entry) * (size_t)a->nEntries);
  a->LeaderCommit = ld->commitIndex;
}

/* HandleAppendEntries, raft_append_entry.go:108-162. */
static void handle_ae(go_raft *rf, const go_ae_args *args, go_ae_reply *reply) {
  memset(reply, 0, sizeof(*reply));
  if (args->Term < rf->currentTerm) {                                 /* :112-115 */
    reply->Term = rf->currentTerm; reply->Success = 0;
    return;
  }
  if (args->Term > rf->currentTerm) { rf->currentTerm = args->Term; rf->votedFor = -1; }
  rf->state = MRAFT_FOLLOWER;                                         /* :120 */
  if (args->PrevLogIndex < dummy_index(rf)) {                         /* :123-127 */
    reply->Term = 0; reply->Success = 0; reply->ConflictIndex = dummy_index(rf) + 1;
    return;
  }
  if (!(args->PrevLogIndex <= last_index(rf) &&                       /* matchLog */
        get_entry(rf, args->PrevLogIndex)->Term == args->PrevLogTerm)) {
    reply->Term = rf->currentTerm; reply->Success = 0;
    const int64_t lastIndex = last_index(rf);
    if (args->PrevLogIndex > lastIndex) {
      reply->ConflictIndex = lastIndex + 1;
    } else {
      const int64_t d = dummy_index(rf), abandoned = get_entry(rf, args->PrevLogIndex)->Term;
      int64_t index = args->PrevLogIndex;
      while (index > d + 1 && get_entry(rf, index)->Term == abandoned) index--;
      reply->ConflictIndex = index;
    }
    return;
  }
  for (int64_t k = 0; k < args->nEntries; ++k) {                      /* :146-155 */
    const go_entry *entry = &args->Entries[k];
    if (entry->Index - dummy_index(rf) >= rf->nlogs || get_entry(rf, entry->Index)->Term != entry->Term) {
      rf->nlogs = entry->Index - dummy_index(rf);                     /* trunc */
      append_entries(rf, args->Entries + k, args->nEntries - k);      /* append */
      break;
    }
  }
  if (args->LeaderCommit > rf->commitIndex) {                         /* :157-160 */
    const int64_t li = last_index(rf);
    rf->commitIndex = args->LeaderCommit < li ? args->LeaderCommit : li;
  }
  reply->Term = rf->currentTerm; reply->Success = 1;
}

/* advanceCommitIndexForLeader, :89-105. */
static void advance_commit(go_raft *rf, int32_t me, int32_t P) {
  for (int64_t i = last_index(rf); i > rf->commitIndex; i--) {
    int64_t num = 0;
    for (int32_t j = 0; j < P; ++j)
      if (j != me && rf->matchIndex[j] >= i) num++;
    if (num + 1 > P / 2 && get_entry(rf, i)->Term == rf->currentTerm) {
      rf->commitIndex = i;
      return;
    }
  }
}

/* processAppendEntriesReply, :66-88. */
static void process_reply(go_raft *rf, int32_t me, int32_t P, int32_t peer, const go_ae_args *args,
                          const go_ae_reply *reply) {
  if (reply->Term > rf->currentTerm) {
    rf->currentTerm = reply->Term; rf->votedFor = -1; rf->state = MRAFT_FOLLOWER;
  } else if (reply->Term == rf->currentTerm && rf->state == MRAFT_LEADER &&
             args->Term == rf->currentTerm && args->PrevLogIndex == rf->nextIndex[peer] - 1) {
    if (reply->Success) {
      rf->matchIndex[peer] = args->nEntries + args->PrevLogIndex;
      rf->nextIndex[peer] = rf->matchIndex[peer] + 1;
      advance_commit(rf, me, P);
    } else {
      rf->nextIndex[peer] = reply->ConflictIndex;
    }
  }
}

int64_t goshape_tick_range(go_cluster *c, const int32_t *leader_peer, int32_t g0, int32_t g1) {
  const int32_t P = c->P;
  int64_t skipped = 0;
  go_ae_args args[8];
  go_ae_reply rep[8];
  go_entry *arena = (go_entry *)malloc(sizeof(go_entry) * (size_t)c->L * 8);
  for (int32_t g = g0; g < g1; ++g) {
    const int32_t lp = leader_peer[g];
    if (lp < 0 || lp >= P) continue;
    go_raft *ld = &c->r[(int64_t)g * P + lp];
    if (ld->state != MRAFT_LEADER) continue;
    int ok = ld->commitIndex >= dummy_index(ld);
    for (int32_t p = 0; p < P && ok; ++p) {
      if (p == lp) continue;
      const int64_t prev = ld->nextIndex[p] - 1;
      if (prev < dummy_index(ld) || prev > last_index(ld)) ok = 0;   /* snapshot / panic */
    }
    if (!ok) { skipped++; continue; }
    for (int32_t p = 0; p < P; ++p) {
      if (p == lp) continue;
      gather(ld, lp, p, &args[p], arena + (size_t)c->L * p);
      go_raft *f = &c->r[(int64_t)g * P + p];
      /* the engine's capacity rule never triggers on the config-#3 workload */
      handle_ae(f, &args[p], &rep[p]);
    }
    for (int32_t p = 0; p < P; ++p) {
      if (p == lp) continue;
      process_reply(ld, lp, P, p, &args[p], &rep[p]);
    }
  }
  free(arena);
  return skipped;
}

#include <pthread.h>

typedef struct {
  go_cluster *c;
  const int32_t *lp;
  int32_t b, e;
  int64_t skipped;
} go_job;

static void *go_worker(void *arg) {
  go_job *j = (go_job *)arg;
  j->skipped = goshape_tick_range(j->c, j->lp, j->b, j->e);
  return NULL;
}

/* Groups split contiguously over nthreads (independent Raft instances). */
int64_t goshape_tick(go_cluster *c, const int32_t *leader_peer, int32_t nthreads) {
  if (nthreads <= 1) return goshape_tick_range(c, leader_peer, 0, c->G);
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  go_job jobs[256];
  for (int32_t t = 0; t < nthreads; ++t) {
    jobs[t].c = c; jobs[t].lp = leader_peer;
    jobs[t].b = (int32_t)((int64_t)c->G * t / nthreads);
    jobs[t].e = (int32_t)((int64_t)c->G * (t + 1) / nthreads);
    pthread_create(&th[t], NULL, go_worker, &jobs[t]);
  }
  int64_t skipped = 0;
  for (int32_t t = 0; t < nthreads; ++t) {
    pthread_join(th[t], NULL);
    skipped += jobs[t].skipped;
  }
  return skipped;
}

/* Restores the pristine SoA state into the already-built cluster in place
 * (slices keep their capacity), groups split over nthreads. Untimed helper of
 * the CPU baseline. */
typedef struct {
  go_cluster *c;
  const mraft_soa *s;
  int64_t b, e;
} go_reset_job;

static void *go_reset_worker(void *arg) {
  go_reset_job *j = (go_reset_job *)arg;
  const int32_t P = j->c->P, L = j->c->L;
  const mraft_soa *s = j->s;
  for (int64_t i = j->b; i < j->e; ++i) {
    go_raft *r = &j->c->r[i];
    r->currentTerm = s->current_term[i]; r->votedFor = s->voted_for[i]; r->state = s->state[i];
    r->commitIndex = s->commit_index[i]; r->lastApplied = s->last_applied[i];
    const int64_t d = s->dummy_index[i], n = (int64_t)s->last_index[i] - d + 1;
    r->nlogs = n;
    const int64_t h = s->log_head ? s->log_head[i] : 0;
    for (int64_t k = 0; k < n; ++k) {
      r->logs[k].Index = d + k;
      r->logs[k].Term = s->log_term[i * L + (h + k) % L];
    }
    for (int32_t q = 0; q < P; ++q) {
      r->nextIndex[q] = s->next_index[i * P + q];
      r->matchIndex[q] = s->match_index[i * P + q];
    }
  }
  return NULL;
}

void goshape_reset(go_cluster *c, const mraft_soa *s, int32_t nthreads) {
  const int64_t n = (int64_t)c->G * c->P;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  go_reset_job jobs[256];
  for (int32_t t = 0; t < nthreads; ++t) {
    jobs[t].c = c; jobs[t].s = s;
    jobs[t].b = n * t / nthreads;
    jobs[t].e = n * (t + 1) / nthreads;
    pthread_create(&th[t], NULL, go_reset_worker, &jobs[t]);
  }
  for (int32_t t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}
