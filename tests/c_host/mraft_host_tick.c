/*
 * mraft_host_tick.c — a plain C11 host of libmraft_hip.so: it includes only
 * include/mraft.h and links the library the way a cgo binding does
 * (INTEGRATION.md), with no HIP header, no C++ and no Python in between.
 *
 * For every seeded tick vector of tests/golden/tick_vectors.bin (written by
 * tests/golden/make_golden.py from tick_vectors.npz: inputs from the seeded
 * generator, expected outputs from the pure-Python restatement of
 * src/raft/raft_append_entry.go:20-162) it runs one replication round of the
 * reference four ways through the boundary, each on a fresh engine
 * (mraft_create = Make, src/raft/raft.go:51-87; mraft_load_state =
 * readPersist, raft.go:217-235; mraft_destroy = Kill, src/raft/utility.go:9-19):
 *
 *   tick      mraft_set_tick_shards(2) -> mraft_replicate_tick_export
 *             (appendOneRound + HandleAppendEntries + processAppendEntriesReply
 *             + GetState, raft.go:237-246), the fused co-resident tick;
 *   messages  the per-message RPC sequence a Go host drives:
 *             mraft_gather_append_args (appendOneRound's args, :20-54) ->
 *             mraft_handle_append_entries_ex by reference (HandleAppendEntries,
 *             :108-162) -> mraft_process_append_replies over one segment per
 *             leader (processAppendEntriesReply + advanceCommitIndexForLeader,
 *             :66-105) -> mraft_export_group_status (GetState);
 *   by value  the same with the entries copied into a caller buffer, as a
 *             host that received the args over the network holds them;
 *   light     the tick again with mraft_set_tick_mode(MRAFT_TICK_LIGHT): the
 *             steady-state groups settled eight per wave, the rest through
 *             the full tick (ABI 6).
 *
 * Each path is compared with the same fixture: the group flags (on the message
 * paths rebuilt from the gather errors, the per-item fold flags and the
 * followers' commitIndex), the exported GetState words and every state array
 * (logs in Index order over the live entries).
 *
 * Usage: mraft_host_tick <tick_vectors.bin> [device]. Exit status 0 = every
 * vector bit-exact on every path; 1 = a mismatch; 2 = an ABI error; 3 = a bad
 * fixture.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mraft.h"

#define N_ARR 12
#define A_COMMIT 3
#define A_DUMMY 5
#define A_LAST 6
#define A_LOG 8

/* The fixture's array order (make_golden.py tick_vectors_bin). */
static const char *const k_names[N_ARR] = {
    "current_term", "voted_for", "state", "commit_index", "last_applied", "dummy_index",
    "last_index", "granted_votes", "log_term", "match_index", "next_index", "persist_dirty"};

typedef struct {
  int32_t G, P, L;
  int32_t *lp, *want_flags, *want_commit, *want_tl;
  int32_t *in[N_ARR], *want[N_ARR];
} vec_t;

enum { PATH_TICK, PATH_MESSAGES, PATH_BY_VALUE, PATH_LIGHT };
static const char *const k_path[4] = {"tick", "messages", "by value", "light tick"};

static int64_t arr_len(int i, int64_t gp, int64_t P, int64_t L) {
  return i == A_LOG ? gp * L : (i == 9 || i == 10) ? gp * P : gp;
}

static int32_t **slot_of(mraft_soa *s, int i) {
  int32_t **t[N_ARR] = {&s->current_term, &s->voted_for, &s->state, &s->commit_index,
                        &s->last_applied, &s->dummy_index, &s->last_index, &s->granted_votes,
                        &s->log_term, &s->match_index, &s->next_index, &s->persist_dirty};
  return t[i];
}

static void *zalloc(int64_t n, size_t size) { return calloc((size_t)(n > 0 ? n : 1), size); }

static int32_t *read_i32(FILE *f, int64_t n) {
  int32_t *p = (int32_t *)zalloc(n, sizeof(int32_t));
  if (!p || (n > 0 && fread(p, sizeof(int32_t), (size_t)n, f) != (size_t)n)) {
    free(p);
    return NULL;
  }
  return p;
}

#define ABI(call)                                                                   \
  do {                                                                              \
    int rc_ = (call);                                                               \
    if (rc_ != MRAFT_OK) {                                                          \
      fprintf(stderr, "%s -> %d: %s\n", #call, rc_, mraft_last_error_string());     \
      return 2;                                                                     \
    }                                                                               \
  } while (0)

#define NEED(p)          \
  do {                   \
    if (!(p)) return 3;  \
  } while (0)

static int mismatch(int v, int path, const char *what, int64_t at, int32_t got, int32_t want) {
  fprintf(stderr, "vector %d (%s): %s differs at %lld: %d vs %d\n", v, k_path[path], what, (long long)at,
          (int)got, (int)want);
  return 1;
}

static int read_vector(FILE *f, vec_t *t) {
  int32_t dims[3];
  if (fread(dims, sizeof dims, 1, f) != 1) return 3;
  t->G = dims[0];
  t->P = dims[1];
  t->L = dims[2];
  const int64_t gp = (int64_t)t->G * t->P;
  NEED(t->lp = read_i32(f, t->G));
  NEED(t->want_flags = read_i32(f, t->G));
  NEED(t->want_commit = read_i32(f, t->G));
  NEED(t->want_tl = read_i32(f, t->G));
  for (int i = 0; i < N_ARR; ++i) NEED(t->in[i] = read_i32(f, arr_len(i, gp, t->P, t->L)));
  for (int i = 0; i < N_ARR; ++i) NEED(t->want[i] = read_i32(f, arr_len(i, gp, t->P, t->L)));
  return 0;
}

static void free_vector(vec_t *t) {
  for (int i = 0; i < N_ARR; ++i) {
    free(t->in[i]);
    free(t->want[i]);
  }
  free(t->lp);
  free(t->want_flags);
  free(t->want_commit);
  free(t->want_tl);
}

/* Make + readPersist of the fixture's inputs. The fixture predates the ring
   and the terms_sorted proof: heads 0 (Index dummy at row position 0), no
   snapshot pending; terms_sorted is recomputed by mraft_load_state from the
   logs whatever the source holds. */
static int open_engine(const vec_t *t, int device, mraft_engine **h) {
  const int64_t gp = (int64_t)t->G * t->P;
  int32_t *zeros = (int32_t *)zalloc(gp, sizeof(int32_t));
  NEED(zeros);
  ABI(mraft_create(t->G, t->P, t->L, device, 0, h));
  mraft_soa src;
  memset(&src, 0, sizeof src);
  for (int i = 0; i < N_ARR; ++i) *slot_of(&src, i) = t->in[i];
  src.log_head = zeros;
  src.has_snapshot = zeros;
  src.terms_sorted = zeros;
  ABI(mraft_load_state(*h, &src, MRAFT_HOST));
  free(zeros);
  return 0;
}

/* mraft_store_state + comparison with the fixture; destroys the engine. */
static int check_engine(const vec_t *t, int v, int path, mraft_engine *h, const int32_t *flags,
                        const int32_t *commit, const int32_t *tl) {
  const int32_t G = t->G, P = t->P, L = t->L;
  const int64_t gp = (int64_t)G * P;
  int32_t *got[N_ARR];
  int32_t *head = (int32_t *)zalloc(gp, sizeof(int32_t)), *hsnap = (int32_t *)zalloc(gp, sizeof(int32_t)),
          *srt = (int32_t *)zalloc(gp, sizeof(int32_t));
  NEED(head && hsnap && srt);
  mraft_soa dst;
  memset(&dst, 0, sizeof dst);
  for (int i = 0; i < N_ARR; ++i) {
    NEED(got[i] = (int32_t *)zalloc(arr_len(i, gp, P, L), sizeof(int32_t)));
    *slot_of(&dst, i) = got[i];
  }
  dst.log_head = head;
  dst.has_snapshot = hsnap;
  dst.terms_sorted = srt;
  ABI(mraft_store_state(h, &dst, MRAFT_HOST));
  ABI(mraft_destroy(h));

  for (int32_t g = 0; g < G; ++g) {
    if (flags[g] != t->want_flags[g]) return mismatch(v, path, "group_flags", g, flags[g], t->want_flags[g]);
    if (commit[g] != t->want_commit[g]) return mismatch(v, path, "export commit", g, commit[g], t->want_commit[g]);
    if (tl[g] != t->want_tl[g]) return mismatch(v, path, "export term<<1|leader", g, tl[g], t->want_tl[g]);
  }
  for (int i = 0; i < N_ARR; ++i) {
    if (i == A_LOG) continue; /* logs: below, in Index order */
    for (int64_t k = 0; k < arr_len(i, gp, P, L); ++k)
      if (got[i][k] != t->want[i][k]) return mismatch(v, path, k_names[i], k, got[i][k], t->want[i][k]);
  }
  /* logs: Index dummy..last of every replica, at ring position
     (head + Index - dummy) mod L in the engine, at Index - dummy in the fixture */
  const int32_t *dummy = t->want[A_DUMMY], *last = t->want[A_LAST], *wlog = t->want[A_LOG];
  for (int64_t s = 0; s < gp; ++s) {
    if (head[s] < 0 || head[s] >= L) return mismatch(v, path, "log_head", s, head[s], 0);
    for (int32_t i = dummy[s]; i <= last[s]; ++i) {
      const int64_t k = i - dummy[s];
      const int32_t a = got[A_LOG][s * L + (head[s] + k) % L], b = wlog[s * L + k];
      if (a != b) return mismatch(v, path, "log_term (slot*L + Index - dummy)", s * L + k, a, b);
    }
    /* terms_sorted is a proof: 1 only over non-decreasing terms after the dummy */
    if (srt[s]) {
      for (int32_t i = dummy[s] + 1; i < last[s]; ++i) {
        const int64_t k = i - dummy[s];
        if (wlog[s * L + k] > wlog[s * L + k + 1]) return mismatch(v, path, "terms_sorted (unsound)", s, 1, 0);
      }
    }
  }
  for (int i = 0; i < N_ARR; ++i) free(got[i]);
  free(head);
  free(hsnap);
  free(srt);
  return 0;
}

static int run_tick(const vec_t *t, int v, int device, int light) {
  const int32_t G = t->G;
  int32_t *flags = (int32_t *)zalloc(G, sizeof(int32_t)), *commit = (int32_t *)zalloc(G, sizeof(int32_t)),
          *tl = (int32_t *)zalloc(G, sizeof(int32_t));
  NEED(flags && commit && tl);
  mraft_engine *h = NULL;
  int rc = open_engine(t, device, &h);
  if (rc) return rc;
  const int32_t shards = G >= 2 ? 2 : 1;
  ABI(mraft_set_tick_shards(h, shards));
  if (mraft_get_tick_shards(h) != shards) {
    fprintf(stderr, "vector %d: mraft_get_tick_shards = %d, want %d\n", v, mraft_get_tick_shards(h), shards);
    return 2;
  }
  if (light) {
    ABI(mraft_set_tick_mode(h, MRAFT_TICK_LIGHT));
    if (mraft_get_tick_mode(h) != MRAFT_TICK_LIGHT || mraft_tick_light_fallbacks(h) != -1) {
      fprintf(stderr, "vector %d: tick mode %d, fallbacks %lld before the first light tick\n", v,
              mraft_get_tick_mode(h), (long long)mraft_tick_light_fallbacks(h));
      return 2;
    }
  }
  ABI(mraft_replicate_tick_export(h, t->lp, flags, commit, tl, MRAFT_HOST));
  if (light && mraft_tick_light_fallbacks(h) < 0) {
    fprintf(stderr, "vector %d: no fallback count after a light tick\n", v);
    return 2;
  }
  rc = check_engine(t, v, light ? PATH_LIGHT : PATH_TICK, h, flags, commit, tl);
  free(flags);
  free(commit);
  free(tl);
  return rc;
}

/* One AppendEntries from every group's leader replica to each other peer, in
   group order (the gather's layout: one leader's messages side by side). */
static int run_messages(const vec_t *t, int v, int device, int by_value) {
  const int32_t G = t->G, P = t->P, L = t->L;
  const int path = by_value ? PATH_BY_VALUE : PATH_MESSAGES;
  int64_t n = 0;
  for (int32_t g = 0; g < G; ++g) n += (t->lp[g] >= 0 && t->lp[g] < P) ? P - 1 : 0;
  int32_t *slots = (int32_t *)zalloc(n, sizeof(int32_t)), *peers = (int32_t *)zalloc(n, sizeof(int32_t)),
          *gerr = (int32_t *)zalloc(n, sizeof(int32_t)), *herr = (int32_t *)zalloc(n, sizeof(int32_t)),
          *fflags = (int32_t *)zalloc(n, sizeof(int32_t)), *ferr = (int32_t *)zalloc(n, sizeof(int32_t));
  mraft_ae_args *args = (mraft_ae_args *)zalloc(n, sizeof(mraft_ae_args));
  mraft_ae_reply *rep = (mraft_ae_reply *)zalloc(n, sizeof(mraft_ae_reply));
  mraft_ae_result *res = (mraft_ae_result *)zalloc(n, sizeof(mraft_ae_result));
  int64_t *seg = (int64_t *)zalloc(n + 1, sizeof(int64_t));
  int32_t *flags = (int32_t *)zalloc(G, sizeof(int32_t)), *commit = (int32_t *)zalloc(G, sizeof(int32_t)),
          *tl = (int32_t *)zalloc(G, sizeof(int32_t));
  NEED(slots && peers && gerr && herr && fflags && ferr && args && rep && res && seg && flags && commit && tl);
  int64_t k = 0;
  for (int32_t g = 0; g < G; ++g) {
    if (t->lp[g] < 0 || t->lp[g] >= P) continue;
    for (int32_t p = 0; p < P; ++p) {
      if (p == t->lp[g]) continue;
      slots[k] = g * P + t->lp[g];
      peers[k++] = p;
    }
  }

  mraft_engine *h = NULL;
  int rc = open_engine(t, device, &h);
  if (rc) return rc;
  ABI(mraft_gather_append_args(h, slots, peers, n, args, gerr, MRAFT_HOST));
  /* a replica that is not the leader sends nothing (appendOneRound returns,
     raft_append_entry.go:22-25): its items leave the batch; the fixture holds
     no InstallSnapshot sends (every next-1 >= dummy) */
  int64_t m = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (gerr[i] == MRAFT_ITEM_BAD_STATE) continue;
    if (gerr[i] != MRAFT_ITEM_OK) return mismatch(v, path, "gather item_err", i, gerr[i], 0);
    slots[m] = slots[i];
    peers[m] = peers[i];
    args[m++] = args[i];
  }
  for (int32_t g = 0; g < G; ++g) flags[g] = 0;
  for (int64_t i = 0; i < m; ++i) flags[slots[i] / P] |= MRAFT_G_ACTIVE;

  int32_t *terms = NULL;
  int64_t n_terms = 0;
  if (by_value) {
    /* the entries as a receiver holds them: their terms, copied out of the
       leader's log (the fixture's input rows, head 0) into one buffer, each
       item at its own offset */
    for (int64_t i = 0; i < m; ++i) n_terms += args[i].n_entries;
    NEED(terms = (int32_t *)zalloc(n_terms, sizeof(int32_t)));
    int64_t at = 0;
    for (int64_t i = 0; i < m; ++i) {
      const int64_t row = (int64_t)slots[i] * L, pos = args[i].entries_offset - row;
      for (int32_t e = 0; e < args[i].n_entries; ++e) terms[at + e] = t->in[A_LOG][row + (pos + e) % L];
      args[i].entries_offset = at;
      at += args[i].n_entries;
    }
  }
  ABI(mraft_handle_append_entries_ex(h, args, m, terms, n_terms, rep, res, herr, MRAFT_HOST));
  for (int64_t i = 0; i < m; ++i) {
    if (herr[i] != MRAFT_ITEM_OK) return mismatch(v, path, "handle item_err", i, herr[i], 0);
    if (res[i].slot != slots[i]) return mismatch(v, path, "result slot", i, res[i].slot, slots[i]);
    if (res[i].peer != peers[i]) return mismatch(v, path, "result peer", i, res[i].peer, peers[i]);
    if (res[i].reply_success != rep[i].success || res[i].reply_term != rep[i].term ||
        res[i].reply_conflict_index != rep[i].conflict_index)
      return mismatch(v, path, "result reply fields", i, res[i].reply_success, rep[i].success);
  }
  /* one segment per leader replica: the records of one slot are adjacent */
  int64_t n_seg = 0;
  for (int64_t i = 0; i < m; ++i)
    if (i == 0 || res[i].slot != res[i - 1].slot) seg[n_seg++] = i;
  seg[n_seg] = m;
  ABI(mraft_process_append_replies(h, res, m, seg, n_seg, fflags, ferr, MRAFT_HOST));
  for (int64_t i = 0; i < m; ++i) {
    if (ferr[i] != MRAFT_ITEM_OK) return mismatch(v, path, "fold item_err", i, ferr[i], 0);
    if (fflags[i] & MRAFT_F_COMMITTED) flags[slots[i] / P] |= MRAFT_G_COMMITTED;
    if (fflags[i] & MRAFT_F_STEPPED_DOWN) flags[slots[i] / P] |= MRAFT_G_STEPPED_DOWN;
  }
  ABI(mraft_export_group_status(h, t->lp, commit, tl, MRAFT_HOST));
  /* a follower that advanced its commitIndex (raft_append_entry.go:157-160) */
  int32_t *fcommit = (int32_t *)zalloc((int64_t)G * P, sizeof(int32_t));
  NEED(fcommit);
  mraft_soa part;
  memset(&part, 0, sizeof part);
  part.commit_index = fcommit;
  ABI(mraft_store_state(h, &part, MRAFT_HOST));
  for (int32_t g = 0; g < G; ++g)
    for (int32_t p = 0; p < P; ++p)
      if (p != t->lp[g] && fcommit[g * P + p] > t->in[A_COMMIT][g * P + p]) flags[g] |= MRAFT_G_FOLLOWER_COMMIT;
  rc = check_engine(t, v, path, h, flags, commit, tl);

  free(slots); free(peers); free(gerr); free(herr); free(fflags); free(ferr);
  free(args); free(rep); free(res); free(seg); free(terms); free(fcommit);
  free(flags); free(commit); free(tl);
  return rc;
}

static int run_vector(FILE *f, int v, int device) {
  vec_t t;
  memset(&t, 0, sizeof t);
  int rc = read_vector(f, &t);
  if (!rc) rc = run_tick(&t, v, device, 0);
  if (!rc) rc = run_tick(&t, v, device, 1);
  if (!rc) rc = run_messages(&t, v, device, 0);
  if (!rc) rc = run_messages(&t, v, device, 1);
  if (!rc) {
    int committed = 0;
    for (int32_t g = 0; g < t.G; ++g) committed += (t.want_flags[g] & MRAFT_G_COMMITTED) != 0;
    printf("vector %d: %d x %d x %d: tick and light tick (2 shards), messages and by value: flags, GetState words and "
           "state bit-exact (%d groups committed)\n",
           v, (int)t.G, (int)t.P, (int)t.L, committed);
  }
  free_vector(&t);
  return rc;
}

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s tick_vectors.bin [device]\n", argv[0]);
    return 3;
  }
  const int device = argc > 2 ? atoi(argv[2]) : 0;
  if (mraft_abi_version() != MRAFT_ABI_VERSION) {
    fprintf(stderr, "library ABI %d, header %d\n", mraft_abi_version(), MRAFT_ABI_VERSION);
    return 2;
  }
  FILE *f = fopen(argv[1], "rb");
  if (!f) {
    perror(argv[1]);
    return 3;
  }
  char magic[4];
  int32_t hdr[2];
  if (fread(magic, 1, 4, f) != 4 || memcmp(magic, "MRTV", 4) != 0 || fread(hdr, sizeof hdr, 1, f) != 1 ||
      hdr[0] != 1 || hdr[1] < 1) {
    fprintf(stderr, "%s: not a version-1 tick vector file\n", argv[1]);
    fclose(f);
    return 3;
  }
  for (int v = 0; v < hdr[1]; ++v) {
    const int rc = run_vector(f, v, device);
    if (rc) {
      if (rc == 3) fprintf(stderr, "%s: truncated at vector %d\n", argv[1], v);
      fclose(f);
      return rc;
    }
  }
  fclose(f);
  printf("ok: %d vectors\n", (int)hdr[1]);
  return 0;
}
