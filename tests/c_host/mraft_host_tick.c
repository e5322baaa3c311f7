/*
 * mraft_host_tick.c — a plain C11 host of libmraft_hip.so: it includes only
 * include/mraft.h and links the library the way a cgo binding does
 * (INTEGRATION.md), with no HIP header, no C++ and no Python in between.
 *
 * For every seeded tick vector of tests/golden/tick_vectors.bin (written by
 * tests/golden/make_golden.py from tick_vectors.npz: inputs from the seeded
 * generator, expected outputs from the pure-Python restatement of
 * src/raft/raft_append_entry.go:20-162) it runs the reference's per-tick
 * sequence through the boundary:
 *   mraft_create (Make, src/raft/raft.go:51-87) -> mraft_load_state
 *   (readPersist, raft.go:217-235) -> mraft_set_tick_shards(2) ->
 *   mraft_replicate_tick_export (appendOneRound + HandleAppendEntries +
 *   processAppendEntriesReply + GetState, raft.go:237-246) -> mraft_store_state
 *   -> mraft_destroy (Kill, src/raft/utility.go:9-19)
 * and compares the group flags, the exported GetState words and every state
 * array (logs in Index order over the live entries) with the fixture.
 *
 * Usage: mraft_host_tick <tick_vectors.bin> [device]. Exit status 0 = every
 * vector bit-exact; 1 = a mismatch; 2 = an ABI error; 3 = a bad fixture.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mraft.h"

#define N_ARR 12

/* The fixture's array order (make_golden.py tick_vectors_bin). */
static const char *const k_names[N_ARR] = {
    "current_term", "voted_for", "state", "commit_index", "last_applied", "dummy_index",
    "last_index", "granted_votes", "log_term", "match_index", "next_index", "persist_dirty"};

static int64_t arr_len(int i, int64_t gp, int64_t P, int64_t L) {
  return i == 8 ? gp * L : (i == 9 || i == 10) ? gp * P : gp;
}

static int32_t **slot_of(mraft_soa *s, int i) {
  int32_t **t[N_ARR] = {&s->current_term, &s->voted_for, &s->state, &s->commit_index,
                        &s->last_applied, &s->dummy_index, &s->last_index, &s->granted_votes,
                        &s->log_term, &s->match_index, &s->next_index, &s->persist_dirty};
  return t[i];
}

static int32_t *read_i32(FILE *f, int64_t n) {
  int32_t *p = (int32_t *)calloc((size_t)(n > 0 ? n : 1), sizeof(int32_t));
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

static int mismatch(int v, const char *what, int64_t at, int32_t got, int32_t want) {
  fprintf(stderr, "vector %d: %s differs at %lld: %d vs %d\n", v, what, (long long)at, (int)got, (int)want);
  return 1;
}

static int run_vector(FILE *f, int v, int device) {
  int32_t dims[3];
  if (fread(dims, sizeof dims, 1, f) != 1) return 3;
  const int32_t G = dims[0], P = dims[1], L = dims[2];
  const int64_t gp = (int64_t)G * P;
  int32_t *lp = read_i32(f, G), *want_flags = read_i32(f, G), *want_commit = read_i32(f, G),
          *want_tl = read_i32(f, G);
  int32_t *in[N_ARR], *want[N_ARR], *got[N_ARR];
  if (!lp || !want_flags || !want_commit || !want_tl) return 3;
  for (int i = 0; i < N_ARR; ++i)
    if (!(in[i] = read_i32(f, arr_len(i, gp, P, L)))) return 3;
  for (int i = 0; i < N_ARR; ++i)
    if (!(want[i] = read_i32(f, arr_len(i, gp, P, L)))) return 3;
  for (int i = 0; i < N_ARR; ++i)
    if (!(got[i] = (int32_t *)calloc((size_t)arr_len(i, gp, P, L), sizeof(int32_t)))) return 3;
  /* the fixture predates the ring and the terms_sorted proof: heads 0 (Index
     dummy at row position 0), no snapshot pending; terms_sorted is recomputed
     by mraft_load_state from the logs whatever the source holds */
  int32_t *zeros = (int32_t *)calloc((size_t)gp, sizeof(int32_t));
  int32_t *head = (int32_t *)calloc((size_t)gp, sizeof(int32_t));
  int32_t *hsnap = (int32_t *)calloc((size_t)gp, sizeof(int32_t));
  int32_t *srt = (int32_t *)calloc((size_t)gp, sizeof(int32_t));
  int32_t *flags = (int32_t *)calloc((size_t)G, sizeof(int32_t));
  int32_t *commit = (int32_t *)calloc((size_t)G, sizeof(int32_t));
  int32_t *tl = (int32_t *)calloc((size_t)G, sizeof(int32_t));
  if (!zeros || !head || !hsnap || !srt || !flags || !commit || !tl) return 3;

  mraft_engine *h = NULL;
  ABI(mraft_create(G, P, L, device, 0, &h));
  mraft_soa src, dst;
  memset(&src, 0, sizeof src);
  memset(&dst, 0, sizeof dst);
  for (int i = 0; i < N_ARR; ++i) {
    *slot_of(&src, i) = in[i];
    *slot_of(&dst, i) = got[i];
  }
  src.log_head = zeros;
  src.has_snapshot = zeros;
  src.terms_sorted = zeros;
  dst.log_head = head;
  dst.has_snapshot = hsnap;
  dst.terms_sorted = srt;
  ABI(mraft_load_state(h, &src, MRAFT_HOST));
  const int32_t shards = G >= 2 ? 2 : 1;
  ABI(mraft_set_tick_shards(h, shards));
  if (mraft_get_tick_shards(h) != shards) {
    fprintf(stderr, "vector %d: mraft_get_tick_shards = %d, want %d\n", v, mraft_get_tick_shards(h), shards);
    return 2;
  }
  ABI(mraft_replicate_tick_export(h, lp, flags, commit, tl, MRAFT_HOST));
  ABI(mraft_store_state(h, &dst, MRAFT_HOST));
  ABI(mraft_destroy(h));

  for (int32_t g = 0; g < G; ++g) {
    if (flags[g] != want_flags[g]) return mismatch(v, "group_flags", g, flags[g], want_flags[g]);
    if (commit[g] != want_commit[g]) return mismatch(v, "export commit", g, commit[g], want_commit[g]);
    if (tl[g] != want_tl[g]) return mismatch(v, "export term<<1|leader", g, tl[g], want_tl[g]);
  }
  for (int i = 0; i < N_ARR; ++i) {
    if (i == 8) continue; /* logs: below, in Index order */
    for (int64_t k = 0; k < arr_len(i, gp, P, L); ++k)
      if (got[i][k] != want[i][k]) return mismatch(v, k_names[i], k, got[i][k], want[i][k]);
  }
  /* logs: Index dummy..last of every replica, at ring position
     (head + Index - dummy) mod L in the engine, at Index - dummy in the fixture */
  const int32_t *dummy = want[5], *last = want[6];
  for (int64_t s = 0; s < gp; ++s) {
    if (head[s] < 0 || head[s] >= L) return mismatch(v, "log_head", s, head[s], 0);
    for (int32_t i = dummy[s]; i <= last[s]; ++i) {
      const int64_t k = i - dummy[s];
      const int32_t a = got[8][s * L + (head[s] + k) % L], b = want[8][s * L + k];
      if (a != b) return mismatch(v, "log_term (slot*L + Index - dummy)", s * L + k, a, b);
    }
    /* terms_sorted is a proof: 1 only over non-decreasing terms after the dummy */
    if (srt[s]) {
      for (int32_t i = dummy[s] + 1; i < last[s]; ++i) {
        const int64_t k = i - dummy[s];
        if (want[8][s * L + k] > want[8][s * L + k + 1]) return mismatch(v, "terms_sorted (unsound)", s, 1, 0);
      }
    }
  }
  int committed = 0;
  for (int32_t g = 0; g < G; ++g) committed += (flags[g] & MRAFT_G_COMMITTED) != 0;
  printf("vector %d: %d x %d x %d, %d tick shards: flags, GetState words and state bit-exact (%d groups committed)\n",
         v, (int)G, (int)P, (int)L, (int)shards, committed);
  for (int i = 0; i < N_ARR; ++i) {
    free(in[i]);
    free(want[i]);
    free(got[i]);
  }
  free(lp); free(want_flags); free(want_commit); free(want_tl);
  free(zeros); free(head); free(hsnap); free(srt); free(flags); free(commit); free(tl);
  return 0;
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
