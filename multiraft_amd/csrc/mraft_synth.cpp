// mraft_synth.cpp — seeded synthetic Multi-Raft workloads (include/mraft_synth.h).
//
// The states are synthetic but shaped like reachable Raft states: log terms
// are non-decreasing (the dummy entry first, raft_log.go:3-12), a follower's
// log is the leader's prefix up to a divergence point followed by a divergent
// tail written by an older leader (terms strictly below the leader's term at
// the divergence), and every AppendEntries is what appendOneRound would build
// from the leader's nextIndex (raft_append_entry.go:20-54).
#include "../../include/mraft_synth.h"

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

namespace {

struct Rng {
  uint64_t s;
  Rng(uint64_t seed, uint64_t g) : s(seed ^ (g * 0xD1B54A32D192ED03ull)) { next(); }
  uint64_t next() {  // splitmix64
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  uint32_t below(uint32_t n) { return n ? (uint32_t)(((next() >> 32) * (uint64_t)n) >> 32) : 0; }
  int32_t range(int32_t lo, int32_t hi) {  // inclusive; lo if hi < lo
    return hi <= lo ? lo : lo + (int32_t)below((uint32_t)(hi - lo + 1));
  }
};

// h-th largest (h = P/2) of matchIndex[j != lp]; the quorum index of a1.
int32_t quorum_match(const int32_t *m, int32_t P, int32_t lp) {
  std::vector<int32_t> v;
  for (int32_t j = 0; j < P; ++j)
    if (j != lp) v.push_back(m[j]);
  int32_t h = P / 2;
  if (h == 0 || v.empty()) return 0;
  std::sort(v.begin(), v.end(), [](int32_t a, int32_t b) { return a > b; });
  return v[(size_t)h - 1];
}

// terms_sorted (include/mraft.h) of a replica whose ring starts at 0: the
// terms of Index dummy+1 .. last never decrease.
int32_t sorted_after_dummy(const int32_t *row, int32_t dummy, int32_t last) {
  for (int32_t i = 1; i < last - dummy; ++i)
    if (row[i] > row[i + 1]) return 0;
  return 1;
}

void gen_group(uint64_t seed, int32_t g, int32_t gl, int32_t P, int32_t L,
               const mraft_soa *st, int32_t *leader_peer, int32_t *item_class) {
  Rng rng(seed, (uint64_t)g);
  const int32_t lp = g % P;
  const int64_t sb = (int64_t)gl * P;
  const int64_t ld = sb + lp;
  int32_t *lt = st->log_term + ld * L;

  // Leader log: dummy {0,0} then geometric runs (mean 16) of increasing terms.
  const int32_t last = L >= 2 ? L / 2 + (int32_t)rng.below((uint32_t)(L - L / 2)) : 0;
  std::vector<int32_t> r((size_t)last + 1, 0);
  if (last >= 1) r[1] = 1;
  for (int32_t s = 2; s <= last; ++s) r[s] = r[s - 1] + (rng.below(16) == 0 ? 1 + (int32_t)rng.below(3) : 0);
  const int32_t off = 4 + (int32_t)rng.below(30000);
  const bool fig8 = rng.below(4) == 0;  // 25%: no entry of the current term yet
  const int32_t T = r[last] + off;
  const int32_t shift = fig8 ? 1 + (int32_t)rng.below(3) : 0;
  lt[0] = 0;
  for (int32_t s = 1; s <= last; ++s) lt[s] = r[s] + off - shift;
  std::fill(lt + last + 1, lt + L, 0);

  int32_t *lmatch = st->match_index + ld * P;
  int32_t *lnext = st->next_index + ld * P;
  leader_peer[gl] = lp;
  if (item_class) item_class[ld] = -1;

  int32_t flasts[8] = {0}, fdummies[8] = {0}, cls[8] = {0};
  for (int32_t p = 0; p < P; ++p) {
    if (p == lp) continue;
    const int64_t f = sb + p;
    int32_t *fl = st->log_term + f * L;
    int32_t c;
    {
      uint32_t u = rng.below(100);
      c = u < 40 ? MRAFT_SYN_MATCH : u < 65 ? MRAFT_SYN_MISMATCH : u < 80 ? MRAFT_SYN_BEYOND
        : u < 90 ? MRAFT_SYN_STALE : u < 95 ? MRAFT_SYN_BELOW_DUMMY : MRAFT_SYN_HEARTBEAT;
    }
    if (last == 0 && c != MRAFT_SYN_STALE) c = MRAFT_SYN_HEARTBEAT;

    int32_t fdummy = 0, dp = last, t = 0, prev = last;
    // Divergence point snapped to a run boundary so that the tail's terms can
    // lie in [lt[dp], lt[dp+1]-1] and the follower log stays non-decreasing.
    auto snap = [&](int32_t d, int32_t lo) {
      while (d > lo && d < last && lt[d + 1] == lt[d]) --d;
      return d;
    };
    switch (c) {
      case MRAFT_SYN_MATCH:
      case MRAFT_SYN_STALE:
        dp = snap(rng.range(0, last), 0);
        t = (int32_t)rng.below(513);
        prev = rng.range(0, dp);
        break;
      case MRAFT_SYN_MISMATCH:
        dp = snap(rng.range(0, last - 1), 0);
        t = 1 + (int32_t)rng.below(512);
        break;
      case MRAFT_SYN_BEYOND:
        dp = snap(rng.range(0, last - 1), 0);
        t = std::min<int32_t>((int32_t)rng.below(513), last - 1 - dp);
        break;
      case MRAFT_SYN_BELOW_DUMMY:
        fdummy = 1 + (int32_t)rng.below((uint32_t)std::min(256, last));
        dp = snap(rng.range(fdummy, last), fdummy);
        t = (int32_t)rng.below(65);
        prev = rng.range(0, fdummy - 1);
        break;
      default:  // heartbeat: identical log, prev = last
        dp = last; t = 0; prev = last;
        break;
    }
    // Tail terms written by an older leader.
    int32_t lo = lt[dp], hi = dp < last ? lt[dp + 1] - 1 : T - 1;
    if (hi < lo) t = 0;
    t = std::min<int32_t>(t, (L - 1) - (dp - fdummy));
    const int32_t flast = dp + t;
    for (int32_t i = fdummy; i <= dp; ++i) fl[i - fdummy] = lt[i];
    int32_t cur = t > 0 ? lo + (int32_t)rng.below((uint32_t)(hi - lo + 1)) : 0;
    for (int32_t i = dp + 1; i <= flast; ++i) {
      fl[i - fdummy] = cur;
      if (cur < hi && rng.below(64) == 0) ++cur;  // runs of mean 64
    }
    std::fill(fl + (flast - fdummy) + 1, fl + L, 0);
    if (c == MRAFT_SYN_MISMATCH) prev = rng.range(dp + 1, std::min(flast, last));
    if (c == MRAFT_SYN_BEYOND) prev = rng.range(flast + 1, last);

    flasts[p] = flast; fdummies[p] = fdummy; cls[p] = c;
    lnext[p] = prev + 1;
    lmatch[p] = rng.range(0, prev);
    if (item_class) item_class[f] = c;
  }
  lmatch[lp] = 0;
  lnext[lp] = last + 1;
  const int32_t M = quorum_match(lmatch, P, lp);
  const int32_t lcommit = rng.range(0, std::min(M, last));

  st->current_term[ld] = T;
  st->voted_for[ld] = lp;
  st->state[ld] = MRAFT_LEADER;
  st->commit_index[ld] = lcommit;
  st->last_applied[ld] = lcommit;
  st->dummy_index[ld] = 0;
  if (st->log_head) st->log_head[ld] = 0;
  if (st->has_snapshot)
    for (int32_t p = 0; p < P; ++p) st->has_snapshot[sb + p] = 0;
  st->last_index[ld] = last;
  st->granted_votes[ld] = 0;
  if (st->persist_dirty)
    for (int32_t p = 0; p < P; ++p) st->persist_dirty[sb + p] = 0;

  for (int32_t p = 0; p < P; ++p) {
    if (p == lp) continue;
    const int64_t f = sb + p;
    const int32_t c = cls[p];
    st->current_term[f] = c == MRAFT_SYN_STALE ? T + 1 + (int32_t)rng.below(3) : T;
    st->voted_for[f] = rng.below(2) ? lp : -1;
    st->state[f] = (c == MRAFT_SYN_STALE && rng.below(2)) ? MRAFT_CANDIDATE : MRAFT_FOLLOWER;
    st->dummy_index[f] = fdummies[p];
    if (st->log_head) st->log_head[f] = 0;
    st->last_index[f] = flasts[p];
    const int32_t fc = rng.range(fdummies[p], std::max(fdummies[p], std::min(flasts[p], lcommit)));
    st->commit_index[f] = fc;
    st->last_applied[f] = fc;
    st->granted_votes[f] = 0;
    std::memset(st->match_index + f * P, 0, sizeof(int32_t) * (size_t)P);
    std::memset(st->next_index + f * P, 0, sizeof(int32_t) * (size_t)P);
  }
  if (st->terms_sorted)
    for (int32_t p = 0; p < P; ++p)
      st->terms_sorted[sb + p] =
          sorted_after_dummy(st->log_term + (sb + p) * L, st->dummy_index[sb + p], st->last_index[sb + p]);
}

}  // namespace

extern "C" int mraft_synth_tick_state(uint64_t seed, int32_t G, int32_t P, int32_t L,
                                      int32_t g_begin, int32_t g_end, const mraft_soa *st,
                                      int32_t *leader_peer, int32_t *item_class,
                                      int32_t nthreads) {
  if (!st || !leader_peer || P < 1 || P > 8 || L < 1 || g_begin < 0 || g_end > G ||
      g_begin > g_end)
    return MRAFT_E_INVAL;
  const mraft_soa *sp = st;
  auto work = [=](int32_t b, int32_t e) {
    for (int32_t g = b; g < e; ++g) gen_group(seed, g, g - g_begin, P, L, sp, leader_peer, item_class);
  };
  int32_t n = g_end - g_begin;
  if (nthreads <= 1 || n < 64) {
    work(g_begin, g_end);
    return MRAFT_OK;
  }
  nthreads = std::min(nthreads, 64);
  std::vector<std::thread> th;
  for (int32_t t = 0; t < nthreads; ++t) {
    int32_t b = g_begin + (int32_t)((int64_t)n * t / nthreads);
    int32_t e = g_begin + (int32_t)((int64_t)n * (t + 1) / nthreads);
    th.emplace_back(work, b, e);
  }
  for (auto &x : th) x.join();
  return MRAFT_OK;
}

extern "C" int64_t mraft_synth_fold_batch(uint64_t seed, int32_t G, int32_t P, int32_t L,
                                          const mraft_soa *st, const int32_t *leader_peer,
                                          mraft_ae_result *out, int64_t *seg_begin) {
  (void)L;
  int64_t n = 0;
  for (int32_t g = 0; g < G; ++g) {
    seg_begin[g] = n;
    Rng rng(seed ^ 0xF01DF01Dull, (uint64_t)g);
    const int32_t lp = leader_peer[g];
    const int64_t ld = (int64_t)g * P + lp;
    const int32_t T = st->current_term[ld], last = st->last_index[ld];
    for (int32_t p = 0; p < P; ++p) {
      if (p == lp) continue;
      mraft_ae_result &it = out[n++];
      it.slot = (int32_t)ld;
      it.peer = p;
      it.args_term = rng.below(20) == 0 ? T - 1 : T;
      it.args_prev_log_index = rng.below(10) == 0 ? rng.range(0, last)
                                                  : st->next_index[ld * P + p] - 1;
      const int32_t prev = it.args_prev_log_index;
      uint32_t u = rng.below(100);
      if (u < 70) {
        it.reply_term = T; it.reply_success = 1; it.reply_conflict_index = 0;
        it.args_n_entries = rng.range(0, std::max(0, last - prev));
      } else if (u < 90) {
        it.reply_term = T; it.reply_success = 0;
        it.reply_conflict_index = rng.range(1, prev + 1);
        it.args_n_entries = rng.range(0, std::max(0, last - prev));
      } else {
        it.reply_term = T + 1 + (int32_t)rng.below(3); it.reply_success = 0;
        it.reply_conflict_index = 0;
        it.args_n_entries = rng.range(0, std::max(0, last - prev));
      }
    }
  }
  seg_begin[G] = n;
  return n;
}

// Election storm (config #5): replicas with terms around a per-group base,
// votedFor in {-1, random} 50/50, short logs whose last entries differ by a
// few indices / terms (so isLogUpToDate goes both ways), and per round 1-3
// distinct timed-out peers per group.
extern "C" int mraft_synth_election_state(uint64_t seed, int32_t G, int32_t P, int32_t L,
                                          int32_t g_begin, int32_t g_end, const mraft_soa *st,
                                          uint8_t *cand_mask, int32_t rounds, int32_t nthreads) {
  if (!st || P < 1 || P > 8 || L < 4 || g_begin < 0 || g_end > G || g_begin > g_end || rounds < 0)
    return MRAFT_E_INVAL;
  const int32_t n = g_end - g_begin;
  auto work = [=](int32_t b, int32_t e) {
    for (int32_t g = b; g < e; ++g) {
      Rng rng(seed ^ 0xE1EC7ull, (uint64_t)g);
      const int64_t sb = (int64_t)(g - g_begin) * P;
      const int32_t T0 = 8 + (int32_t)rng.below(60000);
      const int32_t B = L / 2 + (int32_t)rng.below((uint32_t)(L / 2 - 2));
      for (int32_t p = 0; p < P; ++p) {
        const int64_t s = sb + p;
        st->current_term[s] = T0 + (int32_t)rng.below(3) - 1;
        st->voted_for[s] = rng.below(2) ? -1 : (int32_t)rng.below((uint32_t)P);
        st->state[s] = rng.below(8) == 0 ? MRAFT_CANDIDATE : MRAFT_FOLLOWER;
        st->granted_votes[s] = 0;
        if (st->persist_dirty) st->persist_dirty[s] = 0;
        st->dummy_index[s] = 0;
        if (st->log_head) st->log_head[s] = 0;
        if (st->has_snapshot) st->has_snapshot[s] = 0;
        int32_t last = B + (int32_t)rng.below(5) - 2;
        last = std::max(1, std::min(L - 1, last));
        st->last_index[s] = last;
        st->commit_index[s] = 0;
        st->last_applied[s] = 0;
        const int32_t lt = std::max(1, T0 - (int32_t)rng.below(3) - 1);
        int32_t *row = st->log_term + s * L;
        row[0] = 0;
        for (int32_t k = 1; k <= last; ++k) row[k] = std::max(1, lt - (last - k) / 2);
        for (int32_t k = last + 1; k < L; ++k) row[k] = 0;
        if (st->terms_sorted) st->terms_sorted[s] = sorted_after_dummy(row, 0, last);
        std::memset(st->match_index + s * P, 0, sizeof(int32_t) * (size_t)P);
        std::memset(st->next_index + s * P, 0, sizeof(int32_t) * (size_t)P);
      }
      for (int32_t r = 0; r < rounds; ++r) {
        uint32_t m = 0;
        const int32_t c = 1 + (int32_t)rng.below(3);
        for (int32_t k = 0; k < c; ++k) m |= 1u << rng.below((uint32_t)P);
        cand_mask[(int64_t)r * n + (g - g_begin)] = (uint8_t)m;
      }
    }
  };
  if (nthreads <= 1 || n < 64) {
    work(g_begin, g_end);
    return MRAFT_OK;
  }
  nthreads = std::min(nthreads, 64);
  std::vector<std::thread> th;
  for (int32_t t = 0; t < nthreads; ++t)
    th.emplace_back(work, g_begin + (int32_t)((int64_t)n * t / nthreads),
                    g_begin + (int32_t)((int64_t)n * (t + 1) / nthreads));
  for (auto &x : th) x.join();
  return MRAFT_OK;
}
