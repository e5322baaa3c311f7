// mraft_elect.hip — the election storm (SURVEY.md §8a rows a5-a6, §8d
// config #5) for gfx950: one lane per group; the P replicas' election state
// (term, votedFor, role, grantedVotes, last index/term) lives in registers for
// all R rounds of one launch, so HBM is touched once on entry and once on
// exit. Per round: timeouts -> StartElection (raft_election.go:4-15) in peer
// order, every RequestVote delivered voter by voter in candidate order
// (HandleRequestVote :54-77 with isLogUpToDate, raft_log.go:99-104), every
// candidate's tally in voter order (closure :22-47).
#include "mraft_device.h"
#include "mraft_internal.h"

namespace mraft {

namespace {

template <int P>
__global__ __launch_bounds__(256) void k_election_rounds(Dev s, const uint8_t *__restrict__ cand,
                                                         int R, int32_t *__restrict__ gflags) {
  const int g = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (g >= s.G) return;
  const long long b = (long long)g * P;
  int term[P], voted[P], role[P], votes[P], last[P], lterm[P], became[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    term[p] = s.term[b + p];
    voted[p] = s.voted[b + p];
    role[p] = s.role[b + p];
    votes[p] = s.votes[b + p];
    last[p] = s.last[b + p];
    became[p] = 0;
  }
#pragma unroll
  for (int p = 0; p < P; ++p) lterm[p] = s.log[(b + p) * s.L + (last[p] - s.dummy[b + p])];  // lastEntry
  int fl = 0, pdm = 0;  // pdm: replicas that ran persist() (StartElection :15, HandleRequestVote :57)
  for (int r = 0; r < R; ++r) {
    const int m = cand[(long long)r * s.G + g];
    int isc[P], at[P];
#pragma unroll
    for (int p = 0; p < P; ++p) {                                      // StartElection :6-17
      isc[p] = ((m >> p) & 1) && role[p] != kLeader;
      if (isc[p]) {
        pdm |= 1 << p;
        role[p] = kCandidate;
        term[p] += 1;
        voted[p] = p;
        votes[p] = 1;
      }
      at[p] = term[p];
    }
    int rt[P][P], rg[P][P];  // reply of voter v to candidate c
#pragma unroll
    for (int v = 0; v < P; ++v) {
#pragma unroll
      for (int c = 0; c < P; ++c) {
        rt[c][v] = 0;
        rg[c][v] = 0;
        if (!isc[c] || c == v) continue;
        pdm |= 1 << v;
        if (at[c] < term[v]) {                                         // :59-62
          rt[c][v] = term[v];
          continue;
        }
        if (at[c] > term[v]) {                                         // :63-66
          role[v] = kFollower;
          term[v] = at[c];
          voted[v] = -1;
        }
        rt[c][v] = term[v];                                            // :67
        const bool up = lterm[c] > lterm[v] || (lterm[v] == lterm[c] && last[c] >= last[v]);
        if ((voted[v] == -1 || voted[v] == c) && up) {                 // :69-74
          voted[v] = c;
          rg[c][v] = 1;
        }
      }
    }
#pragma unroll
    for (int c = 0; c < P; ++c) {                                      // tally :24-47
      if (!isc[c]) continue;
#pragma unroll
      for (int v = 0; v < P; ++v) {
        if (v == c) continue;
        if (term[c] == at[c] && role[c] == kCandidate) {               // :29
          if (rg[c][v]) {
            votes[c] += 1;                                             // :31
            if (votes[c] > P / 2) {                                    // :32-38
              role[c] = kLeader;
              became[c] = 1;
              fl |= MRAFT_G_ELECTED;
            }
          } else if (rt[c][v] > term[c]) {                             // :42-45
            role[c] = kFollower;
            term[c] = rt[c][v];
            voted[c] = -1;
            fl |= MRAFT_G_STEPPED_DOWN;
          }
        }
      }
    }
  }
#pragma unroll
  for (int p = 0; p < P; ++p) {
    s.term[b + p] = term[p];
    s.voted[b + p] = voted[p];
    s.role[b + p] = role[p];
    s.votes[b + p] = votes[p];
    if ((pdm >> p) & 1) mark_persist(s, b + p, MRAFT_PERSIST_STATE);
    if (became[p]) {
      for (int j = 0; j < P; ++j) {
        s.match[(b + p) * P + j] = 0;
        s.next[(b + p) * P + j] = last[p] + 1;
      }
    }
  }
  if (gflags) gflags[g] = fl;
}

}  // namespace

void launch_election_rounds(const Dev &s, const uint8_t *cand, int R, int32_t *gflags,
                            hipStream_t st) {
  const dim3 gr((s.G + 255) / 256), bl(256);
  switch (s.P) {
#define MRAFT_EL_CASE(PP) \
  case PP: hipLaunchKernelGGL(k_election_rounds<PP>, gr, bl, 0, st, s, cand, R, gflags); break;
    MRAFT_EL_CASE(1) MRAFT_EL_CASE(2) MRAFT_EL_CASE(3) MRAFT_EL_CASE(4)
    MRAFT_EL_CASE(5) MRAFT_EL_CASE(6) MRAFT_EL_CASE(7) MRAFT_EL_CASE(8)
#undef MRAFT_EL_CASE
    default: break;
  }
}

}  // namespace mraft
