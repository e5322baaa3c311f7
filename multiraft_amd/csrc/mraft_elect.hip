// mraft_elect.hip — the election storm (SURVEY.md §8a rows a5-a6, §8d
// config #5) for gfx950: one lane per replica, eight lanes per group (eight
// groups per wave); each replica's election state (term, votedFor, role,
// grantedVotes, last index/term) lives in registers for all R rounds of one
// launch, so HBM is touched once on entry and once on exit. Per round: timeouts -> StartElection (raft_election.go:4-15) in peer
// order, every RequestVote delivered voter by voter in candidate order
// (HandleRequestVote :54-77 with isLogUpToDate, raft_log.go:99-104), every
// candidate's tally in voter order (closure :22-47).
//
// Round 5 (profiles/r5_e1 README): one lane per group, two lanes per group,
// a dense voter loop, a branch-free vote-key loop and LDS-staged round masks
// were all measured (parity green) and all slower; this layout hides its
// dependent chains with 8 waves per SIMD. Round 6 (profiles/r6_e1): the
// instruction account of the round body matched the counters exactly (84 VALU
// + 19 SALU per wave-round plus 29 + 13 per candidate, 3.0 candidates per
// wave-round), fewer instructions per candidate alone changed nothing, and
// taking the per-candidate LDS round trip out of the delivery loop's
// dependent chain (candidates ranked once per round, held in registers) took
// the storm 9 % down; the loop's conditions as bitwise ops (no exec-mask
// region per candidate: 126 -> 77 SALU per round body) 1.5 % more
// (profiles/r6_d1).
#include "mraft_device.h"
#include "mraft_internal.h"

namespace mraft {

namespace {

template <int P>
__global__ __launch_bounds__(256) void k_election_rounds(Dev s, const uint8_t *__restrict__ cand,
                                                         int R, int32_t *__restrict__ gflags) {
  // Lane p of an 8-lane segment holds replica p of group g (P <= 8): voters
  // and candidates work in parallel, candidate data is broadcast inside the
  // segment (__shfl width 8).
  const int tid = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int g = tid >> 3, p = tid & 7;
  const bool grp = g < s.G;  // uniform over the segment
  const bool act = grp && p < P;
  const long long sl = (long long)g * P + p;
  int term = 0, voted = -1, role = kFollower, votes = 0, last = 0, lterm = 0;
  if (act) {
    term = s.term[sl];
    voted = s.voted[sl];
    role = s.role[sl];
    votes = s.votes[sl];
    last = s.last[sl];
    lterm = term_at(s, sl, s.dummy[sl], s.head[sl], last);             // lastEntry, raft_log.go:50-53
  }
  // votedFor as a bit: 1 << votedFor, 0 for -1, kVJunk for a value outside
  // [-1, P) (no candidate ever equals it, as in Go's compare at :69-74)
  constexpr int kVJunk = 0x100;
  const int pb = 1 << p;
  int vb = voted == -1 ? 0 : ((unsigned)voted < (unsigned)P ? 1 << voted : kVJunk);
  // The logs do not change during an election storm, so isLogUpToDate of
  // every candidate's (lastTerm, lastIndex) against this voter's
  // (raft_log.go:99-104) is fixed for the launch: bit c of upm.
  int upm = 0;
#pragma unroll
  for (int c = 0; c < P; ++c) {
    const int clt = __shfl(lterm, c, 8), clast = __shfl(last, c, 8);
    upm |= (int)(clt > lterm || (clt == lterm && clast >= last)) << c;
  }
  __shared__ int lds_cx[256];
  __shared__ __attribute__((aligned(8))) uint8_t lds_gm[256];
  __shared__ int lds_rt[256];                                  // rank k's args.Term, per segment
  __shared__ __attribute__((aligned(8))) uint8_t lds_rc[256];  // rank k's peer index
  const int seg = (int)(threadIdx.x & 63) & ~7;
  int fl = 0, became = 0, pd = 0;  // pd: persist() ran (StartElection :15, HandleRequestVote :57, :45)
  // The round's timeout mask, loaded one round ahead. (Staging 64 rounds of
  // masks through LDS per cooperative load measured 1 % slower, r5_c1 / r5_e3.)
  int mnext = (grp && R > 0) ? (int)cand[g] : 0;
  for (int r = 0; r < R; ++r) {
    const int m = mnext;
    if (grp && r + 1 < R) mnext = (int)cand[(long long)(r + 1) * s.G + g];
    const int isc = act && ((m >> p) & 1) && role != kLeader;
    if (isc) {                                                         // StartElection :6-17
      role = kCandidate;
      term += 1;
      vb = pb;
      votes = 1;
      pd = 1;
    }
    const int at = term;  // args.Term of this lane's RequestVote (when isc); voter's term before RVs
    int cx[8];
    // One broadcast per replica per round, through this wave's LDS words: its
    // term with the candidate bit on top.
    const int mycx = at;
    lds_cx[threadIdx.x] = mycx;
    __builtin_amdgcn_wave_barrier();
    {
      const int4 a = *reinterpret_cast<const int4 *>(&lds_cx[threadIdx.x & ~7u]);
      const int4 b = *reinterpret_cast<const int4 *>(&lds_cx[(threadIdx.x & ~7u) + 4]);
      cx[0] = a.x; cx[1] = a.y; cx[2] = a.z; cx[3] = a.w;
      cx[4] = b.x; cx[5] = b.y; cx[6] = b.z; cx[7] = b.w;
    }
    // RequestVote deliveries: voter p handles the candidates in peer order
    // (HandleRequestVote :54-77). pmx = max args.Term over candidates c <= p,
    // which with the voter's own pre-delivery term gives every reply.Term the
    // tally below needs (a voter's term after handling c is the max of the
    // two, the stale branch included).
    int gm = 0, pmx = INT32_MIN;
    // The segment's candidate mask (ascending peer order is the delivery order).
    const unsigned long long cb = __ballot(isc);
    const int cm = (int)((cb >> seg) & 0xffull);
    pd |= (int)(act && (cm & ~(1 << p)) != 0);                         // :57, every RV this voter handles
    // The segment's candidates ranked in peer order: rank k's args.Term and
    // peer index staged through LDS once per round and held in registers, so
    // the delivery loop has no LDS round trip per candidate and a compile-time
    // register index per iteration (round 6: 0.164 -> 0.149 ms per storm;
    // round 5's loop walked the candidate mask with a ds_bpermute per
    // candidate in its dependent chain, profiles/r6_e1)
    {
      // every lane writes one rank slot: a candidate its rank (args.Term, its
      // bit), the others the slots past the segment's candidates (INT_MIN, bit
      // 0: a delivery that changes nothing), so the loop needs no validity test
      const int ncand = __builtin_popcount(cm);
      const int rk = __builtin_popcount(cm & (pb - 1));
      const int pos = isc ? rk : ncand + p - rk;
      lds_rt[(threadIdx.x & ~7u) + pos] = isc ? at : INT32_MIN;
      lds_rc[(threadIdx.x & ~7u) + pos] = (uint8_t)(isc ? pb : 0);
      __builtin_amdgcn_wave_barrier();
      const int4 ra = *reinterpret_cast<const int4 *>(&lds_rt[threadIdx.x & ~7u]);
      const int4 rb = *reinterpret_cast<const int4 *>(&lds_rt[(threadIdx.x & ~7u) + 4]);
      const unsigned long long rcs = *reinterpret_cast<const unsigned long long *>(&lds_rc[threadIdx.x & ~7u]);
      __builtin_amdgcn_wave_barrier();
      const int rt[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
      // A candidate's delivery to itself (cb == pb) changes nothing: its term
      // is at >= cat, and at term == at its vote is already its own; the grant
      // bit it sets in gm is masked out of its tally (om). So no c != p test.
#pragma unroll
      for (int k = 0; k < P; ++k) {
        if (!__ballot(k < ncand)) break;
        const int cb = (int)((rcs >> (8 * k)) & 0xffull);
        const int cat = rt[k];
        pmx = cb <= pb ? max(pmx, cat) : pmx;                          // c <= p
        const bool gt = cat > term;                                    // :63-66
        const bool ge = cat >= term;                                   // :59-62 (stale: no change)
        term = gt ? cat : term;
        vb = gt ? 0 : vb;
        const bool grant = ge & (((vb & ~cb) | (cb & ~upm)) == 0);     // :69-74
        vb = grant ? cb : vb;
        gm |= grant ? cb : 0;
      }
      role = term > at ? kFollower : role;                             // :63-66 (some RV carried a higher term)
    }
    // Grants transposed through LDS: byte v of the segment's word = voter v's
    // grant mask; bit v of mine = voter v granted this lane.
    int mine = 0;
    {
      lds_gm[threadIdx.x] = (uint8_t)gm;
      __builtin_amdgcn_wave_barrier();
      const unsigned long long gw = *reinterpret_cast<const unsigned long long *>(&lds_gm[threadIdx.x & ~7u]);
      mine = (int)((((gw >> p) & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56);
      __builtin_amdgcn_wave_barrier();
    }
    // Tally (closure :22-47): candidate p folds its replies in voter order.
    // The guard (:29) can only flip at the first event, becoming leader at the
    // grant that makes a majority (:32-38) or stepping down at the first
    // refusal whose reply.Term exceeds args.Term (:42-45), so the fold is
    // closed-form: whichever of the two positions comes first in voter order.
    {
      const bool ok0 = isc && term == at && role == kCandidate;
      const int om = ((1 << P) - 1) & ~(1 << p);
      int gt = 0, tv = 0;
#pragma unroll
      for (int v = 0; v < P; ++v) gt |= (int)((cx[v]) > at) << v;
      // reply.Term = max(voter's own term, pmx) > at: every refusal when pmx > at.
      const int smask = om & ~mine & (pmx > at ? om : gt);
      int mm = mine & om;
#pragma unroll
      for (int k = 1; k < (P / 2 > 1 ? P / 2 : 1); ++k) mm &= mm - 1;  // the (P/2)-th grant
      const int lpos = mm ? __builtin_ctz(mm) : 32;
      const int spos = smask ? __builtin_ctz(smask) : 32;
      tv = lds_cx[(threadIdx.x & ~7u) + min(spos, 7)];  // used only when spos < P
      const bool lead = ok0 && lpos < spos;
      const bool sd = ok0 && spos < lpos;
      const int upos = lead ? lpos + 1 : spos;                          // < 32 when lead | sd
      const int upto = (lead | sd) ? (int)((1u << (upos & 31)) - 1u) : -1;
      votes += ok0 ? __builtin_popcount(mine & om & upto) : 0;                // :31
      role = lead ? kLeader : sd ? kFollower : role;
      became |= (int)lead;
      fl |= lead ? MRAFT_G_ELECTED : 0;
      term = sd ? max(tv, pmx) : term;
      vb = sd ? 0 : vb;
      fl |= sd ? MRAFT_G_STEPPED_DOWN : 0;
    }
  }
  const unsigned long long el = __ballot(fl & MRAFT_G_ELECTED), sd = __ballot(fl & MRAFT_G_STEPPED_DOWN);
  if (grp && p == 0 && gflags) {
    gflags[g] = (((el >> seg) & 0xffull) ? MRAFT_G_ELECTED : 0) |
                (((sd >> seg) & 0xffull) ? MRAFT_G_STEPPED_DOWN : 0);
  }
  if (!act) return;
  s.term[sl] = term;
  s.voted[sl] = (vb & kVJunk) ? voted : (vb ? __builtin_ctz(vb) : -1);
  s.role[sl] = role;
  s.votes[sl] = votes;
  if (pd) mark_persist(s, sl, MRAFT_PERSIST_STATE);
  if (became) {
#pragma unroll
    for (int j = 0; j < P; ++j) {
      s.match[sl * P + j] = 0;
      s.next[sl * P + j] = last + 1;
    }
  }
}

}  // namespace

void launch_election_rounds(const Dev &s, const uint8_t *cand, int R, int32_t *gflags,
                            hipStream_t st) {
  const dim3 gr((unsigned)(((long long)s.G * 8 + 255) / 256)), bl(256);
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
