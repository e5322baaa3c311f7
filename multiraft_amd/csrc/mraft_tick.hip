// mraft_tick.hip — the fused co-resident replication tick (SURVEY.md §8a rows
// a1-a4) for gfx950: one 64-lane wave per Raft group, one group per 64-thread
// workgroup (a wave's slot is released the moment its group is done; with
// 4-wave workgroups a finished wave held its slot until its siblings ended,
// idling ~18 % of the slots — tools/trace_tick.py).
//
// Per group (wave):
//   header   wave-uniform scalar loads of the leader replica (role, term,
//            commit, last, dummy);
//   phase A  lane per follower: appendOneRound's args gather
//            (raft_append_entry.go:20-54) and HandleAppendEntries up to
//            matchLog (:108-133): term check/adoption, prev < dummy,
//            prev > last, prev-term match;
//   phase B  wave-cooperative: the ConflictIndex backward scans (:136-142) and
//            ONE streaming pass over the leader's log tail that serves every
//            follower's entry merge at once (:149-155): each 256-entry chunk of
//            the leader log is loaded once (dwordx4 per lane) and compared
//            against / copied into every follower whose range covers it, the
//            first mismatch of each follower found by ballot. The reference
//            copies the tail into every follower's args (:50-54); here the
//            leader's entries cross HBM once per group;
//   phase C  lane per follower: follower state write-back, follower commit
//            (:157-160);
//   phase D  wave-uniform fold of the replies in peer order
//            (processAppendEntriesReply, :66-88) with the quorum order
//            statistic over matchIndex in registers, and the current-term gate
//            of advanceCommitIndexForLeader (:89-105): one probe of
//            log[min(M*, last)], a wave-cooperative downward scan only when it
//            misses (Figure-8 groups).
//
// COUNT=true runs the same decisions with no state store and accumulates the
// algorithmic word count of DESIGN.md §4 (reads, writes, active groups).
#include "mraft_device.h"
#include "mraft_internal.h"
#include "mraft_pass.h"

namespace mraft {

namespace {

enum : int {
  IC_NONE = 0,  // no AppendEntries for this item
  IC_SNAP,      // prev < leader dummy: InstallSnapshot path
  IC_PANIC,     // prev > leader last: Go panics
  IC_GO,        // args gathered
  IC_STALE,     // args.Term < currentTerm
  IC_BELOW,     // prev < follower dummy
  IC_BEYOND,    // prev > follower last
  IC_MISMATCH,  // term(prev) differs, ConflictIndex known without a scan
  IC_SCAN,      // term(prev) differs, ConflictIndex needs the backward scan
  IC_MERGE,     // prefix matches, n > 0 entries to merge
  IC_HB,        // prefix matches, heartbeat
  IC_FULL,      // merge would exceed capacity L: rejected
  IC_IS_STALE,  // InstallSnapshot, args.Term < currentTerm (raft_snapshot.go:20-22)
  IC_IS_OLD,    // InstallSnapshot, outdated snapshot (:31-33)
  IC_IS_INSTALL,// InstallSnapshot installed (:35-50)
  IC_IS_PANIC   // InstallSnapshot whose sliceFrom would panic: dropped
};

template <int P>
__device__ __forceinline__ int quorum_match(const int (&m)[P], int lp) {
  // h-th largest (h = P/2) of matchIndex[j != me]: the largest i for which
  // #{j != me : matchIndex[j] >= i} + 1 > P/2 (raft_append_entry.go:91-98).
  constexpr int h = P / 2;
  int best = INT32_MIN;
#pragma unroll
  for (int j = 0; j < P; ++j) {
    if (j == lp) continue;
    int c = 0;
#pragma unroll
    for (int q = 0; q < P; ++q) c += (q != lp && m[q] >= m[j]) ? 1 : 0;
    if (c >= h && m[j] > best) best = m[j];
  }
  return best;
}

__device__ __forceinline__ long long interval_len(long long a, long long b) {
  return b >= a ? b - a + 1 : 0;
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// The state pointers again, read afresh from the kernel-argument segment (the
// tick's first argument is the Dev struct). Phase C/D use this copy, so the
// entry copy of the ~14 array pointers dies after the header instead of being
// held (and spilled) across the streaming pass; the segment pointer is passed
// through an empty asm so the loads are new scalar loads, not the entry ones.
__device__ __forceinline__ Dev reload_dev() {
  const __attribute__((address_space(4))) Dev *kp =
      (const __attribute__((address_space(4))) Dev *)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(kp));
  Dev d;
  d.term = kp->term; d.voted = kp->voted; d.role = kp->role; d.commit = kp->commit;
  d.applied = kp->applied; d.dummy = kp->dummy; d.last = kp->last; d.votes = kp->votes;
  d.log = kp->log; d.match = kp->match; d.next = kp->next; d.pdirty = kp->pdirty;
  d.head = kp->head; d.hsnap = kp->hsnap; d.srt = kp->srt; d.G = kp->G; d.P = kp->P; d.L = kp->L;
  return d;
}

// Reply fold of one group (processAppendEntriesReply, :66-88, in peer order),
// wave-uniform. Inputs per follower slot q come from lane q. The fold keeps
// only what the rest of the tick needs (bit q of gate_m: the reply passed the
// term/state/prev gate; of rs_m: it set matchIndex), so little wave-uniform
// state stays live across the streaming pass; phase D recomputes each lane's
// nextIndex / matchIndex from its own item. COUNT keeps the per-reply arrays
// the algorithmic word count reads.
template <int P, bool COUNT>
struct Fold {
  static constexpr int NI = P - 1;
  static constexpr int NA = COUNT ? NI : 1;
  int term, stepped, any, mstar, gate_m, rs_m;
  int rp[NA], ic[NA];

  // is_m: followers whose reply is an InstallSnapshot reply
  // (processInstallSnapshotReply, raft_snapshot.go:56-69) for
  // LastIncludedIndex lii; their (prev, n) read (lii, 0).
  __device__ __forceinline__ void run(int T, int lp, int (&mm)[P], int have_m, int succ_m, int is_m, int lii,
                                      int rterm, int prev, int n, int rci, int icls) {
    term = T;
    stepped = 0;
    any = 0;
    mstar = INT32_MIN;
    gate_m = 0;
    rs_m = 0;
    int role = kLeader;
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const int pq = q < lp ? q : q + 1;
      int qrp = uni(__shfl(prev, q, 64)), qrn = uni(__shfl(n, q, 64));
      const int qic = uni(__shfl(icls, q, 64));
      if (qic >= IC_IS_STALE) {
        qrp = lii;
        qrn = 0;
      }
      if (COUNT) {
        rp[q < NA ? q : 0] = qrp;
        ic[q < NA ? q : 0] = qic;
      }
      const int rt = uni(__shfl(rterm, q, 64));
      if (!((have_m >> q) & 1)) continue;
      if (rt > term) {                                                   // :67-72, snapshot :59-64
        term = rt;
        role = kFollower;
        stepped = 1;
      } else if ((is_m >> q) & 1) {
        if (role == kLeader && T == term) {                              // snapshot :65-67
          gate_m |= 1 << q;
          rs_m |= 1 << q;
#pragma unroll
          for (int j = 0; j < P; ++j)
            if (j == pq) mm[j] = lii;
        }
      } else if (rt == term && role == kLeader && T == term) {           // :73-74 (prev gate holds)
        gate_m |= 1 << q;
        if ((succ_m >> q) & 1) {
          rs_m |= 1 << q;
#pragma unroll
          for (int j = 0; j < P; ++j)
            if (j == pq) mm[j] = qrp + qrn;                              // :76
          mstar = max(mstar, quorum_match<P>(mm, lp));                   // :78 -> a1
          any = 1;
        }
      }
    }
  }
};

#ifndef MRAFT_TICK_MINW
#define MRAFT_TICK_MINW 8  // __launch_bounds__ minimum waves per SIMD
#endif
#ifndef MRAFT_TICK_ALIGN
#define MRAFT_TICK_ALIGN 32  // pass chunks start on this many entries (32 = one 128-B line)
#endif
#ifndef MRAFT_TICK_TRACE
#define MRAFT_TICK_TRACE 0  // diagnostic build: s_memrealtime stamps per group (tools/trace_tick.py)
#endif
#if MRAFT_TICK_TRACE
__device__ unsigned long long g_tick_trace[65536 * 4];
// the XCD (XCC) this wave runs on, kept in the top bits of the entry stamp
__device__ __forceinline__ unsigned long long tick_xcc() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return (unsigned long long)(v & 15);
}
#define TICK_STAMP(k)                                                                        \
  do {                                                                                       \
    if (!COUNT && g < 65536 && lane == 0) g_tick_trace[g * 4 + (k)] = __builtin_amdgcn_s_memrealtime() | ((k) == 0 ? tick_xcc() << 60 : 0ull); \
  } while (0)
#else
#define TICK_STAMP(k) do {} while (0)
#endif
#ifndef MRAFT_TICK_SCANU
#define MRAFT_TICK_SCANU 1  // ConflictIndex scans past the probe: 64 * SCANU terms per round trip
#endif
#ifndef MRAFT_TICK_CMP_EPL
#define MRAFT_TICK_CMP_EPL 4  // compare chunk: 64 * EPL entries (4: dwordx4 per lane, 2: dwordx2)
#endif
// One wave (group) per 64-thread workgroup: each wave's slot frees as soon as
// its group ends (four per workgroup, the group order without the XCD mapping,
// the compare chunks without software pipelining, two dwordx4 per lane per
// chunk and the state pointers held across the pass all measured slower; git
// history keeps them).

// GetState (raft.go:237-246) of the group's exported replica, fused into the
// tick (mraft_replicate_tick_export): commit and currentTerm<<1 | isLeader.
struct Export {
  int32_t *commit, *term_leader;
  __device__ __forceinline__ void put(int g, int c, int t, int role) const {
    if (commit) {
      commit[g] = c;
      term_leader[g] = (int32_t)(((uint32_t)t << 1) | (role == kLeader ? 1u : 0u));
    }
  }
};

template <int P, bool COUNT>
__global__ __launch_bounds__(64, MRAFT_TICK_MINW) void k_tick_group(Dev s, const int32_t *__restrict__ leader_peer,
                                                    int32_t *__restrict__ gflags,
                                                    unsigned long long *__restrict__ counts,
                                                    Export ex) {
  constexpr int NI = P - 1;
  const int lane = lane_id();
  // Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md
  // §Workgroup dispatch): give each XCD a contiguous range of groups so the
  // scalar SoA lines neighbouring groups share stay in one XCD's L2. Speed
  // only; any placement gives the same results.
  int gb = (int)blockIdx.x;
  {
    const int nb = (int)gridDim.x, x = gb & 7, per = nb >> 3, rem = nb & 7;
    gb = x * per + min(x, rem) + (gb >> 3);
  }
  // (threadIdx.x >> 6 is 0 in a one-wave workgroup; without the term the
  // compiler assigns this kernel's registers differently, so the measured
  // code is kept instruction-for-instruction)
  const int g = uni(gb + (int)(threadIdx.x >> 6));
  if (g >= s.G) return;
#define TICK_EXIT return
#include "mraft_tick_body.inc"
#undef TICK_EXIT
}

// P == 1: no peers, so no AppendEntries and no reply ever reaches a1.
__global__ void k_tick_p1(Dev s, const int32_t *__restrict__ leader_peer,
                          int32_t *__restrict__ gflags, unsigned long long *__restrict__ counts,
                          int count, Export ex) {
  const int g = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (g >= s.G) return;
  const int lp = leader_peer[g];
  int fl = 0;
  unsigned long long R = 0, A = 0;
  if (lp >= 1) {
    fl = MRAFT_G_ERROR;
  } else if (lp == 0) {
    R = 1;
    if (s.role[g] == kLeader) {
      R = 5;
      if (s.commit[g] < s.dummy[g]) fl = MRAFT_G_ERROR;
      else { fl = MRAFT_G_ACTIVE; A = 1; R = 6; }  // + terms_sorted (DESIGN.md §4 header words)
    }
  }
  if (count) {
    atomicAdd(&counts[kCountWords * (blockIdx.x & (kCountStripes - 1)) + 0], R);
    atomicAdd(&counts[kCountWords * (blockIdx.x & (kCountStripes - 1)) + 2], A);
  } else {
    if (gflags) gflags[g] = fl;
    ex.put(g, s.commit[g], s.term[g], s.role[g]);
  }
}

// ------------------------------------------------------------ light tick
// MRAFT_TICK_LIGHT (mraft_set_tick_mode). The tick of a running deployment —
// every follower caught up to its nextIndex, a heartbeat or a few appended
// entries — is a handful of dependent word loads per group and almost no
// streaming, so a wave per group spends its life waiting on them
// (secondary.steady_state_config3: 0.117 ms per 65,536-group tick, 285 GB/s).
// k_tick_lite gives each group eight lanes (eight Raft groups per wave, lane j
// = peer j), so eight groups' chains overlap in one wave. It settles a group
// only when every follower's reply is a success that needs no compare:
// prevLogTerm matches and either n = 0 (heartbeat, IC_HB) or the follower's
// log ends at prev (a pure append: IC_MERGE with an empty compare range, so
// the first mismatch is prev + 1), the append fits the ring, the leader's
// entries to send span at most kLiteSpan Indexes, and a1 settles at its top:
// with every follower at `last`, min(M*, last) = last (the order statistic of
// the last evaluation is `last`), and log[last] is currentTerm, or below it
// under the leader's terms_sorted proof. Every other group (stale or
// adopting-with-conflict replies, snapshots, conflicts, merges that compare,
// Figure-8 scans, capacity) is recognised before any store and appended to a
// device list that k_tick_list runs through the full tick
// (mraft_tick_body.inc). Per group the stores are the full tick's.
constexpr int kLiteSpan = 64;
constexpr int kLiteWaves = 4;  // waves per light workgroup: 32 groups, one list reservation

// START (mraft_start_and_tick): Start (raft.go:90-104) of counts[g] entries at
// the group's leader replica first, inside this launch: the leader lane
// appends them (terms_sorted, lastIndex, persist bit, as k_start) and the
// tick runs on the result — the new entries' terms are currentTerm, known
// without a load (the followers' copies and a1's probe of the new last).
// Groups that fall back carry their Start's stores into the full tick.
template <int P, bool START>
__global__ __launch_bounds__(64 * kLiteWaves, 8) void k_tick_lite(Dev s, const int32_t *__restrict__ leader_peer,
                                                               int32_t *__restrict__ gflags, Export ex,
                                                               int32_t *__restrict__ fb_list,
                                                               unsigned *__restrict__ fb_count, int cap,
                                                               StartIO sio) {
  __shared__ unsigned sh_cnt, sh_base;
  const int lane = lane_id(), j = lane & 7, gbase = lane & ~7, wv = (int)(threadIdx.x >> 6);
  const int xcd = (int)(blockIdx.x & 7);
  int wb = (int)blockIdx.x;  // XCD-contiguous workgroup ranges, as k_tick_group
  {
    const int nb = (int)gridDim.x, x = wb & 7, per = nb >> 3, rem = nb & 7;
    wb = x * per + min(x, rem) + (wb >> 3);
  }
  if (threadIdx.x == 0) sh_cnt = 0;
  const int g = (wb * kLiteWaves + wv) * 8 + (lane >> 3);
  const bool live = g < s.G;
  const int L = s.L;
  // Round trip 1: everything that does not depend on which peer leads. Lane
  // j < P of the group: replica j's scalars, its persist bits and column j of
  // the group's P x P nextIndex block (every candidate leader's view of j).
  const long long r = (long long)g * P + j;
  const bool rl = live && j < P;
  int lpv = -1, rrole = 0, rterm = 0, rcommit = 0, rlast = 0, rdummy = 0, rhead = 0, rsrt = 0, rpd = 0;
  int nx[P];
#pragma unroll
  for (int x = 0; x < P; ++x) nx[x] = 0;
  int kcnt = 0;  // START: entries to append at the leader
  if (live) lpv = leader_peer[g];
  if (START && live) kcnt = sio.counts[g];
  if (rl) {
    rrole = s.role[r]; rterm = s.term[r]; rcommit = s.commit[r]; rlast = s.last[r];
    rdummy = s.dummy[r]; rhead = s.head[r]; rsrt = s.srt[r];
    if (s.pdirty) rpd = s.pdirty[r];
#pragma unroll
    for (int x = 0; x < P; ++x) nx[x] = s.next[((long long)g * P + x) * P + j];
  }
  auto bc = [&](int v, int k) { return __shfl(v, gbase + k, 64); };
  {
    const int c_0 = bc(rcommit, 0), t_0 = bc(rterm, 0), r_0 = bc(rrole, 0);
    if (live && (lpv < 0 || lpv >= P) && j == 0) {
      if (gflags) gflags[g] = lpv >= P ? MRAFT_G_ERROR : 0;
      ex.put(g, c_0, t_0, r_0);  // mraft_export_group_status: replica 0
    }
  }
  bool go = live && lpv >= 0 && lpv < P;
  const int lp = go ? lpv : 0;
  const int role = bc(rrole, lp), T = bc(rterm, lp), c0 = bc(rcommit, lp), last0 = bc(rlast, lp),
            ldummy = bc(rdummy, lp), lhead = bc(rhead, lp), lsrt0 = bc(rsrt, lp);
  // START: mraft_start's decision (k_start) for the group's leader replica
  bool started = false;
  int serr = 0;
  if (START && live) {
    if (lpv >= 0 && lpv < P) {
      if (kcnt < 0) {
        serr = MRAFT_ITEM_BAD_SLOT;
      } else if (kcnt > 0 && role == kLeader) {                          // raft.go:93-95
        if ((int64_t)last0 + kcnt - ldummy > (int64_t)L - 1 || (int64_t)last0 + kcnt > (int64_t)INT32_MAX - 1)
          serr = MRAFT_ITEM_LOG_FULL;
        else
          started = true;
      }
    } else if (lpv >= P && kcnt != 0) {
      serr = MRAFT_ITEM_BAD_SLOT;
    }
    if (j == 0) {
      sio.oi[g] = started ? last0 + 1 : -1;                              // :103
      sio.ot[g] = started ? T : -1;
      sio.ol[g] = started ? 1 : 0;
      sio.err[g] = serr;
    }
  }
  const int last = started ? last0 + kcnt : last0;                       // :96-100
  if (go && (role != kLeader || c0 < ldummy)) {  // appendOneRound returns (:22-25) / MRAFT_ITEM_BAD_STATE
    if (j == 0) {
      if (gflags) gflags[g] = role != kLeader ? 0 : MRAFT_G_ERROR;
      ex.put(g, c0, T, role);
    }
    go = false;
  }
  int nj = 0;
#pragma unroll
  for (int x = 0; x < P; ++x) if (x == lp) nj = nx[x];
  const long long lrow = ((long long)g * P + lp) * L, f = r;
  const int lb = lhead - ldummy;
  const bool isf = go && j < P && j != lp;
  const int fterm = rterm, fdummy = rdummy, flast = rlast, fcommit = rcommit, fhead = rhead;
  const int prev = nj - 1, n = last - prev;                              // :26, :50
  // decided by round trip 1: snapshot, panic, stale, below / beyond the
  // follower's log, a merge that would compare (the follower holds entries
  // past prev) or run past the ring's capacity -> the full tick
  // IC_BELOW (prev below the follower's dummy, :123-127): Go returns before
  // setting reply.Term, so with currentTerm > 0 the leader's gate (:73-74)
  // drops the reply — the follower's own words only (role, term adoption,
  // persist), settled here too
  const bool bel = isf && prev >= ldummy && prev <= last && T >= fterm && prev < fdummy && T > 0;
  bool fb = isf && !bel && (prev < ldummy || prev > last || T < fterm || prev < fdummy || prev > flast ||
                            (n > 0 && (flast != prev || n > kLiteSpan || (long long)last - fdummy > (long long)L - 1)));
  const bool mrg = isf && !fb && !bel && n > 0;
  // successful replies: with at least P/2 of them the last evaluation of a1's
  // order statistic is `last` (so top = min(M*, last) = last); with none, a1
  // never runs; in between (few) a1 runs on an order statistic that still
  // holds older matchIndex words, settled below when it cannot pass commitIndex
  const bool succ = isf && !fb && !bel;
  const int nsucc = __popcll(__ballot(succ) >> gbase & 0xffull);
  const bool few = nsucc > 0 && nsucc < P / 2;
  bool gfb = ((__ballot(fb) >> gbase) & 0xffull) != 0;
  // Round trip 2 (groups still settling here): prevLogTerm at leader and
  // follower, a1's probe log[last] and each merging follower's first four
  // entries to append (its own lane loads the leader's words).
  const bool t2 = go && !gfb;
  int pt = 0, ft = 0, probe = 0, mj = 0;
  int e4[4] = {0, 0, 0, 0};
  // (START: Indexes above last0 are the entries Start appends, currentTerm)
  if (t2) {
    if (few && isf) mj = s.match[((long long)g * P + lp) * P + j];     // the leader's matchIndex[j]
    if (isf && !bel) {
      pt = (START && prev > last0) ? T : s.log[lrow + ring(prev + lb, L)];  // :49
      ft = s.log[f * L + ring(prev - fdummy + fhead, L)];                // :128
    }
    if (mrg) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (u < n) e4[u] = (START && prev + 1 + u > last0) ? T : s.log[lrow + ring(prev + 1 + u + lb, L)];
    }
  }
  // a1's probe (:98) of the pre-Start last: the tick's top when nothing was
  // appended, and Start's terms_sorted rule (k_start) when something was
  if ((t2 || started) && j == lp) probe = s.log[lrow + ring(last0 + lb, L)];
  if (t2 && isf && !bel && ft != pt) fb = true;                          // a conflict: the full tick
  const int pr0 = bc(probe, lp);
  const int t = started ? T : pr0;  // log[last]: an appended entry's term when Start appended
  // the leader's terms_sorted after Start: cleared when an older entry above
  // the dummy carries a term above currentTerm
  const bool sclr = started && last0 > ldummy && pr0 > T;
  const int lsrt = sclr ? 0 : lsrt0;
  if (START && started && j == lp) {
    const long long sl = (long long)g * P + lp;
    if (sclr) s.srt[sl] = 0;
    for (int u = 1; u <= kcnt; ++u) s.log[lrow + ring(last0 + u + lb, L)] = T;
    s.last[sl] = last;
    if (s.pdirty) s.pdirty[sl] = rpd | MRAFT_PERSIST_STATE;             // :101
  }
  int commit = c0, ftop = 0, pq = 0;
  gfb = gfb || ((__ballot(fb) >> gbase) & 0xffull) != 0;
  if (__ballot(t2 && few)) {
    // few successes (fewer than P/2): a1 runs after each of them (:78) on
    // quorum_rt's order statistic — the (P/2)-th largest follower matchIndex —
    // over words each success raises to `last`, the others' older words kept.
    // With no success lowering its word (old <= last) the evaluations' tops
    // rise to the last one's, so a1's ranges cover (commitIndex, top] and its
    // probe of log[top] settles it as for top = last below; otherwise, over
    // each follower's larger word, a bound on every evaluation's top that at
    // or below commitIndex means a1 changes nothing. Else the full tick.
    const int mm = isf ? (succ ? max(mj, last) : mj) : INT32_MIN;
    int c = 0;
#pragma unroll
    for (int q = 0; q < P; ++q) c += (bc((int)isf, q) && bc(mm, q) >= mm) ? 1 : 0;  // followers at or above mine
    int qv = (isf && c >= P / 2) ? mm : INT32_MIN;
#pragma unroll
    for (int q = 0; q < P; ++q) qv = max(qv, bc(qv, q));
    const bool mono = ((__ballot(succ && mj > last) >> gbase) & 0xffull) == 0;
    ftop = min(qv, last);
    if (go && few && ftop > c0) {
      if (!mono) gfb = true;
      else if (j == lp) pq = (START && ftop > last0) ? T : s.log[lrow + ring(ftop + lb, L)];  // :98
    }
    const int pqv = bc(pq, lp);
    if (go && few && !gfb && ftop > c0) {
      if (pqv == T) commit = ftop;                                       // :98-100
      else if (!(lsrt && pqv < T)) gfb = true;                           // a scan: the full tick
    }
  }
  if (go && !gfb && nsucc > 0 && !few && last > c0) {                    // top = last (above)
    if (t == T) commit = last;                                           // :98-100
    else if (!(lsrt && t < T)) gfb = true;                               // a Figure-8 scan: the full tick
  }
  const bool w = go && !gfb;
  // the appended entries, Indexes prev + 1 .. last, by the follower's own lane
  // (:149-155; the compare range is empty); past the first four, four at a time
  if (w && mrg) {
    const long long frow = f * L;
    const int fb0 = prev + 1 - fdummy + fhead;  // ring position of Index prev + 1, before the wrap
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (u < n) s.log[frow + ring(fb0 + u, L)] = e4[u];
    for (int c = 4; c < n; c += 4) {
      int x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        x[u] = c + u >= n ? 0 : (START && prev + 1 + c + u > last0) ? T : s.log[lrow + ring(prev + 1 + c + u + lb, L)];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (c + u < n) s.log[frow + ring(fb0 + c + u, L)] = x[u];
    }
  }
  bool fcadv = false;
  if (w && isf) {
    if (s.pdirty) s.pdirty[f] = rpd | MRAFT_PERSIST_STATE;              // :111 (mark_persist)
    if (T > fterm) { s.term[f] = T; s.voted[f] = -1; }                   // :116-118
    s.role[f] = kFollower;                                               // :120
  }
  if (w && isf && !bel) {
    int newlast = flast;
    if (n > 0) {
      newlast = last;                                                    // prev + n
      s.last[f] = newlast;
      // terms_sorted after appending from prev + 1 (the tick's rule, mk = 0)
      const bool fl = lsrt != 0 && (prev != ldummy || pt <= e4[0]);  // e4[0]: the entry at prev + 1
      const int sw = !fl ? 0 : prev == fdummy ? 1 : -1;
      if (sw >= 0) s.srt[f] = sw;
    }
    if (c0 > fcommit) {                                                  // :157-160
      s.commit[f] = min(c0, newlast);
      fcadv = true;
    }
    s.next[((long long)g * P + lp) * P + j] = last + 1;                  // :76-77
    s.match[((long long)g * P + lp) * P + j] = last;
  }
  const bool anyadv = ((__ballot(fcadv) >> gbase) & 0xffull) != 0;
  if (w && j == 0) {
    if (commit != c0) s.commit[(long long)g * P + lp] = commit;
    if (gflags)
      gflags[g] = MRAFT_G_ACTIVE | (commit != c0 ? MRAFT_G_COMMITTED : 0) | (anyadv ? MRAFT_G_FOLLOWER_COMMIT : 0);
    ex.put(g, commit, T, kLeader);
  }
  // The groups for the full tick: one LDS count per wave, one global atomic
  // per workgroup on its XCD's counter (one device-wide counter hit by every
  // wave serialised the launch: 72 us for 65,536 groups, profiles/r6_l4), the
  // list entries in the XCD's region of cap groups.
  const bool push = go && gfb && j == 0;
  const unsigned long long pmask = __ballot(push);
  unsigned woff = 0;
  if (pmask && lane == first_lane(pmask)) woff = atomicAdd(&sh_cnt, (unsigned)__popcll(pmask));
  woff = (unsigned)__shfl((int)woff, pmask ? first_lane(pmask) : 0, 64);
  __syncthreads();
  if (threadIdx.x == 0) sh_base = sh_cnt ? atomicAdd(&fb_count[xcd * 32], sh_cnt) : 0u;
  __syncthreads();
  if (push) fb_list[(long long)xcd * cap + sh_base + woff + (unsigned)__popcll(pmask & ((1ull << lane) - 1))] = g;
}

// The light tick's fallback: the groups k_tick_lite listed (eight XCD lists
// of cap entries, their counts 32 words apart), each through the full tick
// (one wave per group, grid-stride over the device counts, so any grid is
// exact; the host sizes it from the previous tick's count). The first
// workgroup zeroes the counters the next light tick uses and publishes this
// tick's count to the host's pinned word.
template <int P>
__global__ __launch_bounds__(64, MRAFT_TICK_MINW) void k_tick_list(Dev s, const int32_t *__restrict__ leader_peer,
                                                   int32_t *__restrict__ gflags,
                                                   unsigned long long *__restrict__ counts, Export ex,
                                                   const int32_t *__restrict__ list, const unsigned *__restrict__ cnt,
                                                   unsigned *__restrict__ cnt_next, long long *__restrict__ hint,
                                                   int cap) {
  constexpr bool COUNT = false;
  constexpr int NI = P - 1;
  const int lane = lane_id();
  unsigned c8[8], nl = 0;
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    c8[x] = (unsigned)uni((int)cnt[x * 32]);
    nl += c8[x];
  }
  if (blockIdx.x == 0) {
    if (lane < 8) cnt_next[lane * 32] = 0;
    if (lane == 0 && hint) __hip_atomic_store(hint, (long long)nl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  for (unsigned k = blockIdx.x; k < nl; k += gridDim.x) {
    unsigned base = 0;
    int x = 0;
#pragma unroll
    for (int y = 0; y < 7; ++y)
      if (x == y && k >= base + c8[y]) { base += c8[y]; x = y + 1; }
    const int g = uni(list[(long long)x * cap + (k - base)]);
#define TICK_EXIT continue
#include "mraft_tick_body.inc"
#undef TICK_EXIT
  }
}

template <int P>
void launch_tick_light_p(const Dev &s, const int32_t *lpeer, int32_t *gflags, Export ex, const LiteBufs &lb,
                         const StartIO *sio, hipStream_t st) {
  if (sio)
    hipLaunchKernelGGL((k_tick_lite<P, true>), dim3((unsigned)lite_blocks(s.G)), dim3(64 * kLiteWaves), 0, st, s,
                       lpeer, gflags, ex, lb.list, lb.cnt, lite_cap(s.G), *sio);
  else
    hipLaunchKernelGGL((k_tick_lite<P, false>), dim3((unsigned)lite_blocks(s.G)), dim3(64 * kLiteWaves), 0, st, s,
                       lpeer, gflags, ex, lb.list, lb.cnt, lite_cap(s.G), StartIO{});
  hipLaunchKernelGGL(k_tick_list<P>, dim3((unsigned)lb.grid), dim3(64), 0, st, s, lpeer, gflags,
                     (unsigned long long *)nullptr, ex, (const int32_t *)lb.list, (const unsigned *)lb.cnt,
                     lb.cnt_next, lb.hint, lite_cap(s.G));
}

template <int P, bool COUNT>
void launch_tick_p(const Dev &s, const int32_t *lpeer, int32_t *gflags, unsigned long long *counts,
                   Export ex, hipStream_t st) {
  hipLaunchKernelGGL((k_tick_group<P, COUNT>), dim3(s.G), dim3(64), 0, st, s, lpeer, gflags, counts, ex);
}

template <bool COUNT>
void launch_tick_c(const Dev &s, const int32_t *lpeer, int32_t *gflags, unsigned long long *counts,
                   Export ex, hipStream_t st) {
  switch (s.P) {
    case 2: launch_tick_p<2, COUNT>(s, lpeer, gflags, counts, ex, st); break;
    case 3: launch_tick_p<3, COUNT>(s, lpeer, gflags, counts, ex, st); break;
    case 4: launch_tick_p<4, COUNT>(s, lpeer, gflags, counts, ex, st); break;
    case 5: launch_tick_p<5, COUNT>(s, lpeer, gflags, counts, ex, st); break;
    case 6: launch_tick_p<6, COUNT>(s, lpeer, gflags, counts, ex, st); break;
    case 7: launch_tick_p<7, COUNT>(s, lpeer, gflags, counts, ex, st); break;
    case 8: launch_tick_p<8, COUNT>(s, lpeer, gflags, counts, ex, st); break;
    default: {
      const int blocks = (s.G + 255) / 256;
      hipLaunchKernelGGL(k_tick_p1, dim3(blocks), dim3(256), 0, st, s, lpeer, gflags, counts,
                         COUNT ? 1 : 0, ex);
    }
  }
}

}  // namespace

#if MRAFT_TICK_TRACE
extern "C" int mraft_debug_tick_trace(void *dst, long long nbytes) {
  if (nbytes > (long long)sizeof(g_tick_trace)) nbytes = sizeof(g_tick_trace);
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_tick_trace), (size_t)nbytes, 0, hipMemcpyDeviceToHost) ==
                 hipSuccess ? 0 : -3;
}
#endif

void launch_replicate_tick(const Dev &s, const int32_t *lpeer, int32_t *gflags, int32_t *exp_commit,
                           int32_t *exp_term_leader, hipStream_t st) {
  launch_tick_c<false>(s, lpeer, gflags, nullptr, Export{exp_commit, exp_term_leader}, st);
}

void launch_replicate_tick_light(const Dev &s, const int32_t *lpeer, int32_t *gflags, int32_t *exp_commit,
                                 int32_t *exp_term_leader, const LiteBufs &lb, const StartIO *sio, hipStream_t st) {
  const Export ex{exp_commit, exp_term_leader};
  switch (s.P) {
    case 2: launch_tick_light_p<2>(s, lpeer, gflags, ex, lb, sio, st); break;
    case 3: launch_tick_light_p<3>(s, lpeer, gflags, ex, lb, sio, st); break;
    case 4: launch_tick_light_p<4>(s, lpeer, gflags, ex, lb, sio, st); break;
    case 5: launch_tick_light_p<5>(s, lpeer, gflags, ex, lb, sio, st); break;
    case 6: launch_tick_light_p<6>(s, lpeer, gflags, ex, lb, sio, st); break;
    case 7: launch_tick_light_p<7>(s, lpeer, gflags, ex, lb, sio, st); break;
    case 8: launch_tick_light_p<8>(s, lpeer, gflags, ex, lb, sio, st); break;
    default:  // P == 1: k_tick_p1 is a lane per group already
      if (sio) launch_start_groups(s, lpeer, *sio, st);
      launch_tick_c<false>(s, lpeer, gflags, nullptr, ex, st);
  }
}

void launch_replicate_tick_count(const Dev &s, const int32_t *lpeer, unsigned long long *counts,
                                 hipStream_t st) {
  launch_tick_c<true>(s, lpeer, nullptr, counts, Export{nullptr, nullptr}, st);
}

}  // namespace mraft

MRAFT_BOUNDS_READER(mraft_debug_bounds_tick)
