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
  const int L = s.L;
  TICK_STAMP(0);

  // ------------------------------------------------------------ header
  const int lp = uni(leader_peer[g]);
  if (lp < 0 || lp >= P) {
    if (!COUNT && lane == 0) {
      if (gflags) gflags[g] = lp >= P ? MRAFT_G_ERROR : 0;
      if (ex.commit) {
        const long long s0 = (long long)g * P;  // mraft_export_group_status: replica 0
        ex.put(g, s.commit[s0], s.term[s0], s.role[s0]);
      }
    }
    return;
  }
  const long long ld = (long long)g * P + lp;
  const long long lrow = ld * L;
  // Every load that depends only on the leader index, issued together.
  const int role = uni(s.role[ld]), T = uni(s.term[ld]), c0 = uni(s.commit[ld]),
            last = uni(s.last[ld]), ldummy = uni(s.dummy[ld]), lhead = uni(s.head[ld]),
            lsrt = uni(s.srt[ld]);
  const int lb = lhead - ldummy;  // leader Index i at lrow + ring(i + lb): the log ring
  int mm[P];
#pragma unroll
  for (int j = 0; j < P; ++j) mm[j] = uni(s.match[ld * P + j]);
  const int p = lane < lp ? lane : lane + 1;
  const long long f = (long long)g * P + p;
  int nxt = 0, fterm = 0, fdummy = 0, flast = 0, fcommit = 0, fhead = 0;
  if (lane < NI) {
    nxt = s.next[ld * P + p];
    fterm = s.term[f];
    fdummy = s.dummy[f];
    flast = s.last[f];
    fcommit = s.commit[f];
    fhead = s.head[f];
  }
  long long hR = 1;  // algorithmic words of the header (wave-uniform)
  if (role != kLeader || c0 < ldummy) {
    // not a leader: appendOneRound returns (:22-25); commit < dummy: outside
    // the reachable states (include/mraft.h MRAFT_ITEM_BAD_STATE).
    if (COUNT) {
      if (lane == 0) atomicAdd(&counts[0], (unsigned long long)(role != kLeader ? 1 : 5));
    } else if (lane == 0) {
      if (gflags) gflags[g] = role != kLeader ? 0 : MRAFT_G_ERROR;
      ex.put(g, c0, T, role);
    }
    return;
  }
  hR = 6 + NI;  // role, term, commit, last, dummy, terms_sorted, nextIndex[q]

  // ------------------------------------------------------------ phase A
  int icls = IC_NONE;
  const int prev = nxt - 1;                                              // :26
  if (lane < NI) icls = prev < ldummy ? IC_SNAP : (prev > last ? IC_PANIC : IC_GO);  // :27, :41
  const int snap_m = (int)__ballot(icls == IC_SNAP);  // lanes >= NI never set a bit: 32 bits suffice
  if (__ballot(icls == IC_PANIC)) {  // a3 would panic: the whole group is skipped
    if (COUNT) {
      if (lane == 0) atomicAdd(&counts[0], (unsigned long long)hR);
    } else if (lane == 0) {
      if (gflags) gflags[g] = MRAFT_G_ERROR | (snap_m ? MRAFT_G_NEED_SNAPSHOT : 0);
      ex.put(g, c0, T, role);
    }
    return;
  }
  int flags = MRAFT_G_ACTIVE | (snap_m ? MRAFT_G_NEED_SNAPSHOT : 0);
  const int probe_last = uni(s.log[lrow + ring(last + lb, L)]);  // speculative a1 probe
  int prev_term = 0, ft = 0;
  if (icls == IC_GO) {
    prev_term = s.log[lrow + ring(prev + lb, L)];                        // :49
    if (prev >= fdummy && prev <= flast) ft = s.log[f * L + ring(prev - fdummy + fhead, L)];
  }
  const int n = last - prev;                                             // :50
  int rterm = 0, rsucc = 0, rci = 0;
  bool adopt = false;
  // InstallSnapshot (raft_append_entry.go:27-34 -> raft_snapshot.go:15-54),
  // LastIncludedIndex = leader dummyIndex, LastIncludedTerm = dummyTerm.
  const int lit = snap_m ? uni(s.log[lrow + lhead]) : 0;
  if (icls == IC_SNAP) {
    if (T >= fterm && ldummy > fcommit && ldummy <= flast && ldummy < fdummy) {
      icls = IC_IS_PANIC;                                                // sliceFrom panics
    } else if (T < fterm) {                                              // :20-22
      icls = IC_IS_STALE;
      rterm = fterm;
    } else {
      adopt = T > fterm;                                                 // :23-26
      rterm = T;
      icls = ldummy <= fcommit ? IC_IS_OLD : IC_IS_INSTALL;              // :31-33
    }
  }
  if (icls == IC_GO) {
    if (T < fterm) {                                                     // :112-115
      icls = IC_STALE;
      rterm = fterm;
    } else {
      adopt = T > fterm;                                                 // :116-118
      if (prev < fdummy) {                                               // :123-127
        icls = IC_BELOW;
        rci = fdummy + 1;
      } else {
        rterm = T;
        if (prev > flast) {                                              // :131-133
          icls = IC_BEYOND;
          rci = flast + 1;
        } else if (ft != prev_term) {                                    // :128
          if (prev > fdummy + 1) icls = IC_SCAN;
          else { icls = IC_MISMATCH; rci = prev; }
        } else {
          rsucc = 1;
          icls = n > 0 ? IC_MERGE : IC_HB;
        }
      }
    }
  }

  // ------------------------------------------------------------ phase B
  int scan_extra = 0;
  // ConflictIndex scans (:136-142): the first 64 terms below prev of every
  // scanning follower in one round trip (most runs end there), then each
  // longer run on its own, 64 * MRAFT_TICK_SCANU terms per round trip (64
  // measured 1.4 % faster than 256: fewer lines fetched past the run's end
  // outweigh the extra round trips). (Running them after the pass with their
  // inputs parked in LDS measured no faster and moved no traffic: r4_v13.)
  auto conflict_scans = [&](const int32_t *__restrict__ logp, unsigned long long m, int qdummy, int qhead, int qft) {
    int pv[NI];
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      pv[q] = 0;
      if ((m >> q) & 1) {
        const long long sf = (long long)g * P + (q < lp ? q : q + 1);
        const int sd = uni(__shfl(qdummy, q, 64)), sp = uni(__shfl(prev, q, 64)),
                  sh = uni(__shfl(qhead, q, 64));
        const int32_t *pp = logp + sf * L + ring(max(sp - 1 - lane, sd + 2) - sd + sh, L);  // prev >= dummy + 2
        pv[q] = *pp;
      }
    }
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      if ((m >> q) & 1) {
        const long long sf = (long long)g * P + (q < lp ? q : q + 1);
        const int sd = uni(__shfl(qdummy, q, 64)), sp = uni(__shfl(prev, q, 64)), sa = uni(__shfl(qft, q, 64)),
                  sh = uni(__shfl(qhead, q, 64));
        const int lo = sd + 2, hi = sp - 1;
        const unsigned long long mm = __ballot(hi - lane >= lo && pv[q] != sa);
        int ci;
        if (mm) {
          ci = hi - first_lane(mm);
        } else if (hi - 64 < lo) {
          ci = sd + 1;
        } else {
          const int r = wave_scan_down_ne<MRAFT_TICK_SCANU>(logp + sf * L, sd, sh, L, lo, hi - 64, sa);
          ci = r < lo ? sd + 1 : r;
        }
        if (lane == q) {
          rci = ci;
          if (COUNT) scan_extra = sp - (ci > sd + 1 ? ci : sd + 2);
        }
      }
    }
  };
  const unsigned long long scan_m = __ballot(icls == IC_SCAN);
  if (scan_m) conflict_scans(s.log, scan_m, fdummy, fhead, ft);

  // prev == the follower's dummy, for phase C's terms_sorted rule (a ballot:
  // no per-lane word kept live across the pass)
  const unsigned long long pd_m = __ballot(prev == fdummy);
  // Per-follower pass parameters (wave-uniform).
  const int merge_m = (int)__ballot(icls == IC_MERGE);
  Fol<NI> fo;
  fo.log = s.log;
  fo.slot0 = (long long)g * P;
  fo.skip = lp;
  fo.L = L;
  fo.cmp = merge_m;
  fo.copy = 0;
  fo.capok = 0;
  fo.full = 0;
  int mlo = last + 1, maybe_full = 0;
  bool vec = (L & 3) == 0 && (reinterpret_cast<uintptr_t>(s.log) & 15) == 0;
#pragma unroll
  for (int q = 0; q < NI; ++q) {
    const int sp = uni(__shfl(prev, q, 64)), sd = uni(__shfl(fdummy, q, 64)),
              sl = uni(__shfl(flast, q, 64)), sh = uni(__shfl(fhead, q, 64));
    fo.base[q] = sh - sd;
    fo.start[q] = sp + 1;
    fo.cend[q] = min(last, sl) + 1;  // compared while the follower has the slot
    fo.cfrom[q] = 0;                 // 0: no mismatch (the pass's relative Indexes are > 0)
    const bool capok = (long long)last - sd <= (long long)L - 1;
    fo.capok |= capok ? 1 << q : 0;
    if ((merge_m >> q) & 1) {
      mlo = min(mlo, fo.start[q]);
      vec = vec && (((fo.base[q] - lb) & 3) == 0);  // 4-entry groups aligned alike in both rings
      maybe_full |= !capok;
    }
  }

  // Fold before the pass when no follower can be rejected for capacity (then
  // every merge replies success whatever its mismatch point), so the exact
  // commit scan of a Figure-8 group rides along the same streaming pass.
  Fold<P, COUNT> fd;
  int commit = c0, top = 0, slo = 1, shi = 0;
  int settled = 0;  // a1 decided by its top term alone (sorted terms, include/mraft.h)
  const int is_m = (int)__ballot(icls >= IC_IS_STALE && icls <= IC_IS_INSTALL);
  const int have0 = (int)__ballot(icls >= IC_STALE && icls <= IC_HB) | is_m;
  const int succ0 = (int)__ballot(icls >= IC_STALE && icls <= IC_HB && rsucc);
  if (!maybe_full) {
    fd.run(T, lp, mm, have0, succ0, is_m, ldummy, rterm, prev, n, rci, icls);
    if (fd.any) {
      top = min(fd.mstar, last);
      if (top > c0) {
        const int t = top == last ? probe_last : uni(s.log[lrow + ring(top + lb, L)]);  // :98
        if (t == T) commit = top;
        else if (lsrt && t < T) settled = 1;  // no lower entry carries currentTerm
        else { slo = c0 + 1; shi = top - 1; }
      }
    }
  }
  int found = -1;
  TICK_STAMP(1);
  if (merge_m || slo <= shi) {
    const int plo = min(mlo, slo <= shi ? slo : mlo);
    const int phi = merge_m ? last : shi;
    // The pass runs on Indexes relative to B = pass_bias(plo) (mraft_pass.h:
    // no chunk end overflows int32 near 2^31); the rows absorb B.
    const int B = pass_bias(plo);
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      if (!((merge_m >> q) & 1)) continue;  // (only merging followers are ever addressed)
      fo.base[q] += B;
      fo.start[q] -= B;
      fo.cend[q] -= B;
    }
    const RingRow lsrc{s.log, lrow, lb + B, L};
    const int pl = plo - B, ph = phi - B, nend = last + 1 - B;
    const int sl = slo <= shi ? slo - B : 1, sh = slo <= shi ? shi - B : 0;
    // Chunks start on a 128-B line of the leader's row (physical position of
    // plo rounded down; the ring wraps at a multiple of 4 entries, so every
    // lane's dwordx4 stays contiguous).
    if (vec) {
      int c = pl - (int)((lrow + ring(plo + lb, L)) & (MRAFT_TICK_ALIGN - 1));
      if (c <= ph && fo.cmp) c = pass_pipe<COUNT, MRAFT_TICK_CMP_EPL>(lsrc, fo, nend, sl, sh, T, found, c, pl, ph);
      copy_loop<true, COUNT>(lsrc, fo, c, nend, pl, ph, sl, sh, T, found);
    } else {
      int c = pl;
      for (; c <= ph && fo.cmp; c += 256) pass_chunk<1, false, COUNT>(lsrc, fo, nend, sl, sh, T, found, c, pl, ph);
      copy_loop<false, COUNT>(lsrc, fo, c, nend, pl, ph, sl, sh, T, found);
    }
    if (found >= 0) found += B;  // the a1 hit back in Raft Indexes
  }
  TICK_STAMP(2);
  const Dev s2 = reload_dev();  // phase C/D re-read the state pointers (not held across the pass)
  int mk = -1;  // this lane's follower: first mismatching entry of its merge
#pragma unroll
  for (int q = 0; q < NI; ++q) {
    if (lane == q && icls == IC_MERGE) {
      mk = (fo.cfrom[q] > 0 || ((fo.full >> q) & 1)) ? fo.cfrom[q] - fo.start[q] : -1;
      if ((fo.full >> q) & 1) icls = IC_FULL;
    }
  }
  if (!maybe_full) {
    if (slo <= shi && found > c0) commit = found;
  } else {
    const int have1 = (int)__ballot(icls >= IC_STALE && icls <= IC_HB) | is_m;
    const int succ1 = (int)__ballot(icls >= IC_STALE && icls <= IC_HB && rsucc);
#pragma unroll
    for (int j = 0; j < P; ++j) mm[j] = uni(s2.match[ld * P + j]);  // re-read: not kept live across the pass
    fd.run(T, lp, mm, have1, succ1, is_m, ldummy, rterm, prev, n, rci, icls);
    if (fd.any) {
      top = min(fd.mstar, last);
      if (top > c0) {
        const int t = uni(s2.log[lrow + ring(top + lb, L)]);
        if (t == T) {
          commit = top;
        } else if (uni(s2.srt[ld]) && t < T) {
          settled = 1;
        } else {
          const int i = wave_scan_down_eq(s2.log + lrow, ldummy, lhead, L, c0 + 1, top - 1, T);
          if (i > c0) commit = i;
        }
      }
    }
  }

  // ------------------------------------------------------------ phase C
  int fcadv = 0;
  long long cR = 0, cW = 0;  // algorithmic words of this lane's follower item (COUNT)
  if (icls >= IC_STALE && icls <= IC_HB) {
    // deferred :111 (a load, OR and store: as a non-returning atomic OR it
    // measured no faster here, r4_v7)
    if (!COUNT) mark_persist(s2, f, MRAFT_PERSIST_STATE);
    if (icls == IC_STALE) {
      cR = 1;
    } else {
      if (!COUNT) {
        if (adopt) { s2.term[f] = T; s2.voted[f] = -1; }
        s2.role[f] = kFollower;                                           // :120
      }
      cR = 2;                                                            // term, dummy
      cW = (adopt ? 2 : 0) + 1;                                          // role
      if (icls != IC_BELOW) cR += 1;                                     // last
      if (icls >= IC_MISMATCH) cR += 1;                                  // log[prev]
      if (icls == IC_SCAN) cR += scan_extra;
      if (icls == IC_MERGE || icls == IC_HB) {
        int newlast = flast;
        if (icls == IC_MERGE) {
          const int kc = min(n, flast - prev);
          cR += (mk < 0) ? n : (mk < kc ? mk + 1 : mk);                 // compared follower terms
          if (mk >= 0) {
            newlast = prev + n;
            if (!COUNT) s2.last[f] = newlast;
            cW += (n - mk) + 1;
            // terms_sorted after appending from Index prev+1+mk: the args'
            // flag (prevLogTerm, entries sorted: the leader's proof, with the
            // dummy's term compared explicitly), or the new entries are the
            // whole log when that Index is the dummy's successor
            bool fl = lsrt != 0;
            if (fl && prev == ldummy)
              fl = s2.log[lrow + ring(prev + lb, L)] <= s2.log[lrow + ring(prev + 1 + lb, L)];
            const bool at_dummy = ((pd_m >> lane) & 1) != 0;
            const int sw = !fl ? 0 : (mk == 0 && at_dummy) ? 1 : -1;
            if (sw >= 0) {
              if (!COUNT) s2.srt[f] = sw;
              cW += 1;
            }
          }
        }
        cR += 1;                                                         // :157-160
        if (c0 > fcommit) {
          fcadv = 1;
          cW += 1;
          if (!COUNT) s2.commit[f] = min(c0, newlast);
        }
      }
    }
  }
  if (icls >= IC_IS_STALE && icls <= IC_IS_INSTALL) {
    cR = 1;                                                              // term
    if (!COUNT) {
      const int bits = (adopt ? MRAFT_PERSIST_STATE : 0) |                 // raft_snapshot.go:26
                       (icls == IC_IS_INSTALL ? MRAFT_PERSIST_STATE | MRAFT_PERSIST_SNAPSHOT : 0);  // :47
      mark_persist(s2, f, bits);
    }
    if (icls != IC_IS_STALE) {
      if (!COUNT) {
        if (adopt) { s2.term[f] = T; s2.voted[f] = -1; }
        s2.role[f] = kFollower;                                           // :28
      }
      cR += 1;                                                           // commit
      cW = (adopt ? 2 : 0) + 1;
      if (icls == IC_IS_INSTALL) {
        const bool newlog = ldummy > flast;                              // :35-37
        // sliceFrom(LastIncludedIndex) (:38-40) is an O(1) rebase of the
        // ring: the head moves to the entry at LastIncludedIndex, no term
        // moves; a new log ([dummy] only, :35-37) keeps its head.
        // (head and dummy re-read here rather than kept live across the pass)
        const int fh = s2.head[f], nh = newlog ? fh : ring(fh + (ldummy - s2.dummy[f]), L);
        if (!COUNT) {
          s2.log[f * L + nh] = lit;                                       // :44-45 dummy term
          if (newlog) { s2.last[f] = ldummy; s2.srt[f] = 1; }           // [dummy] only: sorted
          else s2.head[f] = nh;                                           // a suffix: unchanged
          s2.hsnap[f] = 1;                                                // raft_snapshot.go:52 hasSnapshot
          s2.dummy[f] = ldummy;
          s2.commit[f] = ldummy;                                          // :42
          s2.applied[f] = ldummy;                                         // :43
        }
        cR += 1;                                                         // last
        cW += 3;
        if (newlog) {
          cW += 3;                                                       // dummy term, last, terms_sorted
        } else {
          cR += 1;                                                       // dummy
          cW += 1;                                                       // dummy term
        }
      }
    }
  }
  if (__ballot(icls == IC_IS_INSTALL)) flags |= MRAFT_G_SNAPSHOT_INSTALLED;
  if (__ballot(icls == IC_IS_PANIC)) flags |= MRAFT_G_FOLLOWER_PANIC;
  if (__ballot(icls == IC_FULL)) flags |= MRAFT_G_LOG_FULL;
  if (__ballot(fcadv != 0)) flags |= MRAFT_G_FOLLOWER_COMMIT;

  // ------------------------------------------------------------ phase D
  if (commit != c0) flags |= MRAFT_G_COMMITTED;
  if (fd.stepped) flags |= MRAFT_G_STEPPED_DOWN;
  if (!COUNT) {
    if (lane == 0) {
      if (fd.stepped) {
        s2.term[ld] = fd.term;
        s2.voted[ld] = -1;
        s2.role[ld] = kFollower;
        mark_persist(s2, ld, MRAFT_PERSIST_STATE);                        // :72, snapshot :64
      }
      if (commit != c0) s2.commit[ld] = commit;
      if (gflags) gflags[g] = flags;
      ex.put(g, commit, fd.stepped ? fd.term : T, fd.stepped ? kFollower : kLeader);
    }
    TICK_STAMP(3);
    // nextIndex / matchIndex of this lane's follower (:76-77, :82; snapshot
    // :66-67): success -> prev + n (+1), failure -> ConflictIndex, snapshot
    // -> LastIncludedIndex (+1).
    if (lane < NI && ((fd.gate_m >> lane) & 1)) {
      const bool isr = ((is_m >> lane) & 1) != 0, ok = ((fd.rs_m >> lane) & 1) != 0;
      const int mv = isr ? ldummy : prev + n;
      s2.next[ld * P + p] = ok ? mv + 1 : rci;
      if (ok) s2.match[ld * P + p] = mv;
    }
  } else {
    // Leader-side words, wave-uniform.
    long long gR = hR + (fd.any ? NI : 0), gW = (fd.stepped ? 3 : 0) + (commit != c0 ? 1 : 0);
#pragma unroll
    for (int q = 0; q < NI; ++q) gW += ((fd.gate_m >> q) & 1) ? (((fd.rs_m >> q) & 1) ? 2 : 1) : 0;
    // Leader log words: union of {prev_q} (PrevLogTerm), [prev_q+1, last]
    // (entries consumed by merges) and the commit scan [stop, top].
    long long A = (long long)last + 1;
#pragma unroll
    for (int q = 0; q < NI; ++q)
      if (fd.ic[q] == IC_MERGE) A = min(A, (long long)fd.rp[q] + 1);
    long long a1lo = 1, a1hi = 0;
    if (fd.any && top > c0) {
      a1hi = top;
      a1lo = (commit != c0) ? commit : settled ? top : c0 + 1;
    }
    long long u = interval_len(A, last) + interval_len(a1lo, a1hi);
    u -= interval_len(max(A, a1lo), min((long long)last, a1hi));
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      if (fd.ic[q] < IC_STALE) continue;  // log[prev] per gathered item, log[dummy] per snapshot
      bool dup = false;
#pragma unroll
      for (int q2 = 0; q2 < q; ++q2) dup |= (fd.ic[q2] >= IC_STALE && fd.rp[q2] == fd.rp[q]);
      const long long x = fd.rp[q];
      const bool inside = (x >= A && x <= last) || (x >= a1lo && x <= a1hi);
      if (!dup && !inside) u += 1;
    }
    gR += u;
    const unsigned long long R = wave_sum((unsigned long long)cR) + (unsigned long long)gR;
    const unsigned long long W = wave_sum((unsigned long long)cW) + (unsigned long long)gW;
    if (lane == 0) {
      atomicAdd(&counts[0], R);
      atomicAdd(&counts[1], W);
      atomicAdd(&counts[2], 1ull);
    }
  }
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
    atomicAdd(&counts[0], R);
    atomicAdd(&counts[2], A);
  } else {
    if (gflags) gflags[g] = fl;
    ex.put(g, s.commit[g], s.term[g], s.role[g]);
  }
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

void launch_replicate_tick_count(const Dev &s, const int32_t *lpeer, unsigned long long *counts,
                                 hipStream_t st) {
  launch_tick_c<true>(s, lpeer, nullptr, counts, Export{nullptr, nullptr}, st);
}

}  // namespace mraft

MRAFT_BOUNDS_READER(mraft_debug_bounds_tick)
