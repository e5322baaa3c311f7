// mraft_tick.hip — the fused co-resident replication tick (SURVEY.md §8a rows
// a1-a4) for gfx950.
//
// One 64-lane wave owns GPW = 64/(P-1) whole groups, so every AppendEntries
// item of its groups (one per follower) and the leader's reply fold stay
// inside the wave; no inter-wave or inter-workgroup communication exists.
//   phase A  lane per item:  appendOneRound's args gather (raft_append_entry.go
//            :20-54) and HandleAppendEntries up to matchLog (:108-133): term
//            check/adoption, prev < dummy, prev > last, prev-term match;
//   phase B  wave per item:  the variable-length work — the ConflictIndex scan
//            (:136-142) and the entry merge + truncate/append (:149-155) —
//            streamed 256 terms per iteration, mismatch found by ballot;
//   phase C  lane per item:  follower state write-back, follower commit
//            (:157-160), reply;
//   phase D  lane per group: processAppendEntriesReply (:66-88) in peer order,
//            the quorum order statistic over matchIndex held in registers, and
//            the current-term gate of advanceCommitIndexForLeader (:89-105):
//            one probe of log[min(M*, last)], a wave-cooperative downward scan
//            only when that probe misses (Figure-8 groups).
// The AppendEntries entries are never copied: the follower reads the leader's
// log row in place (the reference copies them into the args, :50-54).
//
// COUNT=true runs the same decisions without any state store and accumulates
// the algorithmic word count of DESIGN.md §4 (reads, writes, active groups).
#include "mraft_device.h"
#include "mraft_internal.h"

namespace mraft {

namespace {

enum : int {
  IC_NONE = 0,   // no AppendEntries for this item
  IC_SNAP,       // prev < leader dummy: InstallSnapshot path
  IC_PANIC,      // prev > leader last: Go panics
  IC_GO,         // args gathered
  IC_STALE,      // args.Term < currentTerm
  IC_BELOW,      // prev < follower dummy
  IC_BEYOND,     // prev > follower last
  IC_MISMATCH,   // term(prev) differs, ConflictIndex known without a scan
  IC_SCAN,       // term(prev) differs, ConflictIndex needs the backward scan
  IC_MERGE,      // prefix matches, n > 0 entries to merge
  IC_HB,         // prefix matches, heartbeat
  IC_FULL        // merge would exceed capacity L: rejected
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

__device__ __forceinline__ long long interval_len(long long a, long long b) { return b >= a ? b - a + 1 : 0; }

template <int P, bool COUNT>
__global__ __launch_bounds__(256) void k_replicate_tick(Dev s, const int32_t *__restrict__ leader_peer,
                                                        int32_t *__restrict__ gflags,
                                                        unsigned long long *__restrict__ counts) {
  constexpr int NI = P - 1;
  constexpr int GPW = 64 / NI;
  const int lane = lane_id();
  const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int G = s.G, L = s.L;
  const int g0 = wave * GPW;
  if (g0 >= G) return;

  // ------------------------------------------------------------ phase A
  const int gi = lane / NI, kk = lane % NI;
  const int g = g0 + gi;
  const bool item_lane = lane < GPW * NI && g < G;

  int lp = -1, lterm = 0, lcommit = 0, llast = 0, ldummy = 0;
  int gstat = 0;  // 0 inactive (no leader / not a leader), 1 active, 2 error
  int has_lp = 0;
  int p = 0, prev = 0, lnext = 0;
  int icls = IC_NONE;
  if (item_lane) {
    lp = leader_peer[g];
    if (lp >= P) {
      gstat = 2;
    } else if (lp >= 0) {
      has_lp = 1;
      const long long ld = (long long)g * P + lp;
      if (s.role[ld] == kLeader) {
        lterm = s.term[ld];
        lcommit = s.commit[ld];
        llast = s.last[ld];
        ldummy = s.dummy[ld];
        if (lcommit < ldummy) {
          gstat = 2;  // outside the reachable states (include/mraft.h BAD_STATE)
        } else {
          gstat = 1;
          p = kk < lp ? kk : kk + 1;
          lnext = s.next[ld * P + p];
          prev = lnext - 1;                                            // :26
          icls = prev < ldummy ? IC_SNAP : (prev > llast ? IC_PANIC : IC_GO);  // :27, :41
        }
      }
    }
  }
  const unsigned long long gbits = (NI >= 64) ? ~0ull : ((1ull << NI) - 1);
  const unsigned long long panic_m = __ballot(icls == IC_PANIC);
  const int gshift = item_lane ? gi * NI : 0;
  if (item_lane && gstat == 1 && ((panic_m >> gshift) & gbits)) gstat = 2;  // a3 would panic

  const int T = lterm, LC = lcommit;
  int n = 0, f = 0, fdummy = 0, flast = 0, ft = 0;
  bool adopt = false;
  int rterm = 0, rsucc = 0, rci = 0;
  if (gstat == 1 && icls == IC_GO) {
    const long long ld = (long long)g * P + lp;
    const int prev_term = s.log[ld * L + (prev - ldummy)];             // :49
    n = llast - prev;                                                  // :50
    f = g * P + p;
    const int fterm = s.term[f];
    if (T < fterm) {                                                   // :112-115
      icls = IC_STALE;
      rterm = fterm;
    } else {
      adopt = T > fterm;                                               // :116-118
      fdummy = s.dummy[f];
      if (prev < fdummy) {                                             // :123-127
        icls = IC_BELOW;
        rterm = 0;
        rci = fdummy + 1;
      } else {
        flast = s.last[f];
        rterm = T;
        if (prev > flast) {                                            // :131-133
          icls = IC_BEYOND;
          rci = flast + 1;
        } else {
          ft = s.log[(long long)f * L + (prev - fdummy)];
          if (ft != prev_term) {                                       // :128
            if (prev > fdummy + 1) icls = IC_SCAN;
            else { icls = IC_MISMATCH; rci = prev; }
          } else {
            rsucc = 1;
            icls = n > 0 ? IC_MERGE : IC_HB;
          }
        }
      }
    }
  }

  // ------------------------------------------------------------ phase B
  int scan_extra = 0;
  {
    unsigned long long m = __ballot(icls == IC_SCAN);
    while (m) {
      const int src = first_lane(m);
      m &= m - 1;
      const int sf = shfl_i(f, src), sd = shfl_i(fdummy, src), sp = shfl_i(prev, src),
                sa = shfl_i(ft, src);
      const int ci = wave_conflict_scan(s.log + (long long)sf * L, sd, sp, sa);
      if (lane == src) {
        rci = ci;
        if (COUNT) scan_extra = sp - (ci > sd + 1 ? ci : sd + 2);
      }
    }
  }
  int mk = -1;  // first mismatching entry of the merge, -1 if all match
  {
    unsigned long long m = __ballot(icls == IC_MERGE);
    while (m) {
      const int src = first_lane(m);
      m &= m - 1;
      const int sf = shfl_i(f, src), sd = shfl_i(fdummy, src), sl = shfl_i(flast, src),
                sp = shfl_i(prev, src), sn = shfl_i(n, src);
      const int sg = g0 + src / NI, slp = shfl_i(lp, src), sld = shfl_i(ldummy, src);
      const int32_t *E = s.log + ((long long)sg * P + slp) * L + (sp + 1 - sld);
      int32_t *F = s.log + (long long)sf * L + (sp + 1 - sd);
      const int kc = min(sn, sl - sp);
      int k = wave_merge_compare(E, F, kc);
      if (k < 0 && kc < sn) k = kc;                                    // beyond the end
      const bool full = k >= 0 && (long long)sp + sn - sd > (long long)L - 1;
      if (!COUNT && k >= 0 && !full) wave_copy(E + k, F + k, sn - k);  // trunc + append
      if (lane == src) {
        mk = k;
        if (full) icls = IC_FULL;
      }
    }
  }

  // ------------------------------------------------------------ phase C
  int fcadv = 0;
  long long fR = 0, fW = 0;
  if (icls >= IC_STALE && icls <= IC_HB) {
    if (icls == IC_STALE) {
      fR = 1;
    } else {
      if (!COUNT) {
        if (adopt) { s.term[f] = T; s.voted[f] = -1; }
        s.role[f] = kFollower;                                         // :120
      }
      fR = 2;                                                          // term, dummy
      fW = (adopt ? 2 : 0) + 1;
      if (icls != IC_BELOW) fR += 1;                                   // last
      if (icls >= IC_MISMATCH) fR += 1;                                // log[prev]
      if (icls == IC_SCAN) fR += scan_extra;
      if (icls == IC_MERGE || icls == IC_HB) {
        int newlast = flast;
        if (icls == IC_MERGE) {
          const int kc = min(n, flast - prev);
          fR += (mk < 0) ? n : (mk < kc ? mk + 1 : mk);               // compared follower terms
          if (mk >= 0) {
            newlast = prev + n;
            if (!COUNT) s.last[f] = newlast;
            fW += (n - mk) + 1;
          }
        }
        const int fc = s.commit[f];                                    // :157-160
        fR += 1;
        if (LC > fc) {
          fcadv = 1;
          fW += 1;
          if (!COUNT) s.commit[f] = min(LC, newlast);
        }
      }
    }
  }
  const bool have = icls >= IC_STALE && icls <= IC_HB;

  // ------------------------------------------------------------ phase D
  const unsigned long long snap_m = __ballot(icls == IC_SNAP);
  const unsigned long long full_m = __ballot(icls == IC_FULL);
  const unsigned long long fc_m = __ballot(fcadv != 0);

  int rh[NI], rt[NI], rs[NI], rc[NI], rp[NI], rn[NI], rx[NI], ic[NI];
#pragma unroll
  for (int q = 0; q < NI; ++q) {
    const int src = (lane < GPW ? lane : 0) * NI + q;
    rh[q] = shfl_i(have ? 1 : 0, src);
    rt[q] = shfl_i(rterm, src);
    rs[q] = shfl_i(rsucc, src);
    rc[q] = shfl_i(rci, src);
    rp[q] = shfl_i(prev, src);
    rn[q] = shfl_i(n, src);
    rx[q] = shfl_i(lnext, src);
    ic[q] = shfl_i(icls, src);
  }
  const int src0 = (lane < GPW ? lane : 0) * NI;
  const int d_gstat = shfl_i(gstat, src0), d_lp = shfl_i(lp, src0), d_has = shfl_i(has_lp, src0);
  const int d_T = shfl_i(lterm, src0), d_c0 = shfl_i(lcommit, src0),
            d_last = shfl_i(llast, src0), d_dummy = shfl_i(ldummy, src0);
  const int g2 = g0 + lane;
  const bool glane = lane < GPW && g2 < G;
  const int gsh = (lane < GPW ? lane : 0) * NI;

  long long gR = 0, gW = 0, gA = 0;
  int need_scan = 0, top = 0, commit = d_c0;
  int term = d_T, role = kLeader, stepped = 0;
  int mm[P];
  int any = 0, gate[NI];
#pragma unroll
  for (int q = 0; q < NI; ++q) gate[q] = 0;
#pragma unroll
  for (int j = 0; j < P; ++j) mm[j] = 0;
  int flags = 0;
  const long long ldg = (long long)g2 * P + d_lp;
  if (glane) {
    if (d_gstat == 2) {
      flags = MRAFT_G_ERROR | (((snap_m >> gsh) & gbits) ? MRAFT_G_NEED_SNAPSHOT : 0);
      if (d_has) gR = 5 + (((panic_m >> gsh) & gbits) ? NI : 0);
    } else if (d_gstat == 0) {
      if (d_has) gR = 1;  // role read: not a leader, appendOneRound returns (:22-25)
    } else {
      flags = MRAFT_G_ACTIVE;
      if ((snap_m >> gsh) & gbits) flags |= MRAFT_G_NEED_SNAPSHOT;
      if ((full_m >> gsh) & gbits) flags |= MRAFT_G_LOG_FULL;
      if ((fc_m >> gsh) & gbits) flags |= MRAFT_G_FOLLOWER_COMMIT;
      int anysucc = 0;
#pragma unroll
      for (int q = 0; q < NI; ++q) anysucc |= rh[q] & rs[q];
      if (anysucc) {
#pragma unroll
        for (int j = 0; j < P; ++j) mm[j] = (j == d_lp) ? 0 : s.match[ldg * P + j];
      }
      int mstar = INT32_MIN;
#pragma unroll
      for (int q = 0; q < NI; ++q) {                                   // a2, peer order
        if (!rh[q]) continue;
        const int pq = q < d_lp ? q : q + 1;
        if (rt[q] > term) {                                            // :67-72
          term = rt[q];
          role = kFollower;
          stepped = 1;
        } else if (rt[q] == term && role == kLeader && d_T == term && rp[q] == rx[q] - 1) {  // :73-74
          gate[q] = 1;
          if (rs[q]) {
#pragma unroll
            for (int j = 0; j < P; ++j)
              if (j == pq) mm[j] = rp[q] + rn[q];                      // :76
            rx[q] = rp[q] + rn[q] + 1;                                 // :77
            const int mq = quorum_match<P>(mm, d_lp);                  // :78 -> a1
            mstar = max(mstar, mq);
            any = 1;
          } else {
            rx[q] = rc[q];                                             // :82
          }
        }
      }
      if (any) {
        top = min(mstar, d_last);
        if (top > d_c0) {
          if (s.log[ldg * L + (top - d_dummy)] == d_T) commit = top;  // :98 gate, one probe
          else need_scan = 1;
        }
      }
    }
  }
  // Wave-cooperative downward scans for groups whose probe missed.
  {
    unsigned long long m = __ballot(need_scan != 0);
    while (m) {
      const int src = first_lane(m);
      m &= m - 1;
      const long long row = (long long)(g0 + src) * P + shfl_i(d_lp, src);
      const int sd = shfl_i(d_dummy, src), stop = shfl_i(top, src), sc0 = shfl_i(d_c0, src),
                sT = shfl_i(d_T, src);
      const int i = wave_scan_down_eq(s.log + row * L, sd, sc0 + 1, stop - 1, sT);
      if (lane == src && i > sc0) commit = i;
    }
  }
  if (glane && d_gstat == 1) {
    if (commit != d_c0) flags |= MRAFT_G_COMMITTED;
    if (stepped) flags |= MRAFT_G_STEPPED_DOWN;
    if (!COUNT) {
      if (stepped) {
        s.term[ldg] = term;
        s.voted[ldg] = -1;
        s.role[ldg] = kFollower;
      }
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        if (!gate[q]) continue;
        const int pq = q < d_lp ? q : q + 1;
        s.next[ldg * P + pq] = rx[q];
        if (rs[q]) s.match[ldg * P + pq] = rp[q] + rn[q];
      }
      if (commit != d_c0) s.commit[ldg] = commit;
    }
    if (COUNT) {
      // Leader-side words.
      gA = 1;
      gR = 5 + NI + (any ? NI : 0);
      gW = (stepped ? 3 : 0) + (commit != d_c0 ? 1 : 0);
#pragma unroll
      for (int q = 0; q < NI; ++q) gW += gate[q] ? (rs[q] ? 2 : 1) : 0;
      // Leader log words: union of {prev_q} (PrevLogTerm), [prev_q+1, last]
      // (entries consumed by merges) and the commit scan [stop, top].
      long long A = (long long)d_last + 1;
#pragma unroll
      for (int q = 0; q < NI; ++q)
        if (ic[q] == IC_MERGE) A = min(A, (long long)rp[q] + 1);
      long long a1lo = 1, a1hi = 0;
      if (any && top > d_c0) {
        a1hi = top;
        a1lo = (commit != d_c0) ? commit : d_c0 + 1;
      }
      long long u = interval_len(A, d_last) + interval_len(a1lo, a1hi);
      const long long olo = max(A, a1lo), ohi = min((long long)d_last, a1hi);
      u -= interval_len(olo, ohi);
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        const bool pt = ic[q] >= IC_STALE;  // a3 read log[prev]
        if (!pt) continue;
        bool dup = false;
#pragma unroll
        for (int q2 = 0; q2 < q; ++q2) dup |= (ic[q2] >= IC_STALE && rp[q2] == rp[q]);
        const long long x = rp[q];
        const bool inside = (x >= A && x <= d_last) || (x >= a1lo && x <= a1hi);
        if (!dup && !inside) u += 1;
      }
      gR += u;
    }
    if (!COUNT && gflags) gflags[g2] = flags;
  } else if (glane && !COUNT && gflags) {
    gflags[g2] = flags;
  }
  if (COUNT) {
    unsigned long long R = (unsigned long long)(fR + gR), W = (unsigned long long)(fW + gW),
                       A = (unsigned long long)gA;
    R = wave_sum(R);
    W = wave_sum(W);
    A = wave_sum(A);
    if (lane == 0) {
      atomicAdd(&counts[0], R);
      atomicAdd(&counts[1], W);
      atomicAdd(&counts[2], A);
    }
  }
}

// P == 1: no peers, so no AppendEntries and no reply ever reaches a1.
__global__ void k_replicate_tick_p1(Dev s, const int32_t *__restrict__ leader_peer,
                                    int32_t *__restrict__ gflags,
                                    unsigned long long *__restrict__ counts, int count) {
  const int g = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (g >= s.G) return;
  const int lp = leader_peer[g];
  int fl = 0;
  unsigned long long R = 0, A = 0;
  if (lp >= 1) fl = MRAFT_G_ERROR;
  else if (lp == 0) {
    R = 1;
    if (s.role[g] == kLeader) {
      R = 5;
      if (s.commit[g] < s.dummy[g]) fl = MRAFT_G_ERROR;
      else { fl = MRAFT_G_ACTIVE; A = 1; }
    }
  }
  if (count) {
    atomicAdd(&counts[0], R);
    atomicAdd(&counts[2], A);
  } else if (gflags) {
    gflags[g] = fl;
  }
}

template <int P, bool COUNT>
void launch_tick_p(const Dev &s, const int32_t *lpeer, int32_t *gflags, unsigned long long *counts,
                   hipStream_t st) {
  constexpr int GPW = 64 / (P - 1);
  const int waves = (s.G + GPW - 1) / GPW;
  const int blocks = (waves + 3) / 4;
  hipLaunchKernelGGL((k_replicate_tick<P, COUNT>), dim3(blocks), dim3(256), 0, st, s, lpeer, gflags,
                     counts);
}

template <bool COUNT>
void launch_tick_c(const Dev &s, const int32_t *lpeer, int32_t *gflags, unsigned long long *counts,
                   hipStream_t st) {
  switch (s.P) {
    case 2: launch_tick_p<2, COUNT>(s, lpeer, gflags, counts, st); break;
    case 3: launch_tick_p<3, COUNT>(s, lpeer, gflags, counts, st); break;
    case 4: launch_tick_p<4, COUNT>(s, lpeer, gflags, counts, st); break;
    case 5: launch_tick_p<5, COUNT>(s, lpeer, gflags, counts, st); break;
    case 6: launch_tick_p<6, COUNT>(s, lpeer, gflags, counts, st); break;
    case 7: launch_tick_p<7, COUNT>(s, lpeer, gflags, counts, st); break;
    case 8: launch_tick_p<8, COUNT>(s, lpeer, gflags, counts, st); break;
    default: {
      const int blocks = (s.G + 255) / 256;
      hipLaunchKernelGGL(k_replicate_tick_p1, dim3(blocks), dim3(256), 0, st, s, lpeer, gflags,
                         counts, COUNT ? 1 : 0);
    }
  }
}

}  // namespace

void launch_replicate_tick(const Dev &s, const int32_t *lpeer, int32_t *gflags, hipStream_t st) {
  launch_tick_c<false>(s, lpeer, gflags, nullptr, st);
}

void launch_replicate_tick_count(const Dev &s, const int32_t *lpeer, unsigned long long *counts,
                                 hipStream_t st) {
  launch_tick_c<true>(s, lpeer, nullptr, counts, st);
}

}  // namespace mraft
