// mraft_tick.hip — the fused co-resident replication tick (SURVEY.md §8a rows
// a1-a4) for gfx950: one 64-lane wave per Raft group, four groups per
// 256-thread workgroup.
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
  IC_FULL       // merge would exceed capacity L: rejected
};

enum : int { M_CMP = 0, M_COPY = 1, M_DONE = 2 };

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

// One chunk of the multi-follower merge pass. VEC: lane j owns entries
// c+4j .. c+4j+3 (one dwordx4 per stream); otherwise lane j owns c+j+64u.
// Leader entry idx lives at log[eo + idx], follower q's at log[fo[q] + idx].
template <int NI, bool VEC, bool COUNT>
__device__ __forceinline__ void merge_chunk(int32_t *__restrict__ log, long long eo,
                                            const long long (&fo)[NI], const int (&start)[NI],
                                            const int (&cend)[NI], const int (&nend)[NI],
                                            int (&mode)[NI], int (&cfrom)[NI],
                                            const int (&capok)[NI], int &fullmask, int c, int hi) {
  const int lane = lane_id();
  int idx[4];
  int e[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) idx[u] = VEC ? c + 4 * lane + u : c + lane + 64 * u;
  if (VEC) {
    int4 v = make_int4(0, 0, 0, 0);
    if (idx[0] <= hi) v = *reinterpret_cast<const int4 *>(log + eo + idx[0]);
    e[0] = v.x; e[1] = v.y; e[2] = v.z; e[3] = v.w;
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u) e[u] = idx[u] <= hi ? log[eo + idx[u]] : 0;
  }
  // Issue every follower's loads before any compare (more bytes in flight).
  int f[NI][4];
#pragma unroll
  for (int q = 0; q < NI; ++q) {
#pragma unroll
    for (int u = 0; u < 4; ++u) f[q][u] = 0;
    if (mode[q] != M_CMP || start[q] > c + 255 || cend[q] <= c) continue;
    if (VEC) {
      if (idx[3] >= start[q] && idx[0] < cend[q]) {
        const int4 v = *reinterpret_cast<const int4 *>(log + fo[q] + idx[0]);
        f[q][0] = v.x; f[q][1] = v.y; f[q][2] = v.z; f[q][3] = v.w;
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (idx[u] >= start[q] && idx[u] < cend[q]) f[q][u] = log[fo[q] + idx[u]];
    }
  }
#pragma unroll
  for (int q = 0; q < NI; ++q) {
    if (mode[q] == M_DONE || start[q] > c + 255) continue;
    if (mode[q] == M_CMP) {
      int im = -1;  // first mismatching entry index in this chunk
      if (cend[q] > c) {
        if (VEC) {
          int first = 4;
#pragma unroll
          for (int u = 3; u >= 0; --u)
            if (idx[u] >= start[q] && idx[u] < cend[q] && e[u] != f[q][u]) first = u;
          const unsigned long long m = __ballot(first < 4);
          if (m) {
            const int l = first_lane(m);
            im = c + 4 * l + __shfl(first, l, 64);
          }
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const unsigned long long m =
                __ballot(idx[u] >= start[q] && idx[u] < cend[q] && e[u] != f[q][u]);
            if (m && im < 0) im = c + 64 * u + first_lane(m);
          }
        }
      }
      if (im < 0 && cend[q] <= c + 255) {
        // Compared region ends in this chunk without a mismatch: either every
        // entry matched (no truncation, the non-FIFO guard) or the follower's
        // log ends before the entries do (mismatch "beyond the end").
        if (cend[q] < nend[q]) im = cend[q];
        else mode[q] = M_DONE;
      }
      if (im >= 0) {
        cfrom[q] = im;
        if (capok[q]) {
          mode[q] = M_COPY;
        } else {
          mode[q] = M_DONE;  // MRAFT_ITEM_LOG_FULL: no state change
          fullmask |= 1 << q;
        }
      }
    }
    if (mode[q] == M_COPY) {
      if (!COUNT) {
        if (VEC) {
          if (idx[0] >= cfrom[q] && idx[3] <= hi) {
            *reinterpret_cast<int4 *>(log + fo[q] + idx[0]) = make_int4(e[0], e[1], e[2], e[3]);
          } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (idx[u] >= cfrom[q] && idx[u] <= hi) log[fo[q] + idx[u]] = e[u];
          }
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (idx[u] >= cfrom[q] && idx[u] <= hi) log[fo[q] + idx[u]] = e[u];
        }
      }
      if (c + 255 >= hi) mode[q] = M_DONE;
    }
  }
}

template <int P, bool COUNT>
__global__ __launch_bounds__(256) void k_tick_group(Dev s, const int32_t *__restrict__ leader_peer,
                                                    int32_t *__restrict__ gflags,
                                                    unsigned long long *__restrict__ counts) {
  constexpr int NI = P - 1;
  const int lane = lane_id();
  const int g = uni((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
  if (g >= s.G) return;
  const int L = s.L;
  long long hR = 0;          // algorithmic words of the header (wave-uniform)
  long long cR = 0, cW = 0;  // algorithmic words of this lane's follower item (COUNT)
  int flags = 0, active = 0;

  // ------------------------------------------------------------ header
  const int lp = uni(leader_peer[g]);
  const long long ld = (long long)g * P + lp;
  int T = 0, c0 = 0, last = 0, ldummy = 0;
  bool go = false;
  if (lp >= P) {
    flags = MRAFT_G_ERROR;
  } else if (lp >= 0) {
    hR = 1;
    if (uni(s.role[ld]) == kLeader) {
      T = uni(s.term[ld]);
      c0 = uni(s.commit[ld]);
      last = uni(s.last[ld]);
      ldummy = uni(s.dummy[ld]);
      hR = 5;
      if (c0 < ldummy) flags = MRAFT_G_ERROR;  // outside the reachable states
      else go = true;
    }
  }
  if (!go) {
    if (COUNT) {
      if (lane == 0) atomicAdd(&counts[0], (unsigned long long)hR);
    } else if (lane == 0 && gflags) {
      gflags[g] = flags;
    }
    return;
  }

  // ------------------------------------------------------------ phase A
  const long long lrow = ld * L;
  int icls = IC_NONE, p = 0, prev = 0, n = 0, fdummy = 0, flast = 0, ft = 0, fterm = 0;
  long long f = 0;
  if (lane < NI) {
    p = lane < lp ? lane : lane + 1;
    prev = s.next[ld * P + p] - 1;                                       // :26
    icls = prev < ldummy ? IC_SNAP : (prev > last ? IC_PANIC : IC_GO);   // :27, :41
  }
  hR += NI;
  const unsigned long long snap_m = __ballot(icls == IC_SNAP);
  if (__ballot(icls == IC_PANIC)) {  // a3 would panic: the whole group is skipped
    if (COUNT) {
      if (lane == 0) atomicAdd(&counts[0], (unsigned long long)hR);
    } else if (lane == 0 && gflags) {
      gflags[g] = MRAFT_G_ERROR | (snap_m ? MRAFT_G_NEED_SNAPSHOT : 0);
    }
    return;
  }
  active = 1;
  flags = MRAFT_G_ACTIVE | (snap_m ? MRAFT_G_NEED_SNAPSHOT : 0);
  int rterm = 0, rsucc = 0, rci = 0;
  bool adopt = false;
  if (icls == IC_GO) {
    f = (long long)g * P + p;
    const int prev_term = s.log[lrow + (prev - ldummy)];                 // :49
    fterm = s.term[f];
    fdummy = s.dummy[f];
    flast = s.last[f];
    n = last - prev;                                                     // :50
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
        } else {
          ft = s.log[f * L + (prev - fdummy)];
          if (ft != prev_term) {                                         // :128
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
      const long long sf = (long long)g * P + (src < lp ? src : src + 1);
      const int sd = __shfl(fdummy, src, 64), sp = __shfl(prev, src, 64), sa = __shfl(ft, src, 64);
      const int ci = wave_conflict_scan(s.log + sf * L, sd, sp, sa);
      if (lane == src) {
        rci = ci;
        if (COUNT) scan_extra = sp - (ci > sd + 1 ? ci : sd + 2);
      }
    }
  }
  int mk = -1;  // this lane's follower: first mismatching entry of its merge
  const int merge_m = (int)__ballot(icls == IC_MERGE);
  if (merge_m) {
    long long fo[NI];
    int start[NI], cend[NI], nend[NI], mode[NI], cfrom[NI], capok[NI];
    int lo = last + 1;
    bool vec = (L & 3) == 0 && (reinterpret_cast<uintptr_t>(s.log) & 15) == 0;
    const long long eo = lrow - ldummy;
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const int qp = q < lp ? q : q + 1;
      const int sp = __shfl(prev, q, 64), sd = __shfl(fdummy, q, 64), sl = __shfl(flast, q, 64);
      fo[q] = ((long long)g * P + qp) * L - sd;
      start[q] = sp + 1;
      nend[q] = last + 1;                      // entries are [prev+1, last]
      cend[q] = min(last, sl) + 1;             // compared while the follower has the slot
      cfrom[q] = 0;
      capok[q] = (long long)last - sd <= (long long)L - 1;
      mode[q] = ((merge_m >> q) & 1) ? M_CMP : M_DONE;
      if (mode[q] == M_CMP) {
        lo = min(lo, start[q]);
        vec = vec && (((fo[q] - eo) & 3) == 0);
      }
    }
    int fullmask = 0;
    if (vec) {
      const int a0 = lo - (int)((eo + lo) & 3);
      for (int c = a0; c <= last; c += 256)
        merge_chunk<NI, true, COUNT>(s.log, eo, fo, start, cend, nend, mode, cfrom, capok, fullmask,
                                     c, last);
    } else {
      for (int c = lo; c <= last; c += 256)
        merge_chunk<NI, false, COUNT>(s.log, eo, fo, start, cend, nend, mode, cfrom, capok,
                                      fullmask, c, last);
    }
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      if (lane == q && icls == IC_MERGE) {
        // k* relative to the first entry; -1 when every entry matched.
        mk = (cfrom[q] > 0 || ((fullmask >> q) & 1)) ? cfrom[q] - start[q] : -1;
        if ((fullmask >> q) & 1) icls = IC_FULL;
      }
    }
  }

  // ------------------------------------------------------------ phase C
  int fcadv = 0;
  const int LC = c0;
  if (icls >= IC_STALE && icls <= IC_HB) {
    if (icls == IC_STALE) {
      cR += 1;
    } else {
      if (!COUNT) {
        if (adopt) { s.term[f] = T; s.voted[f] = -1; }
        s.role[f] = kFollower;                                           // :120
      }
      long long r = 2, w = (adopt ? 2 : 0) + 1;                          // term, dummy; role
      if (icls != IC_BELOW) r += 1;                                      // last
      if (icls >= IC_MISMATCH) r += 1;                                   // log[prev]
      if (icls == IC_SCAN) r += scan_extra;
      if (icls == IC_MERGE || icls == IC_HB) {
        int newlast = flast;
        if (icls == IC_MERGE) {
          const int kc = min(n, flast - prev);
          r += (mk < 0) ? n : (mk < kc ? mk + 1 : mk);                  // compared follower terms
          if (mk >= 0) {
            newlast = prev + n;
            if (!COUNT) s.last[f] = newlast;
            w += (n - mk) + 1;
          }
        }
        const int fc = s.commit[f];                                      // :157-160
        r += 1;
        if (LC > fc) {
          fcadv = 1;
          w += 1;
          if (!COUNT) s.commit[f] = min(LC, newlast);
        }
      }
      cR += r;
      cW += w;
    }
  }
  if (__ballot(icls == IC_FULL)) flags |= MRAFT_G_LOG_FULL;
  if (__ballot(fcadv != 0)) flags |= MRAFT_G_FOLLOWER_COMMIT;

  // ------------------------------------------------------------ phase D
  const bool have = icls >= IC_STALE && icls <= IC_HB;
  int term = T, role = kLeader, stepped = 0, any = 0, mstar = INT32_MIN;
  int mm[P];
  int gate[NI], rs[NI], rp[NI], rn[NI], rx[NI], ic[NI];
  const unsigned long long have_m = __ballot(have);
  const unsigned long long succ_m = __ballot(have && rsucc);
  if (succ_m) {
#pragma unroll
    for (int j = 0; j < P; ++j) mm[j] = (j == lp) ? 0 : uni(s.match[ld * P + j]);
  } else {
#pragma unroll
    for (int j = 0; j < P; ++j) mm[j] = 0;
  }
#pragma unroll
  for (int q = 0; q < NI; ++q) {                                         // a2, peer order
    const int pq = q < lp ? q : q + 1;
    gate[q] = 0;
    rs[q] = (int)((succ_m >> q) & 1);
    rp[q] = uni(__shfl(prev, q, 64));
    rn[q] = uni(__shfl(n, q, 64));
    rx[q] = rp[q] + 1;                                                   // nextIndex[q] (gathered)
    ic[q] = uni(__shfl(icls, q, 64));
    if (!((have_m >> q) & 1)) continue;
    const int rt = uni(__shfl(rterm, q, 64));
    if (rt > term) {                                                     // :67-72
      term = rt;
      role = kFollower;
      stepped = 1;
    } else if (rt == term && role == kLeader && T == term) {             // :73-74 (prev gate holds)
      gate[q] = 1;
      if (rs[q]) {
#pragma unroll
        for (int j = 0; j < P; ++j)
          if (j == pq) mm[j] = rp[q] + rn[q];                            // :76
        rx[q] = rp[q] + rn[q] + 1;                                       // :77
        mstar = max(mstar, quorum_match<P>(mm, lp));                     // :78 -> a1
        any = 1;
      } else {
        rx[q] = uni(__shfl(rci, q, 64));                                 // :82
      }
    }
  }
  int commit = c0, top = 0;
  if (any) {
    top = min(mstar, last);
    if (top > c0) {
      if (uni(s.log[lrow + (top - ldummy)]) == T) {                      // :98, one probe
        commit = top;
      } else {                                                           // Figure-8: exact scan
        const int i = wave_scan_down_eq(s.log + lrow, ldummy, c0 + 1, top - 1, T);
        if (i > c0) commit = i;
      }
    }
  }
  if (commit != c0) flags |= MRAFT_G_COMMITTED;
  if (stepped) flags |= MRAFT_G_STEPPED_DOWN;

  if (!COUNT) {
    if (lane == 0) {
      if (stepped) {
        s.term[ld] = term;
        s.voted[ld] = -1;
        s.role[ld] = kFollower;
      }
      if (commit != c0) s.commit[ld] = commit;
      if (gflags) gflags[g] = flags;
    }
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      const int pq = q < lp ? q : q + 1;
      if (lane == q && gate[q]) {
        s.next[ld * P + pq] = rx[q];
        if (rs[q]) s.match[ld * P + pq] = rp[q] + rn[q];
      }
    }
  } else {
    // Leader-side words, wave-uniform.
    long long gR = hR + (any ? NI : 0), gW = (stepped ? 3 : 0) + (commit != c0 ? 1 : 0);
#pragma unroll
    for (int q = 0; q < NI; ++q) gW += gate[q] ? (rs[q] ? 2 : 1) : 0;
    // Leader log words: union of {prev_q} (PrevLogTerm), [prev_q+1, last]
    // (entries consumed by merges) and the commit scan [stop, top].
    long long A = (long long)last + 1;
#pragma unroll
    for (int q = 0; q < NI; ++q)
      if (ic[q] == IC_MERGE) A = min(A, (long long)rp[q] + 1);
    long long a1lo = 1, a1hi = 0;
    if (any && top > c0) {
      a1hi = top;
      a1lo = (commit != c0) ? commit : c0 + 1;
    }
    long long u = interval_len(A, last) + interval_len(a1lo, a1hi);
    u -= interval_len(max(A, a1lo), min((long long)last, a1hi));
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      if (ic[q] < IC_STALE) continue;  // a3 read log[prev] for every gathered item
      bool dup = false;
#pragma unroll
      for (int q2 = 0; q2 < q; ++q2) dup |= (ic[q2] >= IC_STALE && rp[q2] == rp[q]);
      const long long x = rp[q];
      const bool inside = (x >= A && x <= last) || (x >= a1lo && x <= a1hi);
      if (!dup && !inside) u += 1;
    }
    gR += u;
    const unsigned long long R = wave_sum((unsigned long long)cR) + (unsigned long long)gR;
    const unsigned long long W = wave_sum((unsigned long long)cW) + (unsigned long long)gW;
    if (lane == 0) {
      atomicAdd(&counts[0], R);
      atomicAdd(&counts[1], W);
      atomicAdd(&counts[2], (unsigned long long)active);
    }
  }
}

// P == 1: no peers, so no AppendEntries and no reply ever reaches a1.
__global__ void k_tick_p1(Dev s, const int32_t *__restrict__ leader_peer,
                          int32_t *__restrict__ gflags, unsigned long long *__restrict__ counts,
                          int count) {
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
  const int blocks = (s.G + 3) / 4;
  hipLaunchKernelGGL((k_tick_group<P, COUNT>), dim3(blocks), dim3(256), 0, st, s, lpeer, gflags,
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
      hipLaunchKernelGGL(k_tick_p1, dim3(blocks), dim3(256), 0, st, s, lpeer, gflags, counts,
                         COUNT ? 1 : 0);
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
