// mraft_pass.h — the streaming entry-merge pass shared by the fused tick
// (mraft_tick.hip) and the message-level HandleAppendEntries
// (mraft_kernels.hip): raft_append_entry.go:146-155's compare-then-truncate-
// and-append over one source of entries (`src`: the leader's log row, or a
// network batch) into up to NI follower rows of `log`, 256 entries per wave
// iteration, first mismatch by ballot, and — for the tick — the exact a1
// commit scan riding on the same loads.
#pragma once
#include "mraft_device.h"

namespace mraft {
namespace {

enum : int { M_CMP = 0, M_COPY = 1, M_DONE = 2 };  // a follower's state in the pass

// base + k for a wave-uniform row base and a per-lane k, as a 32-bit unsigned
// byte offset from base - 32 entries: the loads and stores then use the
// SGPR-base + 32-bit VGPR-offset form, one VGPR per stream instead of a 64-bit
// address pair. Valid for k >= -32 on every lane that dereferences it: a
// dwordx4 group that holds the first entry of a range may begin up to 3
// entries before it (a flat entries buffer indexed from its first Index: k < 0
// there while the address is inside the buffer).
// The offset wraps for k >= 2^30 - 32: capacities are capped below that
// (MRAFT_MAX_LOG_CAPACITY), flat sources are built relative to their first
// entry (flat_src) and the pass runs on rebased Indexes (pass_bias), so every
// k formed is within a row length (plus a chunk) of 0. MRAFT_DEBUG_BOUNDS
// builds count every dereferenced k outside [-32, 2^30 - 32) instead of
// trusting that (bounds_note; read with mraft_debug_bounds_violations).
#ifndef MRAFT_DEBUG_BOUNDS
#define MRAFT_DEBUG_BOUNDS 0
#endif
#if MRAFT_DEBUG_BOUNDS
__device__ unsigned long long g_bounds_violations;
__device__ __forceinline__ void bounds_note(long long k) {
  if (k < -32 || k >= (1ll << 30) - 32) atomicAdd(&g_bounds_violations, 1ull);
}
#else
__device__ __forceinline__ void bounds_note(long long) {}
#endif
template <class T>
__device__ __forceinline__ T *at_u(T *base, int k) {
  return reinterpret_cast<T *>(reinterpret_cast<char *>(const_cast<int32_t *>(base - 32)) + (uint32_t)(k + 32) * 4u);
}

// Indexes inside the pass are relative to B = pass_bias(plo) (plo: the pass's
// first Index), so they lie in [kPassBias - 35, kPassBias + L + 256]: a chunk
// end c + 256 cannot overflow int32 however close the Raft Index is to 2^31,
// and 0 stays free as "no Index" (Fol::cfrom). Rows absorb B in their bases.
constexpr int kPassBias = 64;
__device__ __forceinline__ int pass_bias(int plo) { return plo - kPassBias; }

// Where the term of Index idx of a stream lives. Entries come from a
// contiguous buffer (a network batch or staged copy: L = INT32_MAX, never
// wraps, base = -(the pass's first Index) so lane offsets stay small) or from
// a ring (the leader's own row; followers are always rings; include/mraft.h:
// row + (head + idx - dummy) mod L, base = head - dummy).
// Every lane that loads or stores in the pass holds an Index at or above the
// row's dummy (loads and stores are masked to [plo, phi] / [start, cend) /
// [cfrom, nend), and a dwordx4 group aligned in the ring cannot begin below
// it), so idx + base >= 0 there and only the upper wrap is needed; masked
// lanes may form any address, they never dereference it.
struct RingRow {
  const int32_t *p;
  long long row;
  int base, L;
  __device__ __forceinline__ const int32_t *at(int idx) const {
    const int k = idx + base;
    bounds_note(k >= L ? (long long)k - L : k);
    return at_u(p + row, k >= L ? k - L : k);
  }
};

// A flat source whose entry 0 (Index prev + 1) is word `first` of p: at(x) is
// p + first + (x - (prev + 1)), never wrapping (L = INT32_MAX), the lane
// offset relative to entry 0 whatever the Index.
__device__ __forceinline__ RingRow flat_src(const int32_t *p, int64_t first, int prev) {
  return RingRow{p, (long long)first, -(prev + 1), INT32_MAX};
}

// Streaming (read-once / write-once) log accesses of the pass: non-temporal
// loads and stores (plain temporal accesses measured slower in both the tick
// and the handler, round 2; git history keeps the variant).
__device__ __forceinline__ int4 ld4(const int32_t *p) {
  const int4 *q = reinterpret_cast<const int4 *>(p);
  return make_int4(__builtin_nontemporal_load(&q->x), __builtin_nontemporal_load(&q->y),
                   __builtin_nontemporal_load(&q->z), __builtin_nontemporal_load(&q->w));
}
__device__ __forceinline__ int ld1(const int32_t *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st4(int32_t *p, int a, int b, int c, int d) {
  int4 *q = reinterpret_cast<int4 *>(p);
  __builtin_nontemporal_store(a, &q->x);
  __builtin_nontemporal_store(b, &q->y);
  __builtin_nontemporal_store(c, &q->z);
  __builtin_nontemporal_store(d, &q->w);
}
__device__ __forceinline__ void st1(int32_t *p, int a) { __builtin_nontemporal_store(a, p); }
// EPL entries (4 or 2) of one lane: one dwordx4 or dwordx2 access.
template <int EPL>
__device__ __forceinline__ void ldv(const int32_t *p, int (&x)[EPL]) {
  if constexpr (EPL == 4) {
    const int4 v = ld4(p);
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  } else {
    const int2 *q = reinterpret_cast<const int2 *>(p);
    x[0] = __builtin_nontemporal_load(&q->x); x[1] = __builtin_nontemporal_load(&q->y);
  }
}
template <int EPL>
__device__ __forceinline__ void stv(int32_t *p, const int (&x)[EPL]) {
  if constexpr (EPL == 4) {
    st4(p, x[0], x[1], x[2], x[3]);
  } else {
    int2 *q = reinterpret_cast<int2 *>(p);
    __builtin_nontemporal_store(x[0], &q->x); __builtin_nontemporal_store(x[1], &q->y);
  }
}

// The followers a pass serves, with as little wave-uniform state as the pass
// needs (it is live across the whole streaming loop; at 8 waves per SIMD every
// scalar held here is one the compiler would otherwise spill): in the tick,
// follower q's replica slot is slot0 + q, skipping `skip` (the leader's peer
// index), so no 64-bit row offsets are held; the message handler (SLOTS)
// names each receiving slot. A follower's mode is two bits (cmp: still
// comparing; copy: copying from cfrom on; neither: done); capok (the append
// fits the capacity) and full (rejected as MRAFT_ITEM_LOG_FULL) are bits too.
template <int NI, bool SLOTS = false>
struct Fol {
  static constexpr int kNI = NI;
  int32_t *log;
  long long slot0;
  int skip, L;
  int slot[SLOTS ? NI : 1];  // SLOTS: follower q's replica slot
  int base[NI];   // ring base: head - dummy (include/mraft.h)
  int start[NI];  // first compared Index (prev + 1)
  int cend[NI];   // compared while the follower has the Index: [start, cend)
  int cfrom[NI];  // first mismatching Index (copy from here)
  int cmp, copy, capok, full;
  __device__ __forceinline__ int32_t *at(int q, int idx) const {
    const long long row = (SLOTS ? (long long)slot[SLOTS ? q : 0] : slot0 + q + (q >= skip ? 1 : 0)) * (long long)L;
    const int k = idx + base[q];  // >= 0 for every lane that loads or stores (see RingRow)
    bounds_note(k >= L ? (long long)k - L : k);
    return at_u(log + row, k >= L ? k - L : k);
  }
  __device__ __forceinline__ bool is_cmp(int q) const { return (cmp >> q) & 1; }
  __device__ __forceinline__ bool is_copy(int q) const { return (copy >> q) & 1; }
  // follower q's first mismatch is at im: copy from there if the append fits
  __device__ __forceinline__ void mismatch(int q, int im) {
    cfrom[q] = im;
    cmp &= ~(1 << q);
    if ((capok >> q) & 1) copy |= 1 << q;
    else full |= 1 << q;  // MRAFT_ITEM_LOG_FULL: no state change
  }
};

// Descent tracking over the entries a pass streams (the message handler's
// check of an AppendEntries' MRAFT_AE_ENTRIES_SORTED flag, include/mraft.h):
// the highest Index i in (lo, hi] whose predecessor's term is larger,
// term(i - 1) > term(i), over the chunks seen. The chunks of one pass are
// contiguous and ascending and the first starts at or below lo, so `carry`
// (the last term of the previous chunk) is only read where i - 1 >= lo.
// NoDesc (the fused tick: the leader's own proof needs no check) compiles to
// nothing.
struct NoDesc {
  template <int EPL>
  __device__ __forceinline__ void see(const int (&)[EPL], int, int, int) {}
  __device__ __forceinline__ void see_strided(const int (&)[4], int, int, int) {}
};
struct DescTrack {
  int on;     // wave-uniform: some merging message carries the flag
  int carry;  // term of the Index just below the current chunk
  int last;   // highest descent Index seen (INT32_MIN: none)
  // lane j holds Indexes c + EPL*j .. + EPL - 1
  template <int EPL>
  __device__ __forceinline__ void see(const int (&e)[EPL], int c, int lo, int hi) {
    if (!on) return;
    const int lane = lane_id();
    int pl = __shfl_up(e[EPL - 1], 1, 64);
    if (lane == 0) pl = carry;
    int d = INT32_MIN;
#pragma unroll
    for (int u = 0; u < EPL; ++u) {
      const int i = c + EPL * lane + u, b = u ? e[u - 1] : pl;
      if (i - 1 >= lo && i <= hi && b > e[u]) d = i;
    }
    const unsigned long long m = __ballot(d != INT32_MIN);
    if (m) last = max(last, __builtin_amdgcn_readlane(d, 63 - __clzll((long long)m)));
    carry = __builtin_amdgcn_readlane(e[EPL - 1], 63);
  }
  // lane j holds Indexes c + 64*u + j, u = 0..3
  __device__ __forceinline__ void see_strided(const int (&e)[4], int c, int lo, int hi) {
    if (!on) return;
    const int lane = lane_id();
    int d = INT32_MIN;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      int pl = __shfl_up(e[u], 1, 64);
      if (lane == 0) pl = u ? __builtin_amdgcn_readlane(e[u - 1], 63) : carry;
      const int i = c + 64 * u + lane;
      if (i - 1 >= lo && i <= hi && pl > e[u]) d = max(d, i);
    }
    const unsigned long long m = __ballot(d != INT32_MIN);
    if (m) {
      int x = d;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) x = max(x, __shfl_xor(x, o, 64));
      last = max(last, __builtin_amdgcn_readfirstlane(x));
    }
    carry = __builtin_amdgcn_readlane(e[3], 63);
  }
};

// One chunk of the streaming pass over the leader's log. The pass serves
// (1) every follower q's entry merge: compare entries [start_q, cend_q) with
// the follower's log, then (from the first mismatch) copy entries up to `hi`
// into it; and (2) the exact commit scan: the largest index in [slo, shi]
// whose term equals T (kept in `found`, the pass ascends).
// VEC: lane j owns entries c+256v+4j .. +3 (one dwordx4 per stream and v);
// otherwise lane j owns c+64(4v+u)+j. Entry idx is at src.at(idx), follower
// q's term of Index idx at fo.at(q, idx). The tick and the handler call the
// dword form (V = 1, !VEC: rows not 16-B aligned alike, or a flat buffer whose
// ends a dwordx4 would cross); their dwordx4 form is pass_pipe. (A dword-only
// restatement of this template changed the tick kernel's register assignment,
// so the measured code is kept as it is.)
template <int V, bool VEC, bool COUNT, class Src, class F, class D = NoDesc>
__device__ __forceinline__ void pass_chunk(const Src &src, F &fo, int nend, int slo, int shi, int T,
                                           int &found, int c, int plo, int phi, D &&dt = D{}) {
  constexpr int NI = F::kNI;
  constexpr int CW = 256 * V;
  const int lane = lane_id();
  int idx[V][4], e[V][4];
#pragma unroll
  for (int v = 0; v < V; ++v)
#pragma unroll
    for (int u = 0; u < 4; ++u) idx[v][u] = VEC ? c + 256 * v + 4 * lane + u : c + 64 * (4 * v + u) + lane;
  // Leader entries, then every comparing follower's terms: all loads in flight
  // before the first compare.
#pragma unroll
  for (int v = 0; v < V; ++v) {
    if (VEC) {
      int4 x = make_int4(0, 0, 0, 0);
      if (idx[v][3] >= plo && idx[v][0] <= phi) x = ld4(src.at(idx[v][0]));
      e[v][0] = x.x; e[v][1] = x.y; e[v][2] = x.z; e[v][3] = x.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) e[v][u] = (idx[v][u] >= plo && idx[v][u] <= phi) ? ld1(src.at(idx[v][u])) : 0;
    }
  }
#pragma unroll
  for (int v = 0; v < V; ++v) {
    if (VEC) dt.template see<4>(e[v], c + 256 * v, plo, phi);
    else dt.see_strided(e[v], c + 256 * v, plo, phi);
  }
  int f[NI][V][4];
#pragma unroll
  for (int q = 0; q < NI; ++q) {
#pragma unroll
    for (int v = 0; v < V; ++v)
#pragma unroll
      for (int u = 0; u < 4; ++u) f[q][v][u] = 0;
    if (!fo.is_cmp(q) || fo.start[q] > c + CW - 1 || fo.cend[q] <= c) continue;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      if (VEC) {
        if (idx[v][3] >= fo.start[q] && idx[v][0] < fo.cend[q]) {
          const int4 x = ld4(fo.at(q, idx[v][0]));
          f[q][v][0] = x.x; f[q][v][1] = x.y; f[q][v][2] = x.z; f[q][v][3] = x.w;
        }
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (idx[v][u] >= fo.start[q] && idx[v][u] < fo.cend[q]) f[q][v][u] = ld1(fo.at(q, idx[v][u]));
      }
    }
  }
  // Commit scan: highest index of this chunk in [slo, shi] with term T.
  if (slo <= shi && c <= shi && c + CW - 1 >= slo) {
    int hit = -1;
#pragma unroll
    for (int v = V - 1; v >= 0; --v) {
      if (hit >= 0) break;
      if (VEC) {
        int lu = -1;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (idx[v][u] >= slo && idx[v][u] <= shi && e[v][u] == T) lu = u;
        const unsigned long long m = __ballot(lu >= 0);
        if (m) {
          const int l = 63 - __clzll((long long)m);
          hit = c + 256 * v + 4 * l + __shfl(lu, l, 64);
        }
      } else {
#pragma unroll
        for (int u = 3; u >= 0; --u) {
          if (hit >= 0) break;
          const unsigned long long m =
              __ballot(idx[v][u] >= slo && idx[v][u] <= shi && e[v][u] == T);
          if (m) hit = c + 64 * (4 * v + u) + 63 - __clzll((long long)m);
        }
      }
    }
    if (hit >= 0) found = hit;
  }
#pragma unroll
  for (int q = 0; q < NI; ++q) {
    if ((!fo.is_cmp(q) && !fo.is_copy(q)) || fo.start[q] > c + CW - 1) continue;
    if (fo.is_cmp(q)) {
      int im = -1;  // first mismatching entry index in this chunk
      if (fo.cend[q] > c) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          if (im >= 0) break;
          if (VEC) {
            int first = 4;
#pragma unroll
            for (int u = 3; u >= 0; --u)
              if (idx[v][u] >= fo.start[q] && idx[v][u] < fo.cend[q] && e[v][u] != f[q][v][u]) first = u;
            const unsigned long long m = __ballot(first < 4);
            if (m) {
              const int l = first_lane(m);
              im = c + 256 * v + 4 * l + __shfl(first, l, 64);
            }
          } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const unsigned long long m =
                  __ballot(idx[v][u] >= fo.start[q] && idx[v][u] < fo.cend[q] && e[v][u] != f[q][v][u]);
              if (m && im < 0) im = c + 64 * (4 * v + u) + first_lane(m);
            }
          }
        }
      }
      if (im < 0 && fo.cend[q] <= c + CW - 1) {
        // Compared region ends in this chunk without a mismatch: either every
        // entry matched (no truncation: the non-FIFO guard, :146-155) or the
        // follower's log ends before the entries do ("beyond the end").
        if (fo.cend[q] < nend) im = fo.cend[q];
        else fo.cmp &= ~(1 << q);
      }
      if (im >= 0) fo.mismatch(q, im);
    }
    if (fo.is_copy(q)) {
      if (!COUNT) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          if (VEC && idx[v][0] >= fo.cfrom[q] && idx[v][3] < nend) {
            st4(fo.at(q, idx[v][0]), e[v][0], e[v][1], e[v][2], e[v][3]);
          } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (idx[v][u] >= fo.cfrom[q] && idx[v][u] < nend) st1(fo.at(q, idx[v][u]), e[v][u]);
          }
        }
      }
      if (c + CW >= nend) fo.copy &= ~(1 << q);
    }
  }
}

// The compare chunks of the pass (dwordx4 form, 64 * EPL entries per chunk: EPL = 4,
// one dwordx4 per lane and stream, or 2, one dwordx2) software-pipelined:
// chunk c is compared, then chunk c+CW's loads (the leader's entries and the
// words of every follower still comparing after chunk c) are issued, then
// chunk c's stores, so the wave waits for the next loads without waiting for
// its own stores (vmcnt counts both, in order). No word is loaded that
// pass_chunk would not load at the same chunk width; a follower's terms past
// its first mismatch are read up to the end of that chunk (the smaller EPL,
// the fewer: DESIGN.md §5 overfetch account). Runs while some follower
// compares; returns the first chunk not processed (the copy-only loop
// continues there; c stays on the leader row's line grid for EPL >= 2 and
// the caller's 32-entry chunk origin).
template <bool COUNT, int EPL = 4, class Src, class F, class D = NoDesc>
__device__ __forceinline__ int pass_pipe(const Src &src, F &fo, int nend, int slo, int shi, int T, int &found,
                                         int c, int plo, int phi, D &&dt = D{}) {
  constexpr int NI = F::kNI;
  constexpr int CW = 64 * EPL;
  const int lane = lane_id();
  int e[EPL], f[NI][EPL];
  auto load = [&](int cc, int (&ee)[EPL], int (&ff)[NI][EPL]) {
    const int i0 = cc + EPL * lane;
#pragma unroll
    for (int u = 0; u < EPL; ++u) ee[u] = 0;
    if (i0 + EPL - 1 >= plo && i0 <= phi) ldv<EPL>(src.at(i0), ee);
#pragma unroll
    for (int q = 0; q < NI; ++q) {
#pragma unroll
      for (int u = 0; u < EPL; ++u) ff[q][u] = 0;
      if (!fo.is_cmp(q) || fo.start[q] > cc + CW - 1 || fo.cend[q] <= cc) continue;
      if (i0 + EPL - 1 >= fo.start[q] && i0 < fo.cend[q]) ldv<EPL>(fo.at(q, i0), ff[q]);
    }
  };
  load(c, e, f);
  for (;;) {
    const int i0 = c + EPL * lane;
    dt.template see<EPL>(e, c, plo, phi);
    // compare: first mismatch of every follower still comparing
#pragma unroll
    for (int q = 0; q < NI; ++q) {
      if (!fo.is_cmp(q) || fo.start[q] > c + CW - 1) continue;
      int im = -1;
      if (fo.cend[q] > c) {
        int first = EPL;
#pragma unroll
        for (int u = EPL - 1; u >= 0; --u)
          if (i0 + u >= fo.start[q] && i0 + u < fo.cend[q] && e[u] != f[q][u]) first = u;
        const unsigned long long m = __ballot(first < EPL);
        if (m) {
          const int l = first_lane(m);
          im = c + EPL * l + __shfl(first, l, 64);
        }
      }
      if (im < 0 && fo.cend[q] <= c + CW - 1) {
        if (fo.cend[q] < nend) im = fo.cend[q];
        else fo.cmp &= ~(1 << q);
      }
      if (im >= 0) fo.mismatch(q, im);
    }
    // commit scan on this chunk's entries
    if (slo <= shi && c <= shi && c + CW - 1 >= slo) {
      int lu = -1;
#pragma unroll
      for (int u = 0; u < EPL; ++u)
        if (i0 + u >= slo && i0 + u <= shi && e[u] == T) lu = u;
      const unsigned long long m = __ballot(lu >= 0);
      if (m) {
        const int l = 63 - __clzll((long long)m);
        found = c + EPL * l + __shfl(lu, l, 64);
      }
    }
    const int cn = c + CW;
    const bool more = cn <= phi && fo.cmp;
    int en[EPL];
    if (more) load(cn, en, f);
    if (!COUNT) {
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        if (!fo.is_copy(q) || fo.start[q] > c + CW - 1) continue;
        if (i0 >= fo.cfrom[q] && i0 + EPL - 1 < nend) {
          stv<EPL>(fo.at(q, i0), e);
        } else {
#pragma unroll
          for (int u = 0; u < EPL; ++u)
            if (i0 + u >= fo.cfrom[q] && i0 + u < nend) st1(fo.at(q, i0 + u), e[u]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < NI; ++q)
      if (fo.is_copy(q) && fo.start[q] <= c + CW - 1 && cn >= nend) fo.copy &= ~(1 << q);
    if (!more) return cn;
    c = cn;
#pragma unroll
    for (int u = 0; u < EPL; ++u) e[u] = en[u];
  }
}

// Copy-only tail of the pass, once no follower is still comparing: every
// follower still copying receives the leader's entries [c, nend) (its copy
// start is already behind c), and the commit scan [slo, shi] continues on the
// same loads. Software-pipelined: chunk c+256 is loaded before chunk c is
// stored, so a wave never waits for its own stores before issuing the next
// load (gfx9's vmcnt counts both in order). The next chunk is loaded only when
// the loop will run for it: no extra traffic. (Two to four chunks ahead
// measured no faster in round 2 and 3-4 % slower in round 3: the copy is
// memory-system-bound at 8 waves per SIMD and more bytes in flight per wave
// only queue, profiles/r2_experiments, r3_experiments/ab_copydepth_g65536.txt.)
template <bool VEC, bool COUNT, class Src, class F, class D = NoDesc>
__device__ __forceinline__ void copy_loop(const Src &src, const F &fo, int c, int nend, int plo, int phi,
                                          int slo, int shi, int T, int &found, D &&dt = D{}) {
  constexpr int NI = F::kNI;
  constexpr int CW = 256;
  const int lane = lane_id();
  int cmask = fo.copy;
  if constexpr (VEC) {
    if (c > phi || (!cmask && !(slo <= shi && c <= shi))) return;
    int4 cur = make_int4(0, 0, 0, 0);
    if (c + 4 * lane + 3 >= plo && c + 4 * lane <= phi) cur = ld4(src.at(c + 4 * lane));
    for (;;) {
      const int i0 = c + 4 * lane;
      const int cmask_n = c + CW >= nend ? 0 : cmask;
      const int cn = c + CW;
      const bool more = cn <= phi && (cmask_n || (slo <= shi && cn <= shi));
      int4 nxt = make_int4(0, 0, 0, 0);
      if (more && cn + 4 * lane <= phi) nxt = ld4(src.at(cn + 4 * lane));
      {
        const int ce[4] = {cur.x, cur.y, cur.z, cur.w};
        dt.template see<4>(ce, c, plo, phi);
      }
      if (slo <= shi && c <= shi && c + CW - 1 >= slo) {
        const int e[4] = {cur.x, cur.y, cur.z, cur.w};
        int lu = -1;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (i0 + u >= slo && i0 + u <= shi && e[u] == T) lu = u;
        const unsigned long long m = __ballot(lu >= 0);
        if (m) {
          const int l = 63 - __clzll((long long)m);
          found = c + 4 * l + __shfl(lu, l, 64);
        }
      }
      if (!COUNT) {
#pragma unroll
        for (int q = 0; q < NI; ++q) {
          if (!((cmask >> q) & 1)) continue;
          if (i0 + 3 < nend) {
            st4(fo.at(q, i0), cur.x, cur.y, cur.z, cur.w);
          } else {
            const int e[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
            for (int u = 0; u < 4; ++u)
              if (i0 + u < nend) st1(fo.at(q, i0 + u), e[u]);
          }
        }
      }
      if (!more) return;
      cmask = cmask_n;
      c = cn;
      cur = nxt;
    }
  } else {
    for (; c <= phi; c += 64 * 4) {
      if (!cmask && !(slo <= shi && c <= shi)) break;
      int idx[4], e[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        idx[u] = c + 64 * u + lane;
        e[u] = (idx[u] >= plo && idx[u] <= phi) ? ld1(src.at(idx[u])) : 0;
      }
      dt.see_strided(e, c, plo, phi);
      if (slo <= shi && c <= shi && c + CW - 1 >= slo) {
        int hit = -1;
#pragma unroll
        for (int u = 3; u >= 0; --u) {
          if (hit >= 0) break;
          const unsigned long long m = __ballot(idx[u] >= slo && idx[u] <= shi && e[u] == T);
          if (m) hit = c + 64 * u + 63 - __clzll((long long)m);
        }
        if (hit >= 0) found = hit;
      }
      if (!COUNT) {
#pragma unroll
        for (int q = 0; q < NI; ++q) {
          if (!((cmask >> q) & 1)) continue;
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (idx[u] < nend) st1(fo.at(q, idx[u]), e[u]);
        }
      }
      if (c + CW >= nend) cmask = 0;
    }
  }
}

}  // namespace
}  // namespace mraft

// MRAFT_DEBUG_BOUNDS builds: an exported reader of this translation unit's
// violation count (reset = 1 zeroes it after reading; -1 on a HIP error).
#if MRAFT_DEBUG_BOUNDS
#define MRAFT_BOUNDS_READER(fn)                                                                     \
  extern "C" long long fn(int reset) {                                                              \
    unsigned long long v = 0;                                                                       \
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(mraft::g_bounds_violations), sizeof v, 0,               \
                            hipMemcpyDeviceToHost) != hipSuccess)                                   \
      return -1;                                                                                    \
    if (reset) {                                                                                    \
      const unsigned long long z = 0;                                                               \
      if (hipMemcpyToSymbol(HIP_SYMBOL(mraft::g_bounds_violations), &z, sizeof z, 0,               \
                            hipMemcpyHostToDevice) != hipSuccess)                                   \
        return -1;                                                                                  \
    }                                                                                               \
    return (long long)v;                                                                            \
  }
#else
#define MRAFT_BOUNDS_READER(fn)
#endif
