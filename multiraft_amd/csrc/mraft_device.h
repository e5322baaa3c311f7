// mraft_device.h — device-side building blocks shared by the gfx950 kernels.
//
// Wave-cooperative primitives (64-lane wavefronts, 64-bit ballots) used by the
// AppendEntries follower path and the leader's commit scan:
//  * wave_conflict_scan — the ConflictIndex backward scan of
//    raft_append_entry.go:136-142, 256 terms per iteration (4 coalesced
//    dword loads per lane in flight), first mismatch by ballot + find-first-set;
//  * wave_merge_compare — the entry merge of :149-155: compares the entries'
//    terms with the follower's log 256 at a time, first mismatch by ballot;
//  * wave_copy — truncate-and-append (raft_log.go:62-75) as a streaming copy
//    of the leader's tail into the follower's log;
//  * wave_commit_scan — the term gate of advanceCommitIndexForLeader
//    (:89-105): highest index in a range whose term equals currentTerm.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mraft {

constexpr int kLeader = 1, kCandidate = 2, kFollower = 3;  // raft_rpc.go:8-12
constexpr int kWave = 64;
constexpr int kUnroll = 4;                 // loads in flight per lane per stream
constexpr int kChunk = kWave * kUnroll;    // terms per wave iteration

struct Dev {
  int32_t *term, *voted, *role, *commit, *applied, *dummy, *last, *votes;
  int32_t *log, *match, *next;
  int32_t *pdirty;  // persist_dirty (include/mraft.h MRAFT_PERSIST_*); may be null
  int32_t *head;    // log_head: ring position of each replica's dummy entry
  int32_t *hsnap;   // has_snapshot (raft.go:158): set by an installing InstallSnapshot
  int32_t *srt;     // terms_sorted (include/mraft.h MRAFT_TERMS_SORTED): the terms after the dummy never decrease
  int32_t G, P, L;
};

// The log ring (include/mraft.h): Index i of a replica with dummy d and head h
// lives at row + ring(i - d + h, L). Valid for arguments in [-L, 2L): live
// entries have i - d in [0, L), and the pass's masked-out lanes stay within
// one row length of them.
__device__ __forceinline__ int ring(int k, int L) {
  k = k >= L ? k - L : k;
  return k < 0 ? k + L : k;
}

// Term of Index i of replica `slot` (dummy d, head h).
__device__ __forceinline__ int term_at(const Dev &s, int64_t slot, int d, int h, int i) {
  return s.log[slot * s.L + ring(i - d + h, s.L)];
}

// Records a persist() / SaveStateAndSnapshot() call site of the reference for
// replica `slot` (one writer per slot per launch).
__device__ __forceinline__ void mark_persist(const Dev &s, int64_t slot, int bits) {
  if (s.pdirty && bits) s.pdirty[slot] |= bits;
}

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

__device__ __forceinline__ int first_lane(unsigned long long m) { return __ffsll((long long)m) - 1; }

// Largest idx in [lo, hi] with term(idx) != a, scanning downward, in a ring
// row whose Index `base` (the dummy) sits at `head` (row length L); returns
// lo - 1 when every term in the range equals a. Wave-uniform arguments; the
// term of lo must be readable when lo <= hi (lanes past lo re-read it).
template <int U = kUnroll>
__device__ __forceinline__ int wave_scan_down_ne(const int32_t *__restrict__ row, int base, int head,
                                                 int L, int lo, int hi, int a) {
  const int lane = lane_id();
  for (int top = hi; top >= lo; top -= kWave * U) {
    int v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = top - lane - kWave * u;
      const int w = row[ring(max(idx, lo) - base + head, L)];  // unconditional: the loads issue back to back
      v[u] = idx >= lo ? w : a;
    }
    // Every ballot, no exit per vector (which lets the compiler sink each load
    // behind the previous compare: one round trip per 64 terms).
    int r = lo - 1;
#pragma unroll
    for (int u = U - 1; u >= 0; --u) {
      const unsigned long long m = __ballot(v[u] != a);
      r = m ? top - kWave * u - first_lane(m) : r;
    }
    if (r >= lo) return r;
  }
  return lo - 1;
}

// Largest idx in [lo, hi] with term(idx) == a (ring row as above); lo - 1 if none.
__device__ __forceinline__ int wave_scan_down_eq(const int32_t *__restrict__ row, int base, int head,
                                                 int L, int lo, int hi, int a) {
  const int lane = lane_id();
  for (int top = hi; top >= lo; top -= kChunk) {
    int v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int idx = top - lane - kWave * u;
      const int w = row[ring(max(idx, lo) - base + head, L)];
      v[u] = idx >= lo ? w : a + 1;
    }
    int r = lo - 1;
#pragma unroll
    for (int u = kUnroll - 1; u >= 0; --u) {
      const unsigned long long m = __ballot(v[u] == a);
      r = m ? top - kWave * u - first_lane(m) : r;
    }
    if (r >= lo) return r;
  }
  return lo - 1;
}

// ConflictIndex of raft_append_entry.go:136-142 for prev > dummy + 1, where
// a = term(prev): the largest index in [dummy+2, prev-1] whose term differs
// from a, else dummy + 1. The first probe reads one term per lane (64 terms:
// most runs end there), then 256-term iterations.
__device__ __forceinline__ int wave_conflict_scan(const int32_t *__restrict__ frow, int fdummy, int fhead,
                                                  int L, int prev, int a) {
  const int lo = fdummy + 2, hi = prev - 1;
  const int idx = hi - lane_id();
  const int v = idx >= lo ? frow[ring(idx - fdummy + fhead, L)] : a;
  const unsigned long long m = __ballot(v != a);
  if (m) return hi - first_lane(m);
  if (hi - 64 < lo) return fdummy + 1;
  const int r = wave_scan_down_ne(frow, fdummy, fhead, L, lo, hi - 64, a);
  return r < lo ? fdummy + 1 : r;
}

// First k in [0, kc) with E[k] != F[k]; -1 if none.
__device__ __forceinline__ int wave_merge_compare(const int32_t *__restrict__ E,
                                                  const int32_t *__restrict__ F, int kc) {
  const int lane = lane_id();
  for (int base = 0; base < kc; base += kChunk) {
    int e[kUnroll], f[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int k = base + lane + kWave * u, kk = min(k, kc - 1);
      const int x = E[kk], y = F[kk];
      e[u] = k < kc ? x : 0;
      f[u] = k < kc ? y : 0;
    }
    int r = -1;
#pragma unroll
    for (int u = kUnroll - 1; u >= 0; --u) {
      const unsigned long long m = __ballot(e[u] != f[u]);
      r = m ? base + kWave * u + first_lane(m) : r;
    }
    if (r >= 0) return r;
  }
  return -1;
}

// F[k] = E[k] for k in [0, cnt).
__device__ __forceinline__ void wave_copy(const int32_t *__restrict__ E, int32_t *__restrict__ F,
                                          int cnt) {
  const int lane = lane_id();
  for (int base = 0; base < cnt; base += kChunk) {
    int v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      int k = base + lane + kWave * u;
      v[u] = k < cnt ? E[k] : 0;
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      int k = base + lane + kWave * u;
      if (k < cnt) F[k] = v[u];
    }
  }
}

// n terms of a ring row from Index `from` (dummy `base` at `head`) into dst,
// in order: the ring unrolled (persistence read-out, staged entries).
__device__ __forceinline__ void wave_copy_from_ring(const int32_t *__restrict__ row, int base, int head,
                                                    int L, int from, int32_t *__restrict__ dst, int cnt) {
  const int lane = lane_id();
  for (int b = 0; b < cnt; b += kChunk) {
    int v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int k = b + lane + kWave * u;
      v[u] = k < cnt ? row[ring(from + k - base + head, L)] : 0;
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int k = b + lane + kWave * u;
      if (k < cnt) dst[k] = v[u];
    }
  }
}

// Whether the terms of Index [lo, hi] of a ring row (dummy `base` at `head`)
// never decrease (wave-cooperative; terms_sorted, include/mraft.h). Not on a
// hot path: load_state and restore only.
__device__ __forceinline__ bool wave_terms_sorted(const int32_t *__restrict__ row, int base, int head, int L,
                                                  int lo, int hi) {
  // (offsets from lo: an Index loop `b += 64` would overflow int32 within 64
  // of 2^31 - 1, include/mraft.h's Index domain)
  for (int d = 0; d < hi - lo; d += kWave) {
    const int k = d + lane_id();  // Index lo + k
    const bool bad = k < hi - lo && row[ring(lo + k - base + head, L)] > row[ring(lo + k + 1 - base + head, L)];
    if (__ballot(bad)) return false;
  }
  return true;
}

__device__ __forceinline__ int shfl_i(int v, int src) { return __shfl(v, src, 64); }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace mraft
