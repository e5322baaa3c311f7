// probe_place.hip — a synthetic stand-in for the tick's memory traffic, to
// test whether the slow/fast split of log images can be seen
// without the tick's data: one 64-lane wave per group, the tick's XCD-aware
// group order (contiguous range per XCD, all eight advancing in lockstep);
// per group it reads the second half of replica 0's row and the third
// quarter of replicas 1 and 2, and writes the second half of replicas 3 and 4.
// Built as a shared library (tools/Makefile) and driven by bench.py after its
// timed region (roofline.placement_probe); the round-2 experiment drivers that
// also used it are in git history before commit a48e527's housekeeping.
#include <hip/hip_runtime.h>

// mode: the group each workgroup takes (blockIdx b, XCD x = b mod 8, j = b / 8,
// per = G / 8 groups per XCD; G a multiple of 8 * 1024 for modes 4-6):
//   0 contiguous range per XCD, ascending (the tick)        1 g = b (XCDs interleaved)
//   2 as 0, odd XCDs walk their range backwards             3 as 0, odd XCDs start mid-range
//   4 chunks of 64 groups dealt round-robin to the XCDs     5 as 0, 1024-group blocks reversed
//   6 as 0, XCD x starts at x/8 of its range (wrapping)
__device__ __forceinline__ int probe_group(int b, int nb, int mode) {
  const int x = b & 7, j = b >> 3, per = nb >> 3;
  switch (mode) {
    case 1: return b;
    case 2: return x * per + ((x & 1) ? per - 1 - j : j);
    case 3: return x * per + ((x & 1) ? (j + per / 2) % per : j);
    case 4: return ((j >> 6) * 8 + x) * 64 + (j & 63);
    case 5: { const int nblk = per >> 10; return x * per + (nblk - 1 - (j >> 10)) * 1024 + (j & 1023); }
    case 6: return x * per + (j + x * (per / 8)) % per;
    case 7: return x * per + (j & 1) * (per / 2) + (j >> 1);                 // range halves walked together
    case 8: return x * per + (j & 3) * (per / 4) + (j >> 2);                 // range quarters walked together
    case 9: return ((j >> 10) * 8 + x) * 1024 + (j & 1023);                  // 1,024-group chunks dealt round-robin
    case 10: return ((j >> 8) * 8 + x) * 256 + (j & 255);                    // 256-group chunks dealt round-robin
    default: return x * per + j;
  }
}

// traffic patterns (mode / 16): 0 the tick's shape (below); 1 reads only (row 0
// half + rows 1-2 quarter); 2 writes only (rows 3-4 half); 3 one 16-KB row per
// group read (row 0 whole), nothing else; 4 row 0 read whole, row 1 written whole.
__global__ __launch_bounds__(64) void k_probe(int *__restrict__ log, int G, int P, int L, int *__restrict__ sink,
                                              int mode) {
  const int g = probe_group((int)blockIdx.x, (int)gridDim.x, mode & 15);
  if (g >= G) return;
  const int pat = mode >> 4;
  if (pat >= 5) {
    // write-order patterns over rows 1..4 (whole rows): 5 row 4 only; 6 the
    // four rows interleaved per 1-KB chunk (the tick's copy); 7 row after row;
    // 8 interleaved per 4-KB block
    const int ln = threadIdx.x;
    int *r0 = log + (long long)g * P * L;
    const int rows_lo = pat == 5 ? 4 : 1;
    const int blk = pat == 6 ? 256 : pat == 8 ? 1024 : L;
    for (int c0 = 0; c0 < L; c0 += blk)
      for (int q = rows_lo; q < 5; ++q)
        for (int c = c0; c < c0 + blk && c < L; c += 256) {
          int4 *d = reinterpret_cast<int4 *>(r0 + q * L + c + 4 * ln);
          __builtin_nontemporal_store(c, &d->x); __builtin_nontemporal_store(q, &d->y);
          __builtin_nontemporal_store(g, &d->z); __builtin_nontemporal_store(ln, &d->w);
        }
    return;
  }
  if (pat >= 1) {
    const int lane0 = threadIdx.x;
    int *r0 = log + (long long)g * P * L;
    int acc0 = 0;
    const int lo = pat >= 3 ? 0 : L / 2;
    for (int c = lo; c < L; c += 256) {
      const int i = c + 4 * lane0;
      if (pat == 1 || pat >= 3) {
        const int4 *s = reinterpret_cast<const int4 *>(r0 + i);
        int4 v;
        v.x = __builtin_nontemporal_load(&s->x); v.y = __builtin_nontemporal_load(&s->y);
        v.z = __builtin_nontemporal_load(&s->z); v.w = __builtin_nontemporal_load(&s->w);
        acc0 ^= v.x ^ v.w;
        if (pat == 4) {
          int4 *d = reinterpret_cast<int4 *>(r0 + L + i);
          __builtin_nontemporal_store(v.x, &d->x); __builtin_nontemporal_store(v.y, &d->y);
          __builtin_nontemporal_store(v.z, &d->z); __builtin_nontemporal_store(v.w, &d->w);
        }
      }
      if (pat == 1 && c < 3 * L / 4)
        for (int q = 1; q < 3; ++q) {
          const int4 *s = reinterpret_cast<const int4 *>(r0 + q * L + i);
          acc0 ^= __builtin_nontemporal_load(&s->x) ^ __builtin_nontemporal_load(&s->w);
        }
      if (pat == 2)
        for (int q = 3; q < 5; ++q) {
          int4 *d = reinterpret_cast<int4 *>(r0 + q * L + i);
          __builtin_nontemporal_store(c, &d->x); __builtin_nontemporal_store(i, &d->y);
          __builtin_nontemporal_store(q, &d->z); __builtin_nontemporal_store(g, &d->w);
        }
    }
    if (acc0 == 0x7fffffff) sink[0] = acc0;
    return;
  }
  const int lane = threadIdx.x;
  int *r = log + (long long)g * P * L;
  int acc = 0;
  for (int c = L / 2; c < L; c += 256) {
    const int i = c + 4 * lane;
    const int4 *s0 = reinterpret_cast<const int4 *>(r + i);
    int4 v;
    v.x = __builtin_nontemporal_load(&s0->x); v.y = __builtin_nontemporal_load(&s0->y);
    v.z = __builtin_nontemporal_load(&s0->z); v.w = __builtin_nontemporal_load(&s0->w);
    if (c < 3 * L / 4) {
#pragma unroll
      for (int q = 1; q < 3; ++q) {
        const int4 *s = reinterpret_cast<const int4 *>(r + q * L + i);
        acc ^= __builtin_nontemporal_load(&s->x) ^ __builtin_nontemporal_load(&s->w);
      }
    }
#pragma unroll
    for (int q = 3; q < 5; ++q) {
      int4 *d = reinterpret_cast<int4 *>(r + q * L + i);
      __builtin_nontemporal_store(v.x, &d->x); __builtin_nontemporal_store(v.y, &d->y);
      __builtin_nontemporal_store(v.z, &d->z); __builtin_nontemporal_store(v.w, &d->w);
    }
  }
  if (acc == 0x7fffffff) sink[0] = acc;
}

extern "C" int probe_place(void *log, int G, int P, int L, void *sink, float *ms, int mode) {
  if (P < 5) return -1;
  hipEvent_t a, b;
  if (hipEventCreate(&a) || hipEventCreate(&b)) return -3;
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(k_probe, dim3(G), dim3(64), 0, 0, (int *)log, G, P, L, (int *)sink, mode);
    (void)hipEventRecord(b, 0);
    if (hipEventSynchronize(b)) return -3;
    float t;
    (void)hipEventElapsedTime(&t, a, b);
    if (r && t < best) best = t;
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  *ms = best;
  return 0;
}

// Plain streaming write over [p, p + bytes): grid-stride, 16 B per lane, non-temporal.
__global__ void k_write_range(int4 *__restrict__ b, long long n4) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    __builtin_nontemporal_store((int)i, &b[i].x); __builtin_nontemporal_store(1, &b[i].y);
    __builtin_nontemporal_store(2, &b[i].z); __builtin_nontemporal_store(3, &b[i].w);
  }
}

extern "C" int probe_write_range(void *p, long long bytes, float *ms) {
  hipEvent_t a, b;
  if (hipEventCreate(&a) || hipEventCreate(&b)) return -3;
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    (void)hipEventRecord(a, 0);
    hipLaunchKernelGGL(k_write_range, dim3(16384), dim3(256), 0, 0, (int4 *)p, bytes / 16);
    (void)hipEventRecord(b, 0);
    if (hipEventSynchronize(b)) return -3;
    float t;
    (void)hipEventElapsedTime(&t, a, b);
    if (r && t < best) best = t;
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  *ms = best;
  return 0;
}
