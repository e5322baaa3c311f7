// mb_segcopy.hip — what HBM bandwidth does the tick's access pattern allow?
// Copies ~1500-word segments between random 16 KB rows of a 5 GiB log array
// (one wave per group of 4 segments, like the tick's copy phase) and compares
// with a plain sequential dwordx4 copy of the same byte count.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int L = 4096;

template <int VC>
__global__ __launch_bounds__(256) void segcopy(int *__restrict__ log, const int4 *__restrict__ seg, int nseg_groups) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (w >= nseg_groups) return;
  const int4 d = seg[w];  // src row, first dst row, start, end
  const long long src = (long long)d.x * L;
  for (int c = d.z & ~3; c <= d.w; c += 256 * VC) {
    int4 v[VC];
#pragma unroll
    for (int u = 0; u < VC; ++u) {
      const int i = c + 256 * u + 4 * lane;
      v[u] = i <= d.w ? *reinterpret_cast<const int4 *>(log + src + i) : make_int4(0, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long long dst = (long long)(d.y + q) * L;
#pragma unroll
      for (int u = 0; u < VC; ++u) {
        const int i = c + 256 * u + 4 * lane;
        if (i + 3 <= d.w) *reinterpret_cast<int4 *>(log + dst + i) = v[u];
      }
    }
  }
}

__global__ void seqcopy(const int4 *__restrict__ a, int4 *__restrict__ b, long n4) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) b[i] = a[i];
}
// 4 dwordx4 per thread in flight, block-contiguous 16 KB tiles.
__global__ void seqcopy4(const int4 *__restrict__ a, int4 *__restrict__ b, long n4) {
  for (long t = (long)blockIdx.x * 1024; t < n4; t += (long)gridDim.x * 1024) {
    int4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { long i = t + u * 256 + threadIdx.x; v[u] = i < n4 ? a[i] : make_int4(0, 0, 0, 0); }
#pragma unroll
    for (int u = 0; u < 4; ++u) { long i = t + u * 256 + threadIdx.x; if (i < n4) b[i] = v[u]; }
  }
}
// Same with non-temporal loads and/or stores.
template <bool NTL, bool NTS>
__global__ void seqcopy4nt(const int4 *__restrict__ a, int4 *__restrict__ b, long n4) {
  for (long t = (long)blockIdx.x * 1024; t < n4; t += (long)gridDim.x * 1024) {
    int4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      long i = t + u * 256 + threadIdx.x;
      if (i < n4) {
        if (NTL) {
          v[u].x = __builtin_nontemporal_load(&a[i].x); v[u].y = __builtin_nontemporal_load(&a[i].y);
          v[u].z = __builtin_nontemporal_load(&a[i].z); v[u].w = __builtin_nontemporal_load(&a[i].w);
        } else {
          v[u] = a[i];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      long i = t + u * 256 + threadIdx.x;
      if (i < n4) {
        if (NTS) {
          __builtin_nontemporal_store(v[u].x, &b[i].x); __builtin_nontemporal_store(v[u].y, &b[i].y);
          __builtin_nontemporal_store(v[u].z, &b[i].z); __builtin_nontemporal_store(v[u].w, &b[i].w);
        } else {
          b[i] = v[u];
        }
      }
    }
  }
}
__global__ void seqread4(const int4 *__restrict__ a, int *__restrict__ out, long n4) {
  int acc = 0;
  for (long t = (long)blockIdx.x * 1024; t < n4; t += (long)gridDim.x * 1024) {
#pragma unroll
    for (int u = 0; u < 4; ++u) { long i = t + u * 256 + threadIdx.x; if (i < n4) { int4 v = a[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; } }
  }
  if (acc == 0x12345678) out[0] = acc;
}
__global__ void seqwrite4(int4 *__restrict__ b, long n4) {
  for (long t = (long)blockIdx.x * 1024; t < n4; t += (long)gridDim.x * 1024) {
#pragma unroll
    for (int u = 0; u < 4; ++u) { long i = t + u * 256 + threadIdx.x; if (i < n4) b[i] = make_int4(u, 1, 2, 3); }
  }
}

int main() {
  const long G = 65536, P = 5, rows = G * P;
  int *log;
  if (hipMalloc(&log, rows * L * 4)) return 1;
  (void)hipMemset(log, 1, rows * L * 4);
  std::vector<int4> h(G);
  srand(7);
  double bytes = 0;
  for (long g = 0; g < G; ++g) {
    int last = 2048 + rand() % 2048, start = rand() % last;
    h[g] = make_int4((int)(g * P), (int)(g * P + 1), start, last);
    bytes += (double)(last - (start & ~3) + 1) * 4 * 5;  // 1 read + 4 writes
  }
  int4 *seg;
  (void)hipMalloc(&seg, G * sizeof(int4));
  (void)hipMemcpy(seg, h.data(), G * sizeof(int4), hipMemcpyHostToDevice);
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  auto run = [&](const char *name, auto fn, double nbytes) {
    fn(); (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int r = 0; r < 10; ++r) fn();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b);
    printf("%-28s %8.1f us  %6.2f TB/s\n", name, ms * 100, nbytes / (ms / 10 * 1e-3) / 1e12);
  };
  const int blocks = (int)((G + 3) / 4);
  run("segcopy VC=1 (1 KB/it)", [&] { hipLaunchKernelGGL(segcopy<1>, dim3(blocks), dim3(256), 0, 0, log, seg, (int)G); }, bytes);
  run("segcopy VC=2", [&] { hipLaunchKernelGGL(segcopy<2>, dim3(blocks), dim3(256), 0, 0, log, seg, (int)G); }, bytes);
  run("segcopy VC=4", [&] { hipLaunchKernelGGL(segcopy<4>, dim3(blocks), dim3(256), 0, 0, log, seg, (int)G); }, bytes);
  const long n4 = (long)(bytes / 2 / 16);
  run("sequential copy same bytes", [&] { hipLaunchKernelGGL(seqcopy, dim3(8192), dim3(256), 0, 0, (const int4 *)log, (int4 *)(log + 4 * n4 + 1024), n4); }, (double)n4 * 32);
  for (int grid : {4096, 16384}) {
    char nm[64];
    snprintf(nm, sizeof nm, "copy x4 nt-store grid %d", grid);
    run(nm, [&] { hipLaunchKernelGGL((seqcopy4nt<false, true>), dim3(grid), dim3(256), 0, 0, (const int4 *)log, (int4 *)(log + 4 * n4 + 1024), n4); }, (double)n4 * 32);
    snprintf(nm, sizeof nm, "copy x4 nt-load grid %d", grid);
    run(nm, [&] { hipLaunchKernelGGL((seqcopy4nt<true, false>), dim3(grid), dim3(256), 0, 0, (const int4 *)log, (int4 *)(log + 4 * n4 + 1024), n4); }, (double)n4 * 32);
    snprintf(nm, sizeof nm, "copy x4 nt-both grid %d", grid);
    run(nm, [&] { hipLaunchKernelGGL((seqcopy4nt<true, true>), dim3(grid), dim3(256), 0, 0, (const int4 *)log, (int4 *)(log + 4 * n4 + 1024), n4); }, (double)n4 * 32);
  }
  for (int grid : {2048, 4096, 8192, 16384}) {
    char nm[64];
    snprintf(nm, sizeof nm, "copy x4 grid %d", grid);
    run(nm, [&] { hipLaunchKernelGGL(seqcopy4, dim3(grid), dim3(256), 0, 0, (const int4 *)log, (int4 *)(log + 4 * n4 + 1024), n4); }, (double)n4 * 32);
    snprintf(nm, sizeof nm, "read x4 grid %d", grid);
    run(nm, [&] { hipLaunchKernelGGL(seqread4, dim3(grid), dim3(256), 0, 0, (const int4 *)log, log + 16, 2 * n4); }, (double)n4 * 32);
    snprintf(nm, sizeof nm, "write x4 grid %d", grid);
    run(nm, [&] { hipLaunchKernelGGL(seqwrite4, dim3(grid), dim3(256), 0, 0, (int4 *)log, 2 * n4); }, (double)n4 * 32);
  }
  return 0;
}
