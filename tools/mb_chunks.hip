// mb_chunks.hip — is the tick's per-allocation speed (some state
// copies are ~13 % slower, and tools/exp_vmm_alias.py shows it follows the
// physical memory, not the virtual layout) visible to plain streaming kernels?
// Allocates NCOPY x NCH physical chunks of 1 GiB (hipMemCreate), maps each at
// its own VA, and times a streaming read, a streaming write and an in-chunk
// copy (first half -> second half) on every chunk, plus a "5-row" pattern:
// one wave per 16-KB-row quintet reading row 0 and writing rows 1-4 (the
// tick's fan-out shape).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s failed: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void rd(const int4 *__restrict__ a, int *__restrict__ out, long n4) {
  int acc = 0;
  for (long t = (long)blockIdx.x * 1024; t < n4; t += (long)gridDim.x * 1024) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      long i = t + u * 256 + threadIdx.x;
      if (i < n4) {
        int4 v;
        v.x = __builtin_nontemporal_load(&a[i].x); v.y = __builtin_nontemporal_load(&a[i].y);
        v.z = __builtin_nontemporal_load(&a[i].z); v.w = __builtin_nontemporal_load(&a[i].w);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      }
    }
  }
  if (acc == 0x12345678) out[0] = acc;
}
__global__ void wr(int4 *__restrict__ b, long n4) {
  for (long t = (long)blockIdx.x * 1024; t < n4; t += (long)gridDim.x * 1024) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      long i = t + u * 256 + threadIdx.x;
      if (i < n4) {
        __builtin_nontemporal_store(u, &b[i].x); __builtin_nontemporal_store(1, &b[i].y);
        __builtin_nontemporal_store(2, &b[i].z); __builtin_nontemporal_store(3, &b[i].w);
      }
    }
  }
}
__global__ void cp(const int4 *__restrict__ a, int4 *__restrict__ b, long n4) {
  for (long t = (long)blockIdx.x * 1024; t < n4; t += (long)gridDim.x * 1024) {
    int4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      long i = t + u * 256 + threadIdx.x;
      if (i < n4) {
        v[u].x = __builtin_nontemporal_load(&a[i].x); v[u].y = __builtin_nontemporal_load(&a[i].y);
        v[u].z = __builtin_nontemporal_load(&a[i].z); v[u].w = __builtin_nontemporal_load(&a[i].w);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      long i = t + u * 256 + threadIdx.x;
      if (i < n4) {
        __builtin_nontemporal_store(v[u].x, &b[i].x); __builtin_nontemporal_store(v[u].y, &b[i].y);
        __builtin_nontemporal_store(v[u].z, &b[i].z); __builtin_nontemporal_store(v[u].w, &b[i].w);
      }
    }
  }
}
// one 64-lane wave per quintet of 16-KB rows: row 0 read once, written to rows 1..4
__global__ __launch_bounds__(64) void fan(int *__restrict__ base, long nquint) {
  const long g = blockIdx.x;
  if (g >= nquint) return;
  int *row0 = base + g * 5 * 4096;
  const int lane = threadIdx.x;
  for (int c = 0; c < 4096; c += 256) {
    const int i = c + 4 * lane;
    int4 v;
    const int4 *s = reinterpret_cast<const int4 *>(row0 + i);
    v.x = __builtin_nontemporal_load(&s->x); v.y = __builtin_nontemporal_load(&s->y);
    v.z = __builtin_nontemporal_load(&s->z); v.w = __builtin_nontemporal_load(&s->w);
#pragma unroll
    for (int q = 1; q < 5; ++q) {
      int4 *d = reinterpret_cast<int4 *>(row0 + q * 4096 + i);
      __builtin_nontemporal_store(v.x, &d->x); __builtin_nontemporal_store(v.y, &d->y);
      __builtin_nontemporal_store(v.z, &d->z); __builtin_nontemporal_store(v.w, &d->w);
    }
  }
}

int main(int argc, char **argv) {
  const int NCOPY = argc > 1 ? atoi(argv[1]) : 6, NCH = argc > 2 ? atoi(argv[2]) : 5;
  const size_t gran = 1ull << 30;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  std::vector<int *> chunks;
  for (int i = 0; i < NCOPY * NCH; ++i) {
    hipMemGenericAllocationHandle_t h;
    CK(hipMemCreate(&h, gran, &prop, 0));
    void *va;
    CK(hipMemAddressReserve(&va, gran, gran, nullptr, 0));
    CK(hipMemMap(va, gran, 0, h, 0));
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    CK(hipMemSetAccess(va, gran, &acc, 1));
    CK(hipMemset(va, 1, gran));
    chunks.push_back((int *)va);
  }
  int *out;
  CK(hipMalloc(&out, 64));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto timeit = [&](auto fn) {
    fn(); CK(hipDeviceSynchronize());
    float best = 1e9;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(a)); fn(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b));
      best = ms < best ? ms : best;
    }
    return best;
  };
  const long n4 = (long)(gran / 16);
  const long nq = (long)(gran / (5 * 4096 * 4));
  for (int i = 0; i < NCOPY * NCH; ++i) {
    int4 *p = (int4 *)chunks[i];
    const float tr = timeit([&] { hipLaunchKernelGGL(rd, dim3(16384), dim3(256), 0, 0, p, out, n4); });
    const float tw = timeit([&] { hipLaunchKernelGGL(wr, dim3(16384), dim3(256), 0, 0, p, n4); });
    const float tc = timeit([&] { hipLaunchKernelGGL(cp, dim3(16384), dim3(256), 0, 0, p, p + n4 / 2, n4 / 2); });
    const float tf = timeit([&] { hipLaunchKernelGGL(fan, dim3(nq), dim3(64), 0, 0, (int *)p, nq); });
    printf("copy %d chunk %d @ %p: read %.2f TB/s  write %.2f TB/s  copy %.2f TB/s  fan1:4 %.2f TB/s\n", i / NCH,
           i % NCH, (void *)p, gran / (tr * 1e-3) / 1e12, gran / (tw * 1e-3) / 1e12, gran / (tc * 1e-3) / 1e12,
           (double)nq * 5 * 4096 * 4 / (tf * 1e-3) / 1e12);
    fflush(stdout);
  }
  return 0;
}
