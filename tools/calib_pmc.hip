// calib_pmc.hip — calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for
// the access widths the engine uses (tools/profile_round.sh). Each kernel
// streams a known number of bytes from a buffer far larger than the 256 MiB
// Infinity Cache; the ratio counter_bytes / known_bytes is the correction
// applied to the engine's counters (MI355X_MICROARCH.md §HBM: FETCH_SIZE
// reads 1/2 of a 16-B/lane stream; other widths must be calibrated).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void copy_dword(const int *__restrict__ a, int *__restrict__ b, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    b[i] = a[i];
}
__global__ void copy_dwordx4(const int4 *__restrict__ a, int4 *__restrict__ b, long n4) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    b[i] = a[i];
}
__global__ void read_dword(const int *__restrict__ a, int *__restrict__ out, long n) {
  int acc = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    acc ^= a[i];
  if (acc == 0x7fffffff) out[0] = acc;
}

int main() {
  const long n = 512l << 20;  // 512 Mi ints = 2 GiB per buffer
  int *a, *b;
  if (hipMalloc(&a, n * 4) || hipMalloc(&b, n * 4)) { printf("alloc failed\n"); return 1; }
  (void)hipMemset(a, 1, n * 4);
  (void)hipMemset(b, 2, n * 4);
  (void)hipDeviceSynchronize();
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(copy_dword, dim3(8192), dim3(256), 0, 0, a, b, n);
    hipLaunchKernelGGL(copy_dwordx4, dim3(8192), dim3(256), 0, 0, (const int4 *)a, (int4 *)b, n / 4);
    hipLaunchKernelGGL(read_dword, dim3(8192), dim3(256), 0, 0, a, b, n);
  }
  (void)hipDeviceSynchronize();
  printf("{\"known_read_bytes\": %ld, \"known_write_bytes\": %ld}\n", n * 4, n * 4);
  (void)hipFree(a);
  (void)hipFree(b);
  return 0;
}
