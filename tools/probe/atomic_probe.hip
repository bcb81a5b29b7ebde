// Microbenchmark: HBM copy bandwidth, f64 plain-store scatter, f64 atomic scatter (gfx950).
// Decides whether global assembly should scatter with atomics or gather per row.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void copy_k(const double2* __restrict__ a, double2* __restrict__ b, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) b[i] = a[i];
}
__global__ void write_k(double2* __restrict__ b, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) b[i] = make_double2(1.0, 2.0);
}
// each "element" adds 9 doubles (one 3x3 block) into blocks chosen by a hash; lane = one double of a block
// mode 0: atomic add, mode 1: plain store (racy, just for rate)
template <int MODE>
__global__ void scatter_k(double* __restrict__ vals, size_t nblocks, size_t nadds, unsigned seed, int locality) {
  size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t s = (size_t)gridDim.x * blockDim.x;
  for (size_t i = t; i < nadds * 9; i += s) {
    size_t add = i / 9; int c = i % 9;
    // locality: blocks of consecutive adds land in a nearby window
    size_t base = ((add / locality) * 2654435761ull + seed) % nblocks;
    size_t blk = (base + (add % locality) * 7) % nblocks;
    double* p = vals + blk * 9 + c;
    if (MODE == 0) unsafeAtomicAdd(p, 1.0);
    else *p = 1.0;
  }
}
int main() {
  size_t bytes = 4ull << 30;  // 4 GiB
  size_t n2 = bytes / 16;
  double2 *a, *b;
  CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 0, bytes)); CK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float ms;
  for (int g : {1024, 4096, 16384}) {
    copy_k<<<g, 256>>>(a, b, n2); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); for (int r = 0; r < 5; r++) copy_k<<<g, 256>>>(a, b, n2); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1)); printf("copy grid %d: %.1f GB/s (read+write)\n", g, 2.0 * bytes * 5 / (ms * 1e6));
    CK(hipEventRecord(e0)); for (int r = 0; r < 5; r++) write_k<<<g, 256>>>(b, n2); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1)); printf("write grid %d: %.1f GB/s\n", g, 1.0 * bytes * 5 / (ms * 1e6));
  }
  double* vals = (double*)a; size_t nblocks = bytes / 72;
  size_t nadds = 200000000ull;
  for (int loc : {1, 8, 64, 1024}) {
    scatter_k<0><<<16384, 256>>>(vals, nblocks, nadds / 10, 1, loc); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); scatter_k<0><<<16384, 256>>>(vals, nblocks, nadds, 7, loc); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1)); printf("atomic f64 scatter loc %d: %.1f GB/s added, %.2f Gatom/s\n", loc, nadds * 72.0 / (ms * 1e6), nadds * 9.0 / (ms * 1e6));
    CK(hipEventRecord(e0)); scatter_k<1><<<16384, 256>>>(vals, nblocks, nadds, 7, loc); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1)); printf("plain  f64 scatter loc %d: %.1f GB/s stored\n", loc, nadds * 72.0 / (ms * 1e6));
  }
  int dev; hipDeviceProp_t p; CK(hipGetDevice(&dev)); CK(hipGetDeviceProperties(&p, dev));
  printf("device %s CUs %d mem %.1f GB\n", p.gcnArchName, p.multiProcessorCount, p.totalGlobalMem / 1e9);
  return 0;
}
