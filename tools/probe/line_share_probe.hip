// Probe (round 6): do stores from different XCDs into different bytes of one 128-B line, issued at
// about the same time inside one kernel, all reach memory? The gathers' chunk drains store each
// chunk's values; two chunks adjacent in the value array share the 16-B pair / 128-B line at their
// boundary (each stores its own 8-B half). When adjacent chunks run on different XCDs at the same
// time (the neo gather's dealt order; the tail-stealing variant), their L2s each hold a partial line.
// Grid of 8 x G workgroups (blockIdx % 8 = the XCD under round-robin dispatch); line L of the array
// is written by all 8 XCDs: XCD x stores 8-B words x and x + 8 (W = 8) or 16-B words x (W = 16) of
// it, lines assigned so the 8 workgroups of one group write the same lines together. After each
// launch every word is checked against its expected value. Modes: plain, nt (the drains' policy).
// Build: hipcc --offload-arch=gfx950 -O3 -o line_share_probe line_share_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ unsigned long long val(unsigned seed, unsigned long long line, int k) {
  return (line * 16 + k) * 2654435761ull + seed;
}

template <int W, bool NT>
__global__ __launch_bounds__(256) void k_share(unsigned long long* __restrict__ a, unsigned long long nlines,
                                               unsigned seed) {
  const int xc = (int)(blockIdx.x % 8);
  const unsigned long long g = blockIdx.x / 8, ng = gridDim.x / 8;
  for (unsigned long long L = g * 256 + threadIdx.x; L < nlines; L += ng * 256) {
    unsigned long long* p = a + L * 16;
    if constexpr (W == 8) {
      const unsigned long long v0 = val(seed, L, xc), v1 = val(seed, L, xc + 8);
      if (NT) {
        __builtin_nontemporal_store(v0, p + xc);
        __builtin_nontemporal_store(v1, p + xc + 8);
      } else {
        p[xc] = v0;
        p[xc + 8] = v1;
      }
    } else {
      typedef unsigned long long u2 __attribute__((ext_vector_type(2)));
      const u2 v = u2{val(seed, L, 2 * xc), val(seed, L, 2 * xc + 1)};
      u2* q = reinterpret_cast<u2*>(p) + xc;
      if (NT) __builtin_nontemporal_store(v, q);
      else *q = v;
    }
  }
}

__global__ void k_check(const unsigned long long* __restrict__ a, unsigned long long nlines, unsigned seed,
                        unsigned long long* __restrict__ bad) {
  const unsigned long long n = nlines * 16;
  for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    if (a[i] != val(seed, i / 16, (int)(i % 16))) atomicAdd(bad, 1ull);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const unsigned long long nlines = 1ull << 20;  // 128 MiB
  unsigned long long *a = nullptr, *bad = nullptr;
  CK(hipMalloc(&a, nlines * 128));
  CK(hipMalloc(&bad, 8));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const unsigned grids[] = {8u * 32, (unsigned)cus * 4};
  for (int mode = 0; mode < 4; ++mode) {
    for (unsigned grid : grids) {
      unsigned long long tot = 0;
      for (int r = 0; r < reps; ++r) {
        const unsigned seed = 1000u * mode + 17u * r + grid;
        CK(hipMemset(a, 0xFF, nlines * 128));
        CK(hipMemset(bad, 0, 8));
        if (mode == 0) k_share<8, false><<<grid, 256>>>(a, nlines, seed);
        if (mode == 1) k_share<8, true><<<grid, 256>>>(a, nlines, seed);
        if (mode == 2) k_share<16, false><<<grid, 256>>>(a, nlines, seed);
        if (mode == 3) k_share<16, true><<<grid, 256>>>(a, nlines, seed);
        CK(hipGetLastError());
        k_check<<<2048, 256>>>(a, nlines, seed, bad);
        unsigned long long h = 0;
        CK(hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost));
        tot += h;
      }
      printf("%s %s grid %5u: wrong words %llu of %llu\n", mode / 2 ? "16-B" : " 8-B", mode % 2 ? "nt   " : "plain", grid,
             tot, (unsigned long long)reps * nlines * 16);
      fflush(stdout);
    }
  }
  return 0;
}
