// LDS bank model probe (gfx950): clocks per ds_add_f64 wave-instruction for fixed lane -> slot
// patterns of 72-B blocks (the gather accumulator's layout: dword address 18*slot + 2e), to pin
// which lanes conflict (ds_add_f64 and the 9-double block read): 32-lane halves vs 16-lane quarters, and equal slots vs equal residues.
// One 256-thread workgroup per CU (4 waves). Timing only.
// build: hipcc --offload-arch=gfx950 -O3 -o lds_bank_probe lds_bank_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int SLOTS = 398;

__device__ int pattern(int pat, int lane) {
  switch (pat) {
    case 0: return lane;                                // all distinct, residues mod 32 distinct per half
    case 1: return (lane & 15) + 32 * (lane >> 4);      // quarters distinct, 2-way mod 32 in each half
    case 2: return (lane >> 1) + 32 * (lane & 1);       // 2-way mod 32 inside each quarter (pairs)
    case 3: return (lane & 31) * 2 % 64 + (lane >> 5);  // even residues: 2-way mod 32 within half
    case 4: return lane >> 1;                           // pairs share a slot
    case 5: return lane >> 2;                           // 4 lanes share a slot
    case 6: return (lane & 7) + 32 * (lane >> 3);       // 4-way mod 32 in each half, 2-way per quarter
    case 7: return 32 * (lane & 7) + (lane >> 3);       // 8 consecutive lanes equal mod 32
    case 8: return (lane & 31);                         // lane l and l+32 same slot (different halves)
    case 9: return (lane & 15) + 16 * ((lane >> 4) & 1) + 64 * (lane >> 5);  // = pat 0 shape, halves offset 64
    case 10: return (lane * 16) % 64 + (lane >> 2);     // residues mod 16 equal in groups (x*16)
    case 11: return (lane & 15) + 32 * ((lane >> 4) & 1) + 16 * (lane >> 5);  // quarter q residues 16*(q>>1)+..
    default: return lane;
  }
}

template <bool READ>
__global__ __launch_bounds__(1024) void k_probe(int pat, int iters, unsigned long long* out, double* sink) {
  __shared__ double acc[SLOTS * 9];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int t = tid; t < SLOTS * 9; t += blockDim.x) acc[t] = 0.0;
  __syncthreads();
  const int slot = pattern(pat, lane) % SLOTS;
  double v = 1.0 + 1e-3 * tid;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  double sum = 0.0;
  for (int it = 0; it < iters; ++it) {
    double* p = acc + ((slot + (READ ? (it & 1) * 64 : 0)) % SLOTS) * 9;
    if (READ) {
      double t = 0.0;
#pragma unroll
      for (int e = 0; e < 9; ++e) t += p[e];
      sum += t * v;
      asm volatile("" ::: "memory");  // keep the reads in the loop
    } else {
#pragma unroll
      for (int e = 0; e < 9; ++e) atomicAdd(p + e, v);
    }
    v += 1e-9;
  }
  if (sum == 1.2345) sink[0] = sum;
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[blockIdx.x] = t1 - t0;
  if (acc[tid] == 1.2345) sink[0] = acc[tid];
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  const int blocks = 256, threads = argc > 2 ? atoi(argv[2]) : 256;
  unsigned long long* d;
  double* s;
  (void)hipMalloc(&d, sizeof(unsigned long long) * blocks);
  (void)hipMalloc(&s, sizeof(double));
  for (int rd = 0; rd < 2; ++rd)
  for (int pat = 0; pat < 12; ++pat) {
    if (rd) k_probe<true><<<blocks, threads>>>(pat, iters, d, s);
    else k_probe<false><<<blocks, threads>>>(pat, iters, d, s);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(blocks);
    (void)hipMemcpy(h.data(), d, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
    double mean = 0;
    for (auto x : h) mean += (double)x;
    mean /= blocks;
    printf("%s pattern %2d  %7.2f clocks per double per wave\n", rd ? "read" : "atomic", pat, mean / ((double)iters * 9 * (threads / 64)));
  }
  (void)hipFree(d);
  (void)hipFree(s);
  return 0;
}
