// Store / load shape probe (gfx950): what it costs to write 72-B BSR blocks (3x3 f64) and to read
// 80-B cell records when each lane of a wave owns a different block / record, against the
// coalesced shapes the chunk gather uses. Timing only.
//   store modes (GB/s of block bytes written, 2 GiB region, every block written once):
//     0 lane l -> block base+l, 9 x 8-B stores            (contiguous 4.6 KB per wave-instruction group)
//     1 lane l -> block base+l, 4 x 16-B + 1 x 8-B stores  (same bytes, fewer instructions)
//     2 lane l -> block base + (11 l + r) mod 704, 16-B stores (scattered inside a 50 KB window)
//     3 blocks staged through LDS, then 16-B coalesced stores (the chunk gather's store)
//   load modes (GB/s of record bytes read into registers, records 80 B, table 256 MiB):
//     4 lane l -> record (base + l): contiguous
//     5 lane l -> record (base + hash(l, r) mod 256): scattered inside a 20 KB window (L1/L2)
// build: hipcc --offload-arch=gfx950 -O3 -o store_shape_probe store_shape_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d2 __attribute__((ext_vector_type(2)));
typedef double d2u __attribute__((ext_vector_type(2), aligned(8)));

template <int MODE>
__global__ __launch_bounds__(256) void k_store(double* __restrict__ out, int64_t nblk, double seed) {
  constexpr int W = MODE == 3 ? 192 : 704, NR = W / 64;  // window of blocks per wave, rounds
  __shared__ double stage[MODE == 3 ? 4 : 1][MODE == 3 ? W * 9 : 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t nwin = nblk / W;
  for (int64_t win = (int64_t)blockIdx.x * 4 + w; win < nwin; win += (int64_t)gridDim.x * 4) {
    const int64_t base = win * W;
    for (int r = 0; r < NR; ++r) {
      double v[9];
#pragma unroll
      for (int e = 0; e < 9; ++e) v[e] = seed + 1e-3 * e + 1e-6 * r + 1e-9 * lane;
      int64_t blk;
      if (MODE == 2 || MODE == 3) blk = (NR * lane + r) % W;
      else blk = 64 * r + lane;
      if (MODE == 3) {
        double* p = stage[w] + blk * 9;
#pragma unroll
        for (int e = 0; e < 9; ++e) p[e] = v[e];
        continue;
      }
      double* p = out + (base + blk) * 9;
      if (MODE == 0) {
#pragma unroll
        for (int e = 0; e < 9; ++e) __builtin_nontemporal_store(v[e], p + e);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) __builtin_nontemporal_store(d2u{v[2 * e], v[2 * e + 1]}, reinterpret_cast<d2u*>(p + 2 * e));
        __builtin_nontemporal_store(v[8], p + 8);
      }
    }
    if (MODE == 3) {
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      const d2* s2 = reinterpret_cast<const d2*>(stage[w]);
      d2* o2 = reinterpret_cast<d2*>(out + base * 9);  // base * 72 B is 16-B aligned (W even)
      for (int t = lane; t < W * 9 / 2; t += 64) __builtin_nontemporal_store(s2[t], o2 + t);
      __builtin_amdgcn_wave_barrier();
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void k_load(const double* __restrict__ rec, int64_t nrec, int iters, double* sink) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double acc = 0.0;
  const int64_t nwin = nrec / 256;
  uint32_t h = 2654435761u * (uint32_t)(threadIdx.x + 1);
  for (int it = 0; it < iters; ++it)
    for (int64_t win = (int64_t)blockIdx.x * 4 + w; win < nwin; win += (int64_t)gridDim.x * 4) {
      const int64_t base = win * 256;
#pragma unroll 2
      for (int r = 0; r < 4; ++r) {
        int64_t k;
        if (MODE == 4) k = 64 * r + lane;
        else {
          h = h * 1664525u + 1013904223u;
          k = (h >> 8) & 255;
        }
        const d2* p = reinterpret_cast<const d2*>(rec + (base + k) * 10);
#pragma unroll
        for (int e = 0; e < 5; ++e) {
          d2 v = p[e];
          acc += v.x * v.y;
        }
      }
    }
  if (acc == 1.2345) sink[0] = acc;
}

int main() {
  const int64_t bytes = 2ll << 30;
  const int64_t nblk = bytes / 72 / 704 * 704;
  double* out;
  (void)hipMalloc(&out, nblk * 72);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int grid = 1024;
  auto run_store = [&](int mode) {
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(a);
      if (mode == 0) k_store<0><<<grid, 256>>>(out, nblk, 1.0 + rep);
      if (mode == 1) k_store<1><<<grid, 256>>>(out, nblk, 1.0 + rep);
      if (mode == 2) k_store<2><<<grid, 256>>>(out, nblk, 1.0 + rep);
      if (mode == 3) k_store<3><<<grid, 256>>>(out, nblk, 1.0 + rep);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("store mode %d: %.3f ms  %.0f GB/s\n", mode, ms, nblk * 72 / (ms * 1e-3) / 1e9);
  };
  for (int m = 0; m < 4; ++m) run_store(m);
  const int64_t nrec = (256ll << 20) / 80 / 256 * 256;
  double* sink;
  (void)hipMalloc(&sink, 8);
  double* rec = out;
  const int iters = 4;
  for (int mode = 4; mode <= 5; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(a);
      if (mode == 4) k_load<4><<<grid, 256>>>(rec, nrec, iters, sink);
      else k_load<5><<<grid, 256>>>(rec, nrec, iters, sink);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("load mode %d: %.3f ms  %.0f GB/s of records into registers\n", mode, ms,
           (double)nrec * 80 * iters / (ms * 1e-3) / 1e9);
  }
  return 0;
}
