// LDS accumulate-op cost probe (gfx950): shader clocks per wave-instruction, CU-wide, for the ways
// the gather kernel could add a 3x3 FP64 block into its LDS accumulator. One 256-thread workgroup
// per CU (4 waves, one per SIMD) or one wave; each lane adds 9 doubles per iteration.
//   mode 0: ds_add_f64, lane l -> its own slot (conflict-free addresses)
//   mode 1: ds_read_b64 + v_add_f64 + ds_write_b64 (non-atomic), own slot
//   mode 2: ds_add_u64 (integer atomic), own slot
//   mode 3: ds_write_b64 only, own slot
//   mode 4: ds_add_f64, 4 lanes per slot (same-address adds from different lanes)
//   mode 5: ds_add_f64, random slots (birthday conflicts, as in the gather)
// Timing only. build: hipcc --offload-arch=gfx950 -O3 -o lds_atomic_probe lds_atomic_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int SLOTS = 398;  // 3x3 blocks, as the gather's accumulator

template <int MODE>
__global__ __launch_bounds__(256) void k_probe(int iters, unsigned long long* out, double* sink) {
  __shared__ double acc[SLOTS * 9];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int t = tid; t < SLOTS * 9; t += blockDim.x) acc[t] = 0.0;
  __syncthreads();
  unsigned seed = 2654435761u * (unsigned)(tid + 17 * blockIdx.x + 1);
  int slot;
  if (MODE == 4) slot = (lane >> 2) + 16 * wave;
  else if (MODE == 5) slot = (int)((seed >> 7) % SLOTS);
  else slot = (lane + 64 * wave) % SLOTS;
  double v = 1.0 + 1e-3 * tid;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    double* p = acc + slot * 9;
#pragma unroll
    for (int e = 0; e < 9; ++e) {
      if (MODE == 0 || MODE == 4 || MODE == 5) {
        atomicAdd(p + e, v);
      } else if (MODE == 1) {
        p[e] += v;
      } else if (MODE == 2) {
        atomicAdd(reinterpret_cast<unsigned long long*>(p + e), (unsigned long long)(it + 1));
      } else {
        p[e] = v;
      }
    }
    if (MODE == 5) {
      seed = seed * 1664525u + 1013904223u;
      slot = (int)((seed >> 7) % SLOTS);
    }
    v += 1e-9;
  }
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[blockIdx.x] = t1 - t0;
  if (acc[tid] == 1.2345) sink[0] = acc[tid];
}

template <int MODE>
static double run(int threads, int iters, int blocks) {
  unsigned long long* d;
  double* s;
  (void)hipMalloc(&d, sizeof(unsigned long long) * blocks);
  (void)hipMalloc(&s, sizeof(double));
  k_probe<MODE><<<blocks, threads>>>(iters, d, s);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks);
  (void)hipMemcpy(h.data(), d, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
  double mean = 0;
  for (auto x : h) mean += (double)x;
  mean /= blocks;
  (void)hipFree(d);
  (void)hipFree(s);
  return mean / ((double)iters * 9 * (threads / 64));  // clocks per wave-instruction, CU-wide
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  const int blocks = 256;  // one workgroup per CU
  const char* names[] = {"ds_add_f64 own slot", "read+add+write f64", "ds_add_u64 own slot", "ds_write_b64",
                         "ds_add_f64 4 lanes/slot", "ds_add_f64 random slots"};
  for (int threads : {64, 256}) {
    double c[6];
    c[0] = run<0>(threads, iters, blocks);
    c[1] = run<1>(threads, iters, blocks);
    c[2] = run<2>(threads, iters, blocks);
    c[3] = run<3>(threads, iters, blocks);
    c[4] = run<4>(threads, iters, blocks);
    c[5] = run<5>(threads, iters, blocks);
    for (int m = 0; m < 6; ++m)
      printf("waves/CU %d  %-26s %7.2f clocks per wave-instruction\n", threads / 64, names[m], c[m]);
  }
  return 0;
}
