// LDS accumulate / drain op cost probe (gfx950), inline asm so nothing is folded away:
// CU-wide shader clocks per wave-instruction for the ops the row gather's accumulator uses, with
// all lanes active or only a part of them (does a masked lane still cost its LDS cycles?).
// Slots are conflict-free (lane l -> 72-B block l of its wave's range) unless noted.
// One workgroup per CU of `threads` threads (4 or 16 waves). Timing only.
// build: hipcc --offload-arch=gfx950 -O3 -o lds_op_probe lds_op_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int SLOTS = 448;  // 3x3 FP64 blocks (32 KB accumulator)

enum {
  ADD_F64,        // ds_add_f64
  ADD_U64,        // ds_add_u64
  ADD_F64_HALF,   // ds_add_f64, even lanes only
  ADD_F64_Q,      // ds_add_f64, lanes 0-15 of each 32 only (two of four 16-lane groups)
  ADD_F64_RAND,   // ds_add_f64, random slots (the unordered gather's conflicts)
  ADD_U64_RAND,   // ds_add_u64, random slots
  XCHG_B64,       // ds_wrxchg_rtn_b64 (read + zero in one op)
  WRITE_B64,      // ds_write_b64
  WRITE_B128,     // ds_write_b128 (drain zeroing)
  READ_B128,      // ds_read_b128 (drain read)
  READ_B64,       // ds_read_b64 (table read)
  NMODES
};
static const char* kNames[] = {"ds_add_f64", "ds_add_u64", "ds_add_f64 half lanes", "ds_add_f64 2 of 4 groups",
                               "ds_add_f64 random slots", "ds_add_u64 random slots", "ds_wrxchg_rtn_b64",
                               "ds_write_b64", "ds_write_b128", "ds_read_b128", "ds_read_b64"};

template <int MODE>
__global__ __launch_bounds__(1024) void k_probe(int iters, unsigned long long* out, double* sink) {
  __shared__ __attribute__((aligned(16))) double acc[SLOTS * 9];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int t = tid; t < SLOTS * 9; t += blockDim.x) acc[t] = 0.0;
  __syncthreads();
  unsigned seed = 2654435761u * (unsigned)(tid + 17 * blockIdx.x + 1);
  int slot = (lane + 64 * wave) % SLOTS;
  if (MODE == ADD_F64_RAND || MODE == ADD_U64_RAND) slot = (int)((seed >> 7) % SLOTS);
  bool active = true;
  if (MODE == ADD_F64_HALF) active = (lane & 1) == 0;
  if (MODE == ADD_F64_Q) active = (lane & 16) == 0;
  const uint32_t base = (uint32_t)(uintptr_t)acc;
  double v = 1.0 + 1e-3 * tid;
  double sink_v = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    uint32_t a = base + (uint32_t)slot * 72u;
    if (MODE == WRITE_B128 || MODE == READ_B128) a = base + (uint32_t)(((tid * 16 + it * 4096) % (SLOTS * 72 - 16 - 8192)) & ~15);
    if (active) {
      if constexpr (MODE == ADD_F64 || MODE == ADD_F64_HALF || MODE == ADD_F64_Q || MODE == ADD_F64_RAND) {
        asm volatile(
            "ds_add_f64 %0, %1\n ds_add_f64 %0, %1 offset:8\n ds_add_f64 %0, %1 offset:16\n"
            "ds_add_f64 %0, %1 offset:24\n ds_add_f64 %0, %1 offset:32\n ds_add_f64 %0, %1 offset:40\n"
            "ds_add_f64 %0, %1 offset:48\n ds_add_f64 %0, %1 offset:56\n ds_add_f64 %0, %1 offset:64\n" ::"v"(a),
            "v"(v)
            : "memory");
      } else if constexpr (MODE == ADD_U64 || MODE == ADD_U64_RAND) {
        const uint64_t u = (uint64_t)it + 1;
        asm volatile(
            "ds_add_u64 %0, %1\n ds_add_u64 %0, %1 offset:8\n ds_add_u64 %0, %1 offset:16\n"
            "ds_add_u64 %0, %1 offset:24\n ds_add_u64 %0, %1 offset:32\n ds_add_u64 %0, %1 offset:40\n"
            "ds_add_u64 %0, %1 offset:48\n ds_add_u64 %0, %1 offset:56\n ds_add_u64 %0, %1 offset:64\n" ::"v"(a),
            "v"(u)
            : "memory");
      } else if constexpr (MODE == XCHG_B64) {
        double r0, r1, r2;
        asm volatile(
            "ds_wrxchg_rtn_b64 %0, %3, %4\n ds_wrxchg_rtn_b64 %1, %3, %4 offset:8\n ds_wrxchg_rtn_b64 %2, %3, %4 offset:16\n"
            "s_waitcnt lgkmcnt(0)\n"
            : "=&v"(r0), "=&v"(r1), "=&v"(r2)
            : "v"(a), "v"(v)
            : "memory");
        sink_v += r0 + r1 + r2;
      } else if constexpr (MODE == WRITE_B64) {
        asm volatile(
            "ds_write_b64 %0, %1\n ds_write_b64 %0, %1 offset:8\n ds_write_b64 %0, %1 offset:16\n"
            "ds_write_b64 %0, %1 offset:24\n ds_write_b64 %0, %1 offset:32\n ds_write_b64 %0, %1 offset:40\n"
            "ds_write_b64 %0, %1 offset:48\n ds_write_b64 %0, %1 offset:56\n ds_write_b64 %0, %1 offset:64\n" ::"v"(a),
            "v"(v)
            : "memory");
      } else if constexpr (MODE == WRITE_B128) {
        typedef double dv2 __attribute__((ext_vector_type(2)));
        const dv2 z = {v, v};
        asm volatile(
            "ds_write_b128 %0, %1\n ds_write_b128 %0, %1 offset:1024\n ds_write_b128 %0, %1 offset:2048\n"
            "ds_write_b128 %0, %1 offset:3072\n ds_write_b128 %0, %1 offset:4096\n ds_write_b128 %0, %1 offset:5120\n"
            "ds_write_b128 %0, %1 offset:6144\n ds_write_b128 %0, %1 offset:7168\n ds_write_b128 %0, %1 offset:8192\n" ::"v"(a),
            "v"(z)
            : "memory");
      } else if constexpr (MODE == READ_B128) {
        typedef double dv2 __attribute__((ext_vector_type(2)));
        dv2 r0, r1, r2;
        asm volatile(
            "ds_read_b128 %0, %3\n ds_read_b128 %1, %3 offset:1024\n ds_read_b128 %2, %3 offset:2048\n"
            "s_waitcnt lgkmcnt(0)\n"
            : "=&v"(r0), "=&v"(r1), "=&v"(r2)
            : "v"(a)
            : "memory");
        sink_v += r0.x + r1.y + r2.x;
      } else if constexpr (MODE == READ_B64) {
        double r0, r1, r2;
        asm volatile(
            "ds_read_b64 %0, %3\n ds_read_b64 %1, %3 offset:8\n ds_read_b64 %2, %3 offset:16\n"
            "s_waitcnt lgkmcnt(0)\n"
            : "=&v"(r0), "=&v"(r1), "=&v"(r2)
            : "v"(a)
            : "memory");
        sink_v += r0 + r1 + r2;
      }
    }
    if (MODE == ADD_F64_RAND || MODE == ADD_U64_RAND) {
      seed = seed * 1664525u + 1013904223u;
      slot = (int)((seed >> 7) % SLOTS);
    }
    v += 1e-9;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[blockIdx.x] = t1 - t0;
  if (acc[tid] == 1.2345 || sink_v == 1.2345) sink[0] = acc[tid] + sink_v;
}

template <int MODE>
static double run(int threads, int iters, int blocks, unsigned long long* d, double* s) {
  k_probe<MODE><<<blocks, threads>>>(iters, d, s);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks);
  (void)hipMemcpy(h.data(), d, sizeof(unsigned long long) * blocks, hipMemcpyDeviceToHost);
  double mean = 0;
  for (auto x : h) mean += (double)x;
  mean /= blocks;
  const int per_it = (MODE == XCHG_B64 || MODE == READ_B128 || MODE == READ_B64) ? 3 : 9;
  return mean / ((double)iters * per_it * (threads / 64));  // clocks per wave-instruction, CU-wide
}

template <int M>
static void run_all(int threads, int iters, int blocks, unsigned long long* d, double* s) {
  if constexpr (M < NMODES) {
    const double c = run<M>(threads, iters, blocks, d, s);
    printf("waves/CU %2d  %-28s %7.2f clocks per wave-instruction\n", threads / 64, kNames[M], c);
    run_all<M + 1>(threads, iters, blocks, d, s);
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  int dev = 0, cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  unsigned long long* d;
  double* s;
  (void)hipMalloc(&d, sizeof(unsigned long long) * cus);
  (void)hipMalloc(&s, sizeof(double));
  for (int threads : {256, 1024}) run_all<0>(threads, iters, cus, d, s);
  return 0;
}
