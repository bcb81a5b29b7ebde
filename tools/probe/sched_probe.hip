// Probe of k_gather_lin's chunk schedule on the hardware (round 6): a persistent grid pulls chunk ids
// from 8 per-XCD counters exactly as the gather does (lane 0: one atomicAdd of AHEAD ids in the
// prologue, one atomicInc per iteration, ids mapped AHEAD iterations early through an LDS ring, the
// loop ends at the first empty id), and "gathers" a chunk by counting it. Mode 0: each XCD walks its
// own eighth only (the shipped schedule); mode 1: past its eighth a workgroup takes chunks of the
// other XCDs' eighths (tail stealing, the variant under test). Every launch gets fresh stream-ordered
// counters (hipMallocAsync + hipMemsetAsync, freed after the launch, like lin_chunk_desc's scratch).
// Prints, per mode and chunk count, the launches with a chunk never counted or counted twice.
// Build: hipcc --offload-arch=gfx950 -O3 -o sched_probe sched_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int AHEAD = 5, RING = 8;

template <int MODE>
__global__ __launch_bounds__(256) void k_sched(unsigned* __restrict__ ctr, unsigned* __restrict__ hits, unsigned nchunks,
                                               unsigned per, unsigned spin) {
  __shared__ int s_id[RING];
  const int tid = threadIdx.x;
  const int xc = (int)(blockIdx.x % 8);
  unsigned* const lctr = ctr + 32 * xc;
  auto len_of = [&](int x) -> unsigned {
    const unsigned b = (unsigned)x * per;
    return b >= nchunks ? 0u : min(per, nchunks - b);
  };
  auto chunk_of = [&](unsigned j) -> int {
    if (MODE == 0) return (int)(j < per ? min((unsigned)xc * per + j, nchunks) : nchunks);
    if (j < len_of(xc)) return (int)((unsigned)xc * per + j);
    for (int s = 1; s < 8; ++s) {
      const int v = (xc + s) & 7;
      const unsigned lv = len_of(v);
      unsigned* const vc = ctr + 32 * v;
      if (__hip_atomic_load(vc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= lv) continue;
      const unsigned r = atomicInc(vc, 0xFFFFFFFFu);
      if (r < lv) return (int)((unsigned)v * per + r);
    }
    return (int)nchunks;
  };
  if (tid == 0) {
    const unsigned b = atomicAdd(lctr, (unsigned)AHEAD);
    for (int t = 0; t < AHEAD; ++t) s_id[t] = chunk_of(b + t);
  }
  __syncthreads();
  for (int k = 0;; ++k) {
    const int c = __builtin_amdgcn_readfirstlane(s_id[k % RING]);
    if (c >= (int)nchunks) break;
    unsigned rn = 0u;
    if (tid == 0) rn = atomicInc(lctr, 0xFFFFFFFFu);
    // the chunk's work: a hash-dependent spin so workgroups drift apart
    const unsigned w = ((unsigned)c * 2654435761u >> 24) % (spin + 1);
    for (unsigned i = 0; i < w; ++i) __builtin_amdgcn_s_sleep(1);
    if (tid == 0) atomicAdd(hits + c, 1u);
    __syncthreads();
    if (tid == 0) s_id[(k + AHEAD) % RING] = chunk_of(rn);
    __syncthreads();
  }
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? atoi(argv[1]) : 200;
  const unsigned counts[] = {1, 2, 3, 5, 7, 8, 9, 15, 17, 63, 100, 1001, 4097, 65537, 1000003};
  hipStream_t s;
  CK(hipStreamCreate(&s));
  unsigned* hits = nullptr;
  CK(hipMalloc(&hits, sizeof(unsigned) * 1000003));
  std::vector<unsigned> h(1000003);
  int dev = 0, cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  for (int mode = 0; mode < 2; ++mode) {
    for (unsigned n : counts) {
      const unsigned per = (n + 7) / 8;
      const unsigned grid = (unsigned)std::min<long long>(8ll * per, (long long)cus * 4);
      int lost = 0, dup = 0;
      for (int t = 0; t < trials; ++t) {
        unsigned* ctr = nullptr;
        // a scratch block like lin_chunk_desc's: chunk arrays, then the counters
        CK(hipMallocAsync((void**)&ctr, 1024 + 64 * (t % 7), s));
        unsigned* c0 = ctr + 16 * (t % 7);
        CK(hipMemsetAsync(c0, 0, 1024, s));
        CK(hipMemsetAsync(hits, 0, sizeof(unsigned) * n, s));
        if (mode == 0) k_sched<0><<<grid, 256, 0, s>>>(c0, hits, n, per, t % 4);
        else k_sched<1><<<grid, 256, 0, s>>>(c0, hits, n, per, t % 4);
        CK(hipGetLastError());
        CK(hipFreeAsync(ctr, s));
        CK(hipMemcpyAsync(h.data(), hits, sizeof(unsigned) * n, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        bool l = false, d = false;
        for (unsigned i = 0; i < n; ++i) {
          l |= h[i] == 0;
          d |= h[i] > 1;
        }
        lost += l;
        dup += d;
      }
      printf("mode %d nchunks %8u grid %5u: launches with a lost chunk %d, with a duplicate %d (of %d)\n", mode, n, grid,
             lost, dup, trials);
      fflush(stdout);
    }
  }
  return 0;
}
