// FETCH_SIZE calibration for the gather's load shapes (gfx950). MI355X_MICROARCH.md: FETCH_SIZE
// reads 1/2 of the bytes of a wide coalesced streaming read; other widths are uncalibrated. Each
// kernel reads a 4 GiB buffer exactly once (far past the 256 MiB Infinity Cache) in one shape and
// prints the byte count; run under `rocprofv3 --pmc FETCH_SIZE` and divide.
//   wide16   : 16 B per lane, a wave's lanes contiguous (the chunk-store shape, read side)
//   slot10   : 5 x u16 per lane, lanes contiguous at 10 B (k_gather_lin's slot words)
//   rec80    : 5 x 16 B per lane, lanes contiguous at 80 B (the 80-B cell records)
//   u32      : 4 B per lane, contiguous (the entry order)
//   write16  : 16-B non-temporal stores per lane, contiguous (WRITE_SIZE; the chunk stores' shape)
// build: hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef double dv2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_wide16(const dv2* __restrict__ p, int64_t n, double* sink) {
  double s = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const dv2 v = p[i];
    s += v.x + v.y;
  }
  if (s == 1.2345) sink[0] = s;
}

__global__ __launch_bounds__(256) void k_slot10(const uint16_t* __restrict__ p, int64_t nlanes, double* sink) {
  uint32_t s = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nlanes; i += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int t = 0; t < 5; ++t) s += p[i * 5 + t];
  }
  if (s == 12345u) sink[0] = s;
}

__global__ __launch_bounds__(256) void k_rec80(const dv2* __restrict__ p, int64_t nlanes, double* sink) {
  double s = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nlanes; i += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      const dv2 v = p[i * 5 + t];
      s += v.x + v.y;
    }
  }
  if (s == 1.2345) sink[0] = s;
}

__global__ __launch_bounds__(256) void k_u32(const uint32_t* __restrict__ p, int64_t n, double* sink) {
  uint32_t s = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) s += p[i];
  if (s == 12345u) sink[0] = s;
}

__global__ __launch_bounds__(256) void k_write16(dv2* __restrict__ p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(dv2{1.0, 2.0}, p + i);
}

int main() {
  const int64_t bytes = 4ll << 30;
  void* buf = nullptr;
  double* sink = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) return 1;
  hipMemset(buf, 0, bytes);
  hipDeviceSynchronize();
  const int grid = 4096;
  for (int rep = 0; rep < 2; ++rep) {
    k_wide16<<<grid, 256>>>((const dv2*)buf, bytes / 16, sink);
    k_slot10<<<grid, 256>>>((const uint16_t*)buf, bytes / 10, sink);
    k_rec80<<<grid, 256>>>((const dv2*)buf, bytes / 80, sink);
    k_u32<<<grid, 256>>>((const uint32_t*)buf, bytes / 4, sink);
    k_write16<<<grid, 256>>>((dv2*)buf, bytes / 16);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("bytes read per kernel: wide16 %lld slot10 %lld rec80 %lld u32 %lld\n", (long long)bytes,
         (long long)(bytes / 10 * 10), (long long)(bytes / 80 * 80), (long long)bytes);
  hipFree(buf);
  hipFree(sink);
  return 0;
}
