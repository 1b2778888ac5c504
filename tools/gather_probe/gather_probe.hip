// gather_probe.hip — calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the access widths of the
// check kernels (MI355X_MICROARCH.md §HBM: "Other access widths are uncalibrated: calibrate on a
// known byte count in your own access pattern"). Each kernel reads N random, aligned chunks of one
// width from a table far larger than the 256 MiB Infinity Cache (so nearly every chunk is a distinct
// HBM line) and writes one u32 per lane. Known bytes: N x width read, N x 4 written.
//   build: hipcc -O3 --offload-arch=gfx950 -o gather_probe gather_probe.hip
//   run:   rocprofv3 --pmc FETCH_SIZE -- ./gather_probe   (then WRITE_SIZE in a separate pass)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

template <int W>  // bytes per chunk: 4, 16, 32, 64
__global__ void __launch_bounds__(256) k_gather(const unsigned char* __restrict__ tab, unsigned long long n_chunks,
                                                unsigned seed, unsigned* __restrict__ out) {
  const unsigned i = blockIdx.x * 256 + threadIdx.x;
  const unsigned long long c = mix((unsigned long long)i * 0x9E3779B97F4A7C15ull + seed) % n_chunks;
  const unsigned char* p = tab + c * W;
  unsigned acc = 0;
  if constexpr (W == 4) {
    acc = *reinterpret_cast<const unsigned*>(p);
  } else {
    const u64x2* q = reinterpret_cast<const u64x2*>(p);
#pragma unroll
    for (int k = 0; k < W / 16; ++k) {
      const u64x2 v = q[k];
      acc ^= (unsigned)v.x ^ (unsigned)(v.y >> 7);
    }
  }
  out[i] = acc;
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main() {
  const size_t tab_bytes = (size_t)4 << 30;  // 4 GiB: 16x the Infinity Cache
  const unsigned n = 1u << 24;               // lanes per kernel
  unsigned char* tab = nullptr;
  unsigned* out = nullptr;
  CK(hipMalloc(&tab, tab_bytes));
  CK(hipMalloc(&out, (size_t)n * 4));
  CK(hipMemset(tab, 0x5A, tab_bytes));
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](auto kern, int width) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(kern, dim3(n / 256), dim3(256), 0, 0, tab, tab_bytes / width, 1234u + rep, out);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("{\"width\": %d, \"lanes\": %u, \"read_bytes\": %llu, \"write_bytes\": %llu, \"ms\": %.4f, \"GBps\": %.1f}\n",
             width, n, (unsigned long long)n * width, (unsigned long long)n * 4, ms, (double)n * width / (ms * 1e6));
    }
    return 0;
  };
  if (run(k_gather<4>, 4) || run(k_gather<16>, 16) || run(k_gather<32>, 32) || run(k_gather<64>, 64)) return 1;
  CK(hipFree(tab));
  CK(hipFree(out));
  return 0;
}
