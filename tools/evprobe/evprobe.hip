// Compares HIP event timings of one kernel with the profiler's kernel duration:
// (a) hipExtLaunchKernelGGL start/stop events, (b) hipEventRecord markers around the launch,
// (c) one event pair around K back-to-back launches. Run bare and under rocprofv3 --kernel-trace --stats.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define OK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)
__global__ void k_gather(const unsigned* __restrict__ a, unsigned n, unsigned rounds, unsigned* out) {
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned x = i * 2654435761u, s = 0;
  for (unsigned r = 0; r < rounds; ++r) { x = a[(x ^ s) % n]; s += x; }
  out[i] = s;
}
int main(int argc, char** argv) {
  const unsigned n = 1u << 26, threads = 65536, rounds = argc > 1 ? atoi(argv[1]) : 6;
  unsigned *a, *out;
  OK(hipMalloc(&a, (size_t)n * 4));
  OK(hipMalloc(&out, threads * 4));
  std::vector<unsigned> h(n);
  for (unsigned i = 0; i < n; ++i) h[i] = i * 2246822519u + 374761393u;
  OK(hipMemcpy(a, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
  hipStream_t st; OK(hipStreamCreate(&st));
  hipEvent_t e0, e1; OK(hipEventCreate(&e0)); OK(hipEventCreate(&e1));
  const dim3 g(threads / 256), b(256);
  for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(k_gather, g, b, 0, st, a, n, rounds, out);
  OK(hipStreamSynchronize(st));
  const int K = 100;
  double ext = 0, mark = 0; float ms;
  for (int k = 0; k < K; ++k) {
    hipExtLaunchKernelGGL(k_gather, g, b, 0, st, e0, e1, 0, (const unsigned*)a, n, rounds, out);
    OK(hipStreamSynchronize(st)); OK(hipEventElapsedTime(&ms, e0, e1)); ext += ms;
  }
  for (int k = 0; k < K; ++k) {
    OK(hipEventRecord(e0, st)); hipLaunchKernelGGL(k_gather, g, b, 0, st, a, n, rounds, out); OK(hipEventRecord(e1, st));
    OK(hipStreamSynchronize(st)); OK(hipEventElapsedTime(&ms, e0, e1)); mark += ms;
  }
  OK(hipEventRecord(e0, st));
  for (int k = 0; k < K; ++k) hipLaunchKernelGGL(k_gather, g, b, 0, st, a, n, rounds, out);
  OK(hipEventRecord(e1, st)); OK(hipStreamSynchronize(st)); OK(hipEventElapsedTime(&ms, e0, e1));
  printf("{\"rounds\": %u, \"ext_us\": %.2f, \"marker_us\": %.2f, \"burst_us\": %.2f}\n", rounds, ext * 1e3 / K, mark * 1e3 / K, ms * 1e3 / K);
  return 0;
}
