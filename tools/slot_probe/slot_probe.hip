// slot_probe.hip — how fast can a wave fetch its checks' slot lines? Each wave owns 64 "checks";
// each check reads one random 64-B line of table U (8 GiB, the user slots) and one of table D
// (2 GiB, the resource slots). Patterns (FETCH):
//   0  cooperative: 4 lanes x 16 B per 64-B line, 16 lines per instruction (k_closure_join today)
//   1  cooperative, D read as a 32-B half (2 lanes)
//   2  cooperative, both as 32-B halves
//   3  per lane: 4 x 16 B of its own U line, then 4 x 16 B of its own D line
//   4  pattern 0 with nontemporal loads
//   5  cooperative 4 lanes x 16 B, U and D lines of the same check in one instruction's halves
// Timed with the kernel's own events over 40 launches, at 1024 waves (one batch) and 3072 waves.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define OK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33; return x;
}
template <int P>
__global__ void __launch_bounds__(256) k_fetch(const unsigned char* __restrict__ U, unsigned long long nu,
                                               const unsigned char* __restrict__ D, unsigned long long nd,
                                               unsigned seed, unsigned* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) unsigned s[4][64 * 32];
  __shared__ unsigned long long s_u[4][64], s_d[4][64];
  const int wib = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const unsigned i = blockIdx.x * 256 + threadIdx.x;
  const unsigned long long h = mix(i * 0x9E3779B97F4A7C15ull + seed);
  const unsigned long long ua = (unsigned long long)(uintptr_t)(U + (h % nu) * 64);
  const unsigned long long da = (unsigned long long)(uintptr_t)(D + ((h >> 20) % nd) * 64);
  s_u[wib][lane] = ua;
  s_d[wib][lane] = da;
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  unsigned acc = 0;
  if constexpr (P == 0 || P == 4) {
    u32x4 y[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const unsigned k = 16u * r + (lane >> 2), chk = k / 2, part = k & 1;
      const unsigned long long b = part ? s_d[wib][chk] : s_u[wib][chk];
      const u32x4* p = (const u32x4*)(b + (lane & 3) * 16);
      if constexpr (P == 4) y[r] = __builtin_nontemporal_load(p); else y[r] = *p;
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const unsigned k = 16u * r + (lane >> 2), chk = k / 2, part = k & 1;
      *(u32x4*)&s[wib][chk * 32 + part * 16 + (lane & 3) * 4] = y[r];
    }
  } else if constexpr (P == 1) {  // 6 chunks per check: 4 of U, 2 of D
    u32x4 y[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const unsigned c = 64u * r + lane, chk = c / 6, sub = c % 6;
      const unsigned long long b = sub < 4 ? s_u[wib][chk] + sub * 16 : s_d[wib][chk] + (sub - 4) * 16;
      y[r] = *(const u32x4*)b;
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const unsigned c = 64u * r + lane, chk = c / 6, sub = c % 6;
      *(u32x4*)&s[wib][chk * 32 + sub * 4] = y[r];
    }
  } else if constexpr (P == 2) {
    u32x4 y[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const unsigned c = 64u * r + lane, chk = c / 4, sub = c % 4;
      const unsigned long long b = sub < 2 ? s_u[wib][chk] + sub * 16 : s_d[wib][chk] + (sub - 2) * 16;
      y[r] = *(const u32x4*)b;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const unsigned c = 64u * r + lane, chk = c / 4, sub = c % 4;
      *(u32x4*)&s[wib][chk * 32 + sub * 4] = y[r];
    }
  } else if constexpr (P == 3) {
    u32x4 y[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) y[r] = *(const u32x4*)(ua + r * 16);
#pragma unroll
    for (int r = 0; r < 4; ++r) y[4 + r] = *(const u32x4*)(da + r * 16);
#pragma unroll
    for (int r = 0; r < 8; ++r) acc ^= y[r].x + y[r].y * 3 + y[r].z * 5 + y[r].w * 7;
  } else if constexpr (P == 5) {  // instruction r: checks 8r..8r+7, lanes 0-31 U lines, 32-63 D lines
    u32x4 y[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const unsigned chk = 8u * r + ((lane & 31) >> 2);
      const unsigned long long b = lane < 32 ? s_u[wib][chk] : s_d[wib][chk];
      y[r] = *(const u32x4*)(b + (lane & 3) * 16);
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const unsigned chk = 8u * r + ((lane & 31) >> 2);
      *(u32x4*)&s[wib][chk * 32 + (lane < 32 ? 0 : 16) + (lane & 3) * 4] = y[r];
    }
  }
  if constexpr (P != 3) {
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 32; q += 4) {
      const u32x4 v = *(const u32x4*)&s[wib][lane * 32 + q];
      acc ^= v.x + v.y * 3 + v.z * 5 + v.w * 7;
    }
  }
  out[i] = acc;
}
int main(int argc, char** argv) {
  // args: contiguous (0/1), U GiB, D GiB, extra GiB allocated and touched but never read
  const bool contig = argc > 1 && atoi(argv[1]);
  const size_t ub = (size_t)(argc > 2 ? atoi(argv[2]) : 8) << 30, db = (size_t)(argc > 3 ? atoi(argv[3]) : 2) << 30;
  const size_t xb = (size_t)(argc > 4 ? atoi(argv[4]) : 0) << 30;
  unsigned char* X = nullptr;
  if (xb) {
    OK(hipMalloc(&X, xb));
    OK(hipMemset(X, 1, xb));
  }
  unsigned char *U, *D;
  if (contig) {
    OK(hipExtMallocWithFlags((void**)&U, ub, hipDeviceMallocContiguous));
    OK(hipExtMallocWithFlags((void**)&D, db, hipDeviceMallocContiguous));
  } else {
    OK(hipMalloc(&U, ub));
    OK(hipMalloc(&D, db));
  }
  unsigned* out;
  OK(hipMalloc(&out, 3072 * 64 * 4));
  OK(hipMemset(U, 0x3C, ub));
  OK(hipMemset(D, 0x5A, db));
  OK(hipDeviceSynchronize());
  hipStream_t st;
  OK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  OK(hipEventCreate(&e0));
  OK(hipEventCreate(&e1));
  auto run = [&](auto kern, int p) -> int {
    for (int waves : {1024, 3072}) {
      const dim3 g(waves / 4), b(256);
      for (int w = 0; w < 5; ++w) hipLaunchKernelGGL(kern, g, b, 0, st, U, ub / 64, D, db / 64, 77u + w, out);
      OK(hipStreamSynchronize(st));
      double tot = 0, mn = 1e9;
      const int K = 40;
      for (int k = 0; k < K; ++k) {
        hipExtLaunchKernelGGL(kern, g, b, 0, st, e0, e1, 0, (const unsigned char*)U, (unsigned long long)(ub / 64),
                              (const unsigned char*)D, (unsigned long long)(db / 64), 1000u + 7919u * k, out);
        OK(hipStreamSynchronize(st));
        float ms;
        OK(hipEventElapsedTime(&ms, e0, e1));
        tot += ms;
        mn = ms < mn ? ms : mn;
      }
      const double us = tot * 1e3 / K, lines = waves * 128.0;
      printf("{\"pattern\": %d, \"contig\": %d, \"U_GiB\": %zu, \"extra_GiB\": %zu, \"waves\": %d, \"us\": %.2f, \"min_us\": %.2f, \"Glines_s\": %.2f}\n", p, contig,
             ub >> 30, xb >> 30, waves, us, mn * 1e3, lines / us * 1e-3);
    }
    return 0;
  };
  const int only = argc > 5 ? atoi(argv[5]) : -1;  // one pattern (0 or 4), or all
  if (only == 0) return run(k_fetch<0>, 0);
  if (only == 4) return run(k_fetch<4>, 4);
  if (run(k_fetch<0>, 0) || run(k_fetch<1>, 1) || run(k_fetch<2>, 2) || run(k_fetch<3>, 3) || run(k_fetch<4>, 4) ||
      run(k_fetch<5>, 5))
    return 1;
  return 0;
}
