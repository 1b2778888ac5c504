// pcie_probe.hip — where a host batch's PCIe time goes on this box (BASELINE.md:40-41's step moves
// 20 B of items host -> device and 5 B of results device -> host per check).
//
// Prints the topology (the GPU's PCI address and NUMA node, the process's CPU / memory sets, the
// nodes' CPU lists), then for each placement of the pinned buffers (hipHostMalloc default, bound
// to the GPU's node, bound to another node; coherent / non-coherent / uncached) and each placement
// of the calling thread (GPU-local CPUs, remote CPUs) one JSON line:
//   h2d_dma / d2h_dma      hipMemcpyAsync of one 64K batch's items / results, 64 back to back
//   zc_read / zc_write     a kernel reading the items from / writing the results into host memory
//   zc_join                both in one kernel (what the zero-copy join does), 64 back to back
//   zc_one_us              one zc_join alone, launch to event (latency of a lone batch)
//   build: hipcc -O3 --offload-arch=gfx950 -o pcie_probe pcie_probe.hip
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <chrono>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int kN = 65536;             // checks per batch
constexpr size_t kItems = 20ull * kN;  // 1,310,720 B
constexpr int kReps = 64;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// items in: each wave reads its 32 checks' 640 B as 40 lanes x 16 B (the join's item load)
__global__ void __launch_bounds__(256) k_zc_read(const uint4* __restrict__ items, unsigned* __restrict__ sink) {
  const unsigned wave = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  unsigned acc = 0;
  if (lane < 40) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(items) + (size_t)wave * 40 + lane);
    acc = v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

// results out: 1 B + 4 B per check (lanes 0..31 of a wave)
__global__ void __launch_bounds__(256) k_zc_write(unsigned char* __restrict__ perm, int* __restrict__ err) {
  const unsigned wave = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  if (lane < 32) {
    const unsigned i = wave * 32 + lane;
    perm[i] = (unsigned char)(1 + (i & 1));
    err[i] = 0;
  }
}

__global__ void __launch_bounds__(256) k_zc_join(const uint4* __restrict__ items, unsigned char* __restrict__ perm,
                                                 int* __restrict__ err) {
  const unsigned wave = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  __shared__ unsigned s[4][40];
  unsigned acc = 0;
  if (lane < 40) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(items) + (size_t)wave * 40 + lane);
    acc = v.x ^ v.y ^ v.z ^ v.w;
    s[threadIdx.x >> 6][lane] = acc;
  }
  __syncthreads();
  if (lane < 32) {
    const unsigned i = wave * 32 + lane;
    perm[i] = (unsigned char)(1 + (s[threadIdx.x >> 6][lane] & 1));
    err[i] = 0;
  }
}

static std::string slurp(const std::string& p) {
  std::ifstream f(p);
  std::stringstream ss;
  ss << f.rdbuf();
  std::string s = ss.str();
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ')) s.pop_back();
  return s;
}

static std::vector<int> parse_list(const std::string& s) {  // "0-3,8,10-11"
  std::vector<int> v;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    if (tok.empty()) continue;
    const size_t d = tok.find('-');
    const int a = atoi(tok.c_str()), b = d == std::string::npos ? a : atoi(tok.c_str() + d + 1);
    for (int x = a; x <= b; ++x) v.push_back(x);
  }
  return v;
}

static bool pin_thread(const std::vector<int>& cpus, const cpu_set_t& allowed) {
  cpu_set_t s;
  CPU_ZERO(&s);
  int n = 0;
  for (int c : cpus)
    if (CPU_ISSET(c, &allowed)) {
      CPU_SET(c, &s);
      ++n;
    }
  return n > 0 && sched_setaffinity(0, sizeof(s), &s) == 0;
}

// MPOL_BIND (2) to one node, or MPOL_DEFAULT (0)
static bool bind_mem(int node) {
  unsigned long mask[16] = {};
  if (node < 0) return syscall(SYS_set_mempolicy, 0, nullptr, 0) == 0;
  mask[node / 64] |= 1ul << (node % 64);
  return syscall(SYS_set_mempolicy, 2, mask, 1024) == 0;
}

static int page_node(void* p) {  // move_pages with no target: the node holding the page
  void* pages[1] = {p};
  int status[1] = {-1};
  if (syscall(SYS_move_pages, 0, 1, pages, nullptr, status, 0) != 0) return -2;
  return status[0];
}

struct Timer {
  hipEvent_t a, b;
  Timer() {
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
  }
};

int main() {
  CK(hipSetDevice(0));
  char bdf[64] = {};
  CK(hipDeviceGetPCIBusId(bdf, sizeof(bdf), 0));
  for (char* c = bdf; *c; ++c) *c = (char)tolower(*c);
  const std::string dev = std::string("/sys/bus/pci/devices/") + bdf;
  const int gpu_node = atoi(slurp(dev + "/numa_node").c_str());
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  sched_getaffinity(0, sizeof(allowed), &allowed);
  std::vector<std::vector<int>> node_cpus;
  std::string nodes_json = "[";
  for (int n = 0; n < 64; ++n) {
    const std::string cl = slurp("/sys/devices/system/node/node" + std::to_string(n) + "/cpulist");
    if (cl.empty()) break;
    node_cpus.push_back(parse_list(cl));
    int n_allowed = 0;
    for (int c : node_cpus.back()) n_allowed += CPU_ISSET(c, &allowed) ? 1 : 0;
    nodes_json += (n ? "," : "") + std::string("{\"node\":") + std::to_string(n) + ",\"cpus\":\"" + cl +
                  "\",\"allowed\":" + std::to_string(n_allowed) + "}";
  }
  nodes_json += "]";
  const std::string status = slurp("/proc/self/status");
  auto field = [&](const char* k) {
    const size_t p = status.find(k);
    if (p == std::string::npos) return std::string();
    const size_t e = status.find('\n', p);
    std::string v = status.substr(p + strlen(k), e - p - strlen(k));
    while (!v.empty() && (v[0] == ' ' || v[0] == '\t' || v[0] == ':')) v.erase(0, 1);
    return v;
  };
  printf("{\"topology\":{\"bdf\":\"%s\",\"gpu_numa_node\":%d,\"link_speed\":\"%s\",\"link_width\":\"%s\","
         "\"cpus_allowed\":\"%s\",\"mems_allowed\":\"%s\",\"cpu_max\":\"%s\",\"nodes\":%s}}\n",
         bdf, gpu_node, slurp(dev + "/current_link_speed").c_str(), slurp(dev + "/current_link_width").c_str(),
         field("Cpus_allowed_list").c_str(), field("Mems_allowed_list").c_str(),
         slurp("/sys/fs/cgroup/cpu.max").c_str(), nodes_json.c_str());
  fflush(stdout);

  const int n_nodes = (int)node_cpus.size();
  const int local = gpu_node >= 0 && gpu_node < n_nodes ? gpu_node : 0;
  int remote = -1;
  for (int n = 0; n < n_nodes; ++n)
    if (n != local) {
      int k = 0;
      for (int c : node_cpus[n]) k += CPU_ISSET(c, &allowed) ? 1 : 0;
      if (k > 0) {
        remote = n;
        break;
      }
    }

  unsigned char* d_items = nullptr;
  unsigned char* d_res = nullptr;
  unsigned* d_sink = nullptr;
  CK(hipMalloc(&d_items, kItems));
  CK(hipMalloc(&d_res, 5 * kN));
  CK(hipMalloc(&d_sink, 64));
  hipStream_t st, st2;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
  Timer t;
  const int blocks = kN / 32 / 4;  // a wave per 32 checks, 4 waves per block

  struct Kind {
    const char* name;
    unsigned flags;
  } kinds[] = {{"default", hipHostMallocDefault},
               {"coherent", hipHostMallocCoherent},
               {"noncoherent", hipHostMallocNonCoherent},
               {"uncached", hipHostMallocUncached}};
  // placements: (thread node, memory node or -1 = runtime default)
  std::vector<std::pair<int, int>> places = {{local, -1}, {local, local}};
  if (remote >= 0) {
    places.push_back({remote, -1});
    places.push_back({local, remote});
    places.push_back({remote, remote});
  }
  for (auto [tn, mn] : places) {
    const bool pinned_ok = pin_thread(node_cpus[tn], allowed);
    for (const Kind& kd : kinds) {
      if (mn >= 0 && !bind_mem(mn)) {
        printf("{\"error\":\"set_mempolicy node %d refused\"}\n", mn);
        continue;
      }
      const unsigned fl = kd.flags | (mn >= 0 ? hipHostMallocNumaUser : 0u);
      void *h_items = nullptr, *h_res = nullptr;
      if (hipHostMalloc(&h_items, kItems, fl) != hipSuccess || hipHostMalloc(&h_res, 5 * kN, fl) != hipSuccess) {
        printf("{\"kind\":\"%s\",\"mem_node\":%d,\"error\":\"hipHostMalloc\"}\n", kd.name, mn);
        (void)hipGetLastError();
        bind_mem(-1);
        continue;
      }
      bind_mem(-1);
      memset(h_items, 1, kItems);
      memset(h_res, 0, 5 * kN);
      const int where = page_node(h_items);
      auto time_loop = [&](auto&& body, hipStream_t s) {
        for (int w = 0; w < 4; ++w) body();
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(t.a, s));
        for (int r = 0; r < kReps; ++r) body();
        CK(hipEventRecord(t.b, s));
        CK(hipEventSynchronize(t.b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, t.a, t.b));
        return ms * 1e3 / kReps;  // us per batch
      };
      const float h2d = time_loop([&] { CK(hipMemcpyAsync(d_items, h_items, kItems, hipMemcpyHostToDevice, st)); }, st);
      const float d2h = time_loop([&] { CK(hipMemcpyAsync(h_res, d_res, 5 * kN, hipMemcpyDeviceToHost, st)); }, st);
      const float zr = time_loop([&] {
        hipLaunchKernelGGL(k_zc_read, dim3(blocks), dim3(256), 0, st, (const uint4*)h_items, d_sink);
      }, st);
      const float zw = time_loop([&] {
        hipLaunchKernelGGL(k_zc_write, dim3(blocks), dim3(256), 0, st, (unsigned char*)h_res, (int*)((char*)h_res + kN));
      }, st);
      const float zj = time_loop([&] {
        hipLaunchKernelGGL(k_zc_join, dim3(blocks), dim3(256), 0, st, (const uint4*)h_items, (unsigned char*)h_res,
                           (int*)((char*)h_res + kN));
      }, st);
      // one batch alone: launch to completion seen by the host (median of 32)
      std::vector<double> one;
      for (int r = 0; r < 35; ++r) {
        const auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(k_zc_join, dim3(blocks), dim3(256), 0, st, (const uint4*)h_items, (unsigned char*)h_res,
                           (int*)((char*)h_res + kN));
        CK(hipStreamSynchronize(st));
        one.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
      }
      std::sort(one.begin() + 3, one.end());
      // DMA in and out concurrently (two streams), 64 pairs
      for (int w = 0; w < 4; ++w) {
        CK(hipMemcpyAsync(d_items, h_items, kItems, hipMemcpyHostToDevice, st));
        CK(hipMemcpyAsync(h_res, d_res, 5 * kN, hipMemcpyDeviceToHost, st2));
      }
      CK(hipDeviceSynchronize());
      const auto c0 = std::chrono::steady_clock::now();
      for (int r = 0; r < kReps; ++r) {
        CK(hipMemcpyAsync(d_items, h_items, kItems, hipMemcpyHostToDevice, st));
        CK(hipMemcpyAsync(h_res, d_res, 5 * kN, hipMemcpyDeviceToHost, st2));
      }
      CK(hipDeviceSynchronize());
      const double both = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c0).count() / kReps;
      auto gbs = [](double bytes, double us) { return bytes / (us * 1e3); };
      printf("{\"kind\":\"%s\",\"thread_node\":%d,\"thread_pinned\":%d,\"mem_policy_node\":%d,\"page_node\":%d,"
             "\"h2d_dma_us\":%.2f,\"h2d_dma_GBs\":%.1f,\"d2h_dma_us\":%.2f,\"d2h_dma_GBs\":%.1f,"
             "\"dma_both_us\":%.2f,\"zc_read_us\":%.2f,\"zc_read_GBs\":%.1f,\"zc_write_us\":%.2f,\"zc_write_GBs\":%.1f,"
             "\"zc_join_us\":%.2f,\"zc_join_checks_per_s\":%.3e,\"zc_one_us_median\":%.2f}\n",
             kd.name, tn, (int)pinned_ok, mn, where, h2d, gbs(kItems, h2d), d2h, gbs(5.0 * kN, d2h), both, zr,
             gbs(kItems, zr), zw, gbs(5.0 * kN, zw), zj, kN / (zj * 1e-6), one[3 + (one.size() - 3) / 2]);
      fflush(stdout);
      CK(hipHostFree(h_items));
      CK(hipHostFree(h_res));
    }
  }
  return 0;
}
