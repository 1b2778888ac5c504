// submit_probe — the host cost of one batch through the C ABI from a compiled caller (what a Go
// caller pays through cgo, without Python): a small nested-group snapshot, batches of N device
// items, D batches in flight (gck_check_submit / gck_check_wait), host time inside each call.
//   build: g++ -O2 -std=c++17 -I include -I /opt/rocm/include -D__HIP_PLATFORM_AMD__ \
//            tools/submit_probe/submit_probe.cpp -o tools/submit_probe/submit_probe \
//            -L gochugaru_amd -lgck -L /opt/rocm/lib -lamdhip64 -Wl,-rpath,'$ORIGIN/../../gochugaru_amd'
//   run:   tools/submit_probe/submit_probe [n=64] [batches=4000]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "gck.h"

#define CK(x)                                                                                    \
  do {                                                                                           \
    int rc_ = (x);                                                                               \
    if (rc_ != GCK_OK) {                                                                         \
      std::fprintf(stderr, "%s: %d %s\n", #x, rc_, gck_last_error());                            \
      return 1;                                                                                  \
    }                                                                                            \
  } while (0)

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 64;
  const int nb = argc > 2 ? std::atoi(argv[2]) : 4000;
  const char* schema =
      "definition user {}\n"
      "definition group { relation member: user | group#member }\n"
      "definition doc { relation viewer: group#member\n permission view = viewer }\n";
  gck_config cfg{};
  cfg.workspaces = 4;
  gck_engine* e = nullptr;
  CK(gck_create(&cfg, &e));
  CK(gck_load_schema(e, schema, std::strlen(schema)));
  std::string t;
  for (int g = 0; g < 200; ++g) {
    for (int k = 0; k < 10; ++k) t += "group:g" + std::to_string(g) + "#member@user:u" + std::to_string((g * 37 + k * 11) % 2000) + "\n";
    if (g > 0) t += "group:g" + std::to_string((g - 1) / 2) + "#member@group:g" + std::to_string(g) + "#member\n";
  }
  for (int d = 0; d < 500; ++d) t += "doc:d" + std::to_string(d) + "#viewer@group:g" + std::to_string(d % 200) + "#member\n";
  CK(gck_begin_snapshot(e, 1));
  CK(gck_add_tuples_text(e, t.data(), t.size()));
  CK(gck_commit_snapshot(e));
  uint16_t t_user, t_doc, r_view;
  CK(gck_type_id(e, "user", 4, &t_user));
  CK(gck_type_id(e, "doc", 3, &t_doc));
  CK(gck_relation_id(e, t_doc, "view", 4, &r_view));
  std::vector<gck_item> items(n);
  for (size_t i = 0; i < n; ++i) {
    std::string d = "d" + std::to_string(i % 500), u = "u" + std::to_string((i * 7) % 2000);
    const char* dp = d.c_str();
    const char* up = u.c_str();
    uint32_t dl = d.size(), ul = u.size(), did, uid;
    CK(gck_intern(e, t_doc, &dp, &dl, 1, 0, &did));
    CK(gck_intern(e, t_user, &up, &ul, 1, 0, &uid));
    items[i] = gck_item{t_doc, r_view, did, t_user, GCK_ELLIPSIS, uid, 0};
  }
  gck_item* d_items;
  uint8_t* d_perm;
  int32_t* d_err;
  if (hipMalloc(&d_items, n * sizeof(gck_item)) || hipMalloc(&d_perm, n) || hipMalloc(&d_err, n * 4)) return 1;
  if (hipMemcpy(d_items, items.data(), n * sizeof(gck_item), hipMemcpyHostToDevice)) return 1;
  hipStream_t st[4];
  for (auto& s : st)
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) return 1;
  gck_consistency cs{GCK_CONSISTENCY_MIN_LATENCY, 0, 0};
  using clk = std::chrono::steady_clock;
  for (int depth : {1, 2, 3, 4}) {
    for (int pass = 0; pass < 2; ++pass) {  // a warm-up pass, then the measured one
      std::deque<gck_batch*> q;
      double ts = 0, tw = 0;
      const auto t0 = clk::now();
      for (int k = 0; k < nb; ++k) {
        if ((int)q.size() >= depth) {
          const auto a = clk::now();
          CK(gck_check_wait(e, q.front()));
          tw += std::chrono::duration<double>(clk::now() - a).count();
          q.pop_front();
        }
        gck_batch* b = nullptr;
        const auto a = clk::now();
        CK(gck_check_submit(e, &cs, d_items, n, nullptr, nullptr, 0, 0, d_perm, d_err, GCK_SUBMIT_DEVICE, st[k % depth], &b));
        ts += std::chrono::duration<double>(clk::now() - a).count();
        q.push_back(b);
      }
      while (!q.empty()) {
        CK(gck_check_wait(e, q.front()));
        q.pop_front();
      }
      const double dt = std::chrono::duration<double>(clk::now() - t0).count();
      if (pass == 1)
        std::printf("{\"n\": %zu, \"inflight\": %d, \"us_per_batch\": %.2f, \"submit_us\": %.2f, \"wait_us\": %.2f}\n", n, depth,
                    dt / nb * 1e6, ts / nb * 1e6, tw / nb * 1e6);
    }
  }
  std::vector<uint8_t> perm(n);
  if (hipMemcpy(perm.data(), d_perm, n, hipMemcpyDeviceToHost)) return 1;
  size_t has = 0;
  for (uint8_t p : perm) has += p == GCK_PERM_HAS;
  std::printf("{\"has\": %zu, \"of\": %zu}\n", has, n);
  gck_destroy(e);
  return 0;
}
