// driver.cpp — a compiled caller of the C ABI's asynchronous batches: the loop a cgo host runs
// (submit, keep `depth` batches in flight, wait for the oldest), so that bench.py can time the
// engine through C calls instead of one ctypes round trip per call (~3-4 us each in CPython,
// ~0.1 us through cgo). It calls only gck_check_submit / gck_check_wait, through the pointers the
// caller passes (the entry points of the libgck instance that created the engine), so it never
// links a second copy of the library.
//   built by make -C gochugaru_amd/csrc as gochugaru_amd/libgck_driver.so
#include <chrono>
#include <cstdint>
#include <deque>

#include "gck.h"

using submit_fn = int (*)(gck_engine*, const gck_consistency*, const gck_item*, size_t, const char* const*,
                          const size_t*, size_t, int64_t, uint8_t*, int32_t*, uint32_t, void*, gck_batch**);
using wait_fn = int (*)(gck_engine*, gck_batch*);
using submit_uniform_fn = int (*)(gck_engine*, const gck_consistency*, const gck_uniform*, const uint32_t*, size_t,
                                  const char* const*, const size_t*, size_t, int64_t, uint64_t*, gck_item_error*,
                                  size_t, size_t*, gck_batch**);

// Optional per-batch timeline of the next loops (gckd_set_trace): for batch k, the seconds after
// the loop's start at which its submit and its wait returned (stamps[2k], stamps[2k + 1]).
static double* g_stamps = nullptr;
static size_t g_cap = 0;

extern "C" {

static inline void stamp(std::chrono::steady_clock::time_point t0, size_t k, int which) {
  if (k < g_cap) g_stamps[2 * k + which] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

void gckd_set_trace(double* stamps, size_t n_batches) {
  g_stamps = stamps;
  g_cap = stamps ? n_batches : 0;
}

// Runs batches k = 0 .. n_batches-1 (device buffers items[k], perm[k], err[k], n checks each) with
// up to `depth` in flight; batch k is submitted on streams[k % depth] with GCK_SUBMIT_DEVICE | flags
// (GCK_SUBMIT_ENGINE_STREAM: on the engine's workspace streams instead), at now_us (0 = the clock). Returns GCK_OK or the first
// error; *seconds = wall time from the first submit to the last wait.
int gckd_run(submit_fn submit, wait_fn wait, gck_engine* e, const gck_consistency* cs, size_t n_batches, const uint64_t* items,
             const uint64_t* perm, const uint64_t* err, size_t n, uint32_t depth, const uint64_t* streams,
             uint32_t flags, int64_t now_us, double* seconds) {
  if (depth == 0) depth = 1;
  std::deque<gck_batch*> q;
  int rc = GCK_OK;
  const auto t0 = std::chrono::steady_clock::now();
  for (size_t k = 0; k < n_batches && rc == GCK_OK; ++k) {
    if (q.size() >= depth) {
      rc = wait(e, q.front());
      stamp(t0, k - depth, 1);
      q.pop_front();
      if (rc != GCK_OK) break;
    }
    gck_batch* b = nullptr;
    rc = submit(e, cs, reinterpret_cast<const gck_item*>(items[k]), n, nullptr, nullptr, 0, now_us,
                reinterpret_cast<uint8_t*>(perm[k]), reinterpret_cast<int32_t*>(err[k]), GCK_SUBMIT_DEVICE | flags,
                reinterpret_cast<void*>(streams[k % depth]), &b);
    if (rc == GCK_OK) q.push_back(b);
    stamp(t0, k, 0);
  }
  size_t kw = n_batches - q.size();
  while (!q.empty()) {  // every submitted batch is waited for, also after an error
    const int r = wait(e, q.front());
    stamp(t0, kw++, 1);
    if (rc == GCK_OK) rc = r;
    q.pop_front();
  }
  if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return rc;
}

// The same loop over host buffers (no GCK_SUBMIT_DEVICE): items[k] / perm[k] / err[k] are host
// pointers — gck_host_alloc memory moves by DMA straight from and into them — and each batch runs
// on the engine's workspace stream: items H2D, kernels, results D2H.
int gckd_run_host(submit_fn submit, wait_fn wait, gck_engine* e, const gck_consistency* cs, size_t n_batches,
                  const uint64_t* items, const uint64_t* perm, const uint64_t* err, size_t n, uint32_t depth,
                  int64_t now_us, double* seconds) {
  if (depth == 0) depth = 1;
  std::deque<gck_batch*> q;
  int rc = GCK_OK;
  const auto t0 = std::chrono::steady_clock::now();
  for (size_t k = 0; k < n_batches && rc == GCK_OK; ++k) {
    if (q.size() >= depth) {
      rc = wait(e, q.front());
      stamp(t0, k - depth, 1);
      q.pop_front();
      if (rc != GCK_OK) break;
    }
    gck_batch* b = nullptr;
    rc = submit(e, cs, reinterpret_cast<const gck_item*>(items[k]), n, nullptr, nullptr, 0, now_us,
                reinterpret_cast<uint8_t*>(perm[k]), reinterpret_cast<int32_t*>(err[k]), 0u, nullptr, &b);
    if (rc == GCK_OK) q.push_back(b);
    stamp(t0, k, 0);
  }
  size_t kw = n_batches - q.size();
  while (!q.empty()) {
    const int r = wait(e, q.front());
    stamp(t0, kw++, 1);
    if (rc == GCK_OK) rc = r;
    q.pop_front();
  }
  if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return rc;
}

// The same loop over uniform requests (gck_check_submit_uniform): request k = header hdrs[k] and
// ns[k] host pairs pairs[k] (u32 ids) in, packed[k] (ceil(ns[k] / 32) words) and errs[k] (err_cap
// records, the count in n_errs[k]) out — what Client.Check sends for runs of relationships of one
// shape, 8 B per check.
int gckd_run_uniform(submit_uniform_fn submit, wait_fn wait, gck_engine* e, const gck_consistency* cs, size_t n_batches,
                     const gck_uniform* hdrs, const uint64_t* pairs, const uint64_t* ns, const uint64_t* packed,
                     const uint64_t* errs, size_t err_cap, size_t* n_errs, uint32_t depth, int64_t now_us,
                     double* seconds) {
  if (depth == 0) depth = 1;
  std::deque<gck_batch*> q;
  int rc = GCK_OK;
  const auto t0 = std::chrono::steady_clock::now();
  for (size_t k = 0; k < n_batches && rc == GCK_OK; ++k) {
    if (q.size() >= depth) {
      rc = wait(e, q.front());
      stamp(t0, k - depth, 1);
      q.pop_front();
      if (rc != GCK_OK) break;
    }
    gck_batch* b = nullptr;
    rc = submit(e, cs, hdrs + k, reinterpret_cast<const uint32_t*>(pairs[k]), (size_t)ns[k], nullptr, nullptr, 0,
                now_us, reinterpret_cast<uint64_t*>(packed[k]), reinterpret_cast<gck_item_error*>(errs[k]), err_cap,
                n_errs ? n_errs + k : nullptr, &b);
    if (rc == GCK_OK) q.push_back(b);
    stamp(t0, k, 0);
  }
  size_t kw = n_batches - q.size();
  while (!q.empty()) {
    const int r = wait(e, q.front());
    stamp(t0, kw++, 1);
    if (rc == GCK_OK) rc = r;
    q.pop_front();
  }
  if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return rc;
}

}  // extern "C"
