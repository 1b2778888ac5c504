// group_bench.cpp — host-only timing of a config-5 Watch batch's grouping (snapshot.cpp
// group_updates: validation, grouping per relation kind, last write per key, sorted keys), the
// host share of the Watch step that needs no GPU to measure.
//   build: make -C tools/group_bench     run: tools/group_bench/group_bench [updates] [reps]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "engine.hpp"

using namespace gck;

static const char* kSchema = R"(
caveat only_on_tuesday(day_of_the_week string) {
  day_of_the_week == "tuesday"
}
definition user {}
definition group {
  relation member: user | group#member
}
definition folder {
  relation parent: folder
  relation viewer: user | group#member | user with only_on_tuesday
  relation editor: user | group#member | user with only_on_tuesday
  permission edit = editor + parent->edit
  permission view = viewer + edit + parent->view
}
definition doc {
  relation parent: folder
  relation owner: user
  relation viewer: user | user:* | group#member | user with only_on_tuesday
  relation editor: user | group#member | user with only_on_tuesday
  permission edit = owner + editor + parent->edit
  permission view = viewer + edit + parent->view
}
)";

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? (size_t)atol(argv[1]) : 9844;
  const int reps = argc > 2 ? atoi(argv[2]) : 400;
  Engine& e = *new Engine();  // (never destroyed: ~Engine lives with the device code)
  e.schema = compile_schema(kSchema);
  const Schema& sc = *e.schema;
  e.interner.resize(sc.types.size());
  auto type = [&](const char* t) { return (uint16_t)sc.find_type(t); };
  const uint16_t user = type("user"), folder = type("folder"), doc = type("doc");
  e.interner[user].count = 1000000;
  e.interner[type("group")].count = 100000;
  e.interner[folder].count = 200000;
  e.interner[doc].count = 2000000;
  e.caveat_instances.push_back({"", ""});
  e.caveat_instances.push_back({"only_on_tuesday", ""});
  const uint16_t kinds[4][2] = {{folder, (uint16_t)sc.find_rel(folder, "viewer")},
                                {folder, (uint16_t)sc.find_rel(folder, "editor")},
                                {doc, (uint16_t)sc.find_rel(doc, "viewer")},
                                {doc, (uint16_t)sc.find_rel(doc, "editor")}};
  std::mt19937_64 rng(7);
  std::vector<std::vector<gck_update>> batches(8);
  for (auto& b : batches) {
    b.resize(n);
    for (gck_update& u : b) {
      const auto& k = kinds[rng() % 4];
      const double r = (double)(rng() % 1000) / 1000.0;
      u = gck_update{};
      u.op = r < 0.45 ? GCK_UPDATE_CREATE : r < 0.9 ? GCK_UPDATE_TOUCH : GCK_UPDATE_DELETE;
      u.tuple.resource_type = k[0];
      u.tuple.relation = k[1];
      u.tuple.resource_id = (uint32_t)(rng() % e.interner[k[0]].count);
      u.tuple.subject_type = user;
      u.tuple.subject_relation = kEllipsis;
      u.tuple.subject_id = (uint32_t)(rng() % 1000000);
      u.tuple.caveat = (rng() % 10 == 0 && u.op != GCK_UPDATE_DELETE) ? 1 : 0;
    }
  }
  std::vector<double> t;
  size_t keys = 0;
  for (int r = 0; r < reps; ++r) {
    const auto& b = batches[r % batches.size()];
    const auto t0 = std::chrono::steady_clock::now();
    const std::vector<UpdateGroup>& g = group_updates(e, b.data(), b.size());
    t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    for (const UpdateGroup& x : g) keys += x.keys.size();
  }
  std::sort(t.begin() + reps / 4, t.end());
  printf("{\"updates\": %zu, \"reps\": %d, \"median_us\": %.1f, \"p10_us\": %.1f, \"keys_per_batch\": %.0f}\n", n, reps,
         t[reps / 4 + (reps - reps / 4) / 2], t[reps / 4 + (reps - reps / 4) / 10], (double)keys / reps);
  return 0;
}

// (engine.hip's phase clock, here so that the host objects link without the device code)
namespace gck {
static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
PhaseClock::PhaseClock(const char* w) : what(w), on(getenv("GCK_DEBUG_PHASES") != nullptr), t0(0), last(0) {
  if (on) t0 = last = now_s();
}
void PhaseClock::mark(const char* phase) {
  if (!on) return;
  const double t = now_s();
  char buf[96];
  snprintf(buf, sizeof(buf), " %s=%.1fus", phase, (t - last) * 1e6);
  line += buf;
  last = t;
}
PhaseClock::~PhaseClock() {
  if (on) fprintf(stderr, "[gck %s] total=%.1fus%s\n", what, (now_s() - t0) * 1e6, line.c_str());
}
// (text parsing registers caveat instances through gck_api.cpp; the bench builds records directly)
uint32_t add_caveat_instance(Engine&, const std::string&, const std::string&) { abort(); }
}  // namespace gck
