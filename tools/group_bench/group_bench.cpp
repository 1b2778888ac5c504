// Host cost of grouping one config-5 Watch batch (snapshot.cpp group_updates), on the CPU: the
// config-5 schema, interner counts of the config-2 graph, 9,844 updates of the churn mix
// (tests/synth_configs.py Mixed.churn: folder/doc viewer/editor, CREATE/TOUCH/DELETE 45/45/10,
// 10 % caveated). No GPU is touched.   make -C tools/group_bench && tools/group_bench/group_bench
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>
#include "engine.hpp"
#include "gck.h"

namespace gck { void validate_tuple(const Engine& e, const gck_tuple& t); }
struct gck_engine {
  gck::Engine impl;
};

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
  gck_config cfg{};
  gck_engine* ge = nullptr;
  if (gck_create(&cfg, &ge) || gck_load_schema(ge, kSchema, strlen(kSchema))) {
    fprintf(stderr, "setup: %s\n", gck_last_error());
    return 1;
  }
  gck::Engine& e = ge->impl;
  uint16_t t_user, t_folder, t_doc, r[4];
  gck_type_id(ge, "user", 4, &t_user);
  gck_type_id(ge, "folder", 6, &t_folder);
  gck_type_id(ge, "doc", 3, &t_doc);
  gck_relation_id(ge, t_folder, "viewer", 6, &r[0]);
  gck_relation_id(ge, t_folder, "editor", 6, &r[1]);
  gck_relation_id(ge, t_doc, "viewer", 6, &r[2]);
  gck_relation_id(ge, t_doc, "editor", 6, &r[3]);
  e.interner[t_user].count = 1000000;
  e.interner[t_folder].count = 200000;
  e.interner[t_doc].count = 2000000;
  gck::add_caveat_instance(e, "only_on_tuesday", "");
  std::mt19937_64 rng(7);
  std::vector<gck_update> ups(n);
  for (size_t i = 0; i < n; ++i) {
    gck_update& u = ups[i];
    const int k = (int)(rng() % 4);
    u.tuple.resource_type = k < 2 ? t_folder : t_doc;
    u.tuple.relation = r[k];
    u.tuple.resource_id = (uint32_t)(rng() % (k < 2 ? 200000 : 2000000));
    u.tuple.subject_type = t_user;
    u.tuple.subject_relation = 0xFFFF;
    u.tuple.subject_id = (uint32_t)(rng() % 1000000);
    const int op = (int)(rng() % 100);
    u.op = op < 45 ? GCK_UPDATE_CREATE : op < 90 ? GCK_UPDATE_TOUCH : GCK_UPDATE_DELETE;
    u.tuple.caveat = (rng() % 10 == 0) ? 1 : 0;
  }
  double best = 1e9, sum = 0;
  const int reps = 200;
  size_t groups = 0;
  for (int k = 0; k < reps; ++k) {
    const auto t0 = std::chrono::steady_clock::now();
    auto g = gck::group_updates(e, ups.data(), ups.size());
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    groups = g.size();
    best = std::min(best, us);
    sum += us;
  }
  double vbest = 1e9;
  for (int k = 0; k < reps; ++k) {
    const auto t0 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < n; ++i) gck::validate_tuple(e, ups[i].tuple);
    vbest = std::min(vbest, std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  printf("validate alone: best %.1f us\n", vbest);
  printf("{\"updates\": %zu, \"groups\": %zu, \"best_us\": %.1f, \"mean_us\": %.1f}\n", n, groups, best, sum / reps);
  gck_destroy(ge);
  return 0;
}
