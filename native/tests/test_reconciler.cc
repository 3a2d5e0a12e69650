// Mi355xPool reconciler decision table (SURVEY.md §4.2 "C++ unit: reconciler decision table,
// observed x desired x health -> actions"): plan_pool() over hand-built device views.
#include "gpupool/provider.h"
#include "gpupool/reconciler.h"
#include "testing.h"

using gpupool::DeviceView;
using gpupool::Json;
using gpupool::Mi355xPoolSpec;
using gpupool::plan_pool;

namespace {

// one observed GPU of the pool: index, health, probe result, pods, state, node
DeviceView gpu(int index, bool healthy = true, bool probe = true, int pods = 0,
               const char* state = "Claimed", const char* node = "n0") {
  DeviceView d;
  d.uuid = std::string(node) + "-gpu" + std::to_string(index);
  d.index = index;
  d.healthy = healthy;
  d.probe_passed = probe;
  d.state = state;
  d.node = node;
  d.pods = Json::array();
  for (int i = 0; i < pods; ++i) d.pods.push_back("default/p" + std::to_string(i));
  return d;
}

Mi355xPoolSpec spec(int replicas, const char* replace = "Replace") {
  Mi355xPoolSpec s;
  s.replicas = replicas;
  s.replace_policy = replace;
  return s;
}

std::string ids(const std::vector<std::string>& v) {
  std::string o;
  for (const auto& x : v) o += (o.empty() ? "" : ",") + x;
  return o;
}

}  // namespace

TEST(plan_scale_up_from_zero_and_steady_state) {
  auto p = plan_pool(spec(4), {});
  EXPECT_TRUE(p.replace.empty() && p.victims.empty());
  EXPECT_EQ(p.keep, 0);
  EXPECT_EQ(p.need, 4);
  p = plan_pool(spec(2), {gpu(0), gpu(1)});  // desired == observed healthy: nothing to do
  EXPECT_TRUE(p.replace.empty() && p.victims.empty());
  EXPECT_EQ(p.keep, 2);
  EXPECT_EQ(p.need, 0);
  p = plan_pool(spec(3), {gpu(0)});  // partial: claim the delta only
  EXPECT_EQ(p.need, 2);
}

TEST(plan_replaces_unhealthy_and_failed_probe) {
  // an ECC/xGMI/thermal fault and a failed probe are both replaced; the pass claims replacements
  auto p = plan_pool(spec(3), {gpu(0), gpu(1, false), gpu(2, true, false)});
  EXPECT_EQ(ids(p.replace), std::string("n0-gpu1,n0-gpu2"));
  EXPECT_EQ(p.keep, 1);
  EXPECT_EQ(p.need, 2);
  // replacePolicy Keep: faulty GPUs stay (and count), nothing is claimed
  p = plan_pool(spec(3, "Keep"), {gpu(0), gpu(1, false), gpu(2, true, false)});
  EXPECT_TRUE(p.replace.empty());
  EXPECT_EQ(p.keep, 3);
  EXPECT_EQ(p.need, 0);
  // a GPU still Probing is in flight, never "bad"
  p = plan_pool(spec(2), {gpu(0), gpu(1, true, false, 0, "Probing")});
  EXPECT_TRUE(p.replace.empty());
  EXPECT_EQ(p.need, 0);
  // ...unless the agent reports it past its probe deadline: then it is replaced, not waited on
  auto overdue = gpu(1, true, false, 0, "Probing");
  overdue.probe_overdue = true;
  p = plan_pool(spec(2), {gpu(0), overdue});
  EXPECT_EQ(ids(p.replace), std::string("n0-gpu1"));
  EXPECT_EQ(p.keep, 1);
  EXPECT_EQ(p.need, 1);
}

TEST(plan_scale_down_victim_order) {
  // 4 -> 2: pod-free GPUs go before busy ones, then the highest index
  auto p = plan_pool(spec(2), {gpu(0, true, true, 1), gpu(1), gpu(2, true, true, 1), gpu(3)});
  EXPECT_EQ(ids(p.victims), std::string("n0-gpu3,n0-gpu1"));
  EXPECT_EQ(p.keep, 2);
  EXPECT_EQ(p.need, 0);
  // with Keep, an unhealthy GPU is the first victim of a scale-down
  p = plan_pool(spec(1, "Keep"), {gpu(0), gpu(1, false, true, 1), gpu(2)});
  EXPECT_EQ(ids(p.victims), std::string("n0-gpu1,n0-gpu2"));
  // every GPU busy: highest index first (the BASELINE config-4 8 -> 4 expectation)
  std::vector<DeviceView> eight;
  for (int i = 0; i < 8; ++i) eight.push_back(gpu(i, true, true, 1));
  p = plan_pool(spec(4), eight);
  EXPECT_EQ(ids(p.victims), std::string("n0-gpu7,n0-gpu6,n0-gpu5,n0-gpu4"));
  // to zero: everything drains
  p = plan_pool(spec(0), {gpu(0), gpu(1)});
  EXPECT_EQ(p.victims.size(), 2u);
  EXPECT_EQ(p.keep, 0);
}

TEST(plan_draining_gpus_are_neither_kept_nor_claimed_again) {
  // a GPU already Draining (cordoned in an earlier pass) does not count toward replicas and is
  // not drained twice; the pass claims its replacement
  auto p = plan_pool(spec(2), {gpu(0), gpu(1, true, true, 1, "Draining")});
  EXPECT_TRUE(p.victims.empty() && p.replace.empty());
  EXPECT_EQ(p.keep, 1);
  EXPECT_EQ(p.need, 1);
}

TEST(plan_spanning_pool_shrinks_its_smallest_node_first) {
  // 3 GPUs on n0, 1 on n1; 4 -> 3: the lone GPU on n1 goes (frees a whole node)
  auto p = plan_pool(spec(3), {gpu(0, true, true, 0, "Claimed", "n0"), gpu(1, true, true, 0, "Claimed", "n0"),
                               gpu(2, true, true, 0, "Claimed", "n0"), gpu(0, true, true, 0, "Claimed", "n1")});
  EXPECT_EQ(ids(p.victims), std::string("n1-gpu0"));
}

TEST(plan_replace_and_scale_down_in_one_pass) {
  // desired drops 3 -> 1 while one GPU is faulty: replace nothing beyond need; the faulty one is
  // cordoned (replace) and one healthy GPU drains, leaving exactly one
  auto p = plan_pool(spec(1), {gpu(0), gpu(1, false), gpu(2)});
  EXPECT_EQ(ids(p.replace), std::string("n0-gpu1"));
  EXPECT_EQ(ids(p.victims), std::string("n0-gpu2"));
  EXPECT_EQ(p.keep, 1);
  EXPECT_EQ(p.need, 0);
}
