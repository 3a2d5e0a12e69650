// Mi355xPool reconciler decision table (SURVEY.md §4.2 "C++ unit: reconciler decision table,
// observed x desired x health -> actions"): plan_pool() over hand-built device views.
#include "gpupool/provider.h"
#include "gpupool/reconciler.h"
#include "testing.h"

#include <algorithm>
#include <map>
#include <random>

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

TEST(pod_index_tracks_live_extended_requests_and_job_pods) {
  using gpupool::Json;
  auto pod = [](const std::string& name, const std::string& node, int gpus, const std::string& phase,
                const std::string& job = "") {
    Json p = Json::parse(R"({"metadata":{"name":"","namespace":"ns","labels":{}},"spec":{"nodeName":"",
      "containers":[{"name":"c","resources":{"limits":{"amd.com/gpu":"0","cpu":"2"}}}]},"status":{"phase":""}})");
    p["metadata"]["name"] = name;
    p["spec"]["nodeName"] = node;
    p["spec"]["containers"].at(0)["resources"]["limits"]["amd.com/gpu"] = std::to_string(gpus);
    p["status"]["phase"] = phase;
    if (!job.empty()) p["metadata"]["labels"]["gpupool.amd.com/job-name"] = job;
    return p;
  };
  gpupool::PodIndex idx;
  idx.on_event("ADDED", pod("a", "n1", 2, "Running"));
  idx.on_event("ADDED", pod("b", "n1", 1, "Pending", "j"));
  idx.on_event("ADDED", pod("c", "n2", 4, "Running", "j"));
  auto u = idx.requested_by_node("amd.com/gpu");
  EXPECT_TRUE(u["n1"] == 3 && u["n2"] == 4);
  idx.on_event("MODIFIED", pod("a", "n1", 2, "Succeeded"));  // terminal: holds nothing
  idx.on_event("DELETED", pod("c", "n2", 4, "Running", "j"));
  u = idx.requested_by_node("amd.com/gpu");
  EXPECT_TRUE(u["n1"] == 1 && !u.count("n2"));
  EXPECT_TRUE(idx.job_pods("ns", "j").size() == 1 && idx.job_pods("other", "j").empty());
  // the informer's projection keeps what the readers use, and relevance
  Json cpu_only = pod("d", "n1", 0, "Running");
  cpu_only["spec"]["containers"].at(0)["resources"]["limits"].erase("amd.com/gpu");
  EXPECT_TRUE(!gpupool::pod_relevant(cpu_only));
  EXPECT_TRUE(gpupool::pod_relevant(pod("e", "n1", 1, "Running")));
  Json t = gpupool::trim_pod(pod("f", "n1", 1, "Running", "j"));
  EXPECT_TRUE(t.path("spec.nodeName").as_string() == "n1");
  EXPECT_TRUE(t.path("spec.containers")[0]["resources"]["limits"]["amd.com/gpu"].as_string() == "1");
  EXPECT_TRUE(t.path("spec.containers")[0]["resources"]["limits"]["cpu"].is_null());
  EXPECT_TRUE(t.path("metadata.labels")["gpupool.amd.com/job-name"].as_string() == "j");
  // init containers: the pod holds max(sum of containers, largest init container), as the
  // scheduler counts it; a pod asking only in an init container is relevant and kept so
  Json init = pod("g", "n3", 1, "Running");
  init["spec"]["initContainers"] = Json::parse(
      R"([{"name":"i1","resources":{"limits":{"amd.com/gpu":"3"}}},{"name":"i2","resources":{"limits":{"amd.com/gpu":"2"}}}])");
  idx.on_event("ADDED", init);
  EXPECT_TRUE(idx.requested_by_node("amd.com/gpu")["n3"] == 3);
  Json only_init = cpu_only;
  only_init["spec"]["initContainers"] = Json::parse(R"([{"name":"i","resources":{"limits":{"amd.com/gpu":"1"}}}])");
  EXPECT_TRUE(gpupool::pod_relevant(only_init));
  EXPECT_TRUE(gpupool::trim_pod(only_init).path("spec.initContainers")[0]["resources"]["limits"]["amd.com/gpu"]
                  .as_string() == "1");
}

// Randomised: after every ADDED / MODIFIED / DELETED event the incremental per-node usage equals a
// recount of the live pods from scratch (phases, node moves of unscheduled pods, init containers,
// requests without limits, pods that ask for nothing), and job membership follows the label.
TEST(pod_index_matches_a_recount_under_random_events) {
  using gpupool::Json;
  std::mt19937 rng(12345);
  auto pick = [&](int n) { return static_cast<int>(rng() % static_cast<unsigned>(n)); };
  const char* phases[] = {"Pending", "Running", "Succeeded", "Failed"};
  const char* nodes[] = {"", "n1", "n2", "n3"};
  std::map<std::string, Json> live;
  gpupool::PodIndex idx;
  for (int step = 0; step < 3000; ++step) {
    const std::string name = "p" + std::to_string(pick(40));
    if (live.count(name) && pick(5) == 0) {
      idx.on_event("DELETED", live[name]);
      live.erase(name);
    } else {
      Json p = Json::parse(R"({"metadata":{"name":"","namespace":"ns","labels":{}},"spec":{"containers":[]},"status":{}})");
      p["metadata"]["name"] = name;
      if (pick(3) == 0) p["metadata"]["labels"]["gpupool.amd.com/job-name"] = pick(2) ? "j1" : "j2";
      const std::string node = nodes[pick(4)];
      if (!node.empty()) p["spec"]["nodeName"] = node;
      p["status"]["phase"] = phases[pick(4)];
      for (int c = 0, n = pick(3); c < n; ++c) {
        Json ctr = Json::object();
        ctr["name"] = "c" + std::to_string(c);
        const std::string part = pick(2) ? "limits" : "requests";
        if (pick(4)) ctr["resources"][part]["amd.com/gpu"] = std::to_string(pick(4));
        p["spec"]["containers"].push_back(ctr);
      }
      if (pick(4) == 0) {
        Json init = Json::object();
        init["name"] = "init";
        init["resources"]["limits"]["amd.com/gpu"] = std::to_string(pick(6));
        p["spec"]["initContainers"] = Json::array();
        p["spec"]["initContainers"].push_back(init);
      }
      idx.on_event(live.count(name) ? "MODIFIED" : "ADDED", p);
      live[name] = p;
    }
    // the recount
    std::map<std::string, int64_t> want;
    for (const auto& kv : live) {
      const Json& p = kv.second;
      const std::string node = p.path("spec.nodeName").as_string();
      const std::string phase = p.path("status.phase").as_string();
      if (node.empty() || phase == "Succeeded" || phase == "Failed") continue;
      int64_t sum = 0, init = 0;
      for (const auto& c : p.path("spec.containers").elements()) {
        const Json& r = c["resources"];
        const std::string v = r["limits"]["amd.com/gpu"].is_string() ? r["limits"]["amd.com/gpu"].as_string()
                              : r["requests"]["amd.com/gpu"].as_string();
        sum += v.empty() ? 0 : std::stoll(v);
      }
      for (const auto& c : p.path("spec.initContainers").elements())
        init = std::max<int64_t>(init, std::stoll(c["resources"]["limits"]["amd.com/gpu"].as_string()));
      const int64_t n = std::max(sum, init);
      if (n > 0) want[node] += n;
    }
    auto got = idx.requested_by_node("amd.com/gpu");
    EXPECT_TRUE(got == want);
    if (got != want) return;
    size_t members = 0;
    for (const auto& kv : live)
      members += kv.second.path("metadata.labels")["gpupool.amd.com/job-name"].as_string() == "j1";
    EXPECT_TRUE(idx.job_pods("ns", "j1").size() == members);
  }
  EXPECT_TRUE(idx.size() == live.size());
}
