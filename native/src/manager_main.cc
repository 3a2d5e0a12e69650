// gpupool-manager: the operator process (the kubebuilder manager the reference never showed —
// "step four" is missing, README.md:162->242). Wires informers (pools of both kinds + Nodes),
// a shared rate-limited work queue with N workers, the providers, an Event recorder, Lease leader
// election, Prometheus /metrics and /healthz, and one long-poll per node agent so device health
// changes trigger reconciles immediately (event-driven, no polling sleeps on the hot path).
// With `job` in --kinds it also runs the Mi355xJob gang scheduler, the Mi355xQueue status
// controller and the demand-driven pool autoscaler (pod + job informers).
//
//   gpupool-manager --apiserver http://127.0.0.1:6443 [--namespace NS] [--workers 4]
//       [--kinds mi355x,azure,job] [--leader-elect] [--metrics-addr :8080] [--health-addr :8081]
//       [--resync 10s] [--fakecloud-state f.json] [--fakecloud-provision-ms N]
//   gpupool-manager --validate obj.json     # validation parity check; prints JSON errors
#include <malloc.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <set>
#include <sstream>
#include <thread>

#include "gpupool/api.h"
#include "gpupool/azure_arm.h"
#include "gpupool/events.h"
#include "gpupool/generated/schema_consts.h"
#include "gpupool/http.h"
#include "gpupool/informer.h"
#include "gpupool/kube.h"
#include "gpupool/leader.h"
#include "gpupool/log.h"
#include "gpupool/metrics.h"
#include "gpupool/podindex.h"
#include "gpupool/provider.h"
#include "gpupool/reconciler.h"
#include "gpupool/trace.h"

using namespace gpupool;

namespace {

std::atomic<bool> g_stop{false};
void on_signal(int) { g_stop = true; }

struct Flags {
  std::string apiserver = "http://127.0.0.1:6443";
  std::string token;
  std::string ns;
  int workers = 4;
  std::string kinds = "mi355x,azure,job";
  bool leader_elect = false;
  bool quota_fail_open = false;
  std::string lease_ns = "gpupool-system";
  std::string identity;
  std::string metrics_addr = "127.0.0.1:0";
  std::string health_addr;
  std::string port_file;
  int resync_ms = 10000;
  int event_delay_ms = 10;
  int progress_ms = 250;
  int cred_retry_ms = 30000;
  int agent_timeout_ms = 60000;
  std::string fakecloud_state;
  std::string fakecloud_faults;
  int fakecloud_provision_ms = 0;
  int fakecloud_deprovision_ms = 0;
  std::string cloud = "fake";  // fake | azure-arm
  std::string azure_arm_endpoint, azure_authority_host, azure_ca_file, azure_ssh_key_file, azure_admin_user;
  int azure_nic_wait_ms = 10000;
  int orphan_sweep_ms = 30000;
  int lease_duration_ms = 15000;
  int renew_deadline_ms = 10000;
  int retry_period_ms = 2000;
  std::string log_level = "info";
  int slow_reconcile_ms = 1000;
  std::string validate;
  // TLS / auth for a real apiserver
  std::string ca_file, client_cert, client_key, token_file, agent_token, agent_token_file, agent_ca_file;
  int token_reload_ms = 60000;
  // node agents: discovery and credentials (provider.h AgentAccess)
  std::string agent_discovery = "annotation", agent_namespace = "gpupool-system",
              agent_selector = "app.kubernetes.io/name=gpupool-agent", agent_scheme = "https",
              agent_signing_key;
  int agent_port = 9443;
  std::string kubeconfig, kube_context;
  bool insecure = false;
  bool apiserver_set = false;
};

int parse_duration_ms(const std::string& s) {
  if (s.empty()) return 0;
  double v = std::stod(s);
  if (s.size() > 2 && s.substr(s.size() - 2) == "ms") return static_cast<int>(v);
  if (s.back() == 's') return static_cast<int>(v * 1000);
  if (s.back() == 'm') return static_cast<int>(v * 60000);
  return static_cast<int>(v);  // bare number = ms
}

const char* kUsage = R"(gpupool-manager: Mi355xPool / AzureVmPool operator

connection, first match wins: --apiserver/$GPUPOOL_APISERVER, --kubeconfig/$KUBECONFIG,
in-cluster ServiceAccount, ~/.kube/config, http://127.0.0.1:6443:
  --apiserver URL              http(s)://host:port or unix:///path   [$GPUPOOL_APISERVER]
  --kubeconfig F [--context C] kubeconfig file and context (default: current-context)
  --token T | --token-file F   bearer token                            [$GPUPOOL_TOKEN]
  --ca-file F                  CA bundle to verify the apiserver certificate
  --client-cert F --client-key F   client certificate authentication
  --insecure-skip-tls-verify   do not verify the apiserver certificate (testing only)
controllers:
  --kinds mi355x,azure,job     reconcilers to run            --namespace NS   watch one namespace
  --workers N (4)              reconcile worker threads      --resync D (10s) steady-state resync
  --event-delay D (10ms)       Events post this long after the pass that records them
  --progress-poll D (250ms)    requeue while scaling/draining
  --credentials-retry D (30s)  AzureVmPool retry after a credentials error
  --agent-timeout D (60s)      node-agent RPC timeout (covers on-claim GPU probes)
  --token-reload D (60s)       re-read --token-file / the ServiceAccount token this often (and on 401)
node agents:
  --agent-discovery pod|annotation (annotation)  pod: the agent Pod's IP on each node (pods of
                               --agent-namespace matching --agent-selector); annotation: the Node's
                               gpupool.amd.com/agent-endpoint (local setups)
  --agent-namespace NS (gpupool-system)  --agent-selector SEL (app.kubernetes.io/name=gpupool-agent)
  --agent-scheme https|http (https)      --agent-port N (9443)
  --agent-signing-key F        Ed25519 key: sign every agent request for its node (no bearer sent)
                               [$GPUPOOL_AGENT_SIGNING_KEY]
  --agent-token-file F         shared bearer for agents without signatures, re-read as it rotates
                               [$GPUPOOL_AGENT_TOKEN]
  --agent-ca-file F            CA that signs https:// agent endpoints [$GPUPOOL_AGENT_CA_FILE]
  --orphan-sweep D (30s)       release claims whose pool no longer exists
  --quota-fail-open            admit scale-ups when ResourceQuotas cannot be read (clusters without
                               quotas); default: block them (Progressing=False, QuotaUnknown)
leader election:
  --leader-elect  --lease-namespace NS (gpupool-system)  --identity ID
  --lease-duration D (15s)  --renew-deadline D (10s)  --retry-period D (2s)
observability:
  --metrics-addr H:P (127.0.0.1:0)  /metrics /healthz /readyz /debug/traces
  --health-addr H:P                 separate /healthz listener
  --port-file F                     write the bound metrics port here
  --log-level debug|info|warn|error --slow-reconcile D (1s) log traces slower than D at info
AzureVmPool cloud:
  --cloud fake|azure-arm (fake)  fake: in-process cloud; azure-arm: the Azure Resource Manager REST API
  --fakecloud-state F  --fakecloud-faults F  --fakecloud-provision-ms N  --fakecloud-deprovision-ms N
  --azure-arm-endpoint URL (https://management.azure.com)
  --azure-authority-host URL (https://login.microsoftonline.com)
  --azure-ca-file F            CA bundle for both (private endpoints, tests)
  --azure-ssh-public-key-file F  VM admin SSH key when the Secret has no AZURE_SSH_PUBLIC_KEY
  --azure-admin-user U (azureuser)  --azure-nic-wait D (10s)
tools:
  --validate obj.json          print validation errors (JSON) for one object and exit
durations: 250ms, 10s, 5m or bare milliseconds.
)";

Flags parse(int argc, char** argv) {
  Flags f;
  auto env = [](const char* k, std::string& dst) {
    if (const char* v = getenv(k)) dst = v;
  };
  env("GPUPOOL_APISERVER", f.apiserver);
  env("GPUPOOL_TOKEN", f.token);
  env("GPUPOOL_NAMESPACE", f.ns);
  env("GPUPOOL_AGENT_TOKEN", f.agent_token);
  env("GPUPOOL_AGENT_CA_FILE", f.agent_ca_file);
  env("GPUPOOL_AGENT_SIGNING_KEY", f.agent_signing_key);
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&]() -> std::string {
      auto eq = a.find('=');
      if (eq != std::string::npos) return a.substr(eq + 1);
      if (i + 1 >= argc) {
        std::cerr << "missing value for " << a << "\n";
        std::exit(2);
      }
      return argv[++i];
    };
    auto is = [&](const char* name) { return a == name || a.rfind(std::string(name) + "=", 0) == 0; };
    if (is("--apiserver")) {
      f.apiserver = val();
      f.apiserver_set = true;
    } else if (is("--ca-file")) f.ca_file = val();
    else if (is("--client-cert")) f.client_cert = val();
    else if (is("--client-key")) f.client_key = val();
    else if (is("--token-file")) f.token_file = val();
    else if (is("--agent-token-file")) f.agent_token_file = val();
    else if (is("--agent-ca-file")) f.agent_ca_file = val();
    else if (is("--token-reload")) f.token_reload_ms = parse_duration_ms(val());
    else if (is("--agent-discovery")) f.agent_discovery = val();
    else if (is("--agent-namespace")) f.agent_namespace = val();
    else if (is("--agent-selector")) f.agent_selector = val();
    else if (is("--agent-scheme")) f.agent_scheme = val();
    else if (is("--agent-port")) f.agent_port = std::stoi(val());
    else if (is("--agent-signing-key")) f.agent_signing_key = val();
    else if (is("--kubeconfig")) f.kubeconfig = val();
    else if (is("--context")) f.kube_context = val();
    else if (a == "--insecure-skip-tls-verify") f.insecure = true;
    else if (is("--token")) f.token = val();
    else if (is("--namespace")) f.ns = val();
    else if (is("--workers")) f.workers = std::stoi(val());
    else if (is("--kinds")) f.kinds = val();
    else if (a == "--leader-elect") f.leader_elect = true;
    else if (a == "--quota-fail-open") f.quota_fail_open = true;
    else if (is("--lease-namespace")) f.lease_ns = val();
    else if (is("--identity")) f.identity = val();
    else if (is("--metrics-addr")) f.metrics_addr = val();
    else if (is("--health-addr")) f.health_addr = val();
    else if (is("--port-file")) f.port_file = val();
    else if (is("--resync")) f.resync_ms = parse_duration_ms(val());
    else if (is("--event-delay")) f.event_delay_ms = parse_duration_ms(val());
    else if (is("--progress-poll")) f.progress_ms = parse_duration_ms(val());
    else if (is("--credentials-retry")) f.cred_retry_ms = parse_duration_ms(val());
    else if (is("--agent-timeout")) f.agent_timeout_ms = parse_duration_ms(val());
    else if (is("--fakecloud-state")) f.fakecloud_state = val();
    else if (is("--fakecloud-faults")) f.fakecloud_faults = val();
    else if (is("--fakecloud-provision-ms")) f.fakecloud_provision_ms = std::stoi(val());
    else if (is("--fakecloud-deprovision-ms")) f.fakecloud_deprovision_ms = std::stoi(val());
    else if (is("--cloud")) f.cloud = val();
    else if (is("--azure-arm-endpoint")) f.azure_arm_endpoint = val();
    else if (is("--azure-authority-host")) f.azure_authority_host = val();
    else if (is("--azure-ca-file")) f.azure_ca_file = val();
    else if (is("--azure-ssh-public-key-file")) f.azure_ssh_key_file = val();
    else if (is("--azure-admin-user")) f.azure_admin_user = val();
    else if (is("--azure-nic-wait")) f.azure_nic_wait_ms = parse_duration_ms(val());
    else if (is("--orphan-sweep")) f.orphan_sweep_ms = parse_duration_ms(val());
    else if (is("--lease-duration")) f.lease_duration_ms = parse_duration_ms(val());
    else if (is("--renew-deadline")) f.renew_deadline_ms = parse_duration_ms(val());
    else if (is("--retry-period")) f.retry_period_ms = parse_duration_ms(val());
    else if (is("--log-level")) f.log_level = val();
    else if (is("--slow-reconcile")) f.slow_reconcile_ms = parse_duration_ms(val());
    else if (is("--validate")) f.validate = val();
    else if (a == "-h" || a == "--help") {
      std::cout << kUsage;
      std::exit(0);
    } else {
      std::cerr << "unknown flag " << a << "\n";
      std::exit(2);
    }
  }
  if (f.agent_discovery != "pod" && f.agent_discovery != "annotation") {
    std::cerr << "--agent-discovery must be pod or annotation\n";
    std::exit(2);
  }
  if (f.cloud != "fake" && f.cloud != "azure-arm") {
    std::cerr << "--cloud must be fake or azure-arm\n";
    std::exit(2);
  }
  if (f.identity.empty()) {
    char host[256] = {0};
    gethostname(host, sizeof host - 1);
    f.identity = std::string(host) + "_" + std::to_string(getpid());
  }
  return f;
}

int run_validate(const std::string& path) {
  std::ifstream in(path);
  std::stringstream ss;
  ss << in.rdbuf();
  Json obj = Json::parse(ss.str());
  std::vector<std::string> errs;
  std::string kind = obj["kind"].as_string();
  if (kind == "Mi355xPool") errs = validate_mi355x(obj);
  else if (kind == "Mi355xJob") errs = validate_job(obj);
  else if (kind == "AzureVmPool") errs = validate_azure(obj);
  else errs.push_back("kind: unsupported " + kind);
  Json out = Json::object();
  Json arr = Json::array();
  for (auto& e : errs) arr.push_back(e);
  out["kind"] = kind;
  out["errors"] = arr;
  std::cout << out.dump() << "\n";
  return errs.empty() ? 0 : 1;
}

// One long-poll loop per node agent: GET /v1/events?since=G blocks until device state changes,
// then every pool with a claim on that node is enqueued.
class AgentWatchers {
 public:
  static constexpr int kMaxFeedBackoffMs = 1000;
  AgentWatchers(RocmProvider& prov, Informer& pools, Controller& ctl) : prov_(prov), pools_(pools), ctl_(ctl) {}
  ~AgentWatchers() { stop_all(); }

  void sync(const std::vector<std::string>& nodes) {
    std::lock_guard<std::mutex> g(mu_);
    std::set<std::string> want(nodes.begin(), nodes.end());
    for (const auto& n : nodes) {
      std::string ep = prov_.endpoint_of(n);
      auto it = w_.find(n);
      if (it != w_.end() && it->second->endpoint == ep) continue;
      if (it != w_.end()) {
        it->second->stop = true;
        it->second->th.join();
        w_.erase(it);
      }
      auto w = std::make_unique<W>();
      w->endpoint = ep;
      W* raw = w.get();
      w->th = std::thread([this, n, raw] { loop(n, raw); });
      w_[n] = std::move(w);
    }
    for (auto it = w_.begin(); it != w_.end();) {
      if (!want.count(it->first)) {
        it->second->stop = true;
        it->second->th.join();
        it = w_.erase(it);
      } else {
        ++it;
      }
    }
  }

  void stop_all() {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : w_) kv.second->stop = true;
    for (auto& kv : w_)
      if (kv.second->th.joinable()) kv.second->th.join();
    w_.clear();
  }

 private:
  struct W {
    std::string endpoint;
    std::atomic<bool> stop{false};
    std::thread th;
  };

  void loop(const std::string& node, W* w) {
    Logger log = Logger("agent-watch").with("node", node);
    int64_t since = -1;
    int backoff = 100;
    bool connected = false;  // the feed answered since the last failure
    while (!w->stop && !g_stop) {
      try {
        // the agent holds the answer up to timeoutSeconds: allow that plus slack before timing out
        std::unique_ptr<HttpClient> cp = prov_.new_client(node, w->endpoint, 10000);
        HttpClient& c = *cp;
        std::string path = "/v1/events?timeoutSeconds=5&since=" + std::to_string(since);
        int status = c.stream_lines(
            path,
            [&](std::string_view line) {
              auto j = Json::try_parse(line);
              if (!j) return true;
              connected = true;
              int64_t gen = (*j)["gen"].as_int(since);
              prov_.note_gen(node, gen);
              const bool changed = gen != since;
              // a generation going backwards is a restarted agent: everything on it may differ
              if (since >= 0 && changed) enqueue_pools(node, (*j)["pools"], gen < since);
              since = gen;
              // after the pools are queued (latency first), refresh the view cache so the next
              // reconcile of a pool on this node needs no observe RPC
              if (changed) prov_.prefetch(node);
              return true;
            },
            &w->stop);
        if (status == 401) prov_.distrust_kx(node);  // the next attempt is Ed25519-signed
        if (status >= 400) throw std::runtime_error("HTTP " + std::to_string(status));
        backoff = 100;
      } catch (const std::exception& e) {
        log.debug("agent long-poll failed", Json::object().set("error", e.what()));
        if (connected) {
          // the agent went away: its cached view no longer stands for anything, and the pools on
          // the node must observe that now (Ready=Unknown, AgentUnreachable) — not after the
          // view cache's age or the next resync
          connected = false;
          prov_.forget_view(node);
          enqueue_pools(node, Json::array(), true);
        }
        // back off while the agent is away (a refused connect is cheap: at most one a second per
        // node), and reconnect at once when a reconcile's RPC reaches it again: a restarted
        // agent's events (re-advertised GPUs, faults) must not wait out a grown backoff
        const uint64_t seen = prov_.answered(node);
        for (int i = 0; i < backoff / 50 && !w->stop && prov_.answered(node) == seen; ++i)
          std::this_thread::sleep_for(std::chrono::milliseconds(50));
        backoff = prov_.answered(node) != seen ? 100 : std::min(backoff * 2, kMaxFeedBackoffMs);
      }
    }
  }

  void enqueue_pools(const std::string& node, const Json& pools, bool node_wide) {
    std::set<std::string> uids;
    for (const auto& u : pools.elements()) uids.insert(u.as_string());
    const bool all = uids.count("*") > 0;
    for (const auto& p : pools_.list()) {
      // the pools the event names (the agent names every pool whose GPUs changed), every pool on
      // the node after an agent restart or a truncated history ("*"), and pools still waiting for
      // capacity ("*free*": a release or an un-cordon anywhere may unblock them). Waking every
      // pool on the node for any event multiplied reconciles ~6x in a burst of claims.
      bool on_node = false;
      if (node_wide || all) {
        on_node = p.path("status.nodeName").as_string() == node;
        for (const auto& n : p.path("status.nodes").elements()) on_node = on_node || n.as_string() == node;
      }
      bool hit = uids.count(p.path("metadata.uid").as_string()) > 0 || on_node ||
                 (all && p.path("status.nodeName").as_string().empty()) ||
                 (uids.count("*free*") > 0 && !condition_true(p.path("status.conditions"), gen::kCondReady));
      if (hit) ctl_.enqueue("Mi355xPool", p.path("metadata.namespace").as_string(), p.path("metadata.name").as_string());
    }
  }

  RocmProvider& prov_;
  Informer& pools_;
  Controller& ctl_;
  std::mutex mu_;
  std::map<std::string, std::unique_ptr<W>> w_;
};

}  // namespace

int main(int argc, char** argv) {
  // glibc gives every thread that allocates its own arena (up to 8 per core): with one event-feed
  // thread per node agent plus the workers, fragmentation across them grew the manager to 309 MiB
  // at 64 nodes / 256 pools and 717 MiB at 128 / 512. Eight shared arenas hold it at 172 MiB at
  // 128 / 512 for ~20 % more CPU; four cost more (malloc lock contention): 146 MiB, +45 % CPU
  // (profiles/r5n_scale_placement_capacity_cpu.json). MALLOC_ARENA_MAX, when set, still wins.
  if (!getenv("MALLOC_ARENA_MAX")) mallopt(M_ARENA_MAX, 8);
  // Test harness only (gpupool/utils/parent_watch.py): exit once the process that started this one
  // is gone — a test runner killed at a timeout never runs its teardown.
  if (const char* pp = getenv("GPUPOOL_EXIT_WITH_PARENT")) {
    const pid_t parent = static_cast<pid_t>(std::atoll(pp));
    unsetenv("GPUPOOL_EXIT_WITH_PARENT");
    if (parent > 0)
      std::thread([parent] {
        while (getppid() == parent) std::this_thread::sleep_for(std::chrono::seconds(1));
        kill(getpid(), SIGTERM);  // the normal shutdown path
        std::this_thread::sleep_for(std::chrono::seconds(20));
        _exit(0);  // a shutdown stuck behind an unreachable apiserver
      }).detach();
  }
  Flags f = parse(argc, argv);
  if (!f.validate.empty()) return run_validate(f.validate);
  Logger::set_level(Logger::parse_level(f.log_level));
  trace::set_slow_threshold(std::chrono::milliseconds(f.slow_reconcile_ms));
  signal(SIGINT, on_signal);
  signal(SIGTERM, on_signal);
  signal(SIGPIPE, SIG_IGN);
  Logger log("manager");
  bool want_mi = f.kinds.find("mi355x") != std::string::npos;
  bool want_az = f.kinds.find("azure") != std::string::npos;
  bool want_job = f.kinds.find("job") != std::string::npos;

  TlsOptions tls;
  tls.ca_file = f.ca_file;
  tls.cert_file = f.client_cert;
  tls.key_file = f.client_key;
  tls.insecure = f.insecure;
  const auto reload = std::chrono::milliseconds(std::max(1000, f.token_reload_ms));
  // apiserver bearer: a file is re-read as it rotates (projected ServiceAccount tokens expire;
  // client-go re-reads them every minute and after a 401 — so do we)
  std::shared_ptr<TokenSource> api_tokens;
  try {
    if (!f.token_file.empty()) api_tokens = TokenSource::file(f.token_file, reload);
    else if (!f.token.empty()) api_tokens = TokenSource::fixed(f.token);
  } catch (const std::exception& e) {
    log.error("apiserver token", Json::object().set("error", e.what()));
    return 2;
  }
  if (!f.apiserver_set && !getenv("GPUPOOL_APISERVER")) {
    std::string server, token, home_cfg;
    TlsOptions ic;
    if (const char* home = getenv("HOME")) home_cfg = std::string(home) + "/.kube/config";
    const char* env_kc = getenv("KUBECONFIG");
    bool use_kc = !f.kubeconfig.empty() || (env_kc && *env_kc);
    if (!use_kc && KubeClient::in_cluster(&server, &token, &ic)) {  // running in a pod
      f.apiserver = server;
      if (!api_tokens) api_tokens = TokenSource::file("/var/run/secrets/kubernetes.io/serviceaccount/token", reload);
      if (tls.ca_file.empty()) tls.ca_file = ic.ca_file;
    } else if (use_kc || (!home_cfg.empty() && std::ifstream(home_cfg).good())) {
      KubeConfig kc;
      try {
        kc = load_kubeconfig(f.kubeconfig, f.kube_context);
      } catch (const std::exception& e) {
        log.error("kubeconfig", Json::object().set("error", e.what()));
        return 2;
      }
      f.apiserver = kc.server;
      if (!api_tokens) {  // explicit flags win over the kubeconfig
        if (!kc.token_file.empty()) api_tokens = TokenSource::file(kc.token_file, reload);
        else if (!kc.token.empty()) api_tokens = TokenSource::fixed(kc.token);
      }
      if (tls.ca_file.empty() && tls.ca_pem.empty()) {
        tls.ca_file = kc.tls.ca_file;
        tls.ca_pem = kc.tls.ca_pem;
      }
      if (tls.cert_file.empty()) {
        tls.cert_file = kc.tls.cert_file;
        tls.key_file = kc.tls.key_file;
        tls.cert_pem = kc.tls.cert_pem;
        tls.key_pem = kc.tls.key_pem;
      }
      tls.insecure = tls.insecure || kc.tls.insecure;
      log.info("using kubeconfig", Json::object().set("context", kc.context).set("server", kc.server));
    }
  }
  // node-agent credentials
  AgentAccess agent_access;
  agent_access.discovery = f.agent_discovery;
  agent_access.scheme = f.agent_scheme;
  agent_access.port = f.agent_port;
  agent_access.tls.ca_file = f.agent_ca_file;
  try {
    if (!f.agent_signing_key.empty()) agent_access.signer = std::make_shared<AgentSigner>(f.agent_signing_key);
    if (!f.agent_token_file.empty()) agent_access.token = TokenSource::file(f.agent_token_file, reload);
    else if (!f.agent_token.empty()) agent_access.token = TokenSource::fixed(f.agent_token);
  } catch (const std::exception& e) {
    log.error("agent credentials", Json::object().set("error", e.what()));
    return 2;
  }
  KubeClient client(f.apiserver, api_tokens, 15000, tls);
  std::atomic<bool> healthy{true}, leading{!f.leader_elect};

  HttpServer metrics;
  metrics.route("/metrics", [](const std::string&, const std::string&, const std::string&) {
    HttpServer::Reply r;
    r.content_type = "text/plain; version=0.0.4";
    r.body = Registry::global().render();
    return r;
  });
  auto health = [&](const std::string&, const std::string&, const std::string&) {
    HttpServer::Reply r;
    r.status = healthy ? 200 : 500;
    r.body = healthy ? "ok\n" : "unhealthy\n";
    return r;
  };
  metrics.route("/healthz", health);
  // recent reconcile traces (newest first); ?n=N, ?key=substring filters by "Kind/ns/name"
  metrics.route("/debug/traces", [](const std::string&, const std::string& target, const std::string&) {
    size_t n = 64;
    std::string key;
    auto q = target.find('?');
    if (q != std::string::npos) {
      std::istringstream qs(target.substr(q + 1));
      std::string kv;
      while (std::getline(qs, kv, '&')) {
        auto eq = kv.find('=');
        if (eq == std::string::npos) continue;
        if (kv.substr(0, eq) == "n") n = static_cast<size_t>(std::max(1, std::atoi(kv.c_str() + eq + 1)));
        else if (kv.substr(0, eq) == "key") key = url_decode(kv.substr(eq + 1));
      }
    }
    Json all = trace::recent(key.empty() ? n : 256);
    Json out = Json::array();
    for (const auto& t : all.elements()) {
      if (out.size() >= n) break;
      if (key.empty() || t["key"].as_string().find(key) != std::string::npos) out.push_back(t);
    }
    HttpServer::Reply r;
    r.content_type = "application/json";
    r.body = out.dump() + "\n";
    return r;
  });
  metrics.route("/readyz", [&](const std::string&, const std::string&, const std::string&) {
    HttpServer::Reply r;
    r.status = leading ? 200 : 503;
    r.body = leading ? "ok\n" : "standby\n";
    return r;
  });
  int mport = metrics.listen(f.metrics_addr);
  std::unique_ptr<HttpServer> health_srv;
  if (!f.health_addr.empty()) {
    health_srv = std::make_unique<HttpServer>();
    health_srv->route("/healthz", health);
    health_srv->listen(f.health_addr);
  }
  if (!f.port_file.empty()) {
    std::ofstream pf(f.port_file + ".tmp");
    pf << mport;
    pf.close();
    std::rename((f.port_file + ".tmp").c_str(), f.port_file.c_str());
  }
  log.info("starting", Json::object().set("apiserver", f.apiserver).set("metricsPort", mport).set("kinds", f.kinds)
                           .set("workers", f.workers).set("identity", f.identity));

  auto run_controllers = [&]() {
    EventRecorder events(&client, "gpupool-manager");
    events.set_delay(std::chrono::milliseconds(f.event_delay_ms));
    Controller ctl(f.workers);
    ReconcilerOptions ropts;
    ropts.resync = std::chrono::milliseconds(f.resync_ms);
    ropts.progress_poll = std::chrono::milliseconds(f.progress_ms);
    ropts.credentials_retry = std::chrono::milliseconds(f.cred_retry_ms);
    ropts.quota_fail_open = f.quota_fail_open;

    Informer nodes(client, res::nodes(), "", std::chrono::milliseconds(f.resync_ms));
    Informer mipools(client, res::mi355xpools(), f.ns, std::chrono::milliseconds(f.resync_ms));
    Informer azpools(client, res::azurevmpools(), f.ns, std::chrono::milliseconds(f.resync_ms));
    Informer quotas(client, res::resourcequotas(), f.ns, std::chrono::milliseconds(f.resync_ms));
    // agent Pods (discovery "pod"): only the DaemonSet's pods in its namespace are cached
    InformerOptions agent_pod_opts;
    agent_pod_opts.label_selector = f.agent_selector;
    Informer agent_pods(client, res::pods(), f.agent_namespace, std::chrono::milliseconds(f.resync_ms),
                        agent_pod_opts);
    AgentAccess access = agent_access;
    if (f.agent_discovery == "pod") access.pods = &agent_pods;
    RocmProvider rocm(nodes, f.agent_timeout_ms, access);
    FakeCloudOptions fco;
    fco.provision = std::chrono::milliseconds(f.fakecloud_provision_ms);
    fco.deprovision = std::chrono::milliseconds(f.fakecloud_deprovision_ms);
    fco.state_file = f.fakecloud_state;
    fco.faults_file = f.fakecloud_faults;
    std::unique_ptr<CloudProvider> cloud_impl;
    if (f.cloud == "azure-arm") {
      AzureArmOptions ao;
      if (!f.azure_arm_endpoint.empty()) ao.arm_endpoint = f.azure_arm_endpoint;
      if (!f.azure_authority_host.empty()) ao.authority_host = f.azure_authority_host;
      if (!f.azure_admin_user.empty()) ao.admin_username = f.azure_admin_user;
      ao.tls.ca_file = f.azure_ca_file;
      ao.nic_wait_ms = f.azure_nic_wait_ms;
      if (!f.azure_ssh_key_file.empty()) {
        std::ifstream kf(f.azure_ssh_key_file);
        std::string key((std::istreambuf_iterator<char>(kf)), std::istreambuf_iterator<char>());
        while (!key.empty() && (key.back() == '\n' || key.back() == '\r' || key.back() == ' ')) key.pop_back();
        ao.ssh_public_key = key;
      }
      cloud_impl = std::make_unique<AzureArmProvider>(ao);
    } else {
      cloud_impl = std::make_unique<FakeCloudProvider>(fco);
    }
    CloudProvider& cloud = *cloud_impl;
    // jobs are driven by their own events, their pods' (the pod index below) and their
    // reconciler's requeues: the informer's RESYNC re-delivery is only a drift net, once a minute
    Informer jobs(client, ResourceRef{gen::kGroup, gen::kVersion, gen::kPluralMi355xJob, true, "Mi355xJob"}, f.ns,
                  std::chrono::milliseconds(f.resync_ms) * 6);
    // the cluster's pods, bounded: only pods that request an extended resource or belong to a
    // Mi355xJob are cached, each as a projection of the fields the readers use (podindex.h) —
    // whole pods of every workload in a 50k-pod cluster would not fit the manager's 512 Mi
    InformerOptions pod_opts;
    pod_opts.filter = pod_relevant;
    pod_opts.transform = trim_pod;
    Informer pods(client, res::pods(), "", std::chrono::milliseconds(f.resync_ms), pod_opts);
    PodIndex pod_index;
    pod_index.attach(pods);
    Informer queues(client, res::mi355xqueues(), "", std::chrono::milliseconds(f.resync_ms));
    Mi355xPoolReconciler mi(client, mipools, rocm, &events, ropts);
    Mi355xJobReconciler jr(client, jobs, nodes, &events, ropts, &pod_index);
    Mi355xQueueReconciler qr(client, queues, jobs, &events, ropts);
    Mi355xPoolAutoscaler as(client, mipools, jobs, pods, &events, ropts);
    AzureVmPoolReconciler az(client, azpools, cloud, &events, ropts);
    AgentWatchers watchers(rocm, mipools, ctl);

    // Node events are frequent (every kubelet and agent heartbeat is a status write) and almost
    // never change what placement reads: wake waiting pools / gangs only when one of those facts
    // moved — labels, schedulability, Ready, the agent endpoint, allocatable.
    std::mutex node_fp_mu;
    std::map<std::string, std::string> node_fp;
    auto node_facts_changed = [&](const std::string& type, const Json& n) {
      const std::string name = n.path("metadata.name").as_string();
      std::string fp;
      if (type != "DELETED") {
        std::string ready;
        for (const auto& c : n.path("status.conditions").elements())
          if (c["type"].as_string() == "Ready") ready = c["status"].as_string();
        fp = n.path("metadata.labels").dump() + "|" + (n.path("spec.unschedulable").as_bool(false) ? "U" : "S") + "|" +
             ready + "|" + n.path("metadata.annotations")[gen::kAnnAgentEndpoint].as_string() + "|" +
             n.path("status.allocatable").dump();
      }
      std::lock_guard<std::mutex> g(node_fp_mu);
      auto it = node_fp.find(name);
      const bool changed = it == node_fp.end() || it->second != fp;
      if (type == "DELETED") node_fp.erase(name);
      else node_fp[name] = fp;
      return changed;
    };
    auto count_node_event = [](bool relevant) {
      static CounterVec& c = Registry::global().counter(
          "gpupool_node_events_total", "Node watch events by whether a placement fact changed.");
      c.inc({{"relevant", relevant ? "true" : "false"}});
    };
    // one fingerprint check per event, shared by the pool and job handlers
    std::atomic<bool> node_relevant{false};
    nodes.add_handler([&](const std::string& type, const Json& n) {
      if (type == "RESYNC") return;
      const bool r = node_facts_changed(type, n);
      node_relevant = r;
      count_node_event(r);
    });
    auto pool_handler = [&ctl](const char* kind, PoolReconcilerBase* r = nullptr) {
      return [&ctl, kind, r](const std::string& type, const Json& obj) {
        if (r && type == "MODIFIED" && r->own_status_write(obj)) return;  // our own status write
        ctl.enqueue(kind, obj.path("metadata.namespace").as_string(), obj.path("metadata.name").as_string());
      };
    };
    if (want_mi) {
      ctl.add_reconciler(&mi);
      mipools.add_handler(pool_handler("Mi355xPool", &mi));
      nodes.add_handler([&](const std::string& type, const Json&) {
        if (type == "RESYNC" || !node_relevant) return;
        watchers.sync(rocm.node_names());
        // node/agent changes can unblock pools waiting for devices
        for (const auto& p : mipools.list())
          if (!condition_true(p.path("status.conditions"), gen::kCondReady))
            ctl.enqueue("Mi355xPool", p.path("metadata.namespace").as_string(), p.path("metadata.name").as_string());
      });
      // quota edits can unblock QuotaExceeded pools in that namespace; the cache is optional
      // (not waited for): until it syncs, quota checks fall back to a LIST
      mi.set_quota_informer(&quotas);
      quotas.add_handler([&](const std::string& type, const Json& q) {
        if (type == "RESYNC") return;
        const std::string qns = q.path("metadata.namespace").as_string();
        for (const auto& p : mipools.list())
          if (p.path("metadata.namespace").as_string() == qns &&
              !condition_true(p.path("status.conditions"), gen::kCondReady))
            ctl.enqueue("Mi355xPool", qns, p.path("metadata.name").as_string());
      });
      if (f.agent_discovery == "pod") {
        agent_pods.add_handler([&](const std::string& type, const Json&) {
          if (type == "RESYNC") return;
          watchers.sync(rocm.node_names());  // an agent (re)started: follow its new address
          for (const auto& p : mipools.list())
            if (!condition_true(p.path("status.conditions"), gen::kCondReady))
              ctl.enqueue("Mi355xPool", p.path("metadata.namespace").as_string(), p.path("metadata.name").as_string());
        });
        agent_pods.start();
      }
      nodes.start();
      mipools.start();
      quotas.start();
    }
    if (want_job) {
      ctl.add_reconciler(&jr);
      ctl.add_reconciler(&qr);
      jobs.add_handler(pool_handler("Mi355xJob"));
      // a job's phase or placement changes its queue's status
      jobs.add_handler([&ctl](const std::string& type, const Json& j) {
        (void)type;
        ctl.enqueue("Mi355xQueue", "", j.path("spec.queue").str_or("default"));
      });
      auto wake_pending = [&]() {
        for (const auto& j : jr.pending()) ctl.enqueue("Mi355xJob", j.first, j.second);
      };
      // job pods drive their job; a pod that ends or goes away frees capacity for waiting gangs
      pods.add_handler([&, wake_pending](const std::string& type, const Json& p) {
        if (type == "RESYNC") return;
        const std::string job = p.path("metadata.labels")[gen::kLabelJob].as_string();
        if (!job.empty()) ctl.enqueue("Mi355xJob", p.path("metadata.namespace").as_string(), job);
        const std::string phase = p.path("status.phase").as_string();
        if (type == "DELETED" || phase == "Succeeded" || phase == "Failed") wake_pending();
      });
      nodes.add_handler([wake_pending, &node_relevant](const std::string& type, const Json&) {
        if (type != "RESYNC" && node_relevant) wake_pending();
      });
      // a gang that ends, is suspended or gives its placement back frees GPUs for waiting ones
      jobs.add_handler([wake_pending, &jr](const std::string& type, const Json& j) {
        if (type == "RESYNC") return;
        const std::string ph = j.path("status.phase").str_or("Pending");
        if (type == "DELETED" || ph == "Succeeded" || ph == "Failed" || ph == "Suspended" ||
            (ph == "Restarting" && j.path("status.placement").size() == 0))
          wake_pending();
        else if (j.path("status.placement").size() > 0)  // placed: those queued behind it go next
          jr.wake_blocked_by(j.path("metadata.namespace").as_string(), j.path("metadata.name").as_string());
      });
      // queue edits (created, opened, capability raised) can admit waiting jobs — spec edits
      // only: the queue's status is rewritten on every job change and admits nothing
      auto queue_gen = std::make_shared<std::map<std::string, int64_t>>();
      auto queue_gen_mu = std::make_shared<std::mutex>();
      queues.add_handler([&ctl, wake_pending, queue_gen, queue_gen_mu](const std::string& type, const Json& q) {
        const std::string name = q.path("metadata.name").as_string();
        ctl.enqueue("Mi355xQueue", "", name);
        if (type == "RESYNC") return;
        const int64_t gen = q.path("metadata.generation").as_int(0);
        bool changed;
        {
          std::lock_guard<std::mutex> g(*queue_gen_mu);
          auto it = queue_gen->find(name);
          changed = type != "MODIFIED" || it == queue_gen->end() || it->second != gen;
          if (type == "DELETED") queue_gen->erase(name);
          else (*queue_gen)[name] = gen;
        }
        if (changed) wake_pending();
      });
      jr.set_waker([&ctl](const std::string& ns, const std::string& name) { ctl.enqueue("Mi355xJob", ns, name); });
      // pool changes (GPUs advertised or released) change capacity too
      mipools.add_handler([wake_pending](const std::string& type, const Json&) {
        if (type != "RESYNC") wake_pending();
      });
      // demand-driven pools: re-evaluated on their own edits and whenever pods or jobs change
      if (want_mi) {
        ctl.add_reconciler(&as);
        mipools.add_handler([&ctl](const std::string& type, const Json& p) {
          (void)type;
          if (p.path("spec.autoscale.enabled").as_bool(false))
            ctl.enqueue("Mi355xPoolAutoscale", p.path("metadata.namespace").as_string(),
                        p.path("metadata.name").as_string());
        });
        auto wake_autoscaled = [&ctl, &as](const std::string& type, const Json&) {
          if (type == "RESYNC") return;
          for (const auto& p : as.autoscaled()) ctl.enqueue("Mi355xPoolAutoscale", p.first, p.second);
        };
        pods.add_handler(wake_autoscaled);
        jobs.add_handler(wake_autoscaled);
      }
      if (!want_mi) {
        nodes.start();
        mipools.start();
      }
      jobs.start();
      pods.start();
      queues.start();
    }
    if (want_mi && !want_job)
      log.warn("pool autoscaling (spec.autoscale) is off: it needs the job controller's pod and job caches",
               Json::object().set("kinds", f.kinds).set("hint", "add 'job' to --kinds"));
    if (want_az) {
      ctl.add_reconciler(&az);
      azpools.add_handler(pool_handler("AzureVmPool", &az));
      azpools.start();
    }
    // Workers start only on synced caches (controller-runtime WaitForCacheSync); the wait is sliced
    // so SIGTERM during an unreachable/untrusted apiserver still exits promptly.
    auto wait_cache = [&](Informer& inf, const char* what) {
      auto warn_at = std::chrono::steady_clock::now() + std::chrono::seconds(30);
      while (!g_stop && !inf.wait_synced(std::chrono::milliseconds(100))) {
        if (std::chrono::steady_clock::now() > warn_at) {
          log.warn("waiting for informer cache sync", Json::object().set("resource", what));
          warn_at = std::chrono::steady_clock::now() + std::chrono::seconds(30);
        }
      }
    };
    if (want_mi) {
      wait_cache(nodes, "nodes");
      wait_cache(mipools, "mi355xpools");
      if (f.agent_discovery == "pod") wait_cache(agent_pods, "agent pods");
    }
    if (want_az) wait_cache(azpools, "azurevmpools");
    if (want_job) {
      wait_cache(jobs, "mi355xjobs");
      wait_cache(pods, "pods");
      wait_cache(queues, "mi355xqueues");
    }
    if (!g_stop) {
      if (want_mi) watchers.sync(rocm.node_names());
      ctl.start();
      log.info("controllers running", Json());
    }
    auto last_sweep = std::chrono::steady_clock::now();
    GaugeVec& depth = Registry::global().gauge("gpupool_workqueue_depth", "Ready keys in the work queue.");
    GaugeVec& cred = Registry::global().gauge(
        "gpupool_credential_reloads", "Times a rotating credential file was re-read with a new value.");
    while (!g_stop && leading) {
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      depth.set({}, static_cast<double>(ctl.queue().len()));
      if (api_tokens) cred.set({{"credential", "apiserver-token"}}, static_cast<double>(api_tokens->reloads()));
      if (agent_access.token)
        cred.set({{"credential", "agent-token"}}, static_cast<double>(agent_access.token->reloads()));
      if (agent_access.signer)
        cred.set({{"credential", "agent-signing-key"}}, static_cast<double>(agent_access.signer->reloads()));
      if (want_mi && std::chrono::steady_clock::now() - last_sweep > std::chrono::milliseconds(f.orphan_sweep_ms)) {
        last_sweep = std::chrono::steady_clock::now();
        try {
          for (const auto& key : mi.sweep_orphans()) ctl.enqueue("Mi355xPool", key.first, key.second);
        } catch (const std::exception& e) {
          log.warn("orphan sweep failed", Json::object().set("error", e.what()));
        }
      }
    }
    log.info("stopping controllers", Json());
    ctl.stop();
    watchers.stop_all();
    jobs.stop();
    pods.stop();
    queues.stop();
    mipools.stop();
    azpools.stop();
    quotas.stop();
    nodes.stop();
    agent_pods.stop();
    events.flush(std::chrono::milliseconds(2000));
  };

  std::thread le_thread;
  std::atomic<bool> lost{false};
  if (f.leader_elect) {
    // Lease election runs beside the controllers: they start once we lead and stop (and the
    // process exits non-zero, like controller-runtime) if the lease is lost.
    le_thread = std::thread([&] {
      LeaderConfig lc;
      lc.ns = f.lease_ns;
      lc.identity = f.identity;
      lc.lease_duration = std::chrono::milliseconds(f.lease_duration_ms);
      lc.renew_deadline = std::chrono::milliseconds(f.renew_deadline_ms);
      lc.retry_period = std::chrono::milliseconds(f.retry_period_ms);
      LeaderElector le(client, lc);
      le.run([&] { leading = true; },
             [&] {
               if (leading) lost = true;
               leading = false;
             },
             &g_stop);
    });
    while (!g_stop && !leading) std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  if (leading) run_controllers();
  g_stop = true;
  if (le_thread.joinable()) le_thread.join();
  metrics.stop();
  log.info("exited", Json::object().set("lostLeadership", lost.load()));
  return lost ? 1 : 0;
}
