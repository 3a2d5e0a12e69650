// C ABI of libmi355x_dev (see native/include/mi355x/dev.h).
#include <poll.h>
#include <sys/inotify.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>

#include "mi355x/dev.h"
#include "model.h"

using gpupool::Json;

struct mi355x_dev {
  std::unique_ptr<mi355x::Backend> backend;
  std::string faults_path;
  Json faults;
  time_t faults_mtime = 0;
  long faults_mtime_ns = 0;
  ino_t faults_ino = 0;
  std::string node;
  std::mutex mu;
  // fault-overlay watch (mi355x_dev_wait_faults): inotify on the overlay's directory
  std::mutex wmu;
  int ino_fd = -1;
  ~mi355x_dev() {
    if (ino_fd >= 0) close(ino_fd);
  }
};

namespace {

char* dup(const std::string& s) {
  char* p = static_cast<char*>(std::malloc(s.size() + 1));
  if (!p) return nullptr;
  std::memcpy(p, s.c_str(), s.size() + 1);
  return p;
}

void set_err(char* err, size_t n, const std::string& msg) {
  if (!err || n == 0) return;
  std::snprintf(err, n, "%s", msg.c_str());
}

void reload_faults(mi355x_dev* d) {
  if (d->faults_path.empty()) return;
  struct stat st {};
  if (stat(d->faults_path.c_str(), &st) != 0) {
    d->faults = Json();  // file removed -> faults cleared
    d->faults_mtime = 0;
    return;
  }
  // a replaced file (rename into place) is a new inode even within one mtime tick
  if (st.st_mtim.tv_sec == d->faults_mtime && st.st_mtim.tv_nsec == d->faults_mtime_ns && st.st_ino == d->faults_ino)
    return;
  std::ifstream f(d->faults_path);
  std::stringstream ss;
  ss << f.rdbuf();
  auto j = Json::try_parse(ss.str());
  if (j) {
    d->faults = *j;
    d->faults_mtime = st.st_mtim.tv_sec;
    d->faults_mtime_ns = st.st_mtim.tv_nsec;
    d->faults_ino = st.st_ino;
  }
}

}  // namespace

extern "C" {

mi355x_dev* mi355x_dev_open(const char* backend, const char* config_json, char* err, size_t errlen) {
  try {
    Json cfg = config_json && *config_json ? Json::parse(config_json) : Json::object();
    std::string b = backend ? backend : "auto";
    auto d = std::make_unique<mi355x_dev>();
    if (b == "fake") {
      d->backend = mi355x::make_fake_backend(cfg);
    } else if (b == "amdsmi") {
      d->backend = mi355x::make_amdsmi_backend(cfg);
    } else if (b == "cli") {
      d->backend = mi355x::make_cli_backend(cfg);
    } else if (b == "auto") {
      d->backend = mi355x::make_amdsmi_backend(cfg);
    } else {
      set_err(err, errlen, "unknown backend: " + b);
      return nullptr;
    }
    d->faults_path = cfg["faults"].as_string();
    d->node = cfg["node"].as_string();
    return d.release();
  } catch (const std::exception& e) {
    set_err(err, errlen, e.what());
    return nullptr;
  }
}

void mi355x_dev_close(mi355x_dev* d) { delete d; }

char* mi355x_dev_snapshot(mi355x_dev* d) {
  if (!d) return nullptr;
  std::lock_guard<std::mutex> g(d->mu);
  try {
    Json s = d->backend->snapshot();
    if (!d->node.empty()) s["node"] = d->node;
    s["ts"] = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
    reload_faults(d);
    if (d->faults.is_object()) mi355x::apply_overlay(s, d->faults);
    return dup(s.dump());
  } catch (const std::exception& e) {
    Json errj = Json::object();
    errj["error"] = e.what();
    return dup(errj.dump());
  }
}

char* mi355x_dev_health_snapshot(mi355x_dev* d) {
  if (!d) return nullptr;
  std::lock_guard<std::mutex> g(d->mu);
  try {
    Json s = d->backend->health_snapshot();
    if (!d->node.empty()) s["node"] = d->node;
    reload_faults(d);
    if (d->faults.is_object()) mi355x::apply_overlay(s, d->faults);
    return dup(s.dump());
  } catch (const std::exception& e) {
    Json errj = Json::object();
    errj["error"] = e.what();
    return dup(errj.dump());
  }
}

char* mi355x_dev_evaluate(const char* device_json, const char* baseline_json, const char* policy_json) {
  try {
    Json dev = Json::parse(device_json ? device_json : "{}");
    Json base = baseline_json && *baseline_json ? Json::parse(baseline_json) : Json::object();
    Json pol = policy_json && *policy_json ? Json::parse(policy_json) : Json::object();
    return dup(mi355x::evaluate(dev, base, pol).dump());
  } catch (const std::exception& e) {
    Json errj = Json::object();
    errj["error"] = e.what();
    errj["healthy"] = false;
    return dup(errj.dump());
  }
}

char* mi355x_dev_evaluate_batch(const char* items_json) {
  try {
    Json items = Json::parse(items_json ? items_json : "[]");
    Json out = Json::array();
    const Json empty = Json::object();
    for (const auto& it : items.elements()) {
      const Json& base = it["baseline"].is_object() ? it["baseline"] : it["device"];
      out.push_back(mi355x::evaluate(it["device"], base, it["policy"].is_object() ? it["policy"] : empty));
    }
    return dup(out.dump());
  } catch (const std::exception& e) {
    Json errj = Json::object();
    errj["error"] = e.what();
    return dup(errj.dump());
  }
}

char* mi355x_dev_select(const char* request_json) {
  try {
    Json req = Json::parse(request_json ? request_json : "{}");
    Json out = Json::object();
    Json sel = Json::array();
    for (int i : mi355x::select_devices(req)) sel.push_back(i);
    out["selected"] = sel;
    return dup(out.dump());
  } catch (const std::exception& e) {
    Json errj = Json::object();
    errj["error"] = e.what();
    errj["selected"] = Json::array();
    return dup(errj.dump());
  }
}

char* mi355x_dev_wait_events(mi355x_dev* d, int timeout_ms) {
  if (!d) return nullptr;
  try {
    return dup(d->backend->wait_events(timeout_ms).dump());
  } catch (const std::exception& e) {
    Json errj = Json::object();
    errj["supported"] = false;
    errj["events"] = Json::array();
    errj["error"] = e.what();
    return dup(errj.dump());
  }
}

char* mi355x_dev_wait_faults(mi355x_dev* d, int timeout_ms) {
  if (!d) return nullptr;
  std::lock_guard<std::mutex> g(d->wmu);
  Json out = Json::object();
  out["supported"] = !d->faults_path.empty();
  out["changed"] = false;
  if (d->faults_path.empty()) return dup(out.dump());
  std::string dir = ".", base = d->faults_path;
  size_t slash = d->faults_path.rfind('/');
  if (slash != std::string::npos) {
    dir = slash ? d->faults_path.substr(0, slash) : "/";
    base = d->faults_path.substr(slash + 1);
  }
  if (d->ino_fd < 0) {
    d->ino_fd = inotify_init1(IN_NONBLOCK | IN_CLOEXEC);
    if (d->ino_fd < 0 || inotify_add_watch(d->ino_fd, dir.c_str(), IN_CLOSE_WRITE | IN_MOVED_TO | IN_DELETE) < 0) {
      if (d->ino_fd >= 0) close(d->ino_fd);
      d->ino_fd = -1;
      out["supported"] = false;
      out["error"] = "inotify on " + dir + " failed";
      return dup(out.dump());
    }
  }
  // other files of the directory (e.g. the writer's temp file) wake the poll too: keep waiting
  // for the overlay itself until the deadline
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  bool changed = false;
  while (!changed) {
    const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - std::chrono::steady_clock::now());
    if (left.count() < 0) break;
    struct pollfd pfd {d->ino_fd, POLLIN, 0};
    if (poll(&pfd, 1, static_cast<int>(left.count())) <= 0 || !(pfd.revents & POLLIN)) break;
    alignas(struct inotify_event) char buf[8192];
    ssize_t n;
    while ((n = read(d->ino_fd, buf, sizeof buf)) > 0) {
      for (char* p = buf; p < buf + n;) {
        auto* ev = reinterpret_cast<struct inotify_event*>(p);
        if (ev->len && base == ev->name) changed = true;
        p += sizeof(struct inotify_event) + ev->len;
      }
    }
  }
  out["changed"] = changed;
  return dup(out.dump());
}

void mi355x_free(char* p) { std::free(p); }

const char* mi355x_dev_version(void) { return "mi355x_dev 0.1.0 (gfx950)"; }

}  // extern "C"
