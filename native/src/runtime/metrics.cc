#include "gpupool/metrics.h"

#include <dirent.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>

namespace gpupool {

namespace {
std::string fmt(double v) {
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  char buf[64];
  std::snprintf(buf, sizeof buf, "%.17g", v);
  return buf;
}
std::string esc(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '\\' || c == '"') o.push_back('\\');
    if (c == '\n') {
      o += "\\n";
      continue;
    }
    o.push_back(c);
  }
  return o;
}
}  // namespace

std::string Metric::label_str(const Labels& l, const std::string& ek, const std::string& ev) {
  if (l.empty() && ek.empty()) return "";
  std::string s = "{";
  bool first = true;
  for (const auto& kv : l) {
    if (!first) s += ",";
    first = false;
    s += kv.first + "=\"" + esc(kv.second) + "\"";
  }
  if (!ek.empty()) {
    if (!first) s += ",";
    s += ek + "=\"" + ev + "\"";
  }
  return s + "}";
}

void CounterVec::inc(const Labels& l, double v) {
  std::lock_guard<std::mutex> g(mu_);
  vals_[l] += v;
}
double CounterVec::get(const Labels& l) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = vals_.find(l);
  return it == vals_.end() ? 0 : it->second;
}
void CounterVec::render(std::string& out) const {
  std::lock_guard<std::mutex> g(mu_);
  out += "# HELP " + name_ + " " + help_ + "\n# TYPE " + name_ + " counter\n";
  for (const auto& kv : vals_) out += name_ + label_str(kv.first) + " " + fmt(kv.second) + "\n";
}

void GaugeVec::set(const Labels& l, double v) {
  std::lock_guard<std::mutex> g(mu_);
  vals_[l] = v;
}
void GaugeVec::erase(const Labels& l) {
  std::lock_guard<std::mutex> g(mu_);
  vals_.erase(l);
}
double GaugeVec::get(const Labels& l) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = vals_.find(l);
  return it == vals_.end() ? 0 : it->second;
}
void GaugeVec::render(std::string& out) const {
  std::lock_guard<std::mutex> g(mu_);
  out += "# HELP " + name_ + " " + help_ + "\n# TYPE " + name_ + " gauge\n";
  for (const auto& kv : vals_) out += name_ + label_str(kv.first) + " " + fmt(kv.second) + "\n";
}

void HistogramVec::observe(const Labels& l, double v) {
  std::lock_guard<std::mutex> g(mu_);
  Series& s = series_[l];
  if (s.counts.empty()) s.counts.assign(buckets_.size(), 0);
  for (size_t i = 0; i < buckets_.size(); ++i)
    if (v <= buckets_[i]) s.counts[i]++;
  s.sum += v;
  s.n++;
}

uint64_t HistogramVec::count(const Labels& l) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = series_.find(l);
  return it == series_.end() ? 0 : it->second.n;
}

double HistogramVec::quantile(const Labels& l, double q) const {
  std::lock_guard<std::mutex> g(mu_);
  auto it = series_.find(l);
  if (it == series_.end() || it->second.n == 0) return NAN;
  const Series& s = it->second;
  double rank = q * static_cast<double>(s.n);
  double prev_b = 0;
  uint64_t prev_c = 0;
  for (size_t i = 0; i < buckets_.size(); ++i) {
    if (static_cast<double>(s.counts[i]) >= rank) {
      uint64_t in_bucket = s.counts[i] - prev_c;
      if (in_bucket == 0) return buckets_[i];
      return prev_b + (buckets_[i] - prev_b) * (rank - static_cast<double>(prev_c)) /
                          static_cast<double>(in_bucket);
    }
    prev_b = buckets_[i];
    prev_c = s.counts[i];
  }
  return buckets_.empty() ? NAN : buckets_.back();
}

void HistogramVec::render(std::string& out) const {
  std::lock_guard<std::mutex> g(mu_);
  out += "# HELP " + name_ + " " + help_ + "\n# TYPE " + name_ + " histogram\n";
  for (const auto& kv : series_) {
    for (size_t i = 0; i < buckets_.size(); ++i)
      out += name_ + "_bucket" + label_str(kv.first, "le", fmt(buckets_[i])) + " " +
             std::to_string(kv.second.counts[i]) + "\n";
    out += name_ + "_bucket" + label_str(kv.first, "le", "+Inf") + " " + std::to_string(kv.second.n) + "\n";
    out += name_ + "_sum" + label_str(kv.first) + " " + fmt(kv.second.sum) + "\n";
    out += name_ + "_count" + label_str(kv.first) + " " + std::to_string(kv.second.n) + "\n";
  }
}

Registry& Registry::global() {
  static Registry r;
  return r;
}

CounterVec& Registry::counter(const std::string& name, const std::string& help) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = by_name_.find(name);
  if (it != by_name_.end()) return dynamic_cast<CounterVec&>(*it->second);
  metrics_.push_back(std::make_unique<CounterVec>(name, help));
  by_name_[name] = metrics_.back().get();
  return static_cast<CounterVec&>(*metrics_.back());
}

GaugeVec& Registry::gauge(const std::string& name, const std::string& help) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = by_name_.find(name);
  if (it != by_name_.end()) return dynamic_cast<GaugeVec&>(*it->second);
  metrics_.push_back(std::make_unique<GaugeVec>(name, help));
  by_name_[name] = metrics_.back().get();
  return static_cast<GaugeVec&>(*metrics_.back());
}

HistogramVec& Registry::histogram(const std::string& name, const std::string& help,
                                  std::vector<double> buckets) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = by_name_.find(name);
  if (it != by_name_.end()) return dynamic_cast<HistogramVec&>(*it->second);
  metrics_.push_back(std::make_unique<HistogramVec>(name, help, std::move(buckets)));
  by_name_[name] = metrics_.back().get();
  return static_cast<HistogramVec&>(*metrics_.back());
}

// Prometheus' standard process metrics (the client libraries' process collector) from /proc/self:
// resident memory, CPU time, threads and open file descriptors — a leak or a thread pile-up in a
// long-running manager shows on the dashboard before it shows as an outage.
static void render_process(std::string& out) {
  long pages = 0, resident = 0;
  if (FILE* f = std::fopen("/proc/self/statm", "r")) {
    if (std::fscanf(f, "%ld %ld", &pages, &resident) != 2) resident = 0;
    std::fclose(f);
  }
  double cpu_s = 0;
  long threads = 0;
  if (FILE* f = std::fopen("/proc/self/stat", "r")) {
    char buf[2048];
    size_t n = std::fread(buf, 1, sizeof buf - 1, f);
    std::fclose(f);
    buf[n] = 0;
    if (const char* p = std::strrchr(buf, ')')) {  // fields restart after the command name
      unsigned long utime = 0, stime = 0;
      long nthreads = 0;
      // state ppid pgrp session tty tpgid flags minflt cminflt majflt cmajflt utime stime cutime cstime
      // priority nice num_threads
      if (std::sscanf(p + 2, "%*c %*d %*d %*d %*d %*d %*u %*u %*u %*u %*u %lu %lu %*d %*d %*d %*d %ld",
                      &utime, &stime, &nthreads) == 3) {
        cpu_s = static_cast<double>(utime + stime) / static_cast<double>(sysconf(_SC_CLK_TCK));
        threads = nthreads;
      }
    }
  }
  long fds = 0;
  if (DIR* d = opendir("/proc/self/fd")) {
    while (struct dirent* e = readdir(d))
      if (e->d_name[0] != '.') ++fds;
    closedir(d);
  }
  char line[512];
  std::snprintf(line, sizeof line,
                "# TYPE process_resident_memory_bytes gauge\nprocess_resident_memory_bytes %ld\n"
                "# TYPE process_cpu_seconds_total counter\nprocess_cpu_seconds_total %.3f\n"
                "# TYPE process_threads gauge\nprocess_threads %ld\n"
                "# TYPE process_open_fds gauge\nprocess_open_fds %ld\n",
                resident * sysconf(_SC_PAGESIZE), cpu_s, threads, fds);
  out += line;
}

std::string Registry::render() const {
  std::lock_guard<std::mutex> g(mu_);
  std::string out;
  for (const auto& m : metrics_) m->render(out);
  render_process(out);
  return out;
}

std::vector<double> exponential_buckets(double start, double factor, int count) {
  std::vector<double> b;
  double v = start;
  for (int i = 0; i < count; ++i) {
    b.push_back(v);
    v *= factor;
  }
  return b;
}

}  // namespace gpupool
