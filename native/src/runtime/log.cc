#include "gpupool/log.h"

#include "gpupool/trace.h"

#include <cstdio>
#include <ctime>

namespace gpupool {

std::atomic<int> Logger::level_{static_cast<int>(LogLevel::Info)};
std::mutex Logger::mu_;

Logger Logger::with(const std::string& key, Json value) const {
  Logger l = *this;
  l.ctx_[key] = std::move(value);
  return l;
}

Logger Logger::named(const std::string& sub) const {
  Logger l = *this;
  l.name_ = name_.empty() ? sub : name_ + "." + sub;
  return l;
}

LogLevel Logger::parse_level(const std::string& s) {
  if (s == "debug") return LogLevel::Debug;
  if (s == "warn" || s == "warning") return LogLevel::Warn;
  if (s == "error") return LogLevel::Error;
  return LogLevel::Info;
}

void Logger::log(LogLevel lvl, const std::string& msg, Json fields) const {
  if (static_cast<int>(lvl) < level_.load()) return;
  static const char* names[] = {"debug", "info", "warn", "error"};
  Json rec = Json::object();
  auto now = std::chrono::system_clock::now();
  double ts = std::chrono::duration<double>(now.time_since_epoch()).count();
  rec["ts"] = ts;
  rec["level"] = names[static_cast<int>(lvl)];
  rec["logger"] = name_;
  rec["msg"] = msg;
  // every line logged inside a reconcile pass carries that pass's reconcileID
  if (trace::Trace* t = trace::Trace::current()) rec["reconcileID"] = t->id();
  for (const auto& kv : ctx_.members()) rec[kv.first] = kv.second;
  for (const auto& kv : fields.members()) rec[kv.first] = kv.second;
  std::string line = rec.dump();
  line.push_back('\n');
  std::lock_guard<std::mutex> g(mu_);
  std::fwrite(line.data(), 1, line.size(), stderr);
  std::fflush(stderr);
}

std::string rfc3339(std::chrono::system_clock::time_point t) {
  std::time_t tt = std::chrono::system_clock::to_time_t(t);
  std::tm tm{};
  gmtime_r(&tt, &tm);
  char buf[32];
  std::strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%SZ", &tm);
  return buf;
}

std::string rfc3339_now() { return rfc3339(std::chrono::system_clock::now()); }

std::string microtime_now() {
  auto now = std::chrono::system_clock::now();
  std::time_t tt = std::chrono::system_clock::to_time_t(now);
  auto us = std::chrono::duration_cast<std::chrono::microseconds>(now.time_since_epoch()).count() % 1000000;
  std::tm tm{};
  gmtime_r(&tt, &tm);
  char buf[48];
  std::strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%S", &tm);
  char out[64];
  std::snprintf(out, sizeof out, "%s.%06lldZ", buf, static_cast<long long>(us));
  return out;
}

bool parse_rfc3339(const std::string& s, std::chrono::system_clock::time_point* out) {
  std::tm tm{};
  int y, mo, d, h, mi;
  double sec;
  if (std::sscanf(s.c_str(), "%d-%d-%dT%d:%d:%lf", &y, &mo, &d, &h, &mi, &sec) != 6) return false;
  tm.tm_year = y - 1900;
  tm.tm_mon = mo - 1;
  tm.tm_mday = d;
  tm.tm_hour = h;
  tm.tm_min = mi;
  tm.tm_sec = static_cast<int>(sec);
  std::time_t tt = timegm(&tm);
  if (tt == static_cast<std::time_t>(-1)) return false;
  auto frac = std::chrono::microseconds(static_cast<long long>((sec - static_cast<int>(sec)) * 1e6));
  *out = std::chrono::system_clock::from_time_t(tt) + frac;
  return true;
}

}  // namespace gpupool
