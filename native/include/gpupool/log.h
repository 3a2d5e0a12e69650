// Structured JSON-lines logging (the controller-runtime ``log.FromContext`` analogue,
// README.md:171). One line per record: {"ts","level","logger","msg", ...fields}.
#pragma once

#include <atomic>
#include <chrono>
#include <mutex>
#include <string>

#include "gpupool/json.h"

namespace gpupool {

enum class LogLevel { Debug = 0, Info = 1, Warn = 2, Error = 3 };

class Logger {
 public:
  explicit Logger(std::string name) : name_(std::move(name)) {}
  Logger with(const std::string& key, Json value) const;
  Logger named(const std::string& sub) const;

  void debug(const std::string& msg, Json fields = Json()) const { log(LogLevel::Debug, msg, std::move(fields)); }
  void info(const std::string& msg, Json fields = Json()) const { log(LogLevel::Info, msg, std::move(fields)); }
  void warn(const std::string& msg, Json fields = Json()) const { log(LogLevel::Warn, msg, std::move(fields)); }
  void error(const std::string& msg, Json fields = Json()) const { log(LogLevel::Error, msg, std::move(fields)); }
  void log(LogLevel lvl, const std::string& msg, Json fields) const;

  static void set_level(LogLevel l) { level_.store(static_cast<int>(l)); }
  static LogLevel parse_level(const std::string& s);

 private:
  std::string name_;
  Json ctx_ = Json::object();
  static std::atomic<int> level_;
  static std::mutex mu_;
};

// RFC3339 UTC "2006-01-02T15:04:05Z" and MicroTime "2006-01-02T15:04:05.000000Z".
std::string rfc3339_now();
std::string rfc3339(std::chrono::system_clock::time_point t);
std::string microtime_now();
// Parses both forms; returns false on failure.
bool parse_rfc3339(const std::string& s, std::chrono::system_clock::time_point* out);

}  // namespace gpupool
