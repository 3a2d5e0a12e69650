// Backend-independent device model: health evaluation, selection, fault overlay.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "gpupool/json.h"

namespace mi355x {

using gpupool::Json;

class Backend {
 public:
  virtual ~Backend() = default;
  virtual std::string name() const = 0;
  // Node snapshot without fault overlay applied.
  virtual Json snapshot() = 0;
  // Asynchronous device events (amdsmi event notification: thermal throttle, GPU pre/post reset,
  // VM fault). Blocks up to timeout_ms; returns {"supported": bool, "events": [{index, type,
  // message}]}. Backends without an event source report supported=false at once.
  virtual Json wait_events(int timeout_ms);
  // The fields health verdicts depend on (ECC counts, xGMI link state, current temperatures,
  // presence), cheap enough to poll ~10x per second; the full snapshot adds telemetry, RAS bad
  // pages and partition state. Default: the full snapshot.
  virtual Json health_snapshot() { return snapshot(); }
};

std::unique_ptr<Backend> make_fake_backend(const Json& cfg);     // throws std::runtime_error
std::unique_ptr<Backend> make_amdsmi_backend(const Json& cfg);   // throws std::runtime_error
std::unique_ptr<Backend> make_cli_backend(const Json& cfg);      // throws std::runtime_error

// Deep-merge a fault overlay {"devices": {"<uuid|index>": {...}}} into a node snapshot.
void apply_overlay(Json& snapshot, const Json& overlay);

// Health verdict (see dev.h).
Json evaluate(const Json& dev, const Json& baseline, const Json& policy);

// Selection (see dev.h); returns empty when fewer than count candidates.
std::vector<int> select_devices(const Json& req);

// Count xGMI links in state 'U' and 'D' from a links array of "U"/"D"/"X" entries.
void count_links(const Json& links, int* up, int* down);

// Deep merge helper (objects merge recursively; other values replace).
void deep_merge(Json& dst, const Json& src);

}  // namespace mi355x
