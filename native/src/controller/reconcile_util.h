// Internal helpers shared by the pool reconcilers (reconciler.cc, mi355x_pool.cc,
// azure_pool.cc): metric families and small formatting helpers. Not part of the public API.
#pragma once

#include <chrono>
#include <string>
#include <vector>

#include "gpupool/metrics.h"
#include "gpupool/reconciler.h"

namespace gpupool {
namespace recutil {

using clock_t_ = std::chrono::steady_clock;
using ms = std::chrono::milliseconds;

std::string join(const std::vector<std::string>& v, const char* sep);
std::string short_id(const DeviceView& d);
HistogramVec& reconcile_hist();
HistogramVec& to_ready_hist();
CounterVec& reconcile_total();
GaugeVec& ready_gauge();
GaugeVec& quota_gauge();
GaugeVec& desired_gauge();
// pool-level GPU utilisation from the agents' telemetry of the pool's claimed GPUs
void set_util_gauges(const Labels& l, const std::vector<DeviceView>& mine);
void erase_util_gauges(const Labels& l);

}  // namespace recutil
}  // namespace gpupool
