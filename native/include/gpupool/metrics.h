// Prometheus text-format metrics registry (manager /metrics; SURVEY.md §5 observability row).
#pragma once

#include <atomic>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace gpupool {

using Labels = std::map<std::string, std::string>;

class Metric {
 public:
  Metric(std::string name, std::string help, std::string type)
      : name_(std::move(name)), help_(std::move(help)), type_(std::move(type)) {}
  virtual ~Metric() = default;
  virtual void render(std::string& out) const = 0;
  const std::string& name() const { return name_; }

 protected:
  static std::string label_str(const Labels& l, const std::string& extra_k = "",
                               const std::string& extra_v = "");
  std::string name_, help_, type_;
};

class CounterVec : public Metric {
 public:
  CounterVec(std::string name, std::string help) : Metric(std::move(name), std::move(help), "counter") {}
  void inc(const Labels& l = {}, double v = 1);
  double get(const Labels& l = {}) const;
  void render(std::string& out) const override;

 private:
  mutable std::mutex mu_;
  std::map<Labels, double> vals_;
};

class GaugeVec : public Metric {
 public:
  GaugeVec(std::string name, std::string help) : Metric(std::move(name), std::move(help), "gauge") {}
  void set(const Labels& l, double v);
  void erase(const Labels& l);
  double get(const Labels& l = {}) const;
  void render(std::string& out) const override;

 private:
  mutable std::mutex mu_;
  std::map<Labels, double> vals_;
};

class HistogramVec : public Metric {
 public:
  HistogramVec(std::string name, std::string help, std::vector<double> buckets)
      : Metric(std::move(name), std::move(help), "histogram"), buckets_(std::move(buckets)) {}
  void observe(const Labels& l, double v);
  // Quantile estimate (linear interpolation within buckets), for logs/tests.
  double quantile(const Labels& l, double q) const;
  uint64_t count(const Labels& l = {}) const;
  void render(std::string& out) const override;

 private:
  struct Series {
    std::vector<uint64_t> counts;
    double sum = 0;
    uint64_t n = 0;
  };
  std::vector<double> buckets_;
  mutable std::mutex mu_;
  std::map<Labels, Series> series_;
};

class Registry {
 public:
  static Registry& global();
  CounterVec& counter(const std::string& name, const std::string& help);
  GaugeVec& gauge(const std::string& name, const std::string& help);
  HistogramVec& histogram(const std::string& name, const std::string& help,
                          std::vector<double> buckets);
  std::string render() const;

 private:
  mutable std::mutex mu_;
  std::vector<std::unique_ptr<Metric>> metrics_;
  std::map<std::string, Metric*> by_name_;
};

std::vector<double> exponential_buckets(double start, double factor, int count);

}  // namespace gpupool
