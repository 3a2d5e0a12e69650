// Tiny self-registering test framework (no gtest in this image).
#pragma once

#include <cstdio>
#include <functional>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace gtest_lite {

struct Case {
  const char* name;
  std::function<void()> fn;
};

inline std::vector<Case>& registry() {
  static std::vector<Case> r;
  return r;
}

struct Reg {
  Reg(const char* n, std::function<void()> f) { registry().push_back({n, std::move(f)}); }
};

struct Failure : std::runtime_error {
  using std::runtime_error::runtime_error;
};

}  // namespace gtest_lite

#define TEST(name)                                                      \
  static void test_##name();                                            \
  static gtest_lite::Reg reg_##name(#name, test_##name);                \
  static void test_##name()

#define EXPECT_TRUE(c)                                                                                     \
  do {                                                                                                     \
    if (!(c)) {                                                                                            \
      std::ostringstream os_;                                                                              \
      os_ << __FILE__ << ":" << __LINE__ << ": expected true: " #c;                                        \
      throw gtest_lite::Failure(os_.str());                                                                \
    }                                                                                                      \
  } while (0)

#define EXPECT_EQ(a, b)                                                                                    \
  do {                                                                                                     \
    auto va_ = (a);                                                                                        \
    auto vb_ = (b);                                                                                        \
    if (!(va_ == vb_)) {                                                                                   \
      std::ostringstream os_;                                                                              \
      os_ << __FILE__ << ":" << __LINE__ << ": expected " #a " == " #b " (" << va_ << " vs " << vb_ << ")"; \
      throw gtest_lite::Failure(os_.str());                                                                \
    }                                                                                                      \
  } while (0)

#define EXPECT_THROW(stmt)                                                         \
  do {                                                                             \
    bool threw_ = false;                                                           \
    try {                                                                          \
      stmt;                                                                        \
    } catch (...) {                                                                \
      threw_ = true;                                                               \
    }                                                                              \
    if (!threw_) {                                                                 \
      std::ostringstream os_;                                                      \
      os_ << __FILE__ << ":" << __LINE__ << ": expected exception from " #stmt;    \
      throw gtest_lite::Failure(os_.str());                                        \
    }                                                                              \
  } while (0)
