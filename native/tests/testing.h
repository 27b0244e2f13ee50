// Minimal test registry for the native unit tests (run by tests/test_native.py).
#pragma once

#include <cstdio>
#include <functional>
#include <string>
#include <vector>

namespace p2pt::testing {

struct Case {
  const char* name;
  std::function<void()> fn;
};
std::vector<Case>& registry();
struct Reg {
  Reg(const char* n, std::function<void()> f) { registry().push_back({n, std::move(f)}); }
};
extern int g_failures;
void fail(const char* file, int line, const std::string& msg);

}  // namespace p2pt::testing

// Sanitizer builds run several times slower: checks on wall-clock-sensitive
// outcomes (drop shares under a rate-limited link, throughputs) only hold in
// plain builds. kTimingChecks gates them; the behaviour checks always run.
#if defined(__SANITIZE_THREAD__) || defined(__SANITIZE_ADDRESS__)
constexpr bool kTimingChecks = false;
#elif defined(__has_feature)
#if __has_feature(thread_sanitizer) || __has_feature(address_sanitizer)
constexpr bool kTimingChecks = false;
#else
constexpr bool kTimingChecks = true;
#endif
#else
constexpr bool kTimingChecks = true;
#endif

#define TEST(name)                                                         \
  static void test_##name();                                               \
  static ::p2pt::testing::Reg reg_##name(#name, test_##name);              \
  static void test_##name()

#define CHECK(cond)                                                                        \
  do {                                                                                     \
    if (!(cond)) ::p2pt::testing::fail(__FILE__, __LINE__, "CHECK(" #cond ") failed");     \
  } while (0)

#define CHECK_EQ(a, b)                                                                              \
  do {                                                                                              \
    auto _va = (a);                                                                                 \
    auto _vb = (b);                                                                                 \
    if (!(_va == _vb)) ::p2pt::testing::fail(__FILE__, __LINE__, "CHECK_EQ(" #a ", " #b ") failed"); \
  } while (0)
