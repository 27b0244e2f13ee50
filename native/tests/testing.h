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
