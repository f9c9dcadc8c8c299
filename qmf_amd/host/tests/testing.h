// Minimal test harness for the host library (gtest is not part of this image).
// TEST(Suite, Name) registers a case; EXPECT_* record failures; EXPECT_DEATH forks.
#pragma once

#include <sys/wait.h>
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <iostream>
#include <string>
#include <vector>

namespace testing {

struct Case {
  std::string name;
  std::function<void()> fn;
};

inline std::vector<Case>& cases() {
  static std::vector<Case> c;
  return c;
}
inline int& failures() {
  static int f = 0;
  return f;
}
struct Registrar {
  Registrar(const char* s, const char* n, std::function<void()> fn) {
    cases().push_back({std::string(s) + "." + n, std::move(fn)});
  }
};

inline void fail(const char* file, int line, const std::string& what) {
  ++failures();
  std::cerr << file << ":" << line << ": FAILED: " << what << "\n";
}

// runs fn in a child with stderr silenced; true if the child aborted / exited non-zero
inline bool dies(const std::function<void()>& fn) {
  std::fflush(nullptr);
  const pid_t pid = fork();
  if (pid == 0) {
    if (!std::freopen("/dev/null", "w", stderr)) std::_Exit(3);
    fn();
    std::_Exit(0);
  }
  int st = 0;
  waitpid(pid, &st, 0);
  return !(WIFEXITED(st) && WEXITSTATUS(st) == 0);
}

inline int runAll(int argc, char** argv) {
  const std::string filter = argc > 1 ? argv[1] : "";
  int ran = 0;
  for (auto& c : cases()) {
    if (!filter.empty() && c.name.find(filter) == std::string::npos) continue;
    const int before = failures();
    c.fn();
    ++ran;
    std::cout << (failures() == before ? "[ OK ] " : "[FAIL] ") << c.name << "\n";
  }
  std::cout << ran << " cases, " << failures() << " failed checks\n";
  return failures() == 0 ? 0 : 1;
}

}  // namespace testing

#define TEST(s, n)                                                              \
  static void test_##s##_##n();                                                 \
  static ::testing::Registrar reg_##s##_##n(#s, #n, test_##s##_##n);            \
  static void test_##s##_##n()

#define EXPECT_TRUE(c) \
  do { if (!(c)) ::testing::fail(__FILE__, __LINE__, #c); } while (0)
#define EXPECT_FALSE(c) EXPECT_TRUE(!(c))
#define EXPECT_EQ(a, b)                                                                 \
  do {                                                                                  \
    if (!((a) == (b))) ::testing::fail(__FILE__, __LINE__, #a " == " #b);               \
  } while (0)
#define EXPECT_NEAR(a, b, tol)                                                          \
  do {                                                                                  \
    if (!(std::fabs((double)(a) - (double)(b)) <= (tol)))                               \
      ::testing::fail(__FILE__, __LINE__,                                               \
                      std::string(#a " ~ " #b ": ") + std::to_string((double)(a)) +     \
                        " vs " + std::to_string((double)(b)));                          \
  } while (0)
#define EXPECT_DOUBLE_EQ(a, b) EXPECT_NEAR(a, b, 4 * 2.2e-16 * std::fabs((double)(b)) + 1e-300)
#define EXPECT_GT(a, b) EXPECT_TRUE((a) > (b))
#define EXPECT_DEATH(stmt) EXPECT_TRUE(::testing::dies([&] { stmt; }))
